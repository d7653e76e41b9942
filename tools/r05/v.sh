#!/bin/bash
# Round 5: configs 2 and 3, source chunk and bin sizes, step wall time with the arms alternated in one process.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 400 python -u tools/ab_kernel.py 2 step 3 - bin_chunk=1024 bin_chunk=1536 bin_chunk=4096 bin_words=1024 bin_words=4096 bin_chunk=1024,bin_words=4096 > $O/ab_c2.txt 2>&1 || { tail -20 $O/ab_c2.txt; exit 1; }
cat $O/ab_c2.txt
timeout -k 10 400 python -u tools/ab_kernel.py 3 step 3 - bin_chunk=2048 bin_chunk=8192 bin_words=9216 > $O/ab_c3.txt 2>&1 || { tail -20 $O/ab_c3.txt; exit 1; }
cat $O/ab_c3.txt
