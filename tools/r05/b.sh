#!/bin/bash
# Round 5, second call: config 2 / 3 step times under the small-kernel variants (scatter_small, bin sizes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 400 python -u tools/sweep_small.py 2 - scatter_small=1 bin_words=2048,scatter_small=1 bin_words=1024,scatter_small=1 bin_words=1024,bin_chunk=512,scatter_small=1 bin_words=2048 > $O/sweep_c2.txt 2>&1 || { tail -20 $O/sweep_c2.txt; exit 1; }
cat $O/sweep_c2.txt
timeout -k 10 400 python -u tools/sweep_small.py 3 - scatter_small=1 bin_words=2048,scatter_small=1 > $O/sweep_c3.txt 2>&1 || { tail -20 $O/sweep_c3.txt; exit 1; }
cat $O/sweep_c3.txt
