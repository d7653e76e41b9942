#!/bin/bash
# Round 5: config 4 (and 5), the heavy-row threshold (heavy_degree), step wall time, arms alternated in one process.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ab; mkdir -p $O
timeout -k 10 500 python -u tools/ab_kernel.py 4 step 2 - heavy_degree=512 heavy_degree=1024 heavy_degree=128 > $O/ab_c4.txt 2>&1 || { tail -20 $O/ab_c4.txt; exit 1; }
cat $O/ab_c4.txt
timeout -k 10 300 python -u tools/ab_kernel.py 5 step 2 - heavy_degree=512 heavy_degree=1024 > $O/ab_c5.txt 2>&1 || { tail -20 $O/ab_c5.txt; exit 1; }
cat $O/ab_c5.txt
