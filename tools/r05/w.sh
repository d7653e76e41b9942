#!/bin/bash
# Round 5: configs 2 / 3 / 4, the heavy-row threshold (heavy_degree: rows above it pulled / pushed by chunks in
# launches of their own), step wall time with the arms alternated in one process.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 400 python -u tools/ab_kernel.py 2 step 3 - heavy_degree=1024 heavy_degree=4096 heavy_degree=100000 > $O/ab_c2.txt 2>&1 || { tail -20 $O/ab_c2.txt; exit 1; }
cat $O/ab_c2.txt
timeout -k 10 400 python -u tools/ab_kernel.py 3 step 3 - heavy_degree=1024 heavy_degree=4096 > $O/ab_c3.txt 2>&1 || { tail -20 $O/ab_c3.txt; exit 1; }
cat $O/ab_c3.txt
