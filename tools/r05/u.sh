#!/bin/bash
# Round 5: the row pull's grid, arms alternated in one process (tools/ab_kernel.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 300 python -u tools/ab_kernel.py 4 pull_light 5 - row_grid=1024 row_grid=2048 row_grid=768 row_grid=1536 row_grid=512 > $O/ab_c4.txt 2>&1 || { tail -20 $O/ab_c4.txt; exit 1; }
cat $O/ab_c4.txt
timeout -k 10 300 python -u tools/ab_kernel.py 5 pull_light 5 - row_grid=1024 row_grid=2048 > $O/ab_c5.txt 2>&1 || { tail -20 $O/ab_c5.txt; exit 1; }
tail -3 $O/ab_c5.txt
