#!/bin/bash
# Round 5: fused heavy pull with one chunk per claim -- config 2 step times, fused against separate.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 400 python -u tools/sweep_small.py 2 - heavy_fuse=0 - heavy_fuse=0 > $O/sweep_c2.txt 2>&1 || { tail -20 $O/sweep_c2.txt; exit 1; }
cat $O/sweep_c2.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c2 -o run -- python3 -u tools/sweep_small.py 2 - > $O/trace_run.txt 2>&1 || { tail -20 $O/trace_run.txt; exit 1; }
python3 tools/kernel_gaps.py $O/c2 0.5 | head -20
