#!/bin/bash
# Round 5: after the empty-trailing-chunk fix -- the group case with torch loaded, then f.sh (partitioned tests,
# config 4 as 8 parts round by round, the --parts 8 line, the full-size partitioned fixtures).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_partitioned.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/c_torch.log 2>&1 || { grep -E "\[gossip\]|Error" $O/c_torch.log | head; tail -5 $O/c_torch.log; exit 1; }
tail -1 $O/c_torch.log
bash tools/r05/f.sh
