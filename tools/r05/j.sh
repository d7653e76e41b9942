#!/bin/bash
# Round 5: small-overlay scatter units split over the grid (scatter_units, scatter_split_direct) and the 16-wave
# small-bin apply (apply_wide): parity variants, then config 2 / 3 step times, arms alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "split_units or apply_wide" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
V2="- scatter_units=1024 scatter_units=2048 scatter_units=2048,scatter_split_direct=1 scatter_units=4096,scatter_small=1 scatter_units=4096,scatter_small=1,scatter_split_direct=1 apply_wide=1 apply_wide=1,scatter_units=2048,scatter_split_direct=1"
timeout -k 10 500 python -u tools/sweep_small.py 2 $V2 $V2 > $O/sweep_c2.txt 2>&1 || { tail -20 $O/sweep_c2.txt; exit 1; }
cat $O/sweep_c2.txt
V3="- scatter_units=8192 scatter_units=8192,scatter_split_direct=1"
timeout -k 10 400 python -u tools/sweep_small.py 3 $V3 $V3 > $O/sweep_c3.txt 2>&1 || { tail -20 $O/sweep_c3.txt; exit 1; }
cat $O/sweep_c3.txt
