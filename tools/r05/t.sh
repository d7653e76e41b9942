#!/bin/bash
# Round 5: the row pull on its resident grid (occupancy x CUs) -- parity of the pull paths, then config 4 / 5 / 3
# rounds with the default against the old fixed grid (row_grid 2048).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for C in 4 5; do
  for A in "" "t.row_grid=2048" ""; do
    timeout -k 10 300 python -u tools/round_profile.py $C $A > $O/rounds_c${C}.txt 2>&1 || { tail -20 $O/rounds_c${C}.txt; exit 1; }
    echo "== c$C $A"; grep -E "pull_light" $O/rounds_c${C}.txt | cut -c1-110
  done
done
timeout -k 10 300 python -u tools/sweep_small.py 3 - row_grid=2048 - row_grid=2048 > $O/sweep_c3.txt 2>&1 || { tail -20 $O/sweep_c3.txt; exit 1; }
cat $O/sweep_c3.txt
