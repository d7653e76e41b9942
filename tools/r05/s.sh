#!/bin/bash
# Round 5: config 4's row pull (round 7) under queue and grid variants, round profiles alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "pull" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
i=0
for A in "" "t.row_queue=256" "t.row_grid=1024" "t.row_grid=1024 t.row_queue=256" "" "t.row_queue=256" "t.row_grid=1024"; do
  i=$((i+1))
  timeout -k 10 300 python -u tools/round_profile.py 4 $A > $O/rounds_$i.txt 2>&1 || { tail -20 $O/rounds_$i.txt; exit 1; }
  echo "== $A"; grep -E "^7 " $O/rounds_$i.txt | cut -c1-120
done
