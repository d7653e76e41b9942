#!/bin/bash
# Round 4: the streamed apply's pipeline shapes at config 4 (alternated per-round profiles) and their parity.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04d}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "apply_pipe or needy_test or stream or slots" > $O/parity.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for rep in 1 2; do
  for v in 0 1 2 3; do
    timeout -k 10 300 python3 -u tools/round_profile.py 4 t.apply_pipe=$v > $O/rounds_p$v.txt 2>&1 || { tail -20 $O/rounds_p$v.txt; exit 1; }
    echo "== apply_pipe $v"; sed -n 6,7p $O/rounds_p$v.txt | cut -c1-120
  done
done
