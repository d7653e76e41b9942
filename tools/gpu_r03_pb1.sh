#!/bin/bash
# Round 3: propagation-blocked push -- full-size parity, then per-round profiles (blocked default vs off).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pb1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -k "blocked or auto" -x -v --timeout 300 --timeout-method thread > $O/full.log 2>&1 || { grep -E "PASS|FAIL|Error|assert|Timeout" $O/full.log | head -30; exit 1; }
grep -E "PASSED|passed" $O/full.log
for c in 4 5 3; do
  for b in auto off; do
    timeout -k 10 300 python3 -u tools/round_profile.py $c blocked=$b > $O/rounds_c${c}_$b.txt 2>&1 || { tail -20 $O/rounds_c${c}_$b.txt; exit 1; }
    echo "== config $c blocked=$b"; cat $O/rounds_c${c}_$b.txt
  done
done
