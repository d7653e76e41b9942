#!/bin/bash
# Round 3: blocked push (static segments) -- small forced run, parity subset, config 4/5/3 round profiles.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pb3; mkdir -p $O
timeout -k 10 90 python3 -u tools/pb_debug.py 2 65536 force > $O/dbg.log 2>&1 || { tail -30 $O/dbg.log; exit 1; }
tail -3 $O/dbg.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "blocked" -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { grep -E "FAIL|Error|assert" $O/parity.log | head -30; exit 1; }
tail -1 $O/parity.log
for c in 4 5 3; do
  timeout -k 10 300 python3 -u tools/round_profile.py $c > $O/rounds_c$c.txt 2>&1 || { tail -20 $O/rounds_c$c.txt; exit 1; }
  echo "== config $c"; cat $O/rounds_c$c.txt
done
