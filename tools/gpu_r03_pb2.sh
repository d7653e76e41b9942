#!/bin/bash
# Round 3: blocked-push debugging -- one small forced run round by round, then the parity subset.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pb2; mkdir -p $O
timeout -k 10 90 python3 -u tools/pb_debug.py 2 65536 force > $O/dbg.log 2>&1; rc=$?
cat $O/dbg.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "blocked" -x -v --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/parity.log | head -40; exit 1; }
grep -cE "PASSED" $O/parity.log
