#!/bin/bash
# Round 4: level 1 of the blocked rounds with two buffers per coarse bin (160 bins) -- staging test, blocked
# parity, full-size forced-blocked parity, config 4's default schedule at full size, per-round profile.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04e}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stage.py -x -q --timeout 120 --timeout-method thread > $O/stage.log 2>&1 || { tail -30 $O/stage.log; exit 1; }
tail -1 $O/stage.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "blocked or deferred" > $O/parity.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 900 python -u -m pytest "tests/test_gpu_fullsize.py::test_fullsize_forced_blocked_matches_oracle" "tests/test_gpu_fullsize.py::test_fullsize_auto_matches_oracle[4]" -x -q --timeout 500 --timeout-method thread > $O/full.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/full.log | head -30; tail -5 $O/full.log; exit 1; }
tail -1 $O/full.log
timeout -k 10 300 python3 -u tools/round_profile.py 4 > $O/rounds_c4.txt 2>&1 || { tail -20 $O/rounds_c4.txt; exit 1; }
cat $O/rounds_c4.txt | cut -c1-160
timeout -k 10 300 python3 -u tools/round_profile.py 5 > $O/rounds_c5.txt 2>&1 || { tail -20 $O/rounds_c5.txt; exit 1; }
cat $O/rounds_c5.txt | cut -c1-160
