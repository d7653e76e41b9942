#!/bin/bash
# Round 4, first GPU pass: the staging protocol test, the blocked-round and ADVICE parity tests, config 4's
# per-round profile (blocked rounds 3-4 with the double-buffered staging; dense rounds in both bin layouts),
# then the P = 8 full-size group test and bench.py --parts 8/4/2 lines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04a}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stage.py -x -q --timeout 120 --timeout-method thread > $O/stage.log 2>&1 || { tail -30 $O/stage.log; exit 1; }
tail -1 $O/stage.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "blocked or deferred or heavy_degree or list_cap or tuning_rejects or needy" > $O/parity.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 600 python -u -m pytest "tests/test_gpu_fullsize.py::test_fullsize_forced_blocked_matches_oracle" "tests/test_gpu_fullsize.py::test_fullsize_auto_matches_oracle[4]" -x -q --timeout 500 --timeout-method thread > $O/full.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/full.log | head -30; tail -5 $O/full.log; exit 1; }
tail -1 $O/full.log
timeout -k 10 300 python3 -u tools/round_profile.py 4 > $O/rounds_c4.txt 2>&1 || { tail -20 $O/rounds_c4.txt; exit 1; }
cat $O/rounds_c4.txt
timeout -k 10 300 python3 -u tools/round_profile.py 4 t.bin_stream=1 > $O/rounds_c4_stream.txt 2>&1 || { tail -20 $O/rounds_c4_stream.txt; exit 1; }
cat $O/rounds_c4_stream.txt
bash tools/gpu_r04_parts.sh $1/parts test
