#!/bin/bash
# Round 4, second GPU pass: staging protocol (three geometries); blocked, group (compact dense exchange), replay
# and ADVICE parity; world-N ranks on one GPU (RCCL); config 4 per-round profile; the two bin layouts at
# configs 3, 5 and 4; config 2 with and without the recorded-schedule replay.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04b}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stage.py -x -q --timeout 120 --timeout-method thread > $O/stage.log 2>&1 || { tail -30 $O/stage.log; exit 1; }
tail -1 $O/stage.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread -k "blocked or deferred or group or replay or heavy_degree or list_cap or tuning_rejects" > $O/parity.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiprocess.py -x -v --timeout 200 --timeout-method thread > $O/mp.log 2>&1; tail -8 $O/mp.log
timeout -k 10 600 python -u -m pytest "tests/test_gpu_fullsize.py::test_fullsize_forced_blocked_matches_oracle" -x -q --timeout 500 --timeout-method thread > $O/full.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/full.log | head -30; tail -5 $O/full.log; exit 1; }
tail -1 $O/full.log
timeout -k 10 300 python3 -u tools/round_profile.py 4 > $O/rounds_c4.txt 2>&1 || { tail -20 $O/rounds_c4.txt; exit 1; }
head -8 $O/rounds_c4.txt
timeout -k 10 300 python3 -u tools/sweep_small.py 2 replay=0 - replay=0 - > $O/sweep2.txt 2>&1 && cat $O/sweep2.txt || { tail $O/sweep2.txt; exit 1; }
for c in 3 5; do
  timeout -k 10 400 python3 -u tools/sweep_small.py $c bin_stream=0 bin_stream=1 bin_stream=0 bin_stream=1 > $O/sweep$c.txt 2>&1 && cat $O/sweep$c.txt || { tail $O/sweep$c.txt; exit 1; }
done
timeout -k 10 600 python3 -u tools/sweep_small.py 4 bin_stream=0 bin_stream=1 > $O/sweep4.txt 2>&1 && cat $O/sweep4.txt || { tail $O/sweep4.txt; exit 1; }
