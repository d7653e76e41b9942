#!/bin/bash
# Round 3: GPU suite, config-2/3 step times, config 4 rounds and bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/quick; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 -u tools/sweep_small.py 2 - > $O/sweep2.txt 2>&1 && cat $O/sweep2.txt || { tail $O/sweep2.txt; exit 1; }
timeout -k 10 300 python3 -u tools/sweep_small.py 3 - > $O/sweep3.txt 2>&1 && cat $O/sweep3.txt || { tail $O/sweep3.txt; exit 1; }
timeout -k 10 300 python3 -u tools/round_profile.py 4 > $O/rounds_c4.txt 2>&1 || { tail -20 $O/rounds_c4.txt; exit 1; }
cat $O/rounds_c4.txt
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $O/bench4.json 2> $O/bench4.err || { tail -20 $O/bench4.err; exit 1; }
cut -c1-300 $O/bench4.json
