#!/bin/bash
# Round 3: needy-list rounds first, then the whole GPU suite, config 4/3 round profiles and the bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/list; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "needy_list or deferred_round_fold or blocked_push" --timeout 120 --timeout-method thread > $O/pytest_list.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/pytest_list.log | head -30; tail -30 $O/pytest_list.log; exit 1; }
tail -2 $O/pytest_list.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for c in 4 3; do
  timeout -k 10 300 python3 -u tools/round_profile.py $c > $O/rounds_c$c.txt 2>&1 || { tail -20 $O/rounds_c$c.txt; exit 1; }
  echo "== config $c"; cat $O/rounds_c$c.txt
done
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $O/bench4.json 2> $O/bench4.err || { tail -20 $O/bench4.err; exit 1; }
cut -c1-300 $O/bench4.json
