#!/bin/bash
# Round 5: a reset after list rounds clears only the last two rounds' list and heavy rows of nw / nx -- the GPU
# suite, then configs 4 and 3 twice each (every replayed step's stats are checked against the recording).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ah; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rs --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in 4 3 4 3; do
  timeout -k 10 300 python3 -u bench.py --config $c --no-cpu-baseline > $O/bench_c$c.json 2> $O/bench_c$c.err || { tail -20 $O/bench_c$c.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_c$c.json').read().splitlines()[-1]);r=d['roofline'];print($c, d['ms_per_step'], d['value'], r.get('frac'), r.get('step_frac'))"
done
