#!/bin/bash
# Round 4 close: smoke(), the GPU suite, and the driver's own bench command on HEAD.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04v}; mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().splitlines()[-1]);r=d['roofline'];print(d['value'], 'GTEPS', d['ms_per_step'], 'ms', 'frac', r.get('frac'), 'traffic', r.get('traffic'), 'cpu', d.get('cpu_baseline',{}).get('value'))"
