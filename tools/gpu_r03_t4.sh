#!/bin/bash
# Round 3: whole GPU suite on the size-aware layout / pull-threshold defaults, then bench lines of configs 1-5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t4/pytest.log 2>&1 || { tail -40 gpurun_out/t4/pytest.log; exit 1; }
tail -2 gpurun_out/t4/pytest.log
for c in 1 2 3 5 4; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/t4/bench_c$c.json 2> gpurun_out/t4/bench_c$c.err || exit 1
  python3 -c "
import json,sys
for l in open('gpurun_out/t4/bench_c$c.json'):
    if l.startswith('{'):
        d=json.loads(l); r=d.get('roofline',{})
        print('config', $c, d['ms_per_step'], d['value'], r.get('frac'), r.get('kernel_ms_per_step'))
"
done
