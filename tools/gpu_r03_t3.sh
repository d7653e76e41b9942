#!/bin/bash
# Round 3: small-overlay parity (tiny path on and off, hand graphs, config 1), then config 1/2 bench lines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "small_overlay or hand_graphs or workload_parity or surface or rebootstrap or rejoin or f10 or closed_form or reload" > gpurun_out/t3/pytest.log 2>&1 || { tail -40 gpurun_out/t3/pytest.log; exit 1; }
tail -2 gpurun_out/t3/pytest.log
for c in 1 2; do
  timeout -k 10 200 python3 -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); r=d.get('roofline',{})
        print('config', $c, d['ms_per_step'], d['value'], r.get('kernel_ms_per_step'))
" || exit 1
done
