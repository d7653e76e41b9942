#!/bin/bash
# Round 3: the whole GPU suite, then bench lines of configs 1 and 2 (no CPU baseline).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t2/pytest.log 2>&1 || { tail -40 gpurun_out/t2/pytest.log; exit 1; }
tail -2 gpurun_out/t2/pytest.log
for c in 1 2; do
  timeout -k 10 200 python3 -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); r=d.get('roofline',{})
        print('config', $c, d['ms_per_step'], d['value'], r.get('kernel_ms_per_step'))
" || exit 1
done
GOSSIP_BIN_STREAM=1 timeout -k 10 200 python3 -u bench.py --config 2 --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); r=d.get('roofline',{})
        print('config 2 stream', d['ms_per_step'], d['value'], r.get('kernel_ms_per_step'))
"
