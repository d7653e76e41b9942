#!/bin/bash
# Round 3 E6: full-step bench (no CPU baseline) of configs 3, 5, 4, default layout vs streamed layout, alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in 3 5 4; do
  for v in - GOSSIP_BIN_STREAM=1 - GOSSIP_BIN_STREAM=1; do
    [ "$v" = "-" ] && v=""
    echo "== config $c [$v]"
    env $v timeout -k 10 200 python3 -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); r=d.get('roofline',{})
        print(d['ms_per_step'], d['value'], r.get('frac'), r.get('kernel_ms_per_step'))
    else: print(l.rstrip()[:200])
" || exit 1
  done
done
