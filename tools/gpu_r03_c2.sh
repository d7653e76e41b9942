#!/bin/bash
# Round 3: config 2 schedule sweep (push/pull switch point) in both binned layouts.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in - GOSSIP_BIN_STREAM=1; do
  for pp in 0 60 110 200; do
    [ "$v" = "-" ] && e="" || e="$v"
    env $e timeout -k 10 200 python3 -u bench.py --config 2 --steps 20 --warmup 3 --no-cpu-baseline --pull-permille $pp 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); r=d.get('roofline',{})
        print('[$v] pull_pm $pp', d['ms_per_step'], d['value'], {k: v for k, v in r.get('kernel_ms_per_step', {}).items()})
" || exit 1
  done
done
