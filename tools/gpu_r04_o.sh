#!/bin/bash
# Round 4: config 2 A/B -- persistent apply on/off, alternated; per-round profile of each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04o}; mkdir -p $O
for v in 1 0 1 0; do
  timeout -k 10 300 python3 -u bench.py --config 2 --steps 20 --warmup 3 --no-cpu-baseline --no-timing --tune apply_persist=$v > $O/bench_c2_p$v.json 2> $O/bench_c2_p$v.err || { tail -20 $O/bench_c2_p$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_c2_p$v.json').read().splitlines()[-1]);print('persist $v', d['ms_per_step'])"
done
for v in 1 0; do
  timeout -k 10 300 python3 -u tools/round_profile.py 2 t.apply_persist=$v > $O/rounds_c2_p$v.txt 2>&1 || { tail -20 $O/rounds_c2_p$v.txt; exit 1; }
  python3 - $O/rounds_c2_p$v.txt <<'PY'
import ast, sys
tot = {}
for line in open(sys.argv[1]):
    parts = line.split(" ", 2)
    if len(parts) < 3 or not parts[0].isdigit():
        continue
    d = ast.literal_eval(parts[2][:parts[2].index("}") + 1])
    for k, v in d.items():
        tot[k] = round(tot.get(k, 0) + v, 3)
print(sys.argv[1].split("/")[-1], tot, round(sum(tot.values()), 3))
PY
done
