#!/bin/bash
# Round 4: per-round profiles of configs 3 and 2 (kernel time per round), for the small-overlay costs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04r}; mkdir -p $O
for c in 3 2; do
  timeout -k 10 300 python3 -u tools/round_profile.py $c > $O/rounds_c$c.txt 2>&1 || { tail -20 $O/rounds_c$c.txt; exit 1; }
done
cut -c1-230 $O/rounds_c3.txt
python3 - $O/rounds_c2.txt <<'PY'
import ast, sys
tot = {}
for line in open(sys.argv[1]):
    parts = line.split(" ", 2)
    if len(parts) < 3 or not parts[0].isdigit():
        continue
    d = ast.literal_eval(parts[2][:parts[2].index("}") + 1])
    for k, v in d.items():
        tot[k] = round(tot.get(k, 0) + v, 3)
print("config 2 totals", tot, round(sum(tot.values()), 3))
PY
