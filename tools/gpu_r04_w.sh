#!/bin/bash
# Round 4: configs 4 and 5 -- the binned/pull switch (bin_permille).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04w}; mkdir -p $O
tot() {
python3 - $1 <<'PY'
import ast, sys
tot = {}
modes = []
for line in open(sys.argv[1]):
    parts = line.split(" ", 2)
    if len(parts) < 3 or not parts[0].isdigit():
        continue
    d = ast.literal_eval(parts[2][:parts[2].index("}") + 1])
    modes.append("b" if "bin_scatter" in d else "p" if ("pull_light" in d or "pull_list" in d) else "B" if "pb_scatter" in d else "s")
    for k, v in d.items():
        tot[k] = round(tot.get(k, 0) + v, 3)
print(sys.argv[1].split("/")[-1], round(sum(tot.values()), 3), "".join(modes), tot)
PY
}
for c in 4 5; do
  for a in bin_permille=4000 bin_permille=8000 bin_permille=16000 bin_permille=32000; do
    timeout -k 10 300 python3 -u tools/round_profile.py $c $a > $O/rounds_c${c}_$a.txt 2>&1 || { tail -20 $O/rounds_c${c}_$a.txt; exit 1; }
    tot $O/rounds_c${c}_$a.txt | cut -c1-260
  done
done
