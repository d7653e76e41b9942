"""Sum per-kernel ms over the rounds of each block of tools/gpu_rounds_env.sh output."""
import ast
import sys
from collections import defaultdict

tot, name = None, None
for line in open(sys.argv[1]):
    if line.startswith("== "):
        if tot is not None:
            print(name, {k: round(v, 3) for k, v in tot.items()}, "sum", round(sum(tot.values()), 3))
        name, tot = line.strip(), defaultdict(float)
    elif tot is not None and " F=" in line and "{" in line:
        d = ast.literal_eval(line[line.index("{"):line.index("}") + 1])
        for k, v in d.items():
            tot[k] += v
if tot is not None:
    print(name, {k: round(v, 3) for k, v in tot.items()}, "sum", round(sum(tot.values()), 3))
