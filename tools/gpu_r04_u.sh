#!/bin/bash
# Round 4: 16-wave apply workgroups when bins <= CUs (config 2), parity; config 2 kernel totals and bench;
# the compact all-gather's exchange bytes at P = 8 against whole slices (gather_permille 0).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04u}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "variants or workload_parity or multiword or hand_graphs" > $O/parity.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 300 python3 -u tools/round_profile.py 2 > $O/rounds_c2.txt 2>&1 || { tail -20 $O/rounds_c2.txt; exit 1; }
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
print("config 2 kernel totals", round(sum(tot.values()), 3), tot)
PY
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config 2 --steps 20 --warmup 3 --no-cpu-baseline --no-timing > $O/bench_c2_$i.json 2> $O/bench_c2_$i.err || { tail -20 $O/bench_c2_$i.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_c2_$i.json').read().splitlines()[-1]);print('config 2', d['ms_per_step'])"
done
for g in 0 600; do
  timeout -k 10 600 python -u bench.py --parts 8 --steps 3 --warmup 1 --no-cpu-baseline --tune gather_permille=$g > $O/bench_p8_g$g.json 2> $O/bench_p8_g$g.err || { tail -20 $O/bench_p8_g$g.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_p8_g$g.json').read().splitlines()[-1]); r=d['roofline']; print('gather_permille=$g', d['ms_per_step'], r.get('exchange_ms_per_step'), r.get('exchange_gb_per_step'))"
done
