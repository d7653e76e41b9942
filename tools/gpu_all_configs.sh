#!/bin/bash
# One bench line per BASELINE.json config (1, 2, 3, 5, 4), each with its CPU baseline legs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/allcfg
mkdir -p $O
nproc > $O/nproc.txt; lscpu > $O/lscpu.txt 2>&1 || true
for c in 1 2 3 5 4; do
    timeout -k 10 400 python3 -u bench.py --config $c --cpu-repeats ${REPS:-3} > $O/c$c.json 2> $O/c$c.err || { tail -20 $O/c$c.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c$c.json'));print($c, d['config']['workload'], d['value'], 'GTEPS', d['ms_per_step'], 'ms', 'cpu', d.get('cpu_baseline',{}).get('value'))"
done
