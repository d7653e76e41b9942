#!/bin/bash
# Round 3: three processes of the default bench (the scatter's speed depends on the slot array's pages).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bench3; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $O/b$i.json 2> $O/b$i.err || { tail -20 $O/b$i.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b$i.json').readline());k=d['roofline']['kernel_ms_per_step'];print($i, d['ms_per_step'], d['value'], 'scatter', round(k['bin_scatter']/2,3), 'apply', round(k['bin_apply']/2,3))"
done
