#!/bin/bash
# Round 4: apply_pipe 2 by default, a deeper shape 3, production apply without probe code; A/B and bench lines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04n}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "variants or workload_parity" > $O/parity.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in 2 3 2 3; do
  timeout -k 10 300 python3 -u tools/round_profile.py 4 t.apply_pipe=$v > $O/rounds_c4_pipe$v.txt 2>&1 || { tail -20 $O/rounds_c4_pipe$v.txt; exit 1; }
  echo "== apply_pipe $v"; grep -E "^(5|6) " $O/rounds_c4_pipe$v.txt | cut -c1-120
done
for c in 2 3 5 4; do
  timeout -k 10 400 python3 -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c$c.json 2> $O/bench_c$c.err || { tail -20 $O/bench_c$c.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_c$c.json').read().splitlines()[-1]);r=d['roofline'];print($c, d['value'], 'GTEPS', d['ms_per_step'], 'ms', 'frac', r.get('frac'), 'step', r.get('step_frac'))"
done
