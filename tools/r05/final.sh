#!/bin/bash
# Round 5 end: smoke(), the GPU suite (skip reasons on record: -rs), bench lines of every config, config 4 and 5
# profiles (kernel trace + PMC passes), and the --parts 2/4/8 lines.  $1 = HEAD commit.  STAGES picks parts.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
H=${1:-unknown}
O=gpurun_out/final_r05; mkdir -p $O
S=${STAGES:-suite bench prof parts}
if [[ $S == *suite* ]]; then
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rs --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
  grep -E "SKIPPED" $O/pytest.log | head -8
  tail -1 $O/pytest.log
fi
if [[ $S == *bench* ]]; then
  nproc > $O/nproc.txt; lscpu > $O/lscpu.txt 2>&1 || true
  for c in ${CONFIGS:-1 2 3 5 4}; do
    timeout -k 10 400 python3 -u bench.py --config $c > $O/bench_config$c.json 2> $O/bench_config$c.err || { tail -20 $O/bench_config$c.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/bench_config$c.json').read().splitlines()[-1]);r=d['roofline'];print($c, d['config']['workload'], d['value'], 'GTEPS', d['ms_per_step'], 'ms', 'frac', r.get('frac'), 'step', r.get('step_frac'), 'cpu', d.get('cpu_baseline',{}).get('value'))"
  done
fi
if [[ $S == *prof* ]]; then
  for c in 4 5; do
    bash tools/r05/profile.sh $c $H > $O/prof_c$c.log 2>&1 || { tail -20 $O/prof_c$c.log; exit 1; }
    tail -16 $O/prof_c$c.log | cut -c1-200
  done
fi
if [[ $S == *parts* ]]; then
  for P in 8 4 2; do
    timeout -k 10 600 python -u bench.py --parts $P --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_parts$P.json 2> $O/bench_parts$P.err || { tail -20 $O/bench_parts$P.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_parts$P.json').read().splitlines()[-1]); r=d['roofline']; print($P, d['ms_per_step'], d['value'], r.get('frac'), sum(r.get('kernel_ms_per_step').values()), r.get('exchange_ms_per_step'), r.get('exchange_link_ms_per_step'), r.get('projected_ms_per_step'))"
  done
fi
