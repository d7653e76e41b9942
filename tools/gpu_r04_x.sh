#!/bin/bash
# Round 4: a replayed run's stat lines go to the history through the zero batch (no copy launch per round):
# replay parity, config 2 and 3 bench lines alternated with the replay off.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04x}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "replay or workload_parity or variants or auto_matches_oracle" > $O/parity.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for r in 1 0 1 0; do
  for c in 2 3; do
    timeout -k 10 300 python3 -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-timing --tune replay=$r > $O/bench_c${c}_r$r.json 2> $O/bench_c${c}_r$r.err || { tail -20 $O/bench_c${c}_r$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/bench_c${c}_r$r.json').read().splitlines()[-1]);print('config $c replay $r', d['ms_per_step'])"
  done
done
