#!/bin/bash
# Round 5: where configs 2 and 3 spend a step -- kernel traces of the bench (no per-kernel events), the busy time
# and the gaps between kernels over the timed steps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05i; mkdir -p $O
for C in 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c$C -o run -- python3 -u bench.py --config $C --no-cpu-baseline --no-timing --steps 5 --warmup 1 > $O/bench_c$C.json 2> $O/bench_c$C.err || { tail -20 $O/bench_c$C.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_c$C.json').read().splitlines()[-1]); print($C, d['ms_per_step'], d['config'].get('rounds_per_step'))"
  python3 tools/kernel_gaps.py $O/c$C 0.66 > $O/gaps_c$C.txt && head -30 $O/gaps_c$C.txt
done
