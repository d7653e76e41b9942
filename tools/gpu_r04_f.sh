#!/bin/bash
# Round 4: partitioned runs -- scatter_direct parity (groups) and --parts 8 A/B of it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04f}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread -k "dense_exchange" > $O/group.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/group.log | head -30; tail -5 $O/group.log; exit 1; }
tail -1 $O/group.log
for d in 0 1; do
  timeout -k 10 600 python -u bench.py --parts 8 --steps 3 --warmup 1 --tune scatter_direct=$d > $O/bench_p8_d$d.json 2> $O/bench_p8_d$d.err || { tail -20 $O/bench_p8_d$d.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_p8_d$d.json').read().splitlines()[-1]); print('direct=$d', d['ms_per_step'], d['roofline'].get('kernel_ms_per_step',{}).get('bin_scatter'), d['roofline'].get('exchange_ms_per_step'))"
done
