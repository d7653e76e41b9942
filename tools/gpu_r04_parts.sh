#!/bin/bash
# Round 4: the partitioned driver at full size on one GPU -- the P = 8 parity test, then
# bench.py --parts 2/4/8 lines (config 4).  $1 = output dir under gpurun_out, $2 = "test" to run the test.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-parts}; mkdir -p $O
if [ "$2" = test ]; then
  timeout -k 10 900 python -u -m pytest "tests/test_gpu_fullsize.py::test_fullsize_partitioned_group_matches_oracle[4-8]" -x -v --timeout 880 --timeout-method thread > $O/p8test.log 2>&1 || { tail -30 $O/p8test.log; exit 1; }
  tail -2 $O/p8test.log
fi
for P in ${PARTS:-8 4 2}; do
  timeout -k 10 600 python -u bench.py --parts $P --steps 5 --warmup 1 > $O/bench_parts$P.json 2> $O/bench_parts$P.err || { tail -20 $O/bench_parts$P.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_parts$P.json').read().splitlines()[-1]); print($P, d['ms_per_step'], d['value'], d['roofline'].get('exchange_ms_per_step'), d['roofline'].get('exchange_gb_per_step'))"
done
