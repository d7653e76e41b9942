#!/bin/bash
# Round 4: BinArgs filled field by field (the tuning keys apply_pipe / scatter_direct / src_stats now reach
# the kernels) -- parity of the variants, then A/B of apply_pipe at config 4 and scatter_direct at P = 8.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04m}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread -k "variants or dense_exchange or workload_parity" > $O/parity.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in 0 1 2 3 0; do
  timeout -k 10 300 python3 -u tools/round_profile.py 4 t.apply_pipe=$v > $O/rounds_c4_pipe$v.txt 2>&1 || { tail -20 $O/rounds_c4_pipe$v.txt; exit 1; }
  echo "== apply_pipe $v"; grep -E "^(5|6) " $O/rounds_c4_pipe$v.txt | cut -c1-120
done
timeout -k 10 300 python3 -u tools/round_profile.py 4 t.src_stats=0 > $O/rounds_c4_src0.txt 2>&1 || { tail -20 $O/rounds_c4_src0.txt; exit 1; }
echo "== src_stats 0"; grep -E "^(5|6) " $O/rounds_c4_src0.txt | cut -c1-120
for d in 0 1; do
  timeout -k 10 600 python -u bench.py --parts 8 --steps 3 --warmup 1 --no-cpu-baseline --tune scatter_direct=$d > $O/bench_p8_d$d.json 2> $O/bench_p8_d$d.err || { tail -20 $O/bench_p8_d$d.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_p8_d$d.json').read().splitlines()[-1]); r=d['roofline']; print('direct=$d', d['ms_per_step'], r.get('kernel_ms_per_step',{}).get('bin_scatter'), r.get('kernel_ms_per_step',{}).get('bin_apply'))"
done
