#!/bin/bash
# Round 4: streamed apply phase clocks (apply_probe) at config 4; scatter with the direct choice compiled out;
# churn with a small strided grid; partitioned --parts 8 A/B of scatter_direct.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04g}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread > $O/group.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/group.log | head -30; tail -5 $O/group.log; exit 1; }
tail -1 $O/group.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "stream or workload_parity or rejoin or apply_probe or blocked or deferred" > $O/parity.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 300 python3 -u tools/round_profile.py 4 t.apply_probe=1 > $O/rounds_c4_probe.txt 2>&1 || { tail -20 $O/rounds_c4_probe.txt; exit 1; }
grep -E "^(3|4|5|6|7) " $O/rounds_c4_probe.txt | cut -c1-400
timeout -k 10 300 python3 -u tools/round_profile.py 4 > $O/rounds_c4.txt 2>&1 || { tail -20 $O/rounds_c4.txt; exit 1; }
grep -E "^(5|6) " $O/rounds_c4.txt | cut -c1-160
timeout -k 10 300 python3 -u tools/round_profile.py 5 > $O/rounds_c5.txt 2>&1 || { tail -20 $O/rounds_c5.txt; exit 1; }
cut -c1-200 $O/rounds_c5.txt
for d in 0 1; do
  timeout -k 10 600 python -u bench.py --parts 8 --steps 3 --warmup 1 --no-cpu-baseline --tune scatter_direct=$d > $O/bench_p8_d$d.json 2> $O/bench_p8_d$d.err || { tail -20 $O/bench_p8_d$d.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_p8_d$d.json').read().splitlines()[-1]); r=d['roofline']; print('direct=$d', d['ms_per_step'], r.get('frac'), r.get('kernel_ms_per_step'), r.get('exchange_ms_per_step'))"
done
