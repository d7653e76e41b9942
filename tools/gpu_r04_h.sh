#!/bin/bash
# Round 4: churn drawn per quad of peers (config 5 fixture regenerated), persistent streamed apply
# (apply_persist) -- parity (variants, workloads, tiny overlays, surface, full size), config 4 A/B of the
# apply, config 5 profile, bench lines of configs 4 and 5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04h}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_surface.py -x -q --timeout 200 --timeout-method thread -k "variants or workload_parity or small_overlay or rejoin or liveness or reload or surface or cli" > $O/parity.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread > $O/group.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/group.log | head -30; tail -5 $O/group.log; exit 1; }
tail -1 $O/group.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 500 --timeout-method thread -k "auto_matches_oracle or group_matches_oracle" > $O/full.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/full.log | head -30; tail -5 $O/full.log; exit 1; }
tail -1 $O/full.log
for v in 1 0; do
  timeout -k 10 300 python3 -u tools/round_profile.py 4 t.apply_persist=$v t.apply_probe=1 > $O/rounds_c4_p$v.txt 2>&1 || { tail -20 $O/rounds_c4_p$v.txt; exit 1; }
  echo "== apply_persist $v"; grep -E "^(5|6) " $O/rounds_c4_p$v.txt | cut -c1-330
done
timeout -k 10 300 python3 -u tools/round_profile.py 5 > $O/rounds_c5.txt 2>&1 || { tail -20 $O/rounds_c5.txt; exit 1; }
cut -c1-200 $O/rounds_c5.txt
for c in 5 4; do
  timeout -k 10 400 python3 -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c$c.json 2> $O/bench_c$c.err || { tail -20 $O/bench_c$c.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_c$c.json').read().splitlines()[-1]);r=d['roofline'];print($c, d['value'], 'GTEPS', d['ms_per_step'], 'ms', 'frac', r.get('frac'), 'step', r.get('step_frac'), r.get('kernel_ms_per_step'))"
done
timeout -k 10 600 python -u bench.py --parts 8 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_p8.json 2> $O/bench_p8.err || { tail -20 $O/bench_p8.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_p8.json').read().splitlines()[-1]); r=d['roofline']; print('P=8', d['ms_per_step'], r.get('frac'), r.get('kernel_ms_per_step'), r.get('exchange_ms_per_step'))"
