#!/bin/bash
# Round 5: the small-overlay single-launch run with the injected-message mask in LDS -- parity of the tiny
# path and config 1's line (its tiny kernel was 0.187 ms per run, 47 rounds).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05af; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_surface.py -k "small_overlay or tiny or golden" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --config 1 --no-cpu-baseline --steps 50 --warmup 5 > $O/bench_c1_$i.json 2> $O/bench_c1_$i.err || { tail -20 $O/bench_c1_$i.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_c1_$i.json').read().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'], r['kernel_ms_per_step'], r['avg_launch_ms'])"
done
