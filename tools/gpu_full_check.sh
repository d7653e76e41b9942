#!/bin/bash
# One GPU call: the whole GPU test suite, then the bench line of each config given
# (default: 4), without the CPU baseline unless CPUB=1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/full
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/full/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/full/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/full/pytest_gpu.log
for c in ${@:-4}; do
  timeout -k 10 400 python -u bench.py --config $c ${CPUB:+} $([ "${CPUB:-0}" = 1 ] || echo --no-cpu-baseline) > gpurun_out/full/bench_c$c.json 2> gpurun_out/full/bench_c$c.err || { tail -20 gpurun_out/full/bench_c$c.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/full/bench_c$c.json')); print($c, d['value'], d['unit'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step'))"
done
