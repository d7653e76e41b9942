#!/bin/bash
# One GPU call: the GPU test suite, the default bench line, then per-round
# kernel times once per env setting given as arguments ("-" = defaults).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/state
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/state/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/state/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/state/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/state/bench.json 2> gpurun_out/state/bench.err || { tail -20 gpurun_out/state/bench.err; exit 1; }
cat gpurun_out/state/bench.json
[ $# -gt 0 ] && bash tools/gpu_rounds_env.sh "$@"
exit 0
