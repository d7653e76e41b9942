#!/bin/bash
# GPU tests (one process, per-test timeout) then one default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${1:+-k "$1"} > gpurun_out/r2/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r2/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r2/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/r2/bench.json 2> gpurun_out/r2/bench.err || { tail -20 gpurun_out/r2/bench.err; exit 1; }
cat gpurun_out/r2/bench.json
