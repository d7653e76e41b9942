#!/bin/bash
# The GPU test suite alone (one process, per-test timeout).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${1:+-k "$1"} > gpurun_out/tests/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/tests/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/tests/pytest_gpu.log
