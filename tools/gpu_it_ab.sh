#!/bin/bash
# GPU parity suite, then the A/B bench (abtest/base vs current).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/it
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/it/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/it/pytest_gpu.log
bash tools/gpu_ab.sh
