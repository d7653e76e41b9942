#!/bin/bash
# Binned-round parity tests, then a bench sweep (sweep_env.sh arguments).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/quick
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bin or full or rebootstrap" > gpurun_out/quick/pytest.log 2>&1 || { tail -30 gpurun_out/quick/pytest.log; exit 1; }
tail -2 gpurun_out/quick/pytest.log
bash tools/sweep_env.sh "$@"
