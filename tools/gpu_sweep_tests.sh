#!/bin/bash
# usage: gpu_sweep_tests.sh "<pytest -k expr or ->" "<ENV1>" "<ENV2>" ...
# A pytest subset (one process), then the default bench once per env setting (tools/sweep_env.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/st
K="$1"; shift
if [ "$K" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/st/pytest.log 2>&1 || { tail -40 gpurun_out/st/pytest.log; exit 1; }
  tail -2 gpurun_out/st/pytest.log
fi
tools/sweep_env.sh "$@"
