#!/bin/bash
# Round 3 A/B: the engine-variant parity tests for the variants named in $K, then
# per-round kernel times of config ${CFG:-4} once per env setting ("-" = defaults).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/var
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/var/pytest.log 2>&1 || { tail -30 gpurun_out/var/pytest.log; exit 1; }
  tail -2 gpurun_out/var/pytest.log
fi
bash tools/gpu_rounds_env.sh "$@"
