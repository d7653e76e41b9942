#!/bin/bash
# The engine-variant parity tests (-k filter $K, default "variants"), then per-round kernel
# times once per env setting given as arguments ("-" = defaults).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/var
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "${K:-variants}" > gpurun_out/var/pytest.log 2>&1 || { tail -30 gpurun_out/var/pytest.log; exit 1; }
tail -2 gpurun_out/var/pytest.log
bash tools/gpu_rounds_env.sh "$@"
