#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rb
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/rb/pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/rb/pytest.log | tail -30; exit 1; }
tail -3 gpurun_out/rb/pytest.log
bash tools/sweep_env.sh -
