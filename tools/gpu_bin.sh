#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bin
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "bin" > gpurun_out/bin/pytest.log 2>&1 || { tail -40 gpurun_out/bin/pytest.log; exit 1; }
tail -2 gpurun_out/bin/pytest.log
timeout -k 10 120 python -u tools/bin_probe.py 4 || exit 1
timeout -k 10 120 python -u tools/bin_probe.py 4 || exit 1
bash tools/sweep_env.sh - -
