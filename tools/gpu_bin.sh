#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c5
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_partitioned.py -x -q --timeout 120 --timeout-method thread -k "rebootstrap" > gpurun_out/c5/pytest.log 2>&1 || { tail -30 gpurun_out/c5/pytest.log; exit 1; }
tail -2 gpurun_out/c5/pytest.log
timeout -k 10 300 python -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --rebootstrap 8 > gpurun_out/c5/c5rb.json 2> gpurun_out/c5/c5rb.err || { tail -5 gpurun_out/c5/c5rb.err; exit 1; }
cut -c1-1400 gpurun_out/c5/c5rb.json
