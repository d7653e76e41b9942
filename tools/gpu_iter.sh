#!/bin/bash
# Iteration call: GPU parity suite, scatter timing of the first binned round, default bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/it
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/it/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/it/pytest_gpu.log
timeout -k 10 240 python -u tools/bin_probe.py 4 > gpurun_out/it/probe.log 2>&1 || { tail -5 gpurun_out/it/probe.log; exit 1; }
cat gpurun_out/it/probe.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/it/bench.json 2> gpurun_out/it/bench.err || { tail -20 gpurun_out/it/bench.err; exit 1; }
cut -c1-1600 gpurun_out/it/bench.json
