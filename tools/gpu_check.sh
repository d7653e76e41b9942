#!/bin/bash
# One GPU call: parity tests, default bench line, rocprofv3 kernel stats of the same bench.
set -o pipefail
mkdir -p gpurun_out/chk
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/chk/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/chk/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/chk/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/chk/bench.json 2> gpurun_out/chk/bench.err || { tail -20 gpurun_out/chk/bench.err; exit 1; }
cat gpurun_out/chk/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/chk/prof -o run -- python3 -u bench.py --no-cpu-baseline > gpurun_out/chk/bench_prof.json 2> gpurun_out/chk/bench_prof.err || { tail -20 gpurun_out/chk/bench_prof.err; exit 1; }
echo done
