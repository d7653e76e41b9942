#!/bin/bash
# Round-end rehearsal: full GPU test suite, smoke(), default bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/full/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/full/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/full/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1 || { tail -20 gpurun_out/full/smoke.log; exit 1; }
tail -1 gpurun_out/full/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err || { tail -20 gpurun_out/full/bench.err; exit 1; }
cat gpurun_out/full/bench.json
