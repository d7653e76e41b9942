#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/c5/pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/c5/pytest.log | tail -30; exit 1; }
tail -2 gpurun_out/c5/pytest.log
timeout -k 10 300 python -u tools/round_profile.py 5 > gpurun_out/c5/rounds5.txt 2>&1 || { tail -5 gpurun_out/c5/rounds5.txt; exit 1; }
cat gpurun_out/c5/rounds5.txt
timeout -k 10 300 python -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5/c5.json 2> gpurun_out/c5/c5.err || { tail -5 gpurun_out/c5/c5.err; exit 1; }
cut -c1-1500 gpurun_out/c5/c5.json
