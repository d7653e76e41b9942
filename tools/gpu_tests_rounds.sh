#!/bin/bash
# GPU tests (one process) then per-round kernel times for config ${CFG:-4} once per env setting ("-" = defaults).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2 gpurun_out/rounds
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/r2/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r2/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r2/pytest_gpu.log
: > gpurun_out/rounds/rounds.log
for v in "$@"; do
    [ "$v" = "-" ] && v=""
    echo "== [$v]" >> gpurun_out/rounds/rounds.log
    env $v timeout -k 10 150 python3 -u tools/round_profile.py ${CFG:-4} >> gpurun_out/rounds/rounds.log 2>&1 || { tail -5 gpurun_out/rounds/rounds.log; exit 1; }
done
cat gpurun_out/rounds/rounds.log
