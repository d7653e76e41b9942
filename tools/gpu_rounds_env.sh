#!/bin/bash
# Per-round kernel times (tools/round_profile.py, config ${CFG:-4}) once per env setting ("-" = defaults).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rounds
: > gpurun_out/rounds/rounds.log
for v in "$@"; do
    [ "$v" = "-" ] && v=""
    echo "== [$v]" >> gpurun_out/rounds/rounds.log
    env $v timeout -k 10 150 python3 -u tools/round_profile.py ${CFG:-4} >> gpurun_out/rounds/rounds.log 2>&1 || { tail -5 gpurun_out/rounds/rounds.log; exit 1; }
done
cat gpurun_out/rounds/rounds.log
