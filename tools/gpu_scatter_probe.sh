#!/bin/bash
# Scatter timing breakdown on config 4 (first binned round, clean and after a
# run), once per setting.  usage: gpu_scatter_probe.sh "<VAR=VAL ...>" ...
# ("-" = defaults).  Useful settings: GOSSIP_SCATTER_U=8, GOSSIP_BIN_UNIT=N,
# GOSSIP_SCATTER_PROBE=1|2|3 (1 staging + stats only, 2 + cb loads,
# 3 + LDS reads; no stores).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sprobe
rm -f gpurun_out/sprobe/probe.log
for v in "$@"; do
    [ "$v" = "-" ] && v=""
    env $v timeout -k 10 150 python3 -u tools/bin_probe.py 4 >> gpurun_out/sprobe/probe.log 2>&1 || { tail -5 gpurun_out/sprobe/probe.log; exit 1; }
done
cat gpurun_out/sprobe/probe.log
