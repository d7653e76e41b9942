#!/bin/bash
# Scatter timing breakdown at config 4: staging only (1), + entry loads (2), + LDS reads (3), full (0); U=8.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/probe
for p in 0 1 2 3; do
  GOSSIP_SCATTER_PROBE=$p timeout -k 10 240 python -u tools/bin_probe.py 4 >> gpurun_out/probe/probe.log 2>&1 || { tail -5 gpurun_out/probe/probe.log; exit 1; }
done
GOSSIP_SCATTER_U=8 timeout -k 10 240 python -u tools/bin_probe.py 4 >> gpurun_out/probe/probe.log 2>&1 || { tail -5 gpurun_out/probe/probe.log; exit 1; }
cat gpurun_out/probe/probe.log
