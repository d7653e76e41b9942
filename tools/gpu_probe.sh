#!/bin/bash
# Scatter timing breakdown per binned round at config 4: full (0), staging only (1), stores to the sink (2).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/probe
: > gpurun_out/probe/probe.log
for p in 0 1 2; do
  GOSSIP_SCATTER_PROBE=$p timeout -k 10 240 python -u tools/bin_probe.py 4 >> gpurun_out/probe/probe.log 2>&1 || { tail -5 gpurun_out/probe/probe.log; exit 1; }
done
cat gpurun_out/probe/probe.log
