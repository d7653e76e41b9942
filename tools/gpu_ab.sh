#!/bin/bash
# A/B on one box: bench.py against the baseline library (abtest/base) and the current one, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
: > gpurun_out/ab/ab.log
for i in 1 2; do
  for v in base cur; do
    if [ $v = base ]; then export GOSSIP_HIP_LIB=$PWD/abtest/base/libgossip_hip.so; else unset GOSSIP_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline ${AB_ARGS} > gpurun_out/ab/$v$i.json 2> gpurun_out/ab/$v$i.err || { tail -20 gpurun_out/ab/$v$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/$v$i.json')); r=d['roofline']; print('$v$i', d['ms_per_step'], 'ms/step', r['kernel_ms_per_step'])" >> gpurun_out/ab/ab.log
  done
done
cat gpurun_out/ab/ab.log
