#!/bin/bash
# A/B/n on one box: bench.py against each library under abtest/<variant>/ (VARIANTS="base nt ..."), alternating, 2 passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abn
: > gpurun_out/abn/ab.log
for i in $(seq 1 ${PASSES:-2}); do
  for v in ${VARIANTS:-base}; do
    export GOSSIP_HIP_LIB=$PWD/abtest/$v/libgossip_hip.so
    timeout -k 10 300 python -u bench.py --no-cpu-baseline ${AB_ARGS} > gpurun_out/abn/$v$i.json 2> gpurun_out/abn/$v$i.err || { tail -20 gpurun_out/abn/$v$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/abn/$v$i.json')); r=d['roofline']; print('$v$i', d['ms_per_step'], 'ms/step', r['kernel_ms_per_step'])" >> gpurun_out/abn/ab.log
  done
done
cat gpurun_out/abn/ab.log
