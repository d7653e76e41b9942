#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bin
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_partitioned.py -x -q --timeout 120 --timeout-method thread -k "bin or full_size or partitioned" > gpurun_out/bin/pytest.log 2>&1 || { tail -40 gpurun_out/bin/pytest.log; exit 1; }
tail -2 gpurun_out/bin/pytest.log
for s in "GOSSIP_X=0" "GOSSIP_BIN_NT=8" "GOSSIP_X=0" "GOSSIP_BIN_NT=8"; do
  env $s timeout -k 10 120 python -u tools/bin_probe.py 4 || exit 1
done
bash tools/sweep_env.sh - GOSSIP_BIN_NT=8 -
