#!/bin/bash
# Round 3 E4: parity of both layouts (source stats in the scatter or the apply), then per-round profiles.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/e4
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "variants or fold" > gpurun_out/e4/pytest_var.log 2>&1 || { tail -30 gpurun_out/e4/pytest_var.log; exit 1; }
tail -1 gpurun_out/e4/pytest_var.log
GOSSIP_BIN_STREAM=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fullsize_auto or fold or workload_parity or multiword or coverage_history" > gpurun_out/e4/pytest_stream.log 2>&1 || { tail -30 gpurun_out/e4/pytest_stream.log; exit 1; }
tail -1 gpurun_out/e4/pytest_stream.log
GOSSIP_SRC_STATS=0 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fullsize_auto or workload_parity or multiword or coverage_history or partitioned" > gpurun_out/e4/pytest_ss0.log 2>&1 || { tail -30 gpurun_out/e4/pytest_ss0.log; exit 1; }
tail -1 gpurun_out/e4/pytest_ss0.log
for v in - GOSSIP_SRC_STATS=0 GOSSIP_BIN_STREAM=1 - GOSSIP_SRC_STATS=0 GOSSIP_BIN_STREAM=1; do
  [ "$v" = "-" ] && v=""
  echo "== [$v]"
  env $v timeout -k 10 150 python3 -u tools/round_profile.py 4 2>&1 | grep -E "^[3-8] " || exit 1
done
