#!/bin/bash
# Round 3 E3: default-layout and streamed-layout parity (variants + full size), then per-round profiles.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/e3
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "variants or fold" > gpurun_out/e3/pytest_var.log 2>&1 || { tail -30 gpurun_out/e3/pytest_var.log; exit 1; }
tail -2 gpurun_out/e3/pytest_var.log
GOSSIP_BIN_STREAM=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fullsize_auto or fold or workload_parity" > gpurun_out/e3/pytest_stream.log 2>&1 || { tail -30 gpurun_out/e3/pytest_stream.log; exit 1; }
tail -2 gpurun_out/e3/pytest_stream.log
for v in - GOSSIP_BIN_STREAM=1 - GOSSIP_BIN_STREAM=1; do
  [ "$v" = "-" ] && v=""
  echo "== [$v]"
  env $v timeout -k 10 150 python3 -u tools/round_profile.py 4 2>&1 || exit 1
done
