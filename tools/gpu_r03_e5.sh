#!/bin/bash
# Round 3 E5: streamed-layout parity then per-round profiles, default vs streamed.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/e5
GOSSIP_BIN_STREAM=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fullsize_auto or fold or workload_parity or multiword or coverage_history or variants" > gpurun_out/e5/pytest_stream.log 2>&1 || { tail -30 gpurun_out/e5/pytest_stream.log; exit 1; }
tail -1 gpurun_out/e5/pytest_stream.log
for v in GOSSIP_BIN_STREAM=1 "GOSSIP_BIN_STREAM=1 GOSSIP_XCD_SYNC=0" GOSSIP_BIN_STREAM=1 "GOSSIP_BIN_STREAM=1 GOSSIP_XCD_SYNC=0"; do
  [ "$v" = "-" ] && v=""
  echo "== [$v]"
  env $v timeout -k 10 150 python3 -u tools/round_profile.py 4 2>&1 | grep -E "^[3-8] " || exit 1
done
