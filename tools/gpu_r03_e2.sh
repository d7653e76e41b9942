#!/bin/bash
# Round 3: full-size partitioned tests + streamed-layout variant tests, then per-round profiles
# (default, streamed layout with XCD-contiguous apply, overlap probe).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/e2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "partitioned_group or (variants and STREAM)" > gpurun_out/e2/pytest.log 2>&1
echo "pytest rc=$?"; tail -15 gpurun_out/e2/pytest.log
for v in - GOSSIP_BIN_STREAM=1 GOSSIP_OVERLAP_PROBE=1; do
  [ "$v" = "-" ] && v=""
  echo "== [$v]"
  env $v timeout -k 10 150 python3 -u tools/round_profile.py 4 2>&1 || exit 1
done
