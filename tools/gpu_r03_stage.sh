#!/bin/bash
# Round 3: LDS staging protocol unit test + throughput on the GPU (tools/stage_test.hip)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in "1 20000 0" "96 20000 1" "57 200000 0 1024" "57 200000 0 1024 1" "8 200000 0 1024" "96 100000 0 256" "96 100000 0 256 1"; do
  timeout -k 5 60 tools/stage_test $a; rc=$?; [ $rc -le 1 ] || exit $rc
done
