#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/calib
timeout -k 10 300 tools/calib_store > gpurun_out/calib/store.log 2>&1 || { tail -5 gpurun_out/calib/store.log; exit 1; }
cat gpurun_out/calib/store.log
