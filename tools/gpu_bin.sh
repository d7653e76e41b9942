#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bin
true
true
timeout -k 10 300 python -u bench.py --force-partitioned --no-cpu-baseline > gpurun_out/bin/part.json 2> gpurun_out/bin/part.err || { tail -20 gpurun_out/bin/part.err; exit 1; }
cat gpurun_out/bin/part.json
bash tools/sweep_env.sh -
