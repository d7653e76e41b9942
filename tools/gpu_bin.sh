#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/sweep_env.sh -
BENCH_ARGS="--pull-permille 10" bash tools/sweep_env.sh - 
BENCH_ARGS="--pull-permille 5" bash tools/sweep_env.sh - 
BENCH_ARGS="--pull-permille 20" bash tools/sweep_env.sh - 
BENCH_ARGS="--pull-permille 10 --front-permille 1000" bash tools/sweep_env.sh - 
