#!/bin/bash
# Per-round profile of config 4 + rocprofv3 kernel stats (CSV) of the default bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u tools/round_profile.py 4 > gpurun_out/prof/rounds_c4.txt 2>&1 || { tail -20 gpurun_out/prof/rounds_c4.txt; exit 1; }
cat gpurun_out/prof/rounds_c4.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/rp -o run -- python3 -u bench.py --no-cpu-baseline > gpurun_out/prof/bench_prof.json 2> gpurun_out/prof/bench_prof.err || { tail -20 gpurun_out/prof/bench_prof.err; exit 1; }
cat gpurun_out/prof/bench_prof.json
find gpurun_out/prof/rp -name '*stats*'
