#!/bin/bash
# Round 5: config 2's kernels per step after the replay change (kernel trace of the bench, no events).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ad; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c2 -o run -- python3 -u bench.py --config 2 --no-cpu-baseline --no-timing --steps 10 --warmup 1 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python3 tools/kernel_gaps.py $O/c2 0.8 > $O/gaps_c2.txt && cat $O/gaps_c2.txt
