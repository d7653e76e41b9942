#!/bin/bash
# Round 3: configs 2 and 1 -- per-round kernel times and bench lines (no CPU baseline).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/small; mkdir -p $O
timeout -k 10 200 python3 -u tools/round_profile.py 2 > $O/rounds_c2.txt 2>&1 || { tail -20 $O/rounds_c2.txt; exit 1; }
cat $O/rounds_c2.txt
for c in 2 1; do
  timeout -k 10 200 python3 -u bench.py --config $c --no-cpu-baseline > $O/bench$c.json 2> $O/bench$c.err || { tail -20 $O/bench$c.err; exit 1; }
  cut -c1-260 $O/bench$c.json
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2_trace -o run -- python3 -u bench.py --config 2 --no-cpu-baseline --no-timing --steps 10 --warmup 3 > $O/bench2_trace.json 2> $O/bench2_trace.err || { tail -20 $O/bench2_trace.err; exit 1; }
