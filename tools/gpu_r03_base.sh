#!/bin/bash
# Round 3 (session 2): default bench line and the config-4/5 per-round split on HEAD.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/base; mkdir -p $O
timeout -k 10 300 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cut -c1-600 $O/bench_default.json
for c in 4 5; do
  timeout -k 10 300 python3 -u tools/round_profile.py $c > $O/rounds_c$c.txt 2>&1 || { tail -20 $O/rounds_c$c.txt; exit 1; }
  cat $O/rounds_c$c.txt
done
