#!/bin/bash
# Round-5 profiles of one BASELINE config (default 4): per-round kernel times,
# rocprofv3 kernel trace + stats of the bench command, then FETCH_SIZE and
# WRITE_SIZE in passes of their own, summarised per kernel.
# usage: r05/profile.sh <config> <commit> [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C=${1:-4}; H=${2:-unknown}; shift 2
O=gpurun_out/prof_r05/c$C
mkdir -p $O
timeout -k 10 300 python3 -u tools/round_profile.py $C > $O/rounds.txt 2>&1 || { tail -20 $O/rounds.txt; exit 1; }
cat $O/rounds.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c${C}_trace -o run -- python3 -u bench.py --config $C --no-cpu-baseline --steps 5 --warmup 1 "$@" > $O/bench_trace.json 2> $O/bench_trace.err || { tail -20 $O/bench_trace.err; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c${C}_fetch -o run -- python3 -u bench.py --config $C --no-cpu-baseline --no-timing --steps 3 --warmup 1 "$@" > $O/bench_fetch.json 2> $O/bench_fetch.err || { tail -20 $O/bench_fetch.err; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c${C}_write -o run -- python3 -u bench.py --config $C --no-cpu-baseline --no-timing --steps 3 --warmup 1 "$@" > $O/bench_write.json 2> $O/bench_write.err || { tail -20 $O/bench_write.err; exit 1; }
python3 tools/pmc_summary.py $O $O/pmc_summary.json c$C "round 5, HEAD $H" > /dev/null && python3 -c "
import json; d=json.load(open('$O/pmc_summary.json'))
for k,v in sorted(d['kernels'].items(), key=lambda kv: -kv[1].get('total_ms',0))[:14]:
    print(f\"{k[:48]:48s} n={v.get('launches',0):4d} avg={v.get('avg_ms',0):8.3f} ms  fetch={v.get('fetch_bytes_per_launch_counted',0)/1e9:7.2f} GB  write={v.get('write_bytes_per_launch_counted',0)/1e9:7.2f} GB\")
"
cat $O/bench_trace.json | cut -c1-400
