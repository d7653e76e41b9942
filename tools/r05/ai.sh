#!/bin/bash
# Round 5: the zero fill with four nontemporal 16-B stores in flight per lane -- its average launch under a
# kernel trace of config 4 (compare k_zero2 in profiles/r05/config4_kernel_stats.csv), then the bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ai; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 -u bench.py --config 4 --no-cpu-baseline --no-timing --steps 5 --warmup 1 > $O/bench_trace.json 2> $O/bench_trace.err || { tail -20 $O/bench_trace.err; exit 1; }
grep -h "k_zero2\|fillBuffer" $O/c4/*kernel_stats.csv | cut -c1-200
timeout -k 10 300 python3 -u bench.py --config 4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_c4.json').read().splitlines()[-1]);print(d['ms_per_step'], d['value'])"
