#!/bin/bash
# Round 5 (LDS block tables): balanced blocks (gossip_partition_edges) -- the group / partitioned parity tests including the
# full-size partitioned fixtures, config 4 as 8 parts round by round, and the --parts 8 line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_partitioned.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_group.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/pytest_group.log | head -30; tail -5 $O/pytest_group.log; exit 1; }
tail -1 $O/pytest_group.log
timeout -k 10 400 python -u tools/round_profile_parts.py 4 8 > $O/rounds_c4_p8.txt 2>&1 || { tail -20 $O/rounds_c4_p8.txt; exit 1; }
cut -c1-400 $O/rounds_c4_p8.txt
timeout -k 10 600 python -u bench.py --parts 8 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_parts8.json 2> $O/bench_parts8.err || { tail -20 $O/bench_parts8.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_parts8.json').read().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], d['value'], r.get('frac'), round(sum(r.get('kernel_ms_per_step').values()),2), r.get('exchange_ms_per_step'), r.get('exchange_link_ms_per_step'), r.get('projected_ms_per_step'), r.get('part_kernel_ms_per_step'))"
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k partitioned --timeout 600 --timeout-method thread > $O/pytest_fullsize.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/pytest_fullsize.log | head -30; tail -5 $O/pytest_fullsize.log; exit 1; }
tail -1 $O/pytest_fullsize.log
