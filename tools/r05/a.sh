#!/bin/bash
# Round 5, first call: the new probe-toggle parity test, the variant tests, the group tests (staged exchange,
# tile marks at P > 1), the config-4 round profile, config 4 as 8 parts round by round, and the --parts 8 line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -m gpu -x -q -k "probe_toggle or variants or group or comm_init or record_push" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/round_profile.py 4 > $O/rounds_c4.txt 2>&1 || { tail -20 $O/rounds_c4.txt; exit 1; }
cut -c1-250 $O/rounds_c4.txt
timeout -k 10 400 python -u tools/round_profile_parts.py 4 8 > $O/rounds_c4_p8.txt 2>&1 || { tail -20 $O/rounds_c4_p8.txt; exit 1; }
cut -c1-400 $O/rounds_c4_p8.txt
timeout -k 10 400 python -u tools/round_profile_parts.py 4 8 t.exchange_stages=1 > $O/rounds_c4_p8_s1.txt 2>&1 || { tail -20 $O/rounds_c4_p8_s1.txt; exit 1; }
tail -1 $O/rounds_c4_p8_s1.txt | cut -c1-400
timeout -k 10 600 python -u bench.py --parts 8 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_parts8.json 2> $O/bench_parts8.err || { tail -20 $O/bench_parts8.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_parts8.json').read().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], d['value'], r.get('frac'), r.get('kernel_ms_per_step'), r.get('exchange_ms_per_step'), r.get('exchange_link_ms_per_step'), r.get('projected_ms_per_step'), r.get('part_kernel_ms_per_step'))"
