#!/bin/bash
# Round 5: bench lines of configs 1-3 with the timed loop's steps leaving their stats in the library's buffer
# (the per-round dicts built once after the clock), and the tiny kernel's padded LDS reduce.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ag; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "small_overlay or tiny or golden" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in 1 2 3 1 2 3; do
  timeout -k 10 200 python3 -u bench.py --config $c --no-cpu-baseline > $O/bench_c$c.json 2> $O/bench_c$c.err || { tail -20 $O/bench_c$c.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_c$c.json').read().splitlines()[-1]);r=d['roofline'];print($c, d['ms_per_step'], d['value'], r.get('ms_per_step_with_events'))"
done
