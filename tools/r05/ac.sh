#!/bin/bash
# Round 5: replayed rounds with per-round state rows (no per-round clears) -- parity, then step times.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ac; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for C in 2 3; do
  timeout -k 10 300 python -u tools/ab_kernel.py $C step 3 - > $O/ab_c$C.txt 2>&1 || { tail -20 $O/ab_c$C.txt; exit 1; }
  tail -1 $O/ab_c$C.txt
done
timeout -k 10 300 python3 -u bench.py --config 2 --no-cpu-baseline --no-timing --steps 20 --warmup 2 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c2.json').read().splitlines()[-1]); print('bench c2', d['ms_per_step'])"
