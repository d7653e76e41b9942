#!/bin/bash
# Round 5: compact-exchange tile bitmap as the pulls' frontier bitmap ("gather_front") -- config 4 at P = 8 and 2 per round with the key off (0), heavy rows only (1) and every row (2), then partitioned parity.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ae; mkdir -p $O
for P in 8 2; do
  for g in 0 2 1; do
    timeout -k 10 300 python3 -u tools/round_profile_parts.py 4 $P t.gather_front=$g > $O/parts${P}_g$g.txt 2>&1 || { tail -20 $O/parts${P}_g$g.txt; exit 1; }
    echo "== P=$P gather_front=$g"; tail -14 $O/parts${P}_g$g.txt | cut -c1-220
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_partitioned.py tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
