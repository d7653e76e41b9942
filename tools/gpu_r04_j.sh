#!/bin/bash
# Round 4: bins interleaved over the XCD groups in the streamed apply; scatter and apply per-XCD-group times.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04j}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "apply_probe or apply_one_per_bin or stream or workload_parity" > $O/parity.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in 1 0; do
  timeout -k 10 300 python3 -u tools/round_profile.py 4 t.apply_persist=$v t.apply_probe=1 > $O/rounds_c4_p$v.txt 2>&1 || { tail -20 $O/rounds_c4_p$v.txt; exit 1; }
  echo "== apply_persist $v"; grep -E "^(5|6) " $O/rounds_c4_p$v.txt | cut -c1-700
done
