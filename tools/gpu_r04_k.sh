#!/bin/bash
# Round 4: rows of 32 bins (apply) and of 32 units (scatter) dealt round-robin over the XCD groups.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04k}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "variants or workload_parity or multiword or hand_graphs" > $O/parity.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in 1 0; do
  timeout -k 10 300 python3 -u tools/round_profile.py 4 t.apply_persist=$v t.apply_probe=1 > $O/rounds_c4_p$v.txt 2>&1 || { tail -20 $O/rounds_c4_p$v.txt; exit 1; }
  echo "== apply_persist $v"; grep -E "^(5|6) " $O/rounds_c4_p$v.txt | cut -c1-700
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "dense_exchange or auto_matches_oracle" > $O/full.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/full.log | head -30; tail -5 $O/full.log; exit 1; }
tail -1 $O/full.log
