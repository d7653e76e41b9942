#!/bin/bash
# Round 4: the row pull writes a queued row's nx once (at its finish) -- parity, round 7 time.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04s}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread -k "variants or workload_parity or multiword or hand_graphs or deferred or needy or dense_exchange" > $O/parity.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 500 --timeout-method thread -k "auto_matches_oracle" > $O/full.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/full.log | head -30; tail -5 $O/full.log; exit 1; }
tail -1 $O/full.log
for i in 1 2; do
  timeout -k 10 300 python3 -u tools/round_profile.py 4 > $O/rounds_c4_$i.txt 2>&1 || { tail -20 $O/rounds_c4_$i.txt; exit 1; }
  grep -E "^7 " $O/rounds_c4_$i.txt | cut -c1-100
done
