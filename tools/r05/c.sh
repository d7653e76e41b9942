#!/bin/bash
# Round 5, third call: group / record-push / small-kernel parity, config 4 as 8 parts round by round (record
# push, marked-tile sweeps at P > 1), then the config 2 / 3 small-kernel sweeps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -m gpu -x -q -k "variants or group or record_push" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u tools/round_profile_parts.py 4 8 > $O/rounds_c4_p8.txt 2>&1 || { tail -20 $O/rounds_c4_p8.txt; exit 1; }
cut -c1-400 $O/rounds_c4_p8.txt
bash tools/r05/b.sh
