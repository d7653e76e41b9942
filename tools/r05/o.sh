#!/bin/bash
# Round 5: a binned round's heavy-row pull fused into the persistent apply (heavy_fuse) -- parity variants and
# group tests, then config 2 / 3 step times and config 4 rounds, fused against separate, arms alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -m gpu -x -q -k "heavy or variants or group" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u tools/sweep_small.py 2 - heavy_fuse=0 - heavy_fuse=0 > $O/sweep_c2.txt 2>&1 || { tail -20 $O/sweep_c2.txt; exit 1; }
cat $O/sweep_c2.txt
timeout -k 10 400 python -u tools/sweep_small.py 3 - heavy_fuse=2 - heavy_fuse=2 > $O/sweep_c3.txt 2>&1 || { tail -20 $O/sweep_c3.txt; exit 1; }
cat $O/sweep_c3.txt
timeout -k 10 300 python -u tools/round_profile.py 4 > $O/rounds_c4.txt 2>&1 || { tail -20 $O/rounds_c4.txt; exit 1; }
cut -c1-200 $O/rounds_c4.txt
timeout -k 10 300 python -u tools/round_profile.py 4 t.heavy_fuse=2 > $O/rounds_c4_unfused.txt 2>&1 || { tail -20 $O/rounds_c4_unfused.txt; exit 1; }
cut -c1-200 $O/rounds_c4_unfused.txt
