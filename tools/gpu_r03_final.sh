#!/bin/bash
# Round 3 end: smoke(), the GPU suite, then config 5's profile on HEAD ($1 = commit).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final; mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_profile_r03.sh 5 $1
