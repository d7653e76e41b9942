#!/bin/bash
# Round 5: small overlays in one cooperative launch (gossip_small.hip) -- parity (variants, config 2 at full
# size), then config 2 / 3 step times against the round-by-round engine (small 0), one process.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05y; mkdir -p $O
GOSSIP_SYNC_DEBUG=1 timeout -k 10 120 python -u -c "
import sys; sys.path.insert(0, 'p2p-gossipprotocol_amd')
from gossip_hip import Engine
from gossip_hip.workloads import config
w = config(2, 1 << 16)
e = Engine(w.n, w.n_msgs, device=0, **w.engine_kwargs()); e.build_graph(); e.inject(w.origins, w.inject_rounds); e.reset()
st = e.run(); print('rounds', len(st), st[-1])
" > $O/first.txt 2>&1 || { tail -20 $O/first.txt; exit 1; }
tail -2 $O/first.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "variants or config or fullsize and 2" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/ab_kernel.py 2 step 3 - small=0 > $O/ab_c2.txt 2>&1 || { tail -20 $O/ab_c2.txt; exit 1; }
cat $O/ab_c2.txt
