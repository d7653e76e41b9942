#!/bin/bash
# GPU parity suite, per-round kernel times (abtest/base vs current), A/B bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rp/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/rp/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/rp/pytest_gpu.log
GOSSIP_HIP_LIB=$PWD/abtest/base/libgossip_hip.so timeout -k 10 240 python -u tools/round_profile.py 4 > gpurun_out/rp/base.txt 2>&1 || { tail -5 gpurun_out/rp/base.txt; exit 1; }
timeout -k 10 240 python -u tools/round_profile.py 4 > gpurun_out/rp/cur.txt 2>&1 || { tail -5 gpurun_out/rp/cur.txt; exit 1; }
echo base; cat gpurun_out/rp/base.txt; echo cur; cat gpurun_out/rp/cur.txt
bash tools/gpu_ab.sh
