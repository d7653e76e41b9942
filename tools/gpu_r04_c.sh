#!/bin/bash
# Round 4, third pass: ranks on one GPU through RCCL; the streamed binned layout (now the default) at config 4
# -- PMC of its scatter and apply, half-size bins --; the partitioned bench lines (--parts 8/4/2) with the
# compact exchange and the atomic-free compaction; the loopback harness timed on the box's host cores.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04c}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiprocess.py -x -v --timeout 200 --timeout-method thread > $O/mp.log 2>&1; grep -E "PASS|FAIL|SKIP|passed|failed|skipped" $O/mp.log | tail -8
bash tools/gpu_pmc_rounds.sh ${1:-r04c}/pmc_stream 4 || exit 1
timeout -k 10 300 python3 -u tools/round_profile.py 4 t.bin_words=9216 > $O/rounds_w9216.txt 2>&1 || { tail -20 $O/rounds_w9216.txt; exit 1; }
echo "== bin_words 9216"; sed -n 4,8p $O/rounds_w9216.txt
echo "== default"; sed -n 4,8p $O/pmc_stream/trace.txt
PARTS="8 2" bash tools/gpu_r04_parts.sh ${1:-r04c}/parts || exit 1
nproc > $O/nproc.txt; lscpu | grep -E "Model name|^CPU\(s\)" >> $O/nproc.txt
timeout -k 10 300 python3 -u tools/time_loopback.py > $O/loopback.txt 2>&1 && cat $O/loopback.txt
