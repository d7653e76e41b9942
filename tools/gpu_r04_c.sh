#!/bin/bash
# Round 4, third pass: the streamed binned layout at config 4 -- PMC of its scatter and apply, and bin sizes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04c}; mkdir -p $O
bash tools/gpu_pmc_rounds.sh ${1:-r04c}/pmc_stream 4 t.bin_stream=1 || exit 1
for v in "t.bin_stream=1 t.bin_words=9216" "t.bin_stream=1 t.bin_words=9216 t.bin_chunk=9216" "t.bin_stream=1"; do
  timeout -k 10 300 python3 -u tools/round_profile.py 4 $v > $O/rounds.txt 2>&1 || { tail -20 $O/rounds.txt; exit 1; }
  echo "== $v"; sed -n 4,8p $O/rounds.txt
done
