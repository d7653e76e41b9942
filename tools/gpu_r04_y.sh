#!/bin/bash
# Round 4: A/B of two depths, each built into its own library under build/ab: the streamed scatter's
# pieces per lane in flight (kU 4 -> 8) and blocked level 1's tiles in flight (kPre 4 -> 8); config 4, alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04y}; mkdir -p $O
for v in def su8 pre8 def su8 pre8; do
  if [ $v = def ]; then L=p2p-gossipprotocol_amd/build/libgossip_hip.so; else L=p2p-gossipprotocol_amd/build/ab/libgossip_hip_$v.so; fi
  GOSSIP_HIP_LIB=$PWD/$L timeout -k 10 300 python3 -u tools/round_profile.py 4 > $O/rounds_c4_$v.txt 2>&1 || { tail -20 $O/rounds_c4_$v.txt; exit 1; }
  echo "== $v"; grep -E "^(3|4|5) " $O/rounds_c4_$v.txt | cut -c1-110
done
