#!/bin/bash
# Round 4: A/B of the row pull's occupancy (k_pull_rows with launch bounds asking 5 or 6 waves per SIMD,
# built into separate libraries under build/ab) -- config 4 round 7, alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04q}; mkdir -p $O
for v in def 5 6 def 5 6; do
  if [ $v = def ]; then L=p2p-gossipprotocol_amd/build/libgossip_hip.so; else L=p2p-gossipprotocol_amd/build/ab/libgossip_hip_pw$v.so; fi
  GOSSIP_HIP_LIB=$PWD/$L timeout -k 10 300 python3 -u tools/round_profile.py 4 > $O/rounds_c4_$v.txt 2>&1 || { tail -20 $O/rounds_c4_$v.txt; exit 1; }
  echo "== $v $(grep -E '^7 ' $O/rounds_c4_$v.txt | cut -c1-90)"
done
