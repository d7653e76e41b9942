#!/bin/bash
# Round 3: per-round A/B of engine options on one config (round_profile.py, arms alternated).
# usage: gpu_r03_ab.sh <config> "<optsA>" "<optsB>"   (opts: key=val ... passed to round_profile.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; mkdir -p $O
C=$1; A=$2; B=$3
for i in 1 2; do
  timeout -k 10 300 python3 -u tools/round_profile.py $C $A > $O/a$i.txt 2>&1 || { tail -20 $O/a$i.txt; exit 1; }
  echo "== A$i: $A"; cat $O/a$i.txt
  timeout -k 10 300 python3 -u tools/round_profile.py $C $B > $O/b$i.txt 2>&1 || { tail -20 $O/b$i.txt; exit 1; }
  echo "== B$i: $B"; cat $O/b$i.txt
done
