#!/bin/bash
# Round 5: config 4 as 8 parts -- the record-push threshold per 100 000 (default 5) and block cuts of other cost
# weights (hub edges, peers), each part's kernel total.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05l; mkdir -p $O
i=0
for A in "" "p.hub=1.5 p.peer=2" "p.hub=2 p.peer=2" "p.hub=1.5 p.peer=4" "p.hub=2 p.peer=6"; do
  i=$((i+1))
  timeout -k 10 300 python -u tools/round_profile_parts.py 4 8 $A > $O/rounds_$i.txt 2>&1 || { tail -20 $O/rounds_$i.txt; exit 1; }
  echo "== $A"; grep -E "begins|step sums|^part" $O/rounds_$i.txt | cut -c1-200
done
