#!/bin/bash
# Round 5: config 4 as 8 parts -- the dense rounds' scatter reading other blocks' words straight from the gather
# buffer (scatter_direct) against staging them, and one exchange stage against four.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05m; mkdir -p $O
i=0
for A in "" "t.scatter_direct=1" "t.exchange_stages=1" "t.scatter_direct=1 t.exchange_stages=1"; do
  i=$((i+1))
  timeout -k 10 300 python -u tools/round_profile_parts.py 4 8 $A > $O/rounds_$i.txt 2>&1 || { tail -20 $O/rounds_$i.txt; exit 1; }
  echo "== $A"; grep -E "^[456] |step sums|^part 0" $O/rounds_$i.txt | cut -c1-230
done
