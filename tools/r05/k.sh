#!/bin/bash
# Round 5: config 4 as 8 parts with each part's kernel total, default against the record push in every sparse
# round (px_permille 0: no appended records).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 400 python -u tools/round_profile_parts.py 4 8 > $O/rounds_c4_p8.txt 2>&1 || { tail -20 $O/rounds_c4_p8.txt; exit 1; }
cut -c1-300 $O/rounds_c4_p8.txt
timeout -k 10 400 python -u tools/round_profile_parts.py 4 8 t.px_permille=0 > $O/rounds_c4_p8_px0.txt 2>&1 || { tail -20 $O/rounds_c4_p8_px0.txt; exit 1; }
cut -c1-300 $O/rounds_c4_p8_px0.txt
