#!/bin/bash
# Round 4: SQ counters (one pass, 8 SQ counters) of config 4's rounds: wave cycles split into waiting,
# issue stalls and active issue, LDS stalls and bank conflicts -- for the blocked and dense kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04p}; mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $O/sq -o run -- python3 -u tools/round_profile.py 4 > $O/sq.txt 2>&1 || { tail -20 $O/sq.txt; exit 1; }
f=$(ls $O/sq/*/run_counter_collection.csv $O/sq/run_counter_collection.csv 2>/dev/null | head -1)
python3 tools/sq_summary.py $f k_pb_ k_bin_ k_pull_rows | cut -c1-600
