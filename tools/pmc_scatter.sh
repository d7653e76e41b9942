#!/bin/bash
# PMC passes (one counter group per run) over tools/bin_probe.py (config 4):
# per-launch means for the binned-round kernels.  usage: pmc_scatter.sh [tag]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-pmc}
O=gpurun_out/$T
mkdir -p $O
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "WRITE_SIZE TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum" \
           "FETCH_SIZE" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 -u tools/bin_probe.py 4 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  grep clean $O/p$i.log | head -2
done
python3 tools/pmc_summary2.py $O > $O/summary.txt && cat $O/summary.txt
