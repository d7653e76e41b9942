#!/bin/bash
# PMC passes (one rocprofv3 run each) over the binned-round kernels of one config-4 round profile,
# for the layout given by the environment (e.g. GOSSIP_BIN_STREAM=1).  usage: gpu_r03_pmc.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-def}
O=gpurun_out/pmc_$T
mkdir -p $O
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_ADDR_CONFLICT TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
         "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
         "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TD_TD_BUSY_sum TD_TC_STALL_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --kernel-include-regex "bin_|pull_heavy" --output-format csv -d $O/p$i -o run -- python3 -u tools/round_profile.py 4 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 tools/pmc_table.py $O/p1 $O/p2 $O/p3 $O/p4 > $O/table.txt
cat $O/table.txt
