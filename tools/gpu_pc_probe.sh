#!/bin/bash
# Scatter breakdown (bin_probe: per binned round) for several settings, then one SQ PMC pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pcprobe
mkdir -p $O
rm -f $O/probe.log
for v in "-" "GOSSIP_SCATTER_PROBE=1" "GOSSIP_SCATTER_PROBE=2" "GOSSIP_SCATTER_PROBE=3" "GOSSIP_BIN_NOSKIP=1"; do
    [ "$v" = "-" ] && v=""
    env $v timeout -k 10 150 python3 -u tools/bin_probe.py 4 2>&1 | grep clean >> $O/probe.log || { tail -5 $O/probe.log; exit 1; }
done
cat $O/probe.log
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/p1 -o run -- python3 -u tools/bin_probe.py 4 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum --output-format csv -d $O/p2 -o run -- python3 -u tools/bin_probe.py 4 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
python3 tools/pmc_summary2.py $O k_bin_scatter
