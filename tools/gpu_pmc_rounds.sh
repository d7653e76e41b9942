#!/bin/bash
# Kernel trace + FETCH_SIZE / WRITE_SIZE passes (each its own run) of tools/round_profile.py on one config
# with tuning options; summary per kernel.  usage: gpu_pmc_rounds.sh <out dir> <config> [round_profile args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; C=$2; shift 2
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c${C}_trace -o run -- python3 -u tools/round_profile.py $C "$@" > $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c${C}_fetch -o run -- python3 -u tools/round_profile.py $C "$@" > $O/fetch.txt 2>&1 || { tail -20 $O/fetch.txt; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c${C}_write -o run -- python3 -u tools/round_profile.py $C "$@" > $O/write.txt 2>&1 || { tail -20 $O/write.txt; exit 1; }
python3 tools/pmc_summary.py $O $O/pmc_summary.json c$C "round_profile.py $C $*" > /dev/null && python3 -c "
import json; d=json.load(open('$O/pmc_summary.json'))
for k,v in sorted(d['kernels'].items(), key=lambda kv: -kv[1].get('total_ms',0))[:14]:
    print(f\"{k[:48]:48s} n={v.get('launches',0):4d} avg={v.get('avg_ms',0):8.3f} ms  fetch={v.get('fetch_bytes_per_launch_counted',0)/1e9:7.2f} GB  write={v.get('write_bytes_per_launch_counted',0)/1e9:7.2f} GB\")
"
