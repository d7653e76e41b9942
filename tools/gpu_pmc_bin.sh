#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcbin
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcbin/w -o run -- python3 -u tools/bin_probe.py 4 > gpurun_out/pmcbin/w.log 2>&1 || { tail -5 gpurun_out/pmcbin/w.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcbin/f -o run -- python3 -u tools/bin_probe.py 4 > gpurun_out/pmcbin/f.log 2>&1 || { tail -5 gpurun_out/pmcbin/f.log; exit 1; }
python3 - <<'PY'
import csv, collections, glob
for tag in ("w", "f"):
    f = glob.glob(f"gpurun_out/pmcbin/{tag}/**/*counter_collection.csv", recursive=True)[0]
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        for key in ("k_bin_scatter", "k_bin_apply", "k_pull_light", "k_push_light"):
            if key in k:
                d[key].append(float(r["Counter_Value"]))
    for k, v in d.items():
        print(tag, k, "launches", len(v), "per-launch GB", [round(x * 1024 / 1e9, 2) for x in v][:12])
PY
