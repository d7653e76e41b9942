#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per launch of the binned-round kernels, per library under abtest/<variant>/ (one pass per counter).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcab
for v in ${VARIANTS:-base}; do
  export GOSSIP_HIP_LIB=$PWD/abtest/$v/libgossip_hip.so
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmcab/$v/$c -o run -- python3 -u tools/bin_probe.py 4 > gpurun_out/pmcab/$v.$c.log 2>&1 || { tail -5 gpurun_out/pmcab/$v.$c.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, collections, glob, os
for v in os.environ.get("VARIANTS", "base").split():
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"gpurun_out/pmcab/{v}/{c}/**/*counter_collection.csv", recursive=True)[0]
        d = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            for key in ("k_bin_scatter", "k_bin_apply", "k_pull_heavy"):
                if key in r["Kernel_Name"]:
                    d[key].append(float(r["Counter_Value"]))
        for k, x in d.items():
            print(v, c, k, len(x), [round(y * 1024 / 1e9, 2) for y in x][:10])
PY
