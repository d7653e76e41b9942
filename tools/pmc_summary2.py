"""Per-kernel mean PMC values per launch from rocprofv3 counter_collection.csv passes.
usage: pmc_summary2.py <dir with p*/ subdirs> [kernel substrings...]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
keys = sys.argv[2:] or ["k_bin_scatter", "k_bin_apply", "k_pull_light", "k_push_light", "k_push_heavy", "k_pull_heavy"]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = next((x for x in keys if x in r["Kernel_Name"]), None)
        if k:
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in keys:
    if k not in vals:
        continue
    print(k)
    for c, v in sorted(vals[k].items()):
        m = sum(v) / len(v)
        extra = f"  ({m * 1024 / 1e9:.2f} GB)" if c in ("WRITE_SIZE", "FETCH_SIZE") else ""
        print(f"  {c:40s} n={len(v):3d} mean={m:.4g}{extra}")
