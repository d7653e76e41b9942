#!/usr/bin/env python3
"""Per-kernel averages (per launch) of every counter in rocprofv3 --pmc pass
directories: usage pmc_table.py <dir>... (each holding run_counter_collection.csv
somewhere below).  Kernels are matched by their k_* name with template args."""
import collections
import csv
import re
import sys
from pathlib import Path


def kname(s):
    m = re.search(r"(k_\w+)(<[^>(]*>)?", s)
    return (m.group(1) + (m.group(2) or "")) if m else s[:60]


tab = collections.defaultdict(dict)
for d in sys.argv[1:]:
    for p in Path(d).rglob("*counter_collection.csv"):
        acc = collections.defaultdict(lambda: [0.0, set()])
        for r in csv.DictReader(open(p)):
            k = kname(r["Kernel_Name"])
            a = acc[(k, r["Counter_Name"])]
            a[0] += float(r["Counter_Value"])
            a[1].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        for (k, c), (v, ids) in acc.items():
            tab[k][c] = v / max(1, len(ids))
for k in sorted(tab):
    print(k)
    for c in sorted(tab[k]):
        print(f"    {c:40s} {tab[k][c]:18.4g}")
