#!/usr/bin/env python3
"""Per-kernel averages of SQ counters from a rocprofv3 --pmc pass (run_counter_collection.csv):
value per dispatch, and each counter's share of SQ_WAVE_CYCLES where both are present.
usage: sq_summary.py <run_counter_collection.csv> [kernel-prefix ...]"""
import collections
import csv
import re
import sys


def kname(s):
    m = re.search(r"(k_\w+)(<[^>(]*>)?", s)
    return (m.group(1) + (m.group(2) or "")) if m else s[:60]


tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = kname(r["Kernel_Name"])
    tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
    disp[(k, r["Counter_Name"])].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
want = sys.argv[2:]
kernels = sorted({k for k, _ in tot}, key=lambda k: -tot.get((k, "SQ_WAVE_CYCLES"), 0))
for k in kernels:
    if want and not any(k.startswith(w) for w in want):
        continue
    row = {c: tot[(k, c)] / max(1, len(disp[(k, c)])) for (kk, c) in tot if kk == k}
    wc = row.get("SQ_WAVE_CYCLES")
    print(k, {c: (f"{v:.3g}" + (f" ({v / wc:.2f})" if wc and c != "SQ_WAVE_CYCLES" else "")) for c, v in sorted(row.items())})
