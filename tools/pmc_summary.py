#!/usr/bin/env python3
"""Summarise a rocprofv3 profile directory set (kernel trace + FETCH_SIZE /
WRITE_SIZE passes + the calibration passes of tools/calib_fetch) into one
JSON: per-kernel launches, average duration, counted fetch/write bytes per
launch and the calibration ratios used to read them.

usage: pmc_summary.py <dir with c*_trace/ c*_fetch/ c*_write/ cal_fetch/ cal_write/> <out.json> [prefix] [note]
"""
import csv
import collections
import json
import re
import sys
from pathlib import Path


def kname(s):
    m = re.search(r"(k_\w+)(<[^>(]*>)?", s)
    return (m.group(1) + (m.group(2) or "")) if m else s[:60]


def counters(path):
    d = collections.defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(path)):
        k = kname(r["Kernel_Name"])
        d[(k, r["Counter_Name"])][0] += float(r["Counter_Value"])
        d[(k, r["Counter_Name"])][1] += 1
    return d


def main():
    root, out = Path(sys.argv[1]), Path(sys.argv[2])
    pre = sys.argv[3] if len(sys.argv) > 3 else "c4"
    note = f" ({sys.argv[4]})" if len(sys.argv) > 4 else ""
    res = {"source": str(root) + note, "kernels": {}, "calibration": {}}
    stats = list(csv.DictReader(open(root / f"{pre}_trace" / "run_kernel_stats.csv")))
    for r in stats:
        k = kname(r["Name"])
        res["kernels"][k] = {"launches": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                             "total_ms": float(r["TotalDurationNs"]) / 1e6}
    for ctr, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        p = root / f"{pre}_{sub}" / "run_counter_collection.csv"
        if p.exists():
            for (k, c), (v, n) in counters(p).items():
                res["kernels"].setdefault(k, {})[f"{sub}_bytes_per_launch_counted"] = v * 1024 / n
    cal = {"k_stream16": 2 ** 31, "k_stream4": 2 ** 31, "k_gather8": 2 ** 28 * 8, "k_store8": 2 ** 31}
    for sub in ("fetch", "write"):
        p = root / f"cal_{sub}" / "run_counter_collection.csv"
        if p.exists():
            for (k, c), (v, n) in counters(p).items():
                if k in cal:
                    res["calibration"].setdefault(k, {})[f"{sub}_counted_over_touched"] = v * 1024 / n / cal[k]
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res["calibration"], indent=1))


if __name__ == "__main__":
    main()
