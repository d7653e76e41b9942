"""Kernel busy time and the gaps between kernels from a rocprofv3 kernel trace (CSV).

Usage: kernel_gaps.py <trace dir> [last_n_kernels | fraction]
Prints per-kernel launches / average duration, then over the last N kernels (the timed steps): the span, the
busy time and the idle gaps between consecutive kernels (histogram), so a launch-bound run shows where its
time goes."""
import csv
import glob
import sys
from collections import defaultdict


def main():
    files = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)
    if not files:
        sys.exit(f"no kernel_trace.csv under {sys.argv[1]}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # a count, or a fraction of the trace's kernels (the timed steps at its end)
    arg = sys.argv[2] if len(sys.argv) > 2 else "1.0"
    last = int(len(rows) * float(arg)) if "." in arg else int(arg)
    rows = rows[-last:]
    per = defaultdict(list)
    for s, e, k in rows:
        name = k.replace("void ", "").replace("(anonymous namespace)::", "").replace("gossip::", "")
        per[name.split("(")[0][:70]].append(e - s)
    busy = sum(e - s for s, e, _ in rows)
    span = rows[-1][1] - rows[0][0]
    print(f"kernels {len(rows)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(span - busy) / 1e6:.3f} ms")
    gaps = [max(0, rows[i + 1][0] - rows[i][1]) for i in range(len(rows) - 1)]
    edges = [0, 1000, 2000, 4000, 8000, 16000, 64000, 10 ** 12]
    for lo, hi in zip(edges, edges[1:]):
        g = [x for x in gaps if lo <= x < hi]
        print(f"  gaps {lo / 1e3:6.1f}-{hi / 1e3:8.1f} us: {len(g):6d}  sum {sum(g) / 1e6:.3f} ms")
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:70s} n={len(v):5d} avg={sum(v) / len(v) / 1e3:9.2f} us  sum={sum(v) / 1e6:8.3f} ms")


if __name__ == "__main__":
    main()
