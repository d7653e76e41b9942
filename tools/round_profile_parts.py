"""Per-round kernel and exchange times of one config run as P parts on one GPU
(gossip_group on a single device, device-copy exchanges), summed over the
parts, after one warm run, and each part's kernel total.  Usage: round_profile_parts.py CONFIG P [t.key=value ...] [p.hub=H p.peer=C]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "p2p-gossipprotocol_amd"))
from gossip_hip import Group  # noqa: E402
from gossip_hip.engine import EXCHANGES, KERNELS  # noqa: E402
from gossip_hip.workloads import config  # noqa: E402

w = config(int(sys.argv[1]))
P = int(sys.argv[2])
tuning = {a[2:].split("=")[0]: int(a.split("=")[1]) for a in sys.argv[3:] if a.startswith("t.")}
# p.hub=H,p.peer=C: blocks of equal cost ek (u + H cbrt(u)) + C u (gossip_partition_edges: H = 1, C = 2), A/B only
pm = {a[2:].split("=")[0]: float(a.split("=")[1]) for a in sys.argv[3:] if a.startswith("p.")}
begins = None
if pm:
    import math
    ek = sum(1 - (j / 6) ** 2.5 for j in range(1, 6))
    cost = lambda u: ek * (u + pm.get("hub", 1.0) * u ** (1 / 3)) + pm.get("peer", 2.0) * u  # noqa: E731
    begins = [0]
    for q in range(1, P):
        lo, hi = 0.0, 1.0
        for _ in range(100):
            mid = (lo + hi) / 2
            lo, hi = (mid, hi) if cost(mid) < cost(1.0) * q / P else (lo, mid)
        begins.append(max(begins[-1] + 64, math.ceil(hi * w.n / 64) * 64))
    begins.append(w.n)
    print("begins %", [round(100 * b / w.n, 2) for b in begins], flush=True)
g = Group(w.n, w.n_msgs, [0] * P, tuning=tuning, begins=begins, **w.engine_kwargs())
g.build_graph()
g.inject(w.origins, w.inject_rounds)
if w.kills:
    g.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
g.reset()
g.run()
g.reset()
g.enable_timing(True)
names = KERNELS + EXCHANGES
tot = lambda: {k: sum(g.kernel_time(p, k)[0] for p in range(P)) for k in names}  # noqa: E731
per_part = lambda: [{k: g.kernel_time(p, k)[0] for k in KERNELS} for p in range(P)]  # noqa: E731
base = per_part()
prev = tot()
ksum = {}
while True:
    st, fin = g.step()
    cur = tot()
    d = {k: round(cur[k] - prev[k], 3) for k in names if cur[k] - prev[k] > 0.0005}
    for k, v in d.items():
        ksum[k] = ksum.get(k, 0.0) + v
    kern = sum(v for k, v in d.items() if k in KERNELS)
    print(st["round"], f"F={st['frontier'] / w.n:.4f}", f"kernels={kern:.3f}", d, flush=True)
    prev = cur
    if fin:
        break
print("step sums", {k: round(v, 3) for k, v in sorted(ksum.items(), key=lambda x: -x[1])},
      "kernels", round(sum(v for k, v in ksum.items() if k in KERNELS), 3),
      "exchange", round(sum(v for k, v in ksum.items() if k in EXCHANGES), 3))
# each part's kernels over the step (on P GPUs the slowest part sets the step), its largest kernels
end = per_part()
for p in range(P):
    kp = {k: end[p][k] - base[p][k] for k in KERNELS if end[p][k] - base[p][k] > 0.0005}
    top = sorted(kp.items(), key=lambda x: -x[1])[:7]
    print(f"part {p} kernels {sum(kp.values()):.3f}", {k: round(v, 3) for k, v in top})
g.close()
