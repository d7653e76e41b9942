"""Per-round kernel and exchange times of one config run as P parts on one GPU
(gossip_group on a single device, device-copy exchanges), summed over the
parts, after one warm run.  Usage: round_profile_parts.py CONFIG P [t.key=value ...]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "p2p-gossipprotocol_amd"))
from gossip_hip import Group  # noqa: E402
from gossip_hip.engine import EXCHANGES, KERNELS  # noqa: E402
from gossip_hip.workloads import config  # noqa: E402

w = config(int(sys.argv[1]))
P = int(sys.argv[2])
tuning = {a[2:].split("=")[0]: int(a.split("=")[1]) for a in sys.argv[3:] if a.startswith("t.")}
g = Group(w.n, w.n_msgs, [0] * P, tuning=tuning, **w.engine_kwargs())
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
g.close()
