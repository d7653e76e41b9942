"""Per-round diagnostics: mode, frontier, traversals and per-kernel ms of each round."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "p2p-gossipprotocol_amd"))
from gossip_hip import KERNELS, Engine  # noqa: E402
from gossip_hip.workloads import config  # noqa: E402

idx = int(sys.argv[1]) if len(sys.argv) > 1 else 2
w = config(idx)
e = Engine(w.n, w.n_msgs, device=0, **w.engine_kwargs())
e.build_graph()
e.inject(w.origins, w.inject_rounds)
e.reset()
e.run()
e.reset()
e.enable_timing(True)
prev = {k: 0.0 for k in KERNELS}
pb = {k: 0.0 for k in KERNELS}
E = e.shape()["n_edges"]
while True:
    st, fin = e.step()
    cur = {k: e.kernel_time(k)[0] for k in KERNELS}
    cb = {k: e.kernel_bytes(k) for k in KERNELS}
    d = {k: round(cur[k] - prev[k], 3) for k in KERNELS if cur[k] - prev[k] > 0.001}
    gb = {k: round((cb[k] - pb[k]) / 1e9, 3) for k in KERNELS if cb[k] - pb[k] > 0}
    print(st["round"], "F=%.3f" % (st["frontier"] / w.n), "T/E=%.3f" % (st["traversals"] / E),
          "fresh/n=%.3f" % (st["new_receipts"] / w.n), "cov/(n*M)=%.4f" % (st["covered"] / (w.n * w.n_msgs)), d, gb,
          flush=True)
    prev, pb = cur, cb
    if fin:
        break
