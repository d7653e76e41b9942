"""Times every binned round of config 4 (per-kernel ms, cumulative counters
differenced per round): once on a fresh layout and once after a full run.
Run once per GOSSIP_* setting (GOSSIP_SCATTER_PROBE=1: staging only; 2: slot
stores go to the sink)."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "p2p-gossipprotocol_amd"))
from gossip_hip import Engine  # noqa: E402
from gossip_hip.workloads import config  # noqa: E402

w = config(int(sys.argv[1]) if len(sys.argv) > 1 else 4)
e = Engine(w.n, w.n_msgs, device=0, **w.engine_kwargs())
e.build_graph()
e.inject(w.origins, w.inject_rounds)
tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("GOSSIP_"))
for label in ("clean", "after-run"):
    if label == "after-run":
        e.reset()
        e.run()
    e.reset()
    e.enable_timing(True)
    prev = {k: e.kernel_time(k) for k in ("bin_scatter", "bin_apply")}
    parts = []
    while True:
        st, fin = e.step()
        cur = {k: e.kernel_time(k) for k in prev}
        if cur["bin_scatter"][1] != prev["bin_scatter"][1]:
            parts.append(f"r{st['round']} scatter {cur['bin_scatter'][0] - prev['bin_scatter'][0]:.3f} "
                         f"apply {cur['bin_apply'][0] - prev['bin_apply'][0]:.3f}")
        prev = cur
        if fin:
            break
    print(f"[{tag}] {label}: " + "; ".join(parts), flush=True)
