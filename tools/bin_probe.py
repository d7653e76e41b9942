"""Times the first binned round of config 4 (per-kernel ms): once on a fresh
layout (clean slots) and once after a full run (slots hold the last run's
words).  Run once per GOSSIP_BIN_* setting."""
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
    while True:
        st, fin = e.step()
        t = e.kernel_time("bin_scatter")
        if t[1] or fin:
            break
    print(f"[{tag}] {label} round {st['round']} scatter {t[0]:.3f} ms apply {e.kernel_time('bin_apply')[0]:.3f} ms",
          flush=True)
