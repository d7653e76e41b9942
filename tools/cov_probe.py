"""Per-message final coverage against the live peers for one config (diagnostic)."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "p2p-gossipprotocol_amd"))
from gossip_hip import Engine  # noqa: E402
from gossip_hip.workloads import config  # noqa: E402

w = config(int(sys.argv[1]) if len(sys.argv) > 1 else 5)
e = Engine(w.n, w.n_msgs, device=0, **w.engine_kwargs())
e.build_graph()
e.inject(w.origins, w.inject_rounds)
e.reset()
stats = e.run()
cov = e.coverage()
alive = e.alive()
print("rounds", len(stats), "alive", int(alive.sum()), "of", w.n)
print("coverage min/median/max", int(cov.min()), int(np.median(cov)), int(cov.max()))
print("messages below 99% of alive:", [(i, int(c)) for i, c in enumerate(cov) if c < 0.99 * alive.sum()][:10])
print("injected per round", [s["injected"] for s in stats][:3], "new_receipts", [s["new_receipts"] for s in stats])
