"""Wall time of the real-socket loopback harness (gossip_loopback: TCP peers on 127.0.0.1 with the
reference's wire formats) on BASELINE config 1, beside the round model's deliveries: the socket
path's deliveries per second for comparison with bench.py --config 1.  Measurement only."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "p2p-gossipprotocol_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import oracle_ref  # noqa: E402  (overlay generator and reference model: checker only)

from gossip_hip.loopback import run_loopback  # noqa: E402
from gossip_hip.workloads import config  # noqa: E402

orc = oracle_ref.Oracle(ROOT / "oracle" / "_build" / "libgossip_oracle.so")
w = config(1, pick=orc.pick_origins)
rp, col = orc.gen_workload(w)
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    res = run_loopback(rp, col, w.origins, w.inject_rounds)
    ts.append(time.perf_counter() - t0)
best = min(ts)
print({"workload": w.name, "peers": w.n, "edges": int(len(col)), "deliveries": res["deliveries"],
       "receipts": res["receipts"], "errors": res["errors"], "wall_s": [round(t, 3) for t in ts],
       "deliveries_per_s": round(res["deliveries"] / best, 1)})
