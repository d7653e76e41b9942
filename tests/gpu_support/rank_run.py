"""One rank of a library-driven partitioned run (gossip_comm_init: RCCL inside libgossip_hip), launched by
tests/test_gpu_multiprocess.py with torch.distributed.run.  Every rank uses GPU `--device` (the test box has
one), torch.distributed (gloo) only hands out the RCCL unique id and gathers the results.  Rank 0 writes
the global per-round stats, the gathered reports and every block's seen words to --out."""
import argparse
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "p2p-gossipprotocol_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from gossip_hip import Engine, comm_unique_id, partition  # noqa: E402
from gossip_hip.workloads import config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, required=True)
    ap.add_argument("--peers", type=int, required=True)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--gather", type=int, default=-1)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    w = config(args.config, args.peers)  # the engine's Philox origins (the oracle's pick is the same draw)
    part = partition(w.n, world)
    e = Engine(w.n, w.n_msgs, device=args.device, part=(part[rank], part[rank + 1]),
               tuning={"gather_permille": args.gather}, **w.engine_kwargs())
    e.build_graph()
    e.inject(w.origins, w.inject_rounds)
    if w.kills:
        e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
    uid = [comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    status = "ok"
    try:
        e.comm_init(uid[0], world, rank)
    except Exception as ex:  # (the test reports why RCCL refused)
        status = f"comm_init: {ex}"
    res = {"status": status}
    if status == "ok":
        e.reset()
        stats = e.run()
        reps = e.comm_finalize(stats)
        res.update(stats=stats, reports=reps.tolist(), modes=e.comm_modes())
    seen = e.read_seen() if status == "ok" else np.zeros((0, 1), dtype=np.uint64)
    allres = [None] * world
    dist.all_gather_object(allres, (res, seen))
    if rank == 0:
        Path(args.out).write_text(json.dumps({"ranks": [r for r, _ in allres]}))
        np.save(Path(args.out).with_suffix(".npy"), np.concatenate([s for _, s in allres]) if status == "ok"
                else np.zeros(0, dtype=np.uint64))
    e.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
