"""In-process A/B of engine tuning variants on one kernel (arms alternated in ONE process, so the placement of
the process's buffers is the same for every arm).  Usage:
  ab_kernel.py CONFIG KERNEL REPS key=val[,key=val] ...   ("-" = defaults)
Prints each arm's kernel ms per run (sum over the run's rounds) for every repetition, then the medians."""
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "p2p-gossipprotocol_amd"))
from gossip_hip import Engine  # noqa: E402
from gossip_hip.workloads import config  # noqa: E402

w = config(int(sys.argv[1]))
kern, reps = sys.argv[2], int(sys.argv[3])
arms = [{} if a == "-" else {k: int(v) for k, v in (x.split("=") for x in a.split(","))} for a in sys.argv[4:]]
keys = sorted({k for a in arms for k in a})
e = Engine(w.n, w.n_msgs, device=0, **w.engine_kwargs())
e.build_graph()
e.inject(w.origins, w.inject_rounds)
if w.kills:
    e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
defaults = {"row_grid": 0, "row_queue": 128}
e.reset()
e.run()
e.enable_timing(True)
res = [[] for _ in arms]
for rep in range(reps):
    for i, a in enumerate(arms):
        for k in keys:
            e.set_tuning(k, a.get(k, defaults.get(k, -1)))
        e.reset()
        t0 = e.kernel_time(kern)[0]
        e.run()
        res[i].append(e.kernel_time(kern)[0] - t0)
    print(rep, [round(r[-1], 3) for r in res], flush=True)
for a, r in zip(sys.argv[4:], res):
    print(f"{a:40s} median {statistics.median(r):.3f} ms  min {min(r):.3f}", flush=True)
