"""In-process A/B of engine tuning variants on one kernel (arms alternated in ONE process, so the placement of
the process's buffers is the same for every arm).  Usage:
  ab_kernel.py CONFIG KERNEL REPS key=val[,key=val] ...   ("-" = defaults)
Prints each arm's kernel ms per run (sum over the run's rounds) for every repetition, then the medians.
KERNEL "step": the run's wall time (reset + rounds, host clock, no per-kernel events).  Layout keys (bin_words,
bin_chunk, scatter_units, heavy_degree, heavy_chunk) rebuild the overlay and its layout for their arm."""
import time
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
# the engine's defaults of the keys an arm may set (an arm leaves the others at these)
defaults = {"row_grid": 0, "row_queue": 128, "apply_pipe": 5, "pull_first2": 1, "heavy_exit": 1, "bin_needy_skip": 1,
            "apply_persist": 1, "in_flight": 1, "blocked_pipe": 1,
            "zero_fill": 1}
e.reset()
e.run()
e.enable_timing(True)
LAYOUT = ("bin_words", "bin_chunk", "scatter_units", "heavy_degree", "heavy_chunk")
res = [[] for _ in arms]
if kern == "step":
    e.enable_timing(False)
for rep in range(reps):
    for i, a in enumerate(arms):
        for k in keys:
            e.set_tuning(k, a.get(k, defaults.get(k, -1 if k not in LAYOUT or k == "heavy_degree" else 0)))
        if any(k in LAYOUT for k in keys):
            e.build_graph()
            e.inject(w.origins, w.inject_rounds)
            if w.kills:
                e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
            e.reset()
            e.run()  # (first run of a layout: records the schedule)
        if kern == "step":
            best = 1e9
            for _ in range(5):
                t0 = time.perf_counter()
                e.reset()
                e.run()
                best = min(best, (time.perf_counter() - t0) * 1e3)
            res[i].append(best)
            continue
        e.reset()
        t0 = e.kernel_time(kern)[0]
        e.run()
        res[i].append(e.kernel_time(kern)[0] - t0)
    print(rep, [round(r[-1], 3) for r in res], flush=True)
for a, r in zip(sys.argv[4:], res):
    print(f"{a:40s} median {statistics.median(r):.3f} ms  min {min(r):.3f}", flush=True)
