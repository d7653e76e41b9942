#!/usr/bin/env python3
"""bench.py -- gossip edge-deliveries/s (GTEPS) + rounds-to-full-coverage.

A step = one full propagation of the workload on the resident overlay:
reset (seen/new/alive/... cleared in HBM) -> rounds until no peer learns a
new message (peer.cpp's broadcastMessage/handleClient recursion run to
completion).  The overlay is built once, untimed (it is the seed bootstrap).

Default workload (N=1): BASELINE.json configs[3] -- 2^28 peers, power-law
overlay, 64 concurrent messages from Philox-chosen origins, run to full
coverage -- the largest configuration, and the one the metric's 1/2/4/8-GPU
series is quoted on.  With --gpus N the same 2^28-peer overlay is
vertex-partitioned over N GPUs (strong scaling) and libgossip_hip issues
each round's RCCL collectives itself:
  * under a launcher (torchrun: WORLD_SIZE = N) one process per GPU joins the
    communicator with gossip_comm_init;
  * without one, this process drives GPUs 0..N-1 itself (gossip_group_create,
    ncclCommInitAll) -- and exits non-zero if fewer GPUs are visible.
--parts P (N = 1) runs the same partitioned driver as P parts on ONE GPU, the
exchanges done by device copies: the single-GPU rehearsal of the N-GPU path.

One JSON line on rank 0; see DESIGN.md section 7 for every field.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "p2p-gossipprotocol_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# One xGMI link of the 8-GPU node (a GPU has 7, one to each other GPU).  AMD quotes MI355X's Infinity Fabric as 7
# links and 1075.2 GB/s aggregate, 153.6 GB/s a link, without saying whether that is each way or both ways
# together (MI300X's 128 GB/s a link is both ways, 64 each way).  The projection reports both readings:
XGMI_LINK_GBS = 153.6       # ... 153.6 GB/s each way (the upper bound)
XGMI_LINK_GBS_HALF = 76.8   # ... 153.6 GB/s both ways together: 76.8 each way (the lower bound)
DENSE_KERNELS = ("bin_scatter", "bin_apply", "pull_heavy", "heavy_commit")  # the device work of a binned round


def critical(x: dict, keys) -> float:
    """A round's device time over `keys` on its critical path: a side-stream kernel (SIDE_KERNELS: the heavy rows'
    pull beside a binned round's scatter) counts only if the round has no heavy_commit, whose timer covers the
    wait for it."""
    from gossip_hip.engine import SIDE_KERNELS
    side = x.get("heavy_commit", 0.0) > 0
    return sum(v for k, v in x.items() if k in keys and not (side and k in SIDE_KERNELS))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=4, help="BASELINE.json config index (1-5)")
    ap.add_argument("--n", type=int, default=0, help="override peer count")
    ap.add_argument("--parts", type=int, default=0,
                    help="N = 1 only: run the partitioned driver as this many parts on one GPU (device copies)")
    ap.add_argument("--cpu-sample-n", type=int, default=0, help="CPU baseline sample size, all threads (0: per config)")
    ap.add_argument("--cpu-sample-n1", type=int, default=0, help="CPU baseline sample size, 1 thread (0: per config)")
    ap.add_argument("--cpu-repeats", type=int, default=5)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip per-kernel HIP event timing")
    ap.add_argument("--pull-permille", type=int, default=0, help="push/pull switch point (0 = engine default)")
    ap.add_argument("--front-permille", type=int, default=0, help="frontier-bitmap switch point (0 = default)")
    ap.add_argument("--mode", default="auto", choices=["auto", "push", "pull"])
    ap.add_argument("--rebootstrap", type=int, default=0,
                    help="re-bootstrap after a death with this many extra out-edges per peer (configs 1, 5)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="gossip_set_tuning option for every part (A/B measurements; repeatable)")
    ap.add_argument("--force-partitioned", action="store_true",
                    help="use the library's multi-GPU driver (RCCL collectives) even at WORLD_SIZE 1")
    return ap.parse_args()


# kernel timer name -> rocprofv3 kernel-name prefix in the PMC summary
PMC_KERNELS = {"bin_scatter": ("k_bin_scatter_pc", "k_bin_stream"), "bin_apply": ("k_bin_apply", "k_bin_apply_runs"),
               "pull_light": ("k_pull_rows", "k_pull_light"),  # the row-queue pull is the default
               "push_light": ("k_push_light",), "push_heavy": ("k_push_heavy",), "pull_heavy": ("k_pull_heavy",),
               "heavy_commit": ("k_heavy_commit",)}


def pmc_traffic(workload: str, kernels, n_local: int):
    """HBM bytes per launch of `kernels` (summed: one binned round runs each
    once) from the committed rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE,
    separate runs of this bench command on the same config, newest round
    first) with the gfx950 corrections measured by tools/calib_fetch.hip
    (profiles/r01/calib_fetch_timing.log): FETCH_SIZE counts 1/2 of coalesced
    streamed bytes and one 64-B line per random 8-B gather; WRITE_SIZE counts
    stores 1:1.  The binned kernels read coalesced streams (traffic = 2 x
    fetch + write); pull_heavy's gathers are counted 1:1."""
    cfg = workload.split("_")[0]  # "config4" ...
    cands = [REPO / "profiles" / r / f"{cfg}_pmc_summary.json" for r in ("r06", "r05", "r04", "r03", "r02", "r01")]
    path = next((p for p in cands if p.exists()), None)
    if path is None:
        return None, None
    prof = json.loads(path.read_text())
    total, parts = 0.0, []
    for kernel in kernels:
        keys = [k for k in prof["kernels"] if any(k.startswith(p + "<") or k == p for p in PMC_KERNELS.get(kernel, ()))]
        keys = [k for k in keys if "fetch_bytes_per_launch_counted" in prof["kernels"][k]]
        if not keys:
            if kernel in ("bin_scatter", "bin_apply"):
                return None, None
            parts.append(f"{kernel}: not in the summary")  # (an older summary: no k_heavy_commit)
            continue
        launches = sum(prof["kernels"][k]["launches"] for k in keys)
        fetch = sum(prof["kernels"][k]["fetch_bytes_per_launch_counted"] * prof["kernels"][k]["launches"] for k in keys)
        write = sum(prof["kernels"][k].get("write_bytes_per_launch_counted", 0.0) * prof["kernels"][k]["launches"]
                    for k in keys)
        fetch, write = fetch / launches, write / launches
        total += (2 * fetch if kernel in ("bin_scatter", "bin_apply") else fetch) + write
        avg = sum(prof["kernels"][k]["avg_ms"] * prof["kernels"][k]["launches"] for k in keys) / launches
        parts.append(f"{', '.join(keys)}: {launches} launches, avg {avg:.3f} ms")
    return round(total), f"{path.relative_to(REPO)} ({'; '.join(parts)})"


def rounds_to_full(stats: list[dict]) -> int:
    last = 0
    for s in stats:
        if s["new_receipts"] > 0:
            last = s["round"] + 1
    return last - min(s["round"] for s in stats if s["injected"] > 0) if any(s["injected"] for s in stats) else 0


def _cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores() -> int:
    """CPUs this process may run on (its affinity mask: 16 of the box's 256 on a gpurun box)."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


# CPU baseline samples per BASELINE.json config: (all-threads n, 1-thread n, literal-driver n or 0)
CPU_SAMPLES = {1: (8, 8, 8), 2: (1 << 20, 1 << 18, 1 << 18), 3: (1 << 24, 1 << 20, 0), 4: (1 << 25, 1 << 21, 0),
               5: (1 << 22, 1 << 19, 0)}


def cpu_baseline(args, cfg_idx: int) -> dict:
    """The oracle's 64-bit-mask round driver (gcc -O3 -fopenmp; the restatement
    of peer.cpp:255-318 that the GPU is checked against) on bounded samples of
    the same workload, timed on this host: oracle_sim_run only (the rounds;
    overlay generation, sim allocation and read-backs untimed), median of
    --cpu-repeats fresh runs, at the host's thread budget and at 1 thread.
    Configs 1-2 also time the literal driver (per-peer Message-List hash sets
    with sentTo counts, peer.hpp:23-26,52), single-threaded."""
    import statistics
    sys.path.insert(0, str(REPO / "tests"))
    import oracle_ref  # noqa: E402  (checker / baseline only)
    from gossip_hip.workloads import config

    so = REPO / "oracle" / "_build" / "libgossip_oracle.so"
    orc = oracle_ref.Oracle(so)
    cores = host_cores()
    threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", 0) or cores)
    n_all, n_one, n_lit = CPU_SAMPLES[cfg_idx]
    n_all = args.cpu_sample_n or n_all
    n_one = args.cpu_sample_n1 or n_one
    out = {}
    legs = [("all", n_all, threads, 0, args.cpu_repeats), ("one", n_one, 1, 0, args.cpu_repeats)]
    if n_lit:
        legs.append(("literal", n_lit, 1, 1, 1 if n_lit > 4096 else args.cpu_repeats))
    for label, n, th, variant, reps in legs:
        w = config(cfg_idx, n, pick=orc.pick_origins)
        rp, col = orc.gen_workload(w, threads=threads)
        secs, stats = orc.time_rounds(w, rp, col, threads=th, variant=variant, repeats=reps)
        med = statistics.median(secs)
        d = sum(s["deliveries"] for s in stats)
        t = sum(s["traversals"] for s in stats)
        out[label] = {"gteps": d / med / 1e9, "traversal_gteps": t / med / 1e9, "n": w.n, "edges": int(len(col)),
                      "rounds": len(stats), "median_s": med, "runs_s": [round(x, 4) for x in secs], "threads": th,
                      "sample": f"{w.name} at n={w.n} ({len(col)} edges, {len(stats)} rounds)"}
    a, o = out["all"], out["one"]
    res = {"value": round(a["gteps"], 4), "unit": "GTEPS", "cores": threads, "kind": "port",
           "traversal_gteps": round(a["traversal_gteps"], 4),
           "single_thread": {"value": round(o["gteps"], 4), "traversal_gteps": round(o["traversal_gteps"], 4),
                             "median_s": round(o["median_s"], 4), "runs_s": o["runs_s"], "sample": o["sample"]},
           "host_cores": cores, "machine_cpus": os.cpu_count(), "cpu_model": _cpu_model(),
           "median_s": round(a["median_s"], 4), "runs_s": a["runs_s"],
           "timed": "oracle_sim_run only (rounds); generation, allocation and read-backs excluded",
           "sample": f"{a['sample']}, oracle fast driver, {threads} threads ({cores} CPUs in this process's affinity "
                     f"mask), median of {args.cpu_repeats}"}
    if "literal" in out:
        lt = out["literal"]
        res["literal_driver"] = {"value": round(lt["gteps"], 6), "median_s": round(lt["median_s"], 4),
                                 "runs_s": lt["runs_s"], "threads": 1, "sample": lt["sample"]}
    return res


# ---- the three ways of running the workload --------------------------------------------------
class Single:
    """One ctx owns every peer (gossip_step / gossip_run)."""

    def __init__(self, w, dev, tune):
        from gossip_hip import Engine
        self.eng = Engine(w.n, w.n_msgs, device=dev, **tune, **w.engine_kwargs())
        self.eng.build_graph()
        self.eng.inject(w.origins, w.inject_rounds)
        if w.kills:
            self.eng.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        self.parts, self.n_gpus = 1, 1
        sh = self.eng.shape()
        self.n_edges, self.n_local = sh["n_edges"], [sh["n_local"]]

    def step(self):
        self.eng.reset()
        return self.eng.run()

    def lean_step(self):  # the same step, its stats left in the engine's buffer (no per-round dicts)
        self.eng.reset()
        return self.eng.run_into()

    def last_stats(self):
        return self.eng.last_stats()

    def sync(self):
        import torch
        torch.cuda.synchronize()

    def timing(self, on):
        self.eng.enable_timing(on)

    def ktime(self, p, k):
        return self.eng.kernel_time(k)

    def kbytes(self, p, k):
        return self.eng.kernel_bytes(k)

    def round_step(self):
        return self.eng.step()

    def reset(self):
        self.eng.reset()

    def close(self):
        self.eng.close()


class Grouped(Single):
    """One process drives P parts (gossip_group_*): on P GPUs (RCCL from
    ncclCommInitAll) or, emulated, all on one GPU (device copies)."""

    def __init__(self, w, devices, tune):
        from gossip_hip import Group
        self.g = Group(w.n, w.n_msgs, devices, **tune, **w.engine_kwargs())
        self.g.build_graph()
        self.g.inject(w.origins, w.inject_rounds)
        if w.kills:
            self.g.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        self.devices = devices
        self.parts, self.n_gpus = len(devices), len(set(devices))
        shapes = [self.g.shape(p) for p in range(self.parts)]
        self.n_edges = sum(s["n_edges"] for s in shapes)
        self.n_local = [s["n_local"] for s in shapes]

    def step(self):
        self.g.reset()
        return self.g.run()

    def lean_step(self):
        self.g.reset()
        return self.g.run_into()

    def last_stats(self):
        return self.g.last_stats()

    def sync(self):
        import torch
        for d in sorted(set(self.devices)):
            torch.cuda.synchronize(d)

    def timing(self, on):
        self.g.enable_timing(on)

    def ktime(self, p, k):
        return self.g.kernel_time(p, k)

    def kbytes(self, p, k):
        return self.g.kernel_bytes(p, k)

    def round_step(self):
        return self.g.step()

    def reset(self):
        self.g.reset()

    def close(self):
        self.g.close()


class Ranked(Single):
    """One process per GPU under a launcher: this rank's block, gossip_comm_init."""

    def __init__(self, w, dev, tune, world, rank):
        import torch.distributed as dist

        from gossip_hip import Engine, comm_unique_id, partition_edges
        self.dist, self.world, self.rank = dist, world, rank
        # blocks of about equal work (the powerlaw overlay's edges sit at the low ids), as gossip_group_create
        kw = {**{k: v for k, v in tune.items() if k != "tuning"}, **w.engine_kwargs()}  # (one dict: no duplicate keys)
        part = partition_edges(w.n, w.n_msgs, world, **kw)
        self.eng = Engine(w.n, w.n_msgs, device=dev, part=(part[rank], part[rank + 1]), **tune, **w.engine_kwargs())
        self.eng.build_graph()
        self.eng.inject(w.origins, w.inject_rounds)
        if w.kills:
            self.eng.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        uid = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        self.eng.comm_init(uid[0], world, rank)
        self.parts, self.n_gpus = 1, world
        sh = self.eng.shape()
        import torch
        t = torch.tensor([sh["n_edges"]], dtype=torch.int64)
        dist.all_reduce(t)
        self.n_edges, self.n_local = int(t.item()), [sh["n_local"]]

    def sync(self):
        import torch
        torch.cuda.synchronize()
        self.dist.barrier()


LIVE_COUNTERS = ("#pings", "#pinging_peers")  # 8(d)'s liveness term of a ping round (k_live_count)


def part_agg(run):
    """How per-part device times combine into the run's: the max over the parts
    when each part has its own GPU (they run concurrently), the sum when P parts
    share one GPU (their kernels run one after another on it)."""
    return max if run.parts == run.n_gpus else sum


def per_round_profile(run, n_peers: int) -> list[dict]:
    """One run, stepped round by round with per-kernel timing (untimed pass):
    each round's mode; SURVEY 8(d)'s algorithmic bytes B_r = 32 F_r + 20 T_r,
    plus 6.125 B per ping and 16 B per pinging peer in a ping round; the
    kernels' own design bytes (summed over the round's
    kernels and parts); the device time of its kernels (max over the parts of
    a partitioned run on one GPU per part, the sum over the parts of one run
    emulating P parts on a single GPU, where they run one after another) and
    exchanges; and the round's fraction of the HBM
    peak, frac = B_r / kernel time / peak.  A round whose kernels move fewer
    bytes than 8(d) charges it is marked work_avoiding, with the reason: pull
    rounds (row, list and heavy pulls) stop a row's scan once it holds every
    bit it can still learn, so 8(d)'s 20 B per traversal overstates what they
    touch ("pull"); a ping round's 6.125 B per ping are charged for every ping
    pingLoop sends, while the closed-form liveness only walks the rows of the
    peers whose miss count reaches the limit ("liveness").  Their frac can
    pass 1."""
    from gossip_hip.engine import EXCHANGES, KERNELS
    names = KERNELS + EXCHANGES
    agg = part_agg(run)
    run.reset()
    run.timing(True)
    kb = lambda: [{k: run.kbytes(p, k) for k in KERNELS + LIVE_COUNTERS} for p in range(run.parts)]  # noqa: E731
    prev = [{k: run.ktime(p, k)[0] for k in names} for p in range(run.parts)]
    prev_b = kb()
    rows = []
    while True:
        st, fin = run.round_step()
        cur = [{k: run.ktime(p, k)[0] for k in names} for p in range(run.parts)]
        cur_b = kb()
        d = [{k: c[k] - q[k] for k in names if c[k] - q[k] > 0} for c, q in zip(cur, prev)]
        db = {k: sum(c[k] - q[k] for c, q in zip(cur_b, prev_b)) for k in KERNELS + LIVE_COUNTERS}
        prev, prev_b = cur, cur_b
        mode = "bin" if any("bin_scatter" in x for x in d) else "blocked" if any("pb_scatter" in x for x in d) else \
            "pull" if any("pull_light" in x or "pull_list" in x for x in d) else "push"
        kms = agg(critical(x, KERNELS) for x in d)
        xms = agg(sum(v for k, v in x.items() if k in EXCHANGES) for x in d)
        dense = agg(critical(x, DENSE_KERNELS) for x in d)
        live_b = 6.125 * db["#pings"] + 16 * db["#pinging_peers"]
        alg = 32 * st["frontier"] + 20 * st["traversals"] + live_b
        frac = alg / (kms / 1e3) / 1e9 / HBM_PEAK_GBS if kms > 0 else 0.0
        design = sum(db[k] for k in KERNELS)
        why = "pull" if mode == "pull" else "liveness" if live_b and design < alg else None
        rows.append({"round": st["round"], "mode": mode, "frontier_frac": round(st["frontier"] / n_peers, 4),
                     "traversals": st["traversals"], "alg_bytes": round(alg), "liveness_bytes": round(live_b),
                     "design_bytes": round(design),
                     "kernel_ms": round(kms, 3), "exchange_ms": round(xms, 3), "dense_ms": round(dense, 3),
                     "frac": round(frac, 4), "work_avoiding": why is not None, "avoided": why})
        if fin:
            run.timing(False)
            return rows


def link_projection(run, k_ms, k_b, timed_steps: int, dist) -> dict:
    """What the partitioned run's exchange costs on the 8-GPU node's xGMI mesh:
    per rank, the bytes it receives per step over its P - 1 links (one to each
    other rank, XGMI_LINK_GBS each way) -- exchange_link_ms, the max over the
    ranks.  For a rehearsal of P parts on one GPU (whose exchanges are device
    copies) the projected P-GPU step is the slowest part's kernel time plus
    that link time, with no overlap of the two and no host time:
    projected_ms_per_step."""
    from gossip_hip.engine import EXCHANGES, KERNELS
    world = run.parts if dist is None else run.world
    if world < 2:
        return {}
    gb = max(sum(x[k] for k in EXCHANGES) for x in k_b) / timed_steps / 1e9  # the busiest rank's GB per step
    link = gb / ((world - 1) * XGMI_LINK_GBS) * 1e3
    link_lo = gb / ((world - 1) * XGMI_LINK_GBS_HALF) * 1e3
    out = {"exchange_gb_per_step_busiest_rank": round(gb, 3),
           "exchange_link_ms_per_step": round(link, 3),
           "exchange_link_ms_per_step_half_rate": round(link_lo, 3),
           "exchange_link_model": f"max over ranks of the bytes a rank receives per step / ({world - 1} links x "
                                  f"{XGMI_LINK_GBS} GB/s each way); _half_rate: {XGMI_LINK_GBS_HALF} GB/s each way "
                                  "(AMD's 153.6 GB/s a link read as both ways together)"}
    if run.parts > 1 and run.n_gpus == 1:
        part_k = [sum(x[k][0] for k in KERNELS) / timed_steps for x in k_ms]
        out.update({"part_kernel_ms_per_step": [round(v, 3) for v in part_k],
                    "projected_ms_per_step": round(max(part_k) + link, 3),
                    "projected_ms_per_step_half_rate": round(max(part_k) + link_lo, 3),
                    "projected_model": "slowest part's kernels + exchange_link_ms_per_step, no overlap, no host time"})
    return out


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus != world:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}: {world} ranks run", file=sys.stderr)
    from gossip_hip import device_count
    from gossip_hip.workloads import config

    w = config(args.config, args.n or None, rebootstrap=args.rebootstrap)
    tune = dict(pull_permille=args.pull_permille, front_permille=args.front_permille, mode=args.mode)
    if args.tune:
        tune["tuning"] = {k: int(v) for k, v in (t.split("=", 1) for t in args.tune)}
    dist = None
    if world > 1 or args.force_partitioned:
        # one process per GPU; libgossip_hip drives every round's RCCL collectives
        # itself (gossip_comm_init); torch.distributed (gloo, host side) only hands
        # out the RCCL unique id and keeps the barrier and max-over-ranks timing
        import torch.distributed as dist
        for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29511")):
            os.environ.setdefault(k, v)  # --force-partitioned run without a launcher
        torch.cuda.set_device(local)
        dist.init_process_group("gloo")
        run = Ranked(w, local, tune, world, rank)
    elif args.gpus > 1:
        have = device_count()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, this process sees {have} "
                  f"(one process drives GPUs 0..{args.gpus - 1} through gossip_group_create; or launch "
                  f"{args.gpus} ranks with torchrun)", file=sys.stderr)
            sys.exit(2)
        run = Grouped(w, list(range(args.gpus)), tune)
    elif args.parts > 1:
        torch.cuda.set_device(local)
        run = Grouped(w, [local] * args.parts, tune)
    else:
        torch.cuda.set_device(local)
        run = Single(w, local, tune)

    for _ in range(args.warmup):
        run.step()
    # the headline: K steps with per-kernel timing off (no events in the timed loop).  Each step's per-round
    # stats land in a host buffer the library fills; the Python dicts of the last one are built after the clock
    # (47 rounds of dicts were a third of config 1's step)
    run.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run.lean_step()
    run.sync()
    dt = time.perf_counter() - t0
    stats = run.last_stats()
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    deliveries = sum(s["deliveries"] for s in stats)
    value = args.steps * deliveries / dt / 1e9
    roofline = None
    rounds_prof = None
    if not args.no_timing:
        from gossip_hip.engine import EXCHANGES, KERNELS
        # per-kernel device times from HIP events on each part's stream, in a separate pass of the same steps
        timed_steps = min(args.steps, 5)
        run.timing(True)
        run.sync()
        t1 = time.perf_counter()
        for _ in range(timed_steps):
            run.step()
        run.sync()
        dt_timed = time.perf_counter() - t1
        k_ms = [{k: run.ktime(p, k) for k in KERNELS + EXCHANGES} for p in range(run.parts)]
        k_b = [{k: run.kbytes(p, k) for k in KERNELS + EXCHANGES} for p in range(run.parts)]
        run.timing(False)
        agg = part_agg(run)
        # the per-round pass: which rounds ran binned / pull / push, their 8(d) bytes and device time
        rounds_prof = per_round_profile(run, w.n)
        dense = [r for r in rounds_prof if r["mode"] == "bin"]
        alg = sum(r["alg_bytes"] for r in rounds_prof)
        # the dominant kernel by device time (part 0's; every part runs the same schedule).  A side-stream kernel's
        # events also time its wait for CUs beside the scatter (config 5's heavy-row pull: 0.94 ms per launch by
        # events for 1.5 % of its design bytes), so it is not a candidate when it ran beside a join (critical())
        from gossip_hip.engine import SIDE_KERNELS
        side_used = k_ms[0].get("heavy_commit", (0.0, 0))[1] > 0
        dom = max((k for k in KERNELS if not (side_used and k in SIDE_KERNELS)), key=lambda k: k_ms[0][k][0])
        ms, launches = k_ms[0][dom]
        # without the work-avoiding rounds: a pull round's 8(d) bytes out of the numerator and its kernel and
        # exchange time out of the step; a ping round's liveness bytes out of the numerator (its push or binned
        # work shares the round's time, which stays)
        step_ms = dt / args.steps * 1e3
        wa = [r for r in rounds_prof if r["work_avoiding"]]
        pulls = [r for r in wa if r["avoided"] == "pull"]
        live_all = sum(r["liveness_bytes"] for r in rounds_prof)
        rest_ms = step_ms - sum(r["kernel_ms"] + r["exchange_ms"] for r in pulls)
        rest_b = alg - sum(r["alg_bytes"] for r in pulls) - sum(r["liveness_bytes"] for r in wa
                                                                if r["avoided"] == "liveness")
        peak_all = HBM_PEAK_GBS * run.n_gpus
        roofline = {"bound": "hbm", "peak": peak_all, "unit": "GB/s",
                    "step_frac": round(alg / (dt / args.steps) / 1e9 / peak_all, 4),
                    "step_frac_without_liveness": round((alg - live_all) / (dt / args.steps) / 1e9 / peak_all, 4),
                    "step_frac_without_work_avoiding": round(rest_b / (rest_ms / 1e3) / 1e9 / peak_all, 4)
                    if rest_ms > 0 else None,
                    "work_avoiding_rounds": [r["round"] for r in wa],
                    "step_alg_bytes": round(alg), "step_liveness_bytes": live_all,
                    "timed_steps": timed_steps,
                    "ms_per_step_with_events": round(dt_timed / timed_steps * 1e3, 3),
                    "kernel_ms_per_step": {k: round(agg(x[k][0] for x in k_ms) / timed_steps, 3)
                                           for k in KERNELS if k_ms[0][k][1]},
                    "exchange_ms_per_step": {k: round(agg(x[k][0] for x in k_ms) / timed_steps, 3)
                                             for k in EXCHANGES if k_ms[0][k][1]},
                    "exchange_gb_per_step": {k: round(sum(x[k] for x in k_b) / timed_steps / 1e9, 3)
                                             for k in EXCHANGES if k_ms[0][k][1]}}
        if run.parts > 1 or dist is not None:
            roofline.update(link_projection(run, k_ms, k_b, timed_steps, dist))
        if dense:
            # SURVEY 8(d)'s bytes of the binned rounds over the device time of their kernels
            # (bin_scatter + bin_apply + pull_heavy; part_agg over the parts): the honest dense-round fraction
            d_b = sum(r["alg_bytes"] for r in dense)
            d_ms = sum(r["dense_ms"] for r in dense)
            ach = d_b / (d_ms / 1e3) / 1e9
            traffic, tsrc = pmc_traffic(w.name, DENSE_KERNELS, run.n_local[0]) if run.parts == 1 else (None, None)
            roofline.update({"kernel": "binned round: " + " + ".join(DENSE_KERNELS) + " (pull_heavy beside the scatter "
                                       "on a second stream when heavy_commit runs: its time is then off the round's "
                                       "critical path)",
                             "achieved": round(ach, 2), "frac": round(ach / roofline["peak"], 4),
                             "alg_bytes_per_launch": round(d_b / len(dense)),
                             "avg_launch_ms": round(d_ms / len(dense), 4), "launches": len(dense),
                             "unit_of_work": "one binned round (SURVEY 8(d): 32 B per frontier peer + 20 B per "
                                             "edge traversal)",
                             "traffic": traffic, "traffic_source": tsrc,
                             "dense_rounds": [r["round"] for r in dense]})
        if ms > 0 and launches:
            # the dominant kernel's own design bytes per launch over its HIP-event time
            per_launch = sum(x[dom] for x in k_b) / run.parts / launches
            ach_k = per_launch / (ms / launches / 1e3) / 1e9
            roofline.update({"dominant_kernel": dom, "dominant_avg_launch_ms": round(ms / launches, 4),
                             "dominant_launches": launches, "dominant_design_bytes_per_launch": round(per_launch),
                             "dominant_design_frac": round(ach_k / HBM_PEAK_GBS, 4)})
            if "kernel" not in roofline:  # no binned round: the dominant kernel is the roofline line
                traffic, tsrc = pmc_traffic(w.name, (dom,), run.n_local[0]) if run.parts == 1 else (None, None)
                roofline.update({"kernel": dom, "achieved": round(ach_k * run.n_gpus, 2),
                                 "frac": round(ach_k / HBM_PEAK_GBS, 4), "alg_bytes_per_launch": round(per_launch),
                                 "avg_launch_ms": round(ms / launches, 4), "launches": launches,
                                 "traffic": traffic, "traffic_source": tsrc})

    if rank == 0:
        para = (f"vertex-partition x{run.n_gpus}" if run.parts == run.n_gpus else
                f"vertex-partition x{run.parts} on one GPU (device-copy exchange)")
        launcher = "torchrun (gossip_comm_init)" if dist is not None else \
            "one process, gossip_group (ncclCommInitAll)" if run.n_gpus > 1 else "one process"
        line = {
            "metric": "gossip edge-deliveries/sec (GTEPS) + rounds-to-full-coverage",
            "value": round(value, 3),
            "unit": "GTEPS",
            "n_gpus": run.n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (Philox-generated power-law overlay and origins)",
            "config": {"workload": w.name, "peers": w.n, "edges": run.n_edges,
                       "messages": w.n_msgs, "rounds": len(stats),
                       "rounds_to_full_coverage": rounds_to_full(stats),
                       "deliveries_per_step": deliveries,
                       "traversals_per_step": sum(s["traversals"] for s in stats),
                       "parallelism": para, "launch": launcher},
            "traversal_gteps": round(args.steps * sum(s["traversals"] for s in stats) / dt / 1e9, 3),
        }
        if rounds_prof:
            line["rounds"] = [{k: r[k] for k in ("round", "mode", "frontier_frac", "traversals", "alg_bytes",
                                                 "design_bytes", "kernel_ms", "frac", "work_avoiding")} |
                              ({"liveness_bytes": r["liveness_bytes"]} if r["liveness_bytes"] else {}) |
                              ({"avoided": r["avoided"]} if r["avoided"] else {}) |
                              ({"exchange_ms": r["exchange_ms"]} if run.parts > 1 or dist is not None else {})
                              for r in rounds_prof]
        if roofline:
            line["roofline"] = roofline
        if run.n_gpus == 1 and run.parts == 1 and dist is None and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args, args.config)
        print(json.dumps(line), flush=True)
    if isinstance(run, Ranked):
        reps = run.eng.comm_finalize(stats)
        if rank == 0 and args.force_partitioned:
            print(json.dumps({"partitioned_check": {"modes": run.eng.comm_modes(), "reports": int(len(reps))}}),
                  flush=True)
    run.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
