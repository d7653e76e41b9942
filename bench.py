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
vertex-partitioned over N ranks (strong scaling); libgossip_hip issues each
round's RCCL collectives itself (gossip_comm_init).

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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=4, help="BASELINE.json config index (1-5)")
    ap.add_argument("--n", type=int, default=0, help="override peer count")
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
    ap.add_argument("--force-partitioned", action="store_true",
                    help="use the library's multi-GPU driver (RCCL collectives) even at WORLD_SIZE 1")
    return ap.parse_args()


# kernel timer name -> rocprofv3 kernel-name prefix in the PMC summary
PMC_KERNELS = {"bin_scatter": ("k_bin_scatter_pc",), "bin_apply": ("k_bin_apply",),
               "pull_light": ("k_pull_rows", "k_pull_light"),  # the row-queue pull is the default
               "push_light": ("k_push_light",), "push_heavy": ("k_push_heavy",), "pull_heavy": ("k_pull_heavy",)}


def pmc_traffic(workload: str, kernel: str, alg_bytes_per_launch: float, n_local: int):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (FETCH_SIZE and WRITE_SIZE, separate runs of this bench command on the same
    config: tools/gpu_profile_r02.sh, newest round first) with the
    gfx950 corrections measured by tools/calib_fetch.hip (profiles/r01/
    calib_fetch_timing.log): FETCH_SIZE counts 1/2 of coalesced streamed bytes
    and one 64-B line per random 8-B gather; WRITE_SIZE counts stores 1:1.
    bin_scatter / bin_apply read only coalesced streams (traffic = 2 x fetch +
    write); pull_light mixes streams with random gathers (only its streamed
    reads are doubled)."""
    if kernel not in PMC_KERNELS:
        return None, None
    cfg = workload.split("_")[0]  # "config4" ...
    cands = [REPO / "profiles" / r / f"{cfg}_pmc_summary.json" for r in ("r02", "r01")]
    path = next((p for p in cands if p.exists()), None)
    if path is None:
        return None, None
    prof = json.loads(path.read_text())
    keys = [k for k in prof["kernels"] if any(k.startswith(p + "<") or k == p for p in PMC_KERNELS[kernel])]
    keys = [k for k in keys if "fetch_bytes_per_launch_counted" in prof["kernels"][k]]
    if not keys:
        return None, None
    launches = sum(prof["kernels"][k]["launches"] for k in keys)
    fetch = sum(prof["kernels"][k]["fetch_bytes_per_launch_counted"] * prof["kernels"][k]["launches"] for k in keys)
    write = sum(prof["kernels"][k].get("write_bytes_per_launch_counted", 0.0) * prof["kernels"][k]["launches"]
                for k in keys)
    fetch, write = fetch / launches, write / launches
    if kernel in ("bin_scatter", "bin_apply"):
        t = 2 * fetch + write
    elif kernel == "pull_light":
        scanned = max(alg_bytes_per_launch - 40.0 * n_local, 0.0) / 12.0
        t = fetch + (24.0 * n_local + 4.0 * scanned) / 2 + write
    else:
        t = fetch + write
    avg = sum(prof["kernels"][k]["avg_ms"] * prof["kernels"][k]["launches"] for k in keys) / launches
    return round(t), f"{path.relative_to(REPO)} ({', '.join(keys)}: {launches} launches, avg {avg:.3f} ms)"


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
    nproc = os.cpu_count() or 1
    threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", 0) or nproc)
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
           "nproc": nproc, "cpu_model": _cpu_model(), "median_s": round(a["median_s"], 4), "runs_s": a["runs_s"],
           "timed": "oracle_sim_run only (rounds); generation, allocation and read-backs excluded",
           "sample": f"{a['sample']}, oracle fast driver, {threads} threads of {nproc} visible CPUs, "
                     f"median of {args.cpu_repeats}"}
    if "literal" in out:
        lt = out["literal"]
        res["literal_driver"] = {"value": round(lt["gteps"], 6), "median_s": round(lt["median_s"], 4),
                                 "runs_s": lt["runs_s"], "threads": 1, "sample": lt["sample"]}
    return res


def per_round_profile(eng) -> list[dict]:
    """One run, stepped round by round with per-kernel timing (untimed pass)."""
    from gossip_hip.engine import KERNELS
    eng.reset()
    eng.enable_timing(True)
    prev = {k: eng.kernel_time(k)[0] for k in KERNELS}
    rows = []
    while True:
        st, fin = eng.step()
        cur = {k: eng.kernel_time(k)[0] for k in KERNELS}
        d = {k: cur[k] - prev[k] for k in KERNELS if cur[k] - prev[k] > 0}
        prev = cur
        mode = "bin" if "bin_scatter" in d else "pull" if "pull_light" in d else "push"
        rows.append({"round": st["round"], "mode": mode, "frontier_frac": round(st["frontier"] / eng.n_peers, 4),
                     "traversals": st["traversals"], "alg_bytes": 32 * st["frontier"] + 20 * st["traversals"],
                     "kernel_ms": round(sum(d.values()), 3)})
        if fin:
            return rows


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from gossip_hip import Engine
    from gossip_hip.workloads import config

    w = config(args.config, args.n or None, rebootstrap=args.rebootstrap)
    tune = dict(pull_permille=args.pull_permille, front_permille=args.front_permille, mode=args.mode)
    partitioned = world > 1 or args.force_partitioned
    if partitioned:
        # one process per GPU; libgossip_hip drives every round's RCCL collectives
        # itself (gossip_comm_init); torch.distributed (gloo, host side) only hands
        # out the RCCL unique id and keeps the barrier and max-over-ranks timing
        import torch.distributed as dist

        from gossip_hip import comm_unique_id, partition

        for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29511")):
            os.environ.setdefault(k, v)  # --force-partitioned run without a launcher
        dist.init_process_group("gloo")
        part = partition(w.n, world)
        eng = Engine(w.n, w.n_msgs, device=local, part=(part[rank], part[rank + 1]), **tune, **w.engine_kwargs())
        eng.build_graph()
        eng.inject(w.origins, w.inject_rounds)
        if w.kills:
            eng.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        uid = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init(uid[0], world, rank)

        def one_step():
            eng.reset()
            return eng.run()

        def barrier():
            torch.cuda.synchronize()
            dist.barrier()
    else:
        eng = Engine(w.n, w.n_msgs, device=local, **tune, **w.engine_kwargs())
        eng.build_graph()
        eng.inject(w.origins, w.inject_rounds)
        if w.kills:
            eng.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])

        def one_step():
            eng.reset()
            return eng.run()

        def barrier():
            torch.cuda.synchronize()

    shape = eng.shape()
    n_edges = shape["n_edges"]
    if partitioned:
        t = torch.tensor([n_edges], dtype=torch.int64)
        dist.all_reduce(t)
        n_edges = int(t.item())
    for _ in range(args.warmup):
        one_step()
    # the headline: K steps with per-kernel timing off (no events in the timed loop)
    barrier()
    t0 = time.perf_counter()
    stats = None
    for _ in range(args.steps):
        stats = one_step()
    barrier()
    dt = time.perf_counter() - t0
    if partitioned:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    deliveries = sum(s["deliveries"] for s in stats)
    value = args.steps * deliveries / dt / 1e9
    roofline = None
    timed_steps = 0
    if not args.no_timing:
        # per-kernel device times from HIP events on the ctx stream, in a separate pass of the same steps
        from gossip_hip.engine import KERNELS
        timed_steps = min(args.steps, 5)
        eng.enable_timing(True)
        barrier()
        t1 = time.perf_counter()
        for _ in range(timed_steps):
            one_step()
        barrier()
        dt_timed = time.perf_counter() - t1
        k_ms = {k: eng.kernel_time(k) for k in KERNELS}
        k_b = {k: eng.kernel_bytes(k) for k in KERNELS}
        dom = max(k_ms, key=lambda k: k_ms[k][0])
        ms, launches = k_ms[dom]
        if ms > 0 and launches:
            per_launch_bytes = k_b[dom] / launches
            avg_s = ms / launches / 1e3
            ach = per_launch_bytes / avg_s / 1e9
            traffic, tsrc = pmc_traffic(w.name, dom, per_launch_bytes, shape["n_local"])
            roofline = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "traffic_source": tsrc,
                        "avg_launch_ms": round(ms / launches, 4), "launches": launches,
                        "alg_bytes_per_launch": round(per_launch_bytes),
                        "timed_steps": timed_steps,
                        "ms_per_step_with_events": round(dt_timed / timed_steps * 1e3, 3),
                        "kernel_ms_per_step": {k: round(v[0] / timed_steps, 3) for k, v in k_ms.items() if v[1]},
                        "kernel_frac": {k: round(k_b[k] / (v[0] / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
                                        for k, v in k_ms.items() if v[0] > 0 and k_b[k] > 0}}

    # per-round pass (untimed, P = 1): one step round by round with per-kernel
    # deltas -- which rounds ran binned / pull / push, and SURVEY 8(d)'s
    # algorithmic bytes B_r = 32 F_r + 20 T_r against the kernels' device time
    rounds_prof = None
    if not partitioned and not args.no_timing:
        rounds_prof = per_round_profile(eng)
        traversals = sum(s["traversals"] for s in stats)
        alg = sum(r["alg_bytes"] for r in rounds_prof)
        dense = [r for r in rounds_prof if r["mode"] == "bin"]
        if roofline is not None:
            roofline["step_frac"] = round(alg / (dt / args.steps) / 1e9 / HBM_PEAK_GBS, 4)
            if dense:
                d_b = sum(r["alg_bytes"] for r in dense)
                d_ms = sum(r["kernel_ms"] for r in dense)
                roofline["dense_round"] = {"rounds": [r["round"] for r in dense], "alg_bytes": d_b,
                                           "kernel_ms": round(d_ms, 3),
                                           "frac": round(d_b / (d_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                           "kernels": "bin_scatter + bin_apply + pull_heavy"}

    if rank == 0:
        line = {
            "metric": "gossip edge-deliveries/sec (GTEPS) + rounds-to-full-coverage",
            "value": round(value, 3),
            "unit": "GTEPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (Philox-generated power-law overlay and origins)",
            "config": {"workload": w.name, "peers": w.n, "edges": n_edges,
                       "messages": w.n_msgs, "rounds": len(stats),
                       "rounds_to_full_coverage": rounds_to_full(stats),
                       "deliveries_per_step": deliveries,
                       "traversals_per_step": sum(s["traversals"] for s in stats),
                       "parallelism": f"vertex-partition x{world}"},
            "traversal_gteps": round(args.steps * sum(s["traversals"] for s in stats) / dt / 1e9, 3),
        }
        if rounds_prof:
            line["rounds"] = [{k: r[k] for k in ("round", "mode", "frontier_frac", "traversals", "kernel_ms")}
                              for r in rounds_prof]
        if roofline:
            line["roofline"] = roofline
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args, args.config)
        print(json.dumps(line), flush=True)
    if partitioned:
        reps = eng.comm_finalize(stats)
        if rank == 0 and args.force_partitioned:
            print(json.dumps({"partitioned_check": {"modes": eng.comm_modes(), "reports": int(len(reps))}}), flush=True)
        eng.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
