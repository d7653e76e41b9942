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
vertex-partitioned over N ranks (strong scaling, RCCL all-to-all per round).

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
    ap.add_argument("--cpu-sample-n", type=int, default=1 << 25)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip per-kernel HIP event timing")
    ap.add_argument("--pull-permille", type=int, default=0, help="push/pull switch point (0 = engine default)")
    ap.add_argument("--front-permille", type=int, default=0, help="frontier-bitmap switch point (0 = default)")
    ap.add_argument("--mode", default="auto", choices=["auto", "push", "pull"])
    ap.add_argument("--rebootstrap", type=int, default=0,
                    help="re-bootstrap after a death with this many extra out-edges per peer (configs 1, 5)")
    ap.add_argument("--force-partitioned", action="store_true",
                    help="use the multi-rank driver (RCCL collectives) even at WORLD_SIZE 1")
    return ap.parse_args()


# kernel timer name -> rocprofv3 kernel-name prefix in the PMC summary
PMC_KERNELS = {"bin_scatter": "k_bin_scatter_lds", "bin_apply": "k_bin_apply", "pull_light": "k_pull_light",
               "push_light": "k_push_light", "push_heavy": "k_push_heavy", "pull_heavy": "k_pull_heavy"}


def pmc_traffic(workload: str, kernel: str, alg_bytes_per_launch: float, n_local: int):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (FETCH_SIZE and WRITE_SIZE, separate runs of this same command) with the
    gfx950 corrections measured by tools/calib_fetch.hip (profiles/r01/
    calib_fetch_timing.log): FETCH_SIZE counts 1/2 of coalesced streamed bytes
    and one 64-B line per random 8-B gather; WRITE_SIZE counts stores 1:1.
    bin_scatter / bin_apply read only coalesced streams (traffic = 2 x fetch +
    write); pull_light mixes streams with random gathers (only its streamed
    reads are doubled)."""
    path = REPO / "profiles" / "r01" / "config4_pmc_summary.json"
    if not workload.startswith("config4") or not path.exists() or kernel not in PMC_KERNELS:
        return None, None
    prof = json.loads(path.read_text())
    keys = [k for k in prof["kernels"] if k.startswith(PMC_KERNELS[kernel] + "<") or k == PMC_KERNELS[kernel]]
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


def cpu_baseline(args, cfg_idx: int) -> dict:
    """The oracle's 64-bit-mask round driver (g++ -O3 -fopenmp) on a bounded
    sample of the same workload, timed on this host's cores (rounds only)."""
    sys.path.insert(0, str(REPO / "tests"))
    import oracle_ref  # noqa: E402  (checker / baseline only)
    from gossip_hip.workloads import config

    so = REPO / "oracle" / "_build" / "libgossip_oracle.so"
    orc = oracle_ref.Oracle(so)
    threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", 0) or min(16, os.cpu_count() or 1))
    n = args.cpu_sample_n
    w = config(cfg_idx if cfg_idx != 1 else 3, n, pick=orc.pick_origins)
    rp, col = orc.gen_workload(w, threads=threads)
    t0 = time.perf_counter()
    out = orc.simulate_workload(w, rp, col, variant=0, threads=threads)
    dt = time.perf_counter() - t0
    d = sum(s["deliveries"] for s in out["stats"])
    return {"value": round(d / dt / 1e9, 4), "unit": "GTEPS", "cores": threads, "kind": "port",
            "sample": f"{w.name} workload at n=2^{n.bit_length() - 1} ({n} peers, {len(col)} edges, "
                      f"{len(out['stats'])} rounds), oracle fast driver, {dt:.2f} s incl. state setup"}


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
        import torch.distributed as dist

        from gossip_hip.distributed import PartitionedRun, partition

        for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29511")):
            os.environ.setdefault(k, v)  # --force-partitioned run without a launcher
        dist.init_process_group("nccl", device_id=dev)
        part = partition(w.n, world)
        eng = Engine(w.n, w.n_msgs, device=local, part=(part[rank], part[rank + 1]), **tune, **w.engine_kwargs())
        eng.build_graph()
        eng.inject(w.origins, w.inject_rounds)
        if w.kills:
            eng.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        runner = PartitionedRun(eng, w.n, rank, world, dev)

        def one_step():
            eng.reset()
            return runner.run()

        def barrier():
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()
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
        t = torch.tensor([n_edges], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        n_edges = int(t.item())
    for _ in range(args.warmup):
        one_step()
    if not args.no_timing:
        eng.enable_timing(True)
    barrier()
    t0 = time.perf_counter()
    stats = None
    for _ in range(args.steps):
        stats = one_step()
    barrier()
    dt = time.perf_counter() - t0
    if partitioned:
        import torch.distributed as dist
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    deliveries = sum(s["deliveries"] for s in stats)
    value = args.steps * deliveries / dt / 1e9
    roofline = None
    if not args.no_timing:
        from gossip_hip.engine import KERNELS
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
                        "kernel_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in k_ms.items() if v[1]},
                        "kernel_frac": {k: round(k_b[k] / (v[0] / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
                                        for k, v in k_ms.items() if v[0] > 0 and k_b[k] > 0}}

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
                       "deliveries_per_step": deliveries, "parallelism": f"vertex-partition x{world}"},
        }
        if roofline:
            line["roofline"] = roofline
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args, args.config)
        print(json.dumps(line), flush=True)
    if partitioned:
        import torch.distributed as dist
        reps = runner.finalize(stats)
        if rank == 0 and args.force_partitioned:
            print(json.dumps({"partitioned_check": {"modes": runner.modes, "reports": int(len(reps))}}), flush=True)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
