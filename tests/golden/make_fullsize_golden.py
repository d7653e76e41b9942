#!/usr/bin/env python3
"""Full-size parity fixtures: the oracle's fast round driver (oracle/gossip_oracle.c,
restating peer.cpp:255-318 receive/dedup/push and peer.cpp:320-355,381-405
liveness) run on BASELINE.json configs 2-5 at their full sizes.

TEST INFRASTRUCTURE.  Run in the build container (about 40 GB of RAM and a few
minutes on 8 threads for config 4 at 2^28 peers):

    python tests/golden/make_fullsize_golden.py [--configs 2,3,5,4] [--threads 8]

Writes tests/golden/fullsize.json: per config the overlay checksums (row_ptr,
col), every round's stats (frontier ... digest, covered: the digest pins the
per-round coverage sets), the final per-message coverage, and checksums of the
sorted dead-node reports, the alive flags and the seed registry.  Checksums are
oracle_hash_* (sum_i g(i) * x[i] mod 2^64 with the digest weights of DESIGN.md
section 4).  tests/test_gpu_fullsize.py holds libgossip_hip to these on the GPU.
"""
from __future__ import annotations

import argparse
import json
import platform
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO / "p2p-gossipprotocol_amd"))

import oracle_ref  # noqa: E402
from gossip_hip.workloads import config  # noqa: E402

OUT = HERE / "fullsize.json"


def golden(orc: oracle_ref.Oracle, idx: int, threads: int) -> dict:
    w = config(idx, pick=orc.pick_origins)
    t0 = time.perf_counter()
    rp, col = orc.gen_workload(w, threads=threads)
    t_gen = time.perf_counter() - t0
    csr = {"edges": int(col.size), "row_ptr_hash": orc.hash(rp, threads), "col_hash": orc.hash(col, threads)}
    t0 = time.perf_counter()
    ref = orc.simulate_workload(w, rp, col, threads=threads)
    t_sim = time.perf_counter() - t0
    del rp, col
    reps = ref["reports"]
    out = {
        "workload": w.name, "n": w.n, "n_msgs": w.n_msgs, "rng_seed": w.rng_seed,
        "churn_threshold": w.churn_threshold, "ping_every": w.ping_every, "max_missed": w.max_missed,
        "csr": csr,
        "stats": ref["stats"],
        "coverage": [int(x) for x in ref["coverage"]],
        "reports": {"count": int(reps.shape[0]), "hash": orc.hash(reps, threads)},
        "alive": {"count": int(ref["alive"].sum()), "hash": orc.hash(ref["alive"], threads)},
        "registered": {"count": int(ref["registered"].sum()), "hash": orc.hash(ref["registered"], threads)},
        "seen_popcount": int(np.bitwise_count(ref["seen"]).sum()),
        "oracle_seconds": {"generate": round(t_gen, 1), "simulate": round(t_sim, 1), "threads": threads},
    }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3,5,4")
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    orc = oracle_ref.Oracle(REPO / "oracle" / "_build" / "libgossip_oracle.so")
    data = json.loads(OUT.read_text()) if OUT.exists() else {}
    data.setdefault("_about", "oracle fast driver at BASELINE.json full sizes; made by tests/golden/"
                              "make_fullsize_golden.py; checksums = oracle_hash_* (DESIGN.md section 9)")
    for idx in (int(x) for x in args.configs.split(",")):
        t0 = time.perf_counter()
        data[str(idx)] = golden(orc, idx, args.threads)
        data[str(idx)]["host"] = platform.processor() or platform.machine()
        print(f"config {idx}: {data[str(idx)]['workload']} {len(data[str(idx)]['stats'])} rounds, "
              f"{time.perf_counter() - t0:.1f} s", flush=True)
        OUT.write_text(json.dumps(data, indent=1) + "\n")


if __name__ == "__main__":
    main()
