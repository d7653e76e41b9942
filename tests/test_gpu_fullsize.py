"""Full-size parity (BASELINE.json configs 2-5 at their own sizes): libgossip_hip
through its C-ABI against fixtures of the oracle's fast round driver
(tests/golden/fullsize.json, made by tests/golden/make_fullsize_golden.py).

Every round's stats must match -- frontier, traversals, deliveries (the
reference's sentTo count, peer.cpp:310-316), new receipts and duplicates (the
Message-List check, peer.cpp:277-285), deaths, reports, seed removals
(peer.cpp:320-355,381-405; seed.cpp:158-167) and the coverage digest, which
pins each round's seen sets -- plus the overlay, the final per-message
coverage, the sorted dead-node reports, the alive flags and the registry."""
import json
from pathlib import Path

import numpy as np
import pytest

from gossip_hip import Engine
from gossip_hip.workloads import config, run_engine

pytestmark = pytest.mark.gpu
GOLDEN = json.loads((Path(__file__).resolve().parent / "golden" / "fullsize.json").read_text())


def _check_run(oracle, e, w, g, check_csr):
    if check_csr:
        rp, col = e.read_csr()
        assert int(col.size) == g["csr"]["edges"]
        assert oracle.hash(rp) == g["csr"]["row_ptr_hash"]
        assert oracle.hash(col) == g["csr"]["col_hash"]
        del rp, col
    stats = run_engine(e, w, build=False)
    assert len(stats) == len(g["stats"])
    for got, ref in zip(stats, g["stats"]):
        assert got == ref, (got, ref)
    assert e.coverage().tolist() == g["coverage"]
    reps = e.reports()
    assert int(reps.shape[0]) == g["reports"]["count"]
    assert oracle.hash(reps) == g["reports"]["hash"]
    alive, reg = e.alive(), e.registered()
    assert oracle.hash(alive) == g["alive"]["hash"] and int(alive.sum()) == g["alive"]["count"]
    assert oracle.hash(reg) == g["registered"]["hash"] and int(reg.sum()) == g["registered"]["count"]
    return stats


@pytest.mark.parametrize("idx", [2, 3, 5, 4])
def test_fullsize_auto_matches_oracle(oracle, idx):
    g = GOLDEN[str(idx)]
    w = config(idx)
    assert (w.n, w.n_msgs, w.rng_seed) == (g["n"], g["n_msgs"], g["rng_seed"])
    with Engine(w.n, w.n_msgs, **w.engine_kwargs()) as e:
        e.build_graph()
        stats = _check_run(oracle, e, w, g, check_csr=True)
        e.reset()  # the resident overlay reruns identically (the bench's step)
        assert e.run() == stats


@pytest.mark.parametrize("mode", ["push", "pull", "bin"])
def test_fullsize_config3_schedules_match_oracle(oracle, mode):
    """config 3 (2^24 peers): every forced schedule against the same fixture."""
    g = GOLDEN["3"]
    w = config(3)
    with Engine(w.n, w.n_msgs, mode=mode, **w.engine_kwargs()) as e:
        e.build_graph()
        _check_run(oracle, e, w, g, check_csr=False)


@pytest.mark.parametrize("idx", [3, 5])
def test_fullsize_forced_blocked_matches_oracle(oracle, idx):
    """Every push and binned round propagation-blocked (gossip_blocked.hip) at
    full size: config 3 (2^24 peers) and config 5 (2^26, churn: undelivered
    sends to dead peers) against the same fixtures."""
    g = GOLDEN[str(idx)]
    w = config(idx)
    with Engine(w.n, w.n_msgs, blocked="force", **w.engine_kwargs()) as e:
        e.build_graph()
        _check_run(oracle, e, w, g, check_csr=False)


@pytest.mark.parametrize("idx,P", [(4, 2), (4, 4), (4, 8), (5, 2)])
def test_fullsize_partitioned_group_matches_oracle(oracle, idx, P):
    """The N-GPU path at full size (BASELINE configs 4 and 5): the library's
    partitioned driver (gossip_group, gossip_dist.hip) with P parts on device 0,
    exchanging by device copies -- remote staging, record compaction, the
    all-gathered binned rounds at P > 1, the stats reduction and the report
    merge are the product's -- against the same single-partition fixture:
    every round's stats (seed removals from the merged reports), the final
    coverage, the sorted reports, alive flags and registry, and a rerun from
    reset.  peer.cpp:310-316 -> :277-285 across the partition boundary."""
    from gossip_hip import Group
    g = GOLDEN[str(idx)]
    w = config(idx)
    with Group(w.n, w.n_msgs, [0] * P, **w.engine_kwargs()) as grp:
        grp.build_graph()
        assert sum(grp.shape(p)["n_edges"] for p in range(P)) == g["csr"]["edges"]
        grp.inject(w.origins, w.inject_rounds)
        grp.reset()
        stats = grp.run()
        assert len(stats) == len(g["stats"])
        for got, ref in zip(stats, g["stats"]):
            assert got == ref, (got, ref)
        assert grp.coverage().tolist() == g["coverage"]
        reps = grp.reports()
        assert int(reps.shape[0]) == g["reports"]["count"]
        assert oracle.hash(reps) == g["reports"]["hash"]
        alive, reg = grp.alive(), grp.registered()
        assert oracle.hash(alive) == g["alive"]["hash"] and int(alive.sum()) == g["alive"]["count"]
        assert oracle.hash(reg) == g["registered"]["hash"] and int(reg.sum()) == g["registered"]["count"]
        grp.reset()
        assert grp.run() == stats
