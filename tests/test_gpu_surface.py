"""The drop-in surface on the GPU: `gossip_peer_network network.txt` with the
reference's 20 seeds, 8 peers, 10 messages each, peer 3 killed at round 12
(BASELINE.json configs[0]) -- stats equal the oracle's, and the per-peer /
per-seed log files say what the reference would have logged."""
import json
import subprocess
from pathlib import Path

import pytest

from gossip_hip.workloads import config

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parent.parent
EXE = REPO / "p2p-gossipprotocol_amd" / "build" / "gossip_peer_network"


def test_cli_reference_run(oracle, tmp_path):
    cfg = tmp_path / "network.txt"
    cfg.write_text((REPO / "tests" / "golden" / "network.txt").read_text() +
                   "n_peers=8\nrng_seed=0x5EED0001\nkills=3@12\nmin_rounds=46\n")
    logs = tmp_path / "logs"
    logs.mkdir()
    r = subprocess.run([str(EXE), str(cfg), "--logs", str(logs)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Minimum Required Seeds: 11" in r.stdout
    rounds = [json.loads(l) for l in r.stdout.splitlines() if l.startswith('{"round"')]
    w = config(1, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    assert [(x["round"], x["frontier"], x["deliveries"], x["new_receipts"], x["died"], x["reports"], x["covered"])
            for x in rounds] == [(s["round"], s["frontier"], s["deliveries"], s["new_receipts"], s["died"],
                                  s["reports"], s["covered"]) for s in ref["stats"]]
    # F8: peer 0 connects to nobody; peer 7 to everyone before it
    p0 = (logs / "peer_5000_output.txt").read_text()
    p7 = (logs / "peer_5007_output.txt").read_text()
    assert "Connected to peer" not in p0
    assert p7.count("Connected to peer: 127.0.0.1:") == 7
    assert p7.count("Generated message: Message from 127.0.0.1:5007") == 10
    assert "Received new message" not in p7          # nobody pushes to the last arrival
    assert p0.count("Received new message: Message from 127.0.0.1:5007") == 10
    # peer 3 died at round 12: it generated messages 0..2 only; 4..7 report it at round 45
    p3 = (logs / "peer_5003_output.txt").read_text()
    assert p3.count("Generated message") == 3
    for u in range(4, 8):
        assert "Peer disconnected: 127.0.0.1:5003" in (logs / f"peer_{5000 + u}_output.txt").read_text()
    s0 = (logs / "seed_8000_output.txt").read_text()
    assert s0.count("Registered new peer") == 8
    assert s0.count("Received dead node notification for: 127.0.0.1:5003") == 4
    assert s0.count("Removed dead peer: 127.0.0.1:5003") == 1
    assert "Registered new peer" not in (logs / "seed_8019_output.txt").read_text()  # quorum reached at seed 10


@pytest.mark.parametrize("n_gpus", [1, 2, 3])
def test_cli_partitioned_network(oracle, tmp_path, n_gpus):
    """network.txt with n_gpus: the drop-in CLI runs the overlay vertex-partitioned
    through the library's own multi-GPU driver (gossip_group_*; on a one-GPU box
    every part sits on device 0 and the parts exchange by device copies) -- the
    rounds equal the single-partition oracle's."""
    from gossip_hip.workloads import CHURN_1PCT
    cfg = tmp_path / "network.txt"
    cfg.write_text((REPO / "tests" / "golden" / "network.txt").read_text() +
                   f"n_peers=20000\ngraph=powerlaw\norigins=6\nrng_seed=0x5EED0002\nn_gpus={n_gpus}\n"
                   f"churn_ppm=10000\nping_interval=13\nmin_rounds=40\n")
    r = subprocess.run([str(EXE), str(cfg)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rounds = [json.loads(l) for l in r.stdout.splitlines() if l.startswith('{"round"')]
    import dataclasses
    w = config(2, 20000, pick=oracle.pick_origins)
    w = dataclasses.replace(w, churn_threshold=CHURN_1PCT, ping_every=15, min_rounds=40)  # churn_ppm=10000
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    assert [(x["round"], x["frontier"], x["deliveries"], x["new_receipts"], x["died"], x["reports"], x["covered"])
            for x in rounds] == [(s["round"], s["frontier"], s["deliveries"], s["new_receipts"], s["died"],
                                  s["reports"], s["covered"]) for s in ref["stats"]]


def _ref_wire():
    return json.loads((Path(__file__).resolve().parent / "golden" / "ref_wire.json").read_text())


@pytest.mark.parametrize("idx", [0, 1])
def test_engine_registry_matches_reference_seed(oracle, idx):
    """The engine's seed registry after a whole run (registrations, then the run's dead-node reports -- A2, A10)
    against the REAL reference SeedNode fed the same registrations and reports (tests/golden/ref_wire.json,
    made by tests/golden/make_ref_wire_golden.py from seed.cpp compiled with nlohmann/json 3.1.1): the same
    peers, and as many first removals as the reference printed "Removed dead peer" lines (seed.cpp:162-165)."""
    import numpy as np
    from dataclasses import replace

    from gossip_hip import Engine
    run = _ref_wire()["registry_runs"][idx]
    w = config(1, 8)
    if idx == 1:  # the same workload make_ref_wire_golden.py ran
        w = replace(w, n=300, n_msgs=64, origins=(np.arange(64, dtype=np.uint32) * 4),
                    inject_rounds=np.zeros(64, dtype=np.uint32), churn_threshold=int(0.03 * 2 ** 32), ping_every=3,
                    max_missed=2, min_rounds=20, kills=[(7, 1), (150, 4)], name="ref_bootstrap_300_churn")
    assert w.name == run["workload"] and w.n == run["n"]
    with Engine(w.n, w.n_msgs, device=0, **w.engine_kwargs()) as e:
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        if w.kills:
            e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        e.reset()
        stats = e.run()
        reg = e.registered()
        assert len(e.reports()) == run["reports"]
    ref = {(p["ip"], p["port"]) for p in json.loads(run["reference_final_list"])["peers"]}
    assert {("127.0.0.1", 5000 + i) for i in range(w.n) if reg[i]} == ref
    assert sum(s["seed_removals"] for s in stats) == len(run["reference_removed"])
