"""CPU tests of the oracle (the checker) against the golden vectors and
against itself (literal message-list driver == 64-bit-mask driver)."""
import hashlib
import json
from pathlib import Path

from dataclasses import replace

import numpy as np
import pytest

from gossip_hip.workloads import config

GOLDEN = Path(__file__).resolve().parent / "golden"


def test_philox_kat(oracle):
    for v in json.loads((GOLDEN / "philox_kat.json").read_text())["vectors"]:
        ctr = [int(x, 16) for x in v["ctr"]]
        key = [int(x, 16) for x in v["key"]]
        assert oracle.philox(ctr, key) == [int(x, 16) for x in v["out"]]


def test_sha256_message_hash_vectors():
    # calculateMessageHash (peer.cpp:135-159) = hex(SHA256(content || timestamp || sourceIP))
    for v in json.loads((GOLDEN / "sha256_kat.json").read_text())["vectors"]:
        h = hashlib.sha256((v["content"] + v["timestamp"] + v["source_ip"]).encode()).hexdigest()
        assert h == v["hash"]


@pytest.mark.parametrize("L", [2, 3, 6, 11, 64, 1000, 4096])
def test_threshold_is_exact_ceiling(oracle, L):
    # thr(j,L) is the smallest x with x >= 2^32 (j/L)^2.5  (peer.cpp:219-222)
    from fractions import Fraction
    for j in list(range(1, min(L, 40))) + [L - 1]:
        x = oracle.threshold(j, L)
        target = Fraction(j, L) ** 5 * (1 << 64)   # x^2 >= 2^64 (j/L)^5
        assert x * x >= target and (x - 1) * (x - 1) < target


def test_ref_bootstrap_f8_structure(oracle):
    # F8: edges only point to earlier arrivals; with 11 responses out-deg(i) = i (whp)
    rp, col = oracle.gen("ref_bootstrap", 8, 20, 0x5EED0001)
    assert list(np.diff(rp)) == list(range(8))
    for i in range(8):
        assert list(col[rp[i]:rp[i + 1]]) == list(range(i))
    rp, col = oracle.gen("ref_bootstrap", 200, 20, 7)
    for i in range(200):
        row = col[rp[i]:rp[i + 1]]
        assert np.all(row < i) and np.all(np.diff(row.astype(np.int64)) > 0)


def test_powerlaw_csr_wellformed(oracle):
    n = 1 << 14
    rp, col = oracle.gen("powerlaw", n, 6, 11)
    assert rp[0] == 0 and rp[-1] == len(col)
    deg = np.diff(rp).astype(np.int64)
    src = np.repeat(np.arange(n, dtype=np.uint32), deg)
    assert np.all(col != src)  # no self loops
    for v in range(0, n, 97):
        row = col[rp[v]:rp[v + 1]].astype(np.int64)
        assert np.all(np.diff(row) > 0)
    # symmetric
    fwd = set(zip(src.tolist(), col.tolist()))
    assert all((c, s) in fwd for s, c in list(fwd)[:5000])
    assert 6.0 < len(col) / n < 9.0   # mean degree ~ 8


def _hand_rows(case):
    rows = case["rows"]
    rp = np.zeros(len(rows) + 1, dtype=np.uint64)
    rp[1:] = np.cumsum([len(r) for r in rows])
    col = np.array([c for r in rows for c in r], dtype=np.uint32)
    return rp, col


def hand_cases():
    return json.loads((GOLDEN / "hand_graphs.json").read_text())["cases"]


@pytest.mark.parametrize("case", hand_cases(), ids=lambda c: c["name"])
@pytest.mark.parametrize("variant", [0, 1])
def test_oracle_hand_graphs(oracle, case, variant):
    fields = json.loads((GOLDEN / "hand_graphs.json").read_text())["fields"]
    rp, col = _hand_rows(case)
    out = oracle.simulate(rp, col, case["n"], len(case["origins"]), case["origins"], case["inject_rounds"],
                          ping_every=case.get("ping_every", 0), max_missed=case.get("max_missed", 3),
                          min_rounds=case.get("min_rounds", 0), kills=[tuple(k) for k in case.get("kills", [])],
                          variant=variant)
    got = [[s[f] for f in fields] for s in out["stats"]]
    assert got == case["expect"]
    assert list(out["coverage"]) == case["coverage"]
    assert out["reports"].tolist() == case.get("reports", [])


def _digest(seen, W):
    n = seen.shape[0]
    idx = np.arange(n * W, dtype=np.uint64) + np.uint64(1)
    z = idx * np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = (z ^ (z >> np.uint64(31))) | np.uint64(1)
    return int(np.sum(z * seen.reshape(-1), dtype=np.uint64))


@pytest.mark.parametrize("idx,n", [(1, None), (2, 1 << 12), (3, 1 << 12), (5, 1 << 12)])
def test_oracle_fast_equals_literal(oracle, idx, n):
    w = config(idx, n, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    a = oracle.simulate_workload(w, rp, col, variant=0)
    b = oracle.simulate_workload(w, rp, col, variant=1)
    assert a["stats"] == b["stats"]
    assert np.array_equal(a["seen"], b["seen"])
    assert np.array_equal(a["reports"], b["reports"])
    assert np.array_equal(a["alive"], b["alive"]) and np.array_equal(a["registered"], b["registered"])
    # sentTo bookkeeping (peer.cpp:314) == deliveries
    assert b["sent_to_total"] == sum(s["deliveries"] for s in b["stats"])
    # digest of the final state == last round's push-start digest (that round had no fresh bits)
    last = a["stats"][-1]
    if last["new_receipts"] == 0 and last["died"] == 0:
        assert _digest(a["seen"], (w.n_msgs + 63) // 64) == last["digest"]
    for s in a["stats"]:
        assert s["duplicates"] == s["deliveries"] - s["new_receipts"]


def test_config1_literal_reference_run(oracle):
    # configs[0]: 8 peers, literal bootstrap, 8x10 messages, peer 3 killed at round 12
    w = config(1, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    out = oracle.simulate_workload(w, rp, col, variant=1)
    # F8: origin i's messages cover exactly {0..i} (those generated while alive)
    seen = out["seen"]
    for m in range(w.n_msgs):
        o = int(w.origins[m])
        holders = {v for v in range(8) if (int(seen[v, m // 64]) >> (m % 64)) & 1}
        if o == 3 and w.inject_rounds[m] >= 12:
            assert holders == set()     # dead origin generates nothing (messageGenerationLoop stops)
        else:
            assert holders == set(range(o + 1)) - ({3} if w.inject_rounds[m] >= 12 and o > 3 else set())
    # the 4 later arrivals each hold an edge to peer 3 and report it 3 ping rounds later (15,30,45)
    assert out["reports"].tolist() == [[45, u, 3] for u in range(4, 8)]
    assert out["registered"].tolist() == [1, 1, 1, 0, 1, 1, 1, 1]


def test_pick_origins_distinct(oracle):
    o = oracle.pick_origins(1 << 20, 0x5EED0003, 64)
    assert len(set(o.tolist())) == 64 and o.max() < (1 << 20)


@pytest.mark.parametrize("idx,n,cap", [(5, 1 << 12, 4), (5, 3000, 16), (1, None, 8), (1, 40, 3)])
def test_rebootstrap_literal_equals_fast(oracle, idx, n, cap):
    """Re-bootstrap after a death (handleDeadPeer peer.cpp:398-404): both
    round drivers add the same out-edges and deliver over them identically."""
    w = config(idx, n, pick=oracle.pick_origins, rebootstrap=cap)
    rp, col = oracle.gen_workload(w)
    fast = oracle.simulate_workload(w, rp, col, variant=0)
    lit = oracle.simulate_workload(w, rp, col, variant=1)
    assert fast["stats"] == lit["stats"]
    assert np.array_equal(fast["seen"], lit["seen"])
    assert np.array_equal(fast["extra_counts"], lit["extra_counts"])
    assert np.array_equal(fast["extra_cols"], lit["extra_cols"])
    assert sum(s["reconnects"] for s in fast["stats"]) == int(fast["extra_counts"].sum())
    if idx == 5:   # at n = 8 the literal DAG already links every candidate: nothing new to add
        assert fast["extra_counts"].sum() > 0


def test_rebootstrap_edges_are_new_live_and_bounded(oracle):
    w = config(5, 1 << 12, pick=oracle.pick_origins, rebootstrap=6)
    rp, col = oracle.gen_workload(w)
    out = oracle.simulate_workload(w, rp, col)
    cnt, ex = out["extra_counts"], out["extra_cols"]
    assert int(cnt.max()) <= 6
    reporters = set(out["reports"][:, 1].tolist())
    for u in np.nonzero(cnt)[0].tolist():
        assert u in reporters                                  # only peers that detected a death re-select
        targets = (ex[u, :cnt[u]] & np.uint32(0x7FFFFFFF)).tolist()
        assert len(set(targets)) == len(targets)               # connectedPeers is a map
        assert u not in targets
        assert not set(targets) & set(col[rp[u]:rp[u + 1]].tolist())
    off = oracle.simulate_workload(replace(w, extra_cap=0), rp, col)
    assert all(s["reconnects"] == 0 for s in off["stats"])


@pytest.mark.parametrize("n,cap", [(120, 4095), (64, 1200)])
def test_f10_literal_equals_fast(oracle, n, cap):
    """F10 knob (list_cap): both drivers start the same peers and agree on every round."""
    from gossip_hip.workloads import _batches
    o, r = _batches(np.array([0, 7, n // 2, n - 1], dtype=np.uint32), 10, 5)
    w = replace(config(1), n=n, n_msgs=int(o.size), origins=o, inject_rounds=r, list_cap=cap)
    rp, col = oracle.gen_workload(w)
    fast = oracle.simulate_workload(w, rp, col, variant=0)
    lit = oracle.simulate_workload(w, rp, col, variant=1)
    assert fast["stats"] == lit["stats"]
    assert np.array_equal(fast["seen"], lit["seen"])
    started = oracle.started_under_cap(n, cap)
    assert started < n and not fast["alive"][started:].any() and fast["registered"][started:].all()
    assert not fast["seen"][started:].any()  # never started: never received nor generated


def test_f10_started_count(oracle):
    """peer_list of k 127.0.0.1 peers = 30 + 53 k bytes: 76 fit in 4095 (77 fail)."""
    assert oracle.started_under_cap(4096, 4095) == 76
    assert oracle.started_under_cap(76, 4095) == 76
    assert oracle.started_under_cap(10, 0) == 10
    for k in (1, 2, 50):
        assert oracle.started_under_cap(4096, 30 + 53 * k) == k
        assert oracle.started_under_cap(4096, 30 + 53 * k - 1) == k - 1


@pytest.mark.parametrize("cap", [0, 8])
def test_rejoin_literal_equals_fast(oracle, cap):
    """Join churn (rejoin_threshold): restarted peers with an
    empty Message-List, a dropped row and (cap > 0) fresh out-edges; both
    drivers agree, and sum |sentTo| (restarts included) = sum deliveries."""
    w = replace(config(5, 4096, pick=oracle.pick_origins, rebootstrap=cap), rejoin_threshold=int(0.05 * 2**32),
                min_rounds=30)
    rp, col = oracle.gen_workload(w)
    fast = oracle.simulate_workload(w, rp, col, variant=0)
    lit = oracle.simulate_workload(w, rp, col, variant=1)
    assert fast["stats"] == lit["stats"]
    assert np.array_equal(fast["seen"], lit["seen"])
    assert np.array_equal(fast["extra_cols"], lit["extra_cols"])
    assert sum(s["rejoined"] for s in fast["stats"]) > 100
    assert lit["sent_to_total"] == sum(s["deliveries"] for s in lit["stats"])
    off = oracle.simulate_workload(replace(w, rejoin_threshold=0), rp, col)
    assert all(s["rejoined"] == 0 for s in off["stats"])
    assert int(fast["alive"].sum()) > int(off["alive"].sum())
