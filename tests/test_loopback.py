"""Real-socket loopback harness, CPU only.

gossip_loopback runs the overlay as real TCP peers on 127.0.0.1 with the
reference's wire protocol: register / peer_list JSON with the seeds, gossip
JSON built by the surface's formats, SHA-256 message hashes recomputed by
every receiver, Message-List dedup and broadcast to every out-connection.
Without churn its end state does not depend on delivery order, so it must
equal the round model's: the oracle here, which the GPU tests hold the engine
to.  The F10 case (a 4095-byte peer_list read) pins the oracle's and the
engine's list-size model against the bytes the harness actually exchanges."""
import dataclasses
import re

import numpy as np
import pytest

from gossip_hip.loopback import msg_numbers, run_loopback
from gossip_hip.workloads import config


def _distinct(n, seed, count):  # distinct origins: two messages from one origin and round would share a hash
    return np.random.default_rng(seed).choice(n, count, replace=False).astype(np.uint32)


def _seen_lists(ref, n_msgs, alive=None):
    out = {}
    for v in range(ref["seen"].shape[0]):
        if alive is not None and not alive[v]:
            continue
        out[v] = [m for m in range(n_msgs) if (int(ref["seen"][v][m >> 6]) >> (m & 63)) & 1]
    return out


def _check(oracle, w, list_cap=0, log_dir=None):
    rp, col = oracle.gen_workload(w)
    got = run_loopback(rp, col, w.origins, w.inject_rounds, n_seeds=w.n_seeds, list_cap=list_cap, log_dir=log_dir)
    ref = oracle.simulate_workload(w, rp, col)
    assert got["errors"] == 0
    assert got["refused"] == 0
    assert got["started"] == int(ref["alive"].sum())
    assert got["deliveries"] == sum(s["deliveries"] for s in ref["stats"])
    assert got["receipts"] == sum(s["new_receipts"] for s in ref["stats"])
    want = _seen_lists(ref, w.n_msgs, ref["alive"])
    assert {v: got["seen"].get(v, []) for v in want} == want
    return got, ref


@pytest.mark.parametrize("idx,n", [(2, 192), (3, 256), (1, None)])
def test_loopback_matches_round_model(oracle, idx, n):
    w = config(idx, n, pick=_distinct)
    w = dataclasses.replace(w, kills=[], ping_every=0)  # no churn: the end state is order-independent
    got, _ = _check(oracle, w)
    assert got["started"] == w.n


@pytest.mark.parametrize("n,cap", [(120, 4095), (90, 2048), (40, 4095), (60, 700)])
def test_f10_list_cap(oracle, n, cap):
    """The reference reads a seed's peer_list with one 4 KB recv
    (peer.cpp:188-190): from the 77th registered peer on (127.0.0.1
    addresses) the JSON is cut, the parse fails at every quorum seed and the
    peer never starts.  The harness exchanges the real JSON and
    applies the same read bound; its started count and end state must match
    the round model's list-size model."""
    w = config(1)
    origins = np.array(sorted({3 % n, (n // 3), n // 2, n - 1, min(75, n - 1)}), dtype=np.uint32)
    w = dataclasses.replace(w, n=n, kills=[], ping_every=0, min_rounds=0, list_cap=cap, n_msgs=len(origins),
                            origins=origins, inject_rounds=np.zeros(len(origins), dtype=np.uint32))
    got, ref = _check(oracle, w, list_cap=cap)
    assert got["started"] == oracle.started_under_cap(n, cap)
    if n >= 77 and cap == 4095:
        assert got["started"] == 76  # the F10 count for 127.0.0.1 peers
    # the literal bootstrap lists only earlier peers, so no started peer links to a failed one
    assert got["refused"] == 0


def test_loopback_logs(oracle, tmp_path):
    """Peer logs in the reference's format (logToFile peer.cpp:125-133): one
    "Received new message" per new receipt, one "Generated message" per
    injection, after "Peer node started on port <p>"."""
    w = config(2, 96, pick=_distinct)
    w = dataclasses.replace(w, kills=[], ping_every=0)
    got, _ = _check(oracle, w, log_dir=str(tmp_path))
    line = re.compile(r"^[A-Z][a-z]{2} [A-Z][a-z]{2} [ 0-9]\d \d\d:\d\d:\d\d \d{4}\n$")
    received = generated = 0
    for v in range(w.n):
        text = (tmp_path / f"peer_{5000 + v}_output.txt").read_text()
        entries = text.split("\n: ")
        assert text.startswith(entries[0]) and line.match(entries[0] + "\n")
        msgs = [e.split("\n")[0] for e in entries[1:]]
        assert msgs[0] == f"Peer node started on port {5000 + v}"
        for m in msgs[1:]:
            assert re.fullmatch(r"(Received new|Generated) message: Message from 127\.0\.0\.1:5\d{3}", m), m
        received += sum(m.startswith("Received") for m in msgs)
        generated += sum(m.startswith("Generated") for m in msgs)
    assert received == got["receipts"]
    assert generated == len(w.origins)
    assert (tmp_path / "seed_8000_output.txt").exists()


def test_msg_numbers():
    assert msg_numbers(np.array([4, 4, 7, 4, 7])).tolist() == [0, 1, 0, 2, 1]
