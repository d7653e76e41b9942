"""Driver for gossip_loopback, the build's real-socket loopback harness
(the harness itself is
surface/loopback_main.cpp).

It runs a small overlay as real TCP peers on 127.0.0.1 with the reference's
wire protocol (register / peer_list / gossip JSON, SHA-256 message hashes,
Message-List dedup, broadcast to every out-connection), so the wire formats
and the round model can be cross-checked: without churn the end state does
not depend on delivery order, and must equal the engine's.
"""
from __future__ import annotations

import subprocess
import tempfile
from pathlib import Path

import numpy as np

from ._abi import PKG_ROOT

import os  # noqa: E402

# (GOSSIP_LOOPBACK_BIN: another build of the harness, e.g. the sanitizer build of tests/sanitize/)
BINARY = Path(os.environ.get("GOSSIP_LOOPBACK_BIN", PKG_ROOT / "build" / "gossip_loopback"))


def msg_numbers(origins: np.ndarray) -> np.ndarray:
    """messageCounter of each message at its origin (peer.cpp:358-364): the
    k-th message an origin generates carries msg_number k."""
    seen: dict[int, int] = {}
    out = np.zeros(len(origins), dtype=np.int64)
    for i, o in enumerate(np.asarray(origins).tolist()):
        out[i] = seen.get(o, 0)
        seen[o] = out[i] + 1
    return out


def run_loopback(rp, col, origins, inject_rounds, *, n_seeds: int = 20, list_cap: int = 0,
                 log_dir: str | None = None, timeout: float = 120.0) -> dict:
    """Runs the harness on the overlay (rp, col) with the given injections.

    Returns started (peers that registered with q seeds), deliveries (sum of
    sentTo sizes), receipts (new receipts), refused (edges to peers that did
    not start), errors (malformed or mis-hashed lines; 0 expected) and
    seen: {peer: sorted message indices}."""
    if not BINARY.exists():
        raise FileNotFoundError(f"{BINARY} not built; run __graft_entry__.build()")
    rp = np.asarray(rp, dtype=np.uint64)
    col = np.asarray(col, dtype=np.uint32)
    n = len(rp) - 1
    origins = np.asarray(origins, dtype=np.uint32)
    rounds = np.asarray(inject_rounds, dtype=np.uint32)
    pairs = set(zip(origins.tolist(), rounds.tolist()))
    if len(pairs) != len(origins):
        raise ValueError("two messages share (origin, round): the reference would hash them identically")
    nums = msg_numbers(origins)
    with tempfile.TemporaryDirectory() as td:
        inp = Path(td) / "overlay.txt"
        with open(inp, "w") as f:
            f.write(f"{n} {len(col)}\n")
            f.write(" ".join(map(str, rp.tolist())) + "\n")
            f.write(" ".join(map(str, col.tolist())) + "\n")
            f.write(f"{len(origins)}\n")
            for o, r, k in zip(origins.tolist(), rounds.tolist(), nums.tolist()):
                f.write(f"{o} {r} {k}\n")
        cmd = [str(BINARY), str(inp), "--seeds", str(n_seeds)]
        if list_cap:
            cmd += ["--list-cap", str(list_cap)]
        if log_dir:
            cmd += ["--log-dir", str(log_dir)]
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    if p.returncode != 0:
        raise RuntimeError(f"gossip_loopback failed ({p.returncode}): {p.stderr.strip()}")
    out: dict = {"seen": {}}
    for line in p.stdout.splitlines():  # (seeds with a log dir also echo their log lines, as the reference's do)
        k, *v = line.split() or [""]
        if k == "seen":
            out["seen"][int(v[0])] = [int(x) for x in v[1:]]
        elif k in ("started", "deliveries", "receipts", "refused", "errors"):
            out[k] = int(v[0])
    return out
