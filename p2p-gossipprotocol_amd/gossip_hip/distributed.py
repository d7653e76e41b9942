"""Vertex-partitioned gossip over torch.distributed (RCCL over xGMI on MI355X).

One process per GPU.  Peers are 1D-partitioned into contiguous blocks
[p*n/P, (p+1)*n/P); each rank owns the CSR rows, seen/new words and miss
counters of its block (alive state is global and computed redundantly by
every rank from the same Philox draws, so churn needs no collective).

Per round (the reference's hop broadcastMessage -> handleClient, peer.cpp:
297-318 / 255-295, with the TCP send replaced by one exchange):
  1. engine.round_push()      churn, liveness, injection, local push; masks for
                              remote peers are OR-ed into a dense send buffer
  2. all_to_all_single        rank p's slice of every send buffer -> rank p
  3. engine.round_finish()    test-and-set of the received masks (no atomics)
  4. all_reduce(stats)        one int64 vector; drives the common termination
  5. engine.round_commit()

The driver is generic over the engine: libgossip_hip on cuda tensors (the
product) or, in the CPU tests only, a gloo-backed partition emulation with
the same phase API.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from ._abi import STAT_FIELDS

_SUM_FIELDS = ("frontier", "traversals", "deliveries", "undelivered", "new_receipts", "injected", "died", "reports")
MASK32 = (1 << 32) - 1
MASK64 = (1 << 64) - 1


def partition(n: int, world: int) -> list[int]:
    """Contiguous, balanced vertex blocks: begins[p] = floor(p*n/P)."""
    return [(p * n) // world for p in range(world + 1)]


class PartitionedRun:
    def __init__(self, engine, n: int, rank: int, world: int, device: torch.device, group=None):
        self.engine = engine
        self.n, self.rank, self.world = n, rank, world
        self.device = device
        self.group = group
        self.part = partition(n, world)
        shape = engine.shape()
        X = shape["exchange_words"]
        self.n_local = shape["n_local"]
        assert self.n_local == self.part[rank + 1] - self.part[rank]
        self.send = torch.zeros(n * X, dtype=torch.int64, device=device)
        self.recv = torch.zeros(world * self.n_local * X, dtype=torch.int64, device=device)
        self.in_splits = [(self.part[q + 1] - self.part[q]) * X for q in range(world)]
        self.out_splits = [self.n_local * X] * world
        if device.type == "cuda":
            engine.set_stream(torch.cuda.current_stream(device).cuda_stream)
        engine.set_exchange(self.send.data_ptr(), self.recv.data_ptr(), self.part)
        self.cum_digest = 0
        self.cum_covered = 0

    def _allreduce(self, local: dict) -> dict:
        vals = [local[f] for f in _SUM_FIELDS]
        d = local["digest"] & MASK64
        vals += [d & MASK32, d >> 32, local["covered"]]
        t = torch.tensor(vals, dtype=torch.int64, device=self.device)
        dist.all_reduce(t, group=self.group)
        out = t.tolist()
        g = dict(zip(_SUM_FIELDS, out[: len(_SUM_FIELDS)]))
        lo, hi, cov = out[len(_SUM_FIELDS):]
        self.cum_digest = (self.cum_digest + lo + (hi << 32)) & MASK64
        self.cum_covered += cov
        g["digest"] = self.cum_digest
        g["covered"] = self.cum_covered
        return g

    def step(self) -> tuple[dict, bool]:
        e = self.engine
        e.round_push()
        dist.all_to_all_single(self.recv, self.send, self.out_splits, self.in_splits, group=self.group)
        local = e.round_finish()
        g = self._allreduce(local)
        out = {"round": local["round"], "flags": local["flags"]}
        for f in STAT_FIELDS:
            out[f] = g.get(f, 0)
        out["duplicates"] = out["deliveries"] - out["new_receipts"]
        out["seed_removals"] = 0  # filled from the gathered reports (finalize)
        finished = e.round_commit(out["new_receipts"])
        return out, finished

    def run(self, max_rounds: int = 4096) -> list[dict]:
        self.cum_digest = self.cum_covered = 0
        rounds = []
        for _ in range(max_rounds):
            st, fin = self.step()
            rounds.append(st)
            if fin:
                break
        return rounds

    def finalize(self, rounds: list[dict]) -> np.ndarray:
        """Gather the dead-node reports of every rank, sorted by (round, reporter,
        dead); the seed registry drops a peer on its first report
        (SeedNode::handleDeadNode, seed.cpp:158-167), so seed_removals of a
        round = peers whose first report falls in it."""
        mine = self.engine.reports()
        parts = [None] * self.world
        dist.all_gather_object(parts, mine.tolist(), group=self.group)
        allr = np.array(sorted(tuple(r) for p in parts for r in p), dtype=np.uint32).reshape(-1, 3)
        first = {}
        for r, _, v in allr.tolist():
            first.setdefault(v, r)
        per_round = {}
        for v, r in first.items():
            per_round[r] = per_round.get(r, 0) + 1
        for st in rounds:
            st["seed_removals"] = per_round.get(st["round"], 0)
        return allr

    def gather_seen(self) -> np.ndarray | None:
        """All ranks' seen words on rank 0 (tests/small n only)."""
        mine = self.engine.read_seen()
        parts = [None] * self.world
        dist.all_gather_object(parts, mine, group=self.group)
        return np.concatenate(parts, axis=0) if self.rank == 0 else None
