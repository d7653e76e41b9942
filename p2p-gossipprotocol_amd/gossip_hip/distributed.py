"""Vertex-partitioned gossip over torch.distributed (RCCL over xGMI on MI355X).

One process per GPU.  Peers are 1D-partitioned into contiguous blocks
[p*c, min((p+1)*c, n)), c = ceil(n/P); each rank owns the CSR rows, seen/new words and miss
counters of its block (alive state is global and computed redundantly by
every rank from the same Philox draws, so churn needs no collective).

Per round (the reference's hop broadcastMessage -> handleClient, peer.cpp:
297-318 / 255-295, with the TCP send replaced by one collective):
  1. engine.round_begin(mode)  churn, liveness, injection.  The mode is chosen
                               here from the previous round's GLOBAL new-receipt
                               count, so every rank runs the same one.
  PULL / BIN (dense rounds):
  2. all_gather_into_tensor    every rank's new words -> one buffer indexed by
                               global peer (blocks are ceil(n/P) peers)
  3. engine.round_compute()    each peer ORs its neighbours' words (no atomics):
                               BIN streams them through the rank's slot layout
                               (wide frontier, many pairs still missing), PULL
                               gathers them (late rounds: few needy peers)
  PUSH (sparse rounds):
  2. engine.round_compute()    local push; remote masks OR-ed into a dense
                               staging buffer indexed by global peer, then
                               (PUSH_SPARSE) compacted into {peer, words}
                               records per destination rank
  3. all_to_all_single         PUSH: rank p's slice of every staging buffer;
                               PUSH_SPARSE: record counts, then the records
  4. engine.round_finish()     test-and-set of the received masks/records
  5. all_reduce(stats)         one int64 vector; drives the common termination
  6. engine.round_commit()

The driver is generic over the engine: libgossip_hip on cuda tensors (the
product) or, in the CPU tests only, a gloo-backed partition emulation with
the same phase API.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from ._abi import STAT_FIELDS

_SUM_FIELDS = ("frontier", "traversals", "deliveries", "undelivered", "new_receipts", "injected", "died", "reports",
               "reconnects", "rejoined")
MASK32 = (1 << 32) - 1
MASK64 = (1 << 64) - 1


MODE_PUSH, MODE_PULL, MODE_PUSH_SPARSE, MODE_BIN = 0, 1, 2, 3


def partition(n: int, world: int) -> list[int]:
    """Contiguous vertex blocks of ceil(n/P) peers: begins[p] = min(p*chunk, n),
    so a buffer of P chunks is indexed directly by global peer id."""
    chunk = -(-n // world)
    begins = [min(p * chunk, n) for p in range(world + 1)]
    if any(begins[p + 1] <= begins[p] for p in range(world)):
        raise ValueError(f"{n} peers cannot be split into {world} non-empty blocks of {chunk}")
    return begins


class PartitionedRun:
    def __init__(self, engine, n: int, rank: int, world: int, device: torch.device, group=None,
                 pull_permille: int = 60, pull: bool = True, sparse: bool = True, sparse_permille: int = 250,
                 bin_permille: int = 4000, bin_front_permille: int = 100):
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
        self.chunk = self.part[1]
        self.pull = pull
        self.pull_permille = pull_permille
        if pull:
            self.gather = torch.zeros(world * self.chunk * X, dtype=torch.int64, device=device)
            self.gather_mine = self.gather[rank * self.chunk * X:(rank + 1) * self.chunk * X]
            engine.set_gather(self.gather.data_ptr())
        self.sparse = sparse
        self.sparse_permille = sparse_permille
        self.R = 1 + X  # words per sparse record {peer, words[X]}
        if sparse:
            self.seg = torch.zeros(world * self.chunk * self.R, dtype=torch.int64, device=device)
            self.rec_in = torch.zeros(world * self.n_local * self.R, dtype=torch.int64, device=device)
            engine.set_sparse(self.seg.data_ptr())
        self.bin_permille = bin_permille
        self.bin_front_permille = bin_front_permille
        self.prev_new = 0
        self.injected = 0
        self.modes = []
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
        if self.pull and self.prev_new * 1000 >= self.pull_permille * self.n:
            # binned while the last round's receipts are wide and many (peer, message)
            # pairs are still missing (the same rule as the single-partition engine)
            missing = self.injected * self.n - (self.cum_covered + self.prev_new)
            wide = self.prev_new * 1000 >= self.bin_front_permille * self.n
            want = MODE_BIN if wide and missing * 1000 >= self.bin_permille * self.n else MODE_PULL
        elif self.sparse and self.prev_new * 1000 < self.sparse_permille * self.n:
            want = MODE_PUSH_SPARSE
        else:
            want = MODE_PUSH
        mode = e.round_begin(want)
        self.modes.append(mode)
        if mode in (MODE_PULL, MODE_BIN):
            dist.all_gather_into_tensor(self.gather, self.gather_mine, group=self.group)
            e.round_compute()
            local = e.round_finish()
        elif mode == MODE_PUSH_SPARSE:
            e.round_compute()
            local = self._sparse_exchange(e)
        else:
            e.round_compute()
            dist.all_to_all_single(self.recv, self.send, self.out_splits, self.in_splits, group=self.group)
            local = e.round_finish()
        g = self._allreduce(local)
        self.prev_new = g["new_receipts"]
        self.injected += g["injected"]
        out = {"round": local["round"], "flags": local["flags"]}
        for f in STAT_FIELDS:
            out[f] = g.get(f, 0)
        out["duplicates"] = out["deliveries"] - out["new_receipts"]
        out["seed_removals"] = 0  # filled from the gathered reports (finalize)
        finished = e.round_commit(out["new_receipts"])
        return out, finished

    def _sparse_exchange(self, e) -> dict:
        """Counts first (P int64), then the packed records of every destination."""
        R, chunk = self.R, self.chunk
        counts = [int(c) for c in e.sparse_counts(self.world)]
        c_out = torch.tensor(counts, dtype=torch.int64, device=self.device)
        c_in = torch.zeros(self.world, dtype=torch.int64, device=self.device)
        dist.all_to_all_single(c_in, c_out, group=self.group)
        got = c_in.tolist()
        send = torch.cat([self.seg[q * chunk * R:(q * chunk + counts[q]) * R] for q in range(self.world)])
        total = sum(got)
        recv = self.rec_in[:total * R]
        dist.all_to_all_single(recv, send, [g * R for g in got], [c * R for c in counts], group=self.group)
        return e.round_finish_sparse(recv.data_ptr(), total)

    def run(self, max_rounds: int = 4096) -> list[dict]:
        self.cum_digest = self.cum_covered = 0
        self.prev_new = 0
        self.injected = 0
        self.modes = []
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
