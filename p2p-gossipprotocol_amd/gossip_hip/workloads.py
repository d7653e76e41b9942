"""The five BASELINE.json configurations as concrete round-model workloads.

Time base: one round = one second of the reference's wall clock, so
message_interval 5 s (config.cpp:35, peer.cpp:377) -> a message every 5
rounds, and the ping gate ping_interval 13 s checked on a 5 s tick
(peer.cpp:329-330,353) -> a ping round every ceil(13/5)*5 = 15 rounds.
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace

import numpy as np

CHURN_1PCT = 42949673  # floor(0.01 * 2^32)


def ping_every_rounds(ping_interval_s: int = 13, loop_tick_s: int = 5) -> int:
    """Effective ping period of pingLoop: a 5 s tick (peer.cpp:353) gated by
    'lastPing >= ping_interval' (peer.cpp:329-330)."""
    return -(-ping_interval_s // loop_tick_s) * loop_tick_s


@dataclass
class Workload:
    name: str
    n: int
    graph: str
    n_msgs: int
    origins: np.ndarray
    inject_rounds: np.ndarray
    rng_seed: int
    list_len: int = 6
    n_seeds: int = 20
    kills: list = field(default_factory=list)   # [(peer, round)]
    churn_threshold: int = 0
    ping_every: int = 0
    max_missed: int = 3
    min_rounds: int = 0
    extra_cap: int = 0   # re-bootstrap after a death; 0 = drop-only (the literal reference)
    list_cap: int = 0    # ref_bootstrap: peer_list bytes a peer reads (4095 = the reference's recv, F10); 0 = no cap
    rejoin_threshold: int = 0  # join churn: a dead peer restarts iff philox.x < this; 0 = never

    def engine_kwargs(self) -> dict:
        return dict(rng_seed=self.rng_seed, graph=self.graph, list_len=self.list_len, n_seeds=self.n_seeds,
                    churn_threshold=self.churn_threshold, ping_every=self.ping_every, max_missed=self.max_missed,
                    min_rounds=self.min_rounds, extra_cap=self.extra_cap, list_cap=self.list_cap,
                    rejoin_threshold=self.rejoin_threshold)


def _batches(origins: np.ndarray, per_origin: int, every: int) -> tuple[np.ndarray, np.ndarray]:
    """Message m = origin_index * per_origin + msgNumber, generated at round msgNumber * every."""
    o = np.repeat(origins.astype(np.uint32), per_origin)
    r = np.tile(np.arange(per_origin, dtype=np.uint32) * every, origins.size)
    return o, r


def config(idx: int, n: int | None = None, pick=None, rebootstrap: int = 0) -> Workload:
    """BASELINE.json configs[idx-1]; n overrides the peer count (parity runs).
    pick(n, seed, count) -> origins (defaults to the engine's Philox pick).
    rebootstrap > 0 turns on re-bootstrap after a death with that many extra
    out-edges per peer (configs 1 and 5, the ones with deaths)."""
    w = _config(idx, n, pick)
    return replace(w, extra_cap=rebootstrap, name=w.name + f"_reboot{rebootstrap}") if rebootstrap else w


def _config(idx: int, n: int | None, pick) -> Workload:
    if pick is None:
        from .engine import pick_origins as pick
    if idx == 1:
        n = n or 8
        o, r = _batches(np.arange(n, dtype=np.uint32), 10, 5)
        return Workload("config1_reference_cpu_run", n, "ref_bootstrap", int(o.size), o, r, 0x5EED0001,
                        kills=[(3 % n, 12)], ping_every=ping_every_rounds(), max_missed=3, min_rounds=46)
    if idx == 2:
        n = n or (1 << 20)
        o, r = _batches(pick(n, 0x5EED0002, 6), 10, 5)
        return Workload("config2_1M_powerlaw_6x10", n, "powerlaw", int(o.size), o, r, 0x5EED0002)
    if idx in (3, 4, 5):
        seed = {3: 0x5EED0003, 4: 0x5EED0004, 5: 0x5EED0005}[idx]
        n = n or {3: 1 << 24, 4: 1 << 28, 5: 1 << 26}[idx]
        o = pick(n, seed, 64).astype(np.uint32)
        r = np.zeros(64, dtype=np.uint32)
        name = {3: "config3_16M_64msg", 4: "config4_256M_64msg", 5: "config5_64M_churn"}[idx]
        w = Workload(name, n, "powerlaw", 64, o, r, seed)
        if idx == 5:
            w = replace(w, churn_threshold=CHURN_1PCT, ping_every=3, max_missed=3)
        return w
    raise ValueError(f"no config {idx}")


def run_engine(engine, w: Workload, build: bool = True) -> list[dict]:
    """Drive a single-partition Engine through a workload."""
    if build:
        engine.build_graph()
    engine.inject(w.origins, w.inject_rounds)
    if w.kills:
        engine.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
    engine.reset()
    return engine.run()
