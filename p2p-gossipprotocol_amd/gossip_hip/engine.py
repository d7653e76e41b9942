"""Engine: a thin owner of one gossip_ctx (one vertex partition in HBM).

Mirrors the reference's per-peer surface at simulation scale: the overlay
(selectAndConnectPeers, peer.cpp:214-253), message generation
(messageGenerationLoop, peer.cpp:357-379), forwarding + Message-List dedup
(broadcastMessage/handleClient, peer.cpp:255-318) and liveness
(pingLoop/handleDeadPeer, peer.cpp:320-405) all run inside libgossip_hip.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._abi import DeadReport, GossipConfig, RoundStats, check

_GRAPHS = {"powerlaw": _abi.GRAPH_POWERLAW, "ref_bootstrap": _abi.GRAPH_REF_BOOTSTRAP}
KERNELS = ("push_light", "push_heavy", "push_extra", "src_count", "frontier_bits", "pull_light", "pull_heavy", "pull_list", "list_zero", "bin_scatter",
           "bin_apply", "pb_scatter", "pb_split", "pb_apply", "liveness", "rebootstrap", "rejoin", "churn", "kills",
           "inject", "apply_remote", "commit", "compact_send", "px_scatter", "tiny", "heavy_commit")
# kernels that run on a ctx's second stream beside others (binned rounds at P = 1: the heavy rows' pull beside the
# scatter); a round's critical path counts them only when the round has no join (heavy_commit, whose timer covers
# the wait for the side stream)
SIDE_KERNELS = ("pull_heavy",)
# exchange steps of partitioned rounds, timed on each part's stream (gossip_dist.hip; bytes = received per part)
EXCHANGES = ("all_gather", "all_to_all", "records")


def _u32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint32))


def _ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def comm_unique_id() -> bytes:
    """A fresh RCCL unique id (rank 0 makes it; the others receive it out of band)."""
    buf = (C.c_uint8 * _abi.COMM_ID_BYTES)()
    check(_abi.lib().gossip_comm_unique_id(buf), "gossip_comm_unique_id")
    return bytes(buf)


def partition(n_peers: int, world: int) -> list[int]:
    """The library's vertex blocks: begins[world+1] (ceil(n/world) peers each)."""
    out = np.zeros(world + 1, dtype=np.uint64)
    check(_abi.lib().gossip_partition(n_peers, world, _ptr(out, C.c_uint64)), "gossip_partition")
    return [int(x) for x in out]


def partition_edges(n_peers: int, n_msgs: int, world: int, **kw) -> list[int]:
    """Blocks of about equal work for this overlay (gossip_partition_edges: the
    powerlaw overlay's edges sit at the low ids; others get partition())."""
    cfg = make_config(n_peers, n_msgs, **kw)
    out = np.zeros(world + 1, dtype=np.uint64)
    check(_abi.lib().gossip_partition_edges(C.byref(cfg), world, _ptr(out, C.c_uint64)), "gossip_partition_edges")
    return [int(x) for x in out]


def device_count() -> int:
    """HIP devices visible to this process (gossip_device_count)."""
    n = C.c_int32()
    check(_abi.lib().gossip_device_count(C.byref(n)), "gossip_device_count")
    return n.value


def pick_origins(n_peers: int, rng_seed: int, count: int) -> np.ndarray:
    out = np.zeros(max(count, 1), dtype=np.uint32)
    check(_abi.lib().gossip_pick_origins(n_peers, rng_seed, count, _ptr(out, C.c_uint32)), "gossip_pick_origins")
    return out[:count]


def make_config(n_peers: int, n_msgs: int, *, rng_seed: int = 0, graph: str = "powerlaw", list_len: int = 6,
                n_seeds: int = 20, churn_threshold: int = 0, ping_every: int = 0, max_missed: int = 3,
                max_rounds: int = 4096, min_rounds: int = 0, device: int = -1, coverage_history: bool = False,
                part: tuple[int, int] = (0, 0), report_capacity: int = 0, mode: str = "auto",
                pull_permille: int = 0, front_permille: int = 0, bin_permille: int = 0, bins: bool = True,
                extra_cap: int = 0, list_cap: int = 0, rejoin_threshold: int = 0, blocked: str = "auto",
                blocked_permille: int = 0, uniform_partition: bool = False) -> GossipConfig:
    """gossip_config from keyword arguments (the fields of include/gossip/gossip.h)."""
    cfg = GossipConfig()
    cfg.n_peers = n_peers
    cfg.part_begin, cfg.part_end = part
    cfg.n_msgs = n_msgs
    cfg.rng_seed = rng_seed
    cfg.graph_model = _GRAPHS[graph]
    cfg.list_len = list_len
    cfg.n_seeds = n_seeds
    cfg.churn_threshold = churn_threshold
    cfg.ping_every = ping_every
    cfg.max_missed = max_missed
    cfg.max_rounds = max_rounds
    cfg.min_rounds = min_rounds
    cfg.device = device
    cfg.flags = (_abi.FLAG_COVERAGE_HISTORY if coverage_history else 0) | (0 if bins else _abi.FLAG_NO_BIN) | {
        "auto": 0, "push": _abi.FLAG_FORCE_PUSH, "pull": _abi.FLAG_FORCE_PULL, "bin": _abi.FLAG_FORCE_BIN}[mode] | {
        "auto": 0, "off": _abi.FLAG_NO_BLOCKED, "force": _abi.FLAG_FORCE_BLOCKED}[blocked] | (
        _abi.FLAG_UNIFORM_PARTITION if uniform_partition else 0)
    cfg.report_capacity = report_capacity
    cfg.pull_permille = pull_permille
    cfg.front_permille = front_permille
    cfg.bin_permille = bin_permille
    cfg.extra_cap = extra_cap
    cfg.list_cap = list_cap
    cfg.rejoin_threshold = rejoin_threshold
    cfg.blocked_permille = blocked_permille
    return cfg


class Engine:
    def __init__(self, n_peers: int, n_msgs: int, *, part: tuple[int, int] = (0, 0), tuning: dict | None = None,
                 **kw):
        self._L = _abi.lib()
        cfg = make_config(n_peers, n_msgs, part=part, **kw)
        self.cfg = cfg
        ctx = C.c_void_p()
        check(self._L.gossip_create(C.byref(cfg), C.byref(ctx)), "gossip_create")
        self._ctx = ctx
        for key, value in (tuning or {}).items():
            self.set_tuning(key, value)
        self.n_peers = n_peers
        self.n_msgs = n_msgs
        self.begin, self.end = (part if part != (0, 0) else (0, n_peers))

    # -- lifecycle ----------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_ctx", None) and self._ctx.value:
            self._L.gossip_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ctx(self):
        return self._ctx

    def shape(self) -> dict:
        w, x, nl, ne = C.c_uint32(), C.c_uint32(), C.c_uint64(), C.c_uint64()
        check(self._L.gossip_get_shape(self._ctx, C.byref(w), C.byref(x), C.byref(nl), C.byref(ne)), "get_shape")
        return {"words": w.value, "exchange_words": x.value, "n_local": nl.value, "n_edges": ne.value}

    def set_stream(self, stream_handle: int) -> None:
        check(self._L.gossip_set_stream(self._ctx, C.c_void_p(stream_handle)), "gossip_set_stream")

    # -- overlay --------------------------------------------------------------
    def build_graph(self) -> None:
        check(self._L.gossip_build_graph(self._ctx), "gossip_build_graph")

    def load_csr(self, row_ptr: np.ndarray, col: np.ndarray) -> None:
        rp = np.ascontiguousarray(row_ptr, dtype=np.uint64)
        cl = np.ascontiguousarray(col, dtype=np.uint32)
        if cl.size == 0:
            cl = np.zeros(1, dtype=np.uint32)
        check(self._L.gossip_load_csr(self._ctx, _ptr(rp, C.c_uint64), _ptr(cl, C.c_uint32), rp.size - 1,
                                      int(rp[-1])), "gossip_load_csr")

    def read_csr(self) -> tuple[np.ndarray, np.ndarray]:
        s = self.shape()
        rp = np.zeros(s["n_local"] + 1, dtype=np.uint64)
        col = np.zeros(max(s["n_edges"], 1), dtype=np.uint32)
        check(self._L.gossip_read_csr(self._ctx, _ptr(rp, C.c_uint64), _ptr(col, C.c_uint32)), "gossip_read_csr")
        return rp, col[: s["n_edges"]]

    def read_extra(self) -> tuple[np.ndarray, np.ndarray]:
        """Re-bootstrap edges: counts[n_local], cols[n_local, extra_cap] (bit 31 = dropped again)."""
        nl, K = self.shape()["n_local"], self.cfg.extra_cap
        cnt = np.zeros(nl, dtype=np.uint32)
        cols = np.zeros(max(nl * K, 1), dtype=np.uint32)
        check(self._L.gossip_read_extra(self._ctx, _ptr(cnt, C.c_uint32), _ptr(cols, C.c_uint32)), "gossip_read_extra")
        return cnt, cols[: nl * K].reshape(nl, K)

    # -- schedule ---------------------------------------------------------------
    def inject(self, origin, inject_round) -> None:
        o, r = _u32(origin), _u32(inject_round)
        check(self._L.gossip_inject(self._ctx, _ptr(o, C.c_uint32), _ptr(r, C.c_uint32), o.size), "gossip_inject")

    def schedule_kills(self, peers, rounds) -> None:
        p, r = _u32(peers), _u32(rounds)
        n = p.size
        if n == 0:
            p = r = np.zeros(1, dtype=np.uint32)
        check(self._L.gossip_schedule_kills(self._ctx, _ptr(p, C.c_uint32), _ptr(r, C.c_uint32), n),
              "gossip_schedule_kills")

    # -- rounds -----------------------------------------------------------------
    def reset(self) -> None:
        check(self._L.gossip_reset(self._ctx), "gossip_reset")

    def step(self) -> tuple[dict, bool]:
        st = RoundStats()
        rc = check(self._L.gossip_step(self._ctx, C.byref(st)), "gossip_step")
        return st.as_dict(), rc == 1

    def run(self, cap: int = 4096) -> list[dict]:
        buf = (RoundStats * cap)()
        rounds = C.c_uint32()
        check(self._L.gossip_run(self._ctx, buf, cap, C.byref(rounds)), "gossip_run")
        return [buf[i].as_dict() for i in range(min(rounds.value, cap))]

    def run_into(self, cap: int = 4096) -> int:
        """gossip_run into a buffer kept across calls; returns the rounds run (their stats: last_stats())."""
        if getattr(self, "_run_buf", None) is None or len(self._run_buf) < cap:
            self._run_buf, self._run_n = (RoundStats * cap)(), C.c_uint32()
        check(self._L.gossip_run(self._ctx, self._run_buf, cap, C.byref(self._run_n)), "gossip_run")
        return self._run_n.value

    def last_stats(self) -> list[dict]:
        """The rounds of the last run_into(), as run() returns them ([] before the first)."""
        if getattr(self, "_run_buf", None) is None:
            return []
        return [self._run_buf[i].as_dict() for i in range(min(self._run_n.value, len(self._run_buf)))]

    # partitioned phases (see distributed.py)
    def set_exchange(self, send_ptr: int, recv_ptr: int, part_begins) -> None:
        pb = np.ascontiguousarray(part_begins, dtype=np.uint64)
        check(self._L.gossip_set_exchange(self._ctx, C.c_void_p(send_ptr), C.c_void_p(recv_ptr), pb.size - 1,
                                          _ptr(pb, C.c_uint64)), "gossip_set_exchange")

    def set_gather(self, gather_ptr: int) -> None:
        check(self._L.gossip_set_gather(self._ctx, C.c_void_p(gather_ptr)), "gossip_set_gather")

    def round_begin(self, mode: int) -> int:
        """Phase 1 of a partitioned round; returns the mode actually run (0 push, 1 pull, 2 sparse push, 3 binned, 4 blocked)."""
        got = C.c_int()
        check(self._L.gossip_round_begin(self._ctx, mode, C.byref(got)), "gossip_round_begin")
        return got.value

    def round_compute(self) -> None:
        check(self._L.gossip_round_compute(self._ctx), "gossip_round_compute")

    def set_sparse(self, seg_ptr: int) -> None:
        check(self._L.gossip_set_sparse(self._ctx, C.c_void_p(seg_ptr)), "gossip_set_sparse")

    def sparse_counts(self, world: int) -> np.ndarray:
        out = np.zeros(world, dtype=np.uint64)
        check(self._L.gossip_sparse_counts(self._ctx, _ptr(out, C.c_uint64)), "gossip_sparse_counts")
        return out

    def round_finish_sparse(self, records_ptr: int, n_records: int) -> dict:
        st = RoundStats()
        check(self._L.gossip_round_finish_sparse(self._ctx, C.c_void_p(records_ptr), n_records, C.byref(st)),
              "gossip_round_finish_sparse")
        return st.as_dict()

    def round_push(self) -> None:
        check(self._L.gossip_round_push(self._ctx), "gossip_round_push")

    def round_finish(self) -> dict:
        st = RoundStats()
        check(self._L.gossip_round_finish(self._ctx, C.byref(st)), "gossip_round_finish")
        return st.as_dict()

    def round_commit(self, global_new_receipts: int) -> bool:
        fin = C.c_int()
        check(self._L.gossip_round_commit(self._ctx, global_new_receipts, C.byref(fin)), "gossip_round_commit")
        return bool(fin.value)

    # library-driven multi-GPU rounds (RCCL inside libgossip_hip)
    def comm_init(self, unique_id: bytes, world: int, rank: int) -> None:
        """Join the library's RCCL communicator as `rank` of `world` (collective);
        afterwards step()/run() issue every round's collectives themselves."""
        buf = (C.c_uint8 * _abi.COMM_ID_BYTES).from_buffer_copy(unique_id)
        check(self._L.gossip_comm_init(self._ctx, buf, world, rank), "gossip_comm_init")

    def comm_finalize(self, rounds: list[dict]) -> np.ndarray:
        """Collective: every rank's dead-node reports (sorted) and the global
        seed_removals of each round (filled into `rounds`)."""
        buf = (RoundStats * max(len(rounds), 1))()
        for i, r in enumerate(rounds):
            for f, _ in RoundStats._fields_:
                setattr(buf[i], f, r[f])
        cnt = C.c_uint64()
        check(self._L.gossip_comm_finalize(self._ctx, buf, len(rounds), None, 0, C.byref(cnt)), "gossip_comm_finalize")
        reps = np.zeros((max(cnt.value, 1), 3), dtype=np.uint32)
        check(self._L.gossip_comm_finalize(self._ctx, buf, len(rounds), reps.ctypes.data_as(C.POINTER(DeadReport)),
                                           cnt.value, C.byref(cnt)), "gossip_comm_finalize")
        for i, r in enumerate(rounds):
            r["seed_removals"] = int(buf[i].seed_removals)
        return reps[: cnt.value]

    def comm_modes(self) -> list[int]:
        n = C.c_uint32()
        check(self._L.gossip_comm_modes(self._ctx, None, 0, C.byref(n)), "gossip_comm_modes")
        out = (C.c_int32 * max(n.value, 1))()
        check(self._L.gossip_comm_modes(self._ctx, out, n.value, C.byref(n)), "gossip_comm_modes")
        return list(out)[: n.value]

    # -- results ----------------------------------------------------------------
    def read_seen(self) -> np.ndarray:
        s = self.shape()
        out = np.zeros((s["n_local"], s["words"]), dtype=np.uint64)
        check(self._L.gossip_read_seen(self._ctx, _ptr(out, C.c_uint64)), "gossip_read_seen")
        return out

    def coverage(self) -> np.ndarray:
        out = np.zeros(self.n_msgs, dtype=np.uint64)
        check(self._L.gossip_read_coverage(self._ctx, _ptr(out, C.c_uint64)), "gossip_read_coverage")
        return out

    def coverage_history(self, max_rounds: int = 4096) -> np.ndarray:
        buf = np.zeros((max_rounds, self.n_msgs), dtype=np.uint64)
        r = C.c_uint32()
        check(self._L.gossip_read_coverage_history(self._ctx, _ptr(buf, C.c_uint64), max_rounds, C.byref(r)),
              "gossip_read_coverage_history")
        return buf[: r.value]

    def reports(self) -> np.ndarray:
        cnt = C.c_uint64()
        check(self._L.gossip_read_reports(self._ctx, None, 0, C.byref(cnt)), "gossip_read_reports")
        n = cnt.value
        buf = np.zeros((max(n, 1), 3), dtype=np.uint32)  # DeadReport = 3 x u32
        check(self._L.gossip_read_reports(self._ctx, buf.ctypes.data_as(C.POINTER(DeadReport)), n, C.byref(cnt)),
              "gossip_read_reports")
        return buf[:n]

    def alive(self) -> np.ndarray:
        out = np.zeros(self.n_peers, dtype=np.uint8)
        check(self._L.gossip_read_alive(self._ctx, _ptr(out, C.c_uint8)), "gossip_read_alive")
        return out

    def registered(self) -> np.ndarray:
        out = np.zeros(self.n_peers, dtype=np.uint8)
        check(self._L.gossip_read_registered(self._ctx, _ptr(out, C.c_uint8)), "gossip_read_registered")
        return out

    def set_tuning(self, key: str, value: int) -> None:
        """gossip_set_tuning: a parity-tested engineering option of this ctx (layout keys apply at the
        next build_graph / load_csr)."""
        check(self._L.gossip_set_tuning(self._ctx, key.encode(), int(value)), f"gossip_set_tuning({key})")

    # -- measurement ------------------------------------------------------------
    def enable_timing(self, on: bool = True) -> None:
        check(self._L.gossip_enable_timing(self._ctx, 1 if on else 0), "gossip_enable_timing")

    def kernel_time(self, name: str) -> tuple[float, int]:
        ms, n = C.c_double(), C.c_uint64()
        check(self._L.gossip_kernel_time(self._ctx, name.encode(), C.byref(ms), C.byref(n)), "gossip_kernel_time")
        return ms.value, n.value

    def kernel_bytes(self, name: str) -> float:
        b = C.c_double()
        check(self._L.gossip_kernel_bytes(self._ctx, name.encode(), C.byref(b)), "gossip_kernel_bytes")
        return b.value


class Group:
    """One process driving several vertex blocks (gossip_group_*): one part
    per entry of `devices` (distinct GPUs: RCCL communicators from
    ncclCommInitAll; all the same GPU: device-copy exchange).  Takes the
    Engine's keyword arguments (except part/device); `begins` (n_parts + 1
    block bounds) replaces the default partition (gossip_group_create_parts)."""

    def __init__(self, n_peers: int, n_msgs: int, devices, tuning: dict | None = None, begins=None, **kw):
        self._L = _abi.lib()
        cfg = make_config(n_peers, n_msgs, **kw)
        devs = (C.c_int32 * len(devices))(*devices)
        g = C.c_void_p()
        if begins is None:
            check(self._L.gossip_group_create(C.byref(cfg), len(devices), devs, C.byref(g)), "gossip_group_create")
        else:
            b = (C.c_uint64 * (len(devices) + 1))(*[int(x) for x in begins])
            check(self._L.gossip_group_create_parts(C.byref(cfg), len(devices), devs, b, C.byref(g)),
                  "gossip_group_create_parts")
        self._g = g
        self.n_peers, self.n_msgs = n_peers, n_msgs
        self.W = (n_msgs + 63) // 64
        self.n_parts = len(devices)
        for key, value in (tuning or {}).items():  # every part gets the same options
            for p in range(self.n_parts):
                check(self._L.gossip_set_tuning(self.part_ctx(p), key.encode(), int(value)),
                      f"gossip_set_tuning({key})")

    def close(self) -> None:
        if getattr(self, "_g", None) and self._g.value:
            self._L.gossip_group_destroy(self._g)
            self._g = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def build_graph(self) -> None:
        check(self._L.gossip_group_build_graph(self._g), "gossip_group_build_graph")

    def inject(self, origin, inject_round) -> None:
        o, r = _u32(origin), _u32(inject_round)
        check(self._L.gossip_group_inject(self._g, _ptr(o, C.c_uint32), _ptr(r, C.c_uint32), o.size),
              "gossip_group_inject")

    def schedule_kills(self, peers, rounds) -> None:
        p, r = _u32(peers), _u32(rounds)
        n = p.size
        if n == 0:
            p = r = np.zeros(1, dtype=np.uint32)
        check(self._L.gossip_group_schedule_kills(self._g, _ptr(p, C.c_uint32), _ptr(r, C.c_uint32), n),
              "gossip_group_schedule_kills")

    def reset(self) -> None:
        check(self._L.gossip_group_reset(self._g), "gossip_group_reset")

    def step(self) -> tuple[dict, bool]:
        st = RoundStats()
        rc = check(self._L.gossip_group_step(self._g, C.byref(st)), "gossip_group_step")
        return st.as_dict(), rc == 1

    def run(self, cap: int = 4096) -> list[dict]:
        buf = (RoundStats * cap)()
        rounds = C.c_uint32()
        check(self._L.gossip_group_run(self._g, buf, cap, C.byref(rounds)), "gossip_group_run")
        return [buf[i].as_dict() for i in range(min(rounds.value, cap))]

    def run_into(self, cap: int = 4096) -> int:
        """gossip_group_run into a buffer kept across calls; returns the rounds run (their stats: last_stats())."""
        if getattr(self, "_run_buf", None) is None or len(self._run_buf) < cap:
            self._run_buf, self._run_n = (RoundStats * cap)(), C.c_uint32()
        check(self._L.gossip_group_run(self._g, self._run_buf, cap, C.byref(self._run_n)), "gossip_group_run")
        return self._run_n.value

    def last_stats(self) -> list[dict]:
        """The rounds of the last run_into(), as run() returns them ([] before the first)."""
        if getattr(self, "_run_buf", None) is None:
            return []
        return [self._run_buf[i].as_dict() for i in range(min(self._run_n.value, len(self._run_buf)))]

    def read_seen(self) -> np.ndarray:
        out = np.zeros((self.n_peers, self.W), dtype=np.uint64)
        check(self._L.gossip_group_read_seen(self._g, _ptr(out, C.c_uint64)), "gossip_group_read_seen")
        return out

    def reports(self) -> np.ndarray:
        cnt = C.c_uint64()
        check(self._L.gossip_group_read_reports(self._g, None, 0, C.byref(cnt)), "gossip_group_read_reports")
        buf = np.zeros((max(cnt.value, 1), 3), dtype=np.uint32)
        check(self._L.gossip_group_read_reports(self._g, buf.ctypes.data_as(C.POINTER(DeadReport)), cnt.value,
                                                C.byref(cnt)), "gossip_group_read_reports")
        return buf[: cnt.value]

    def part_ctx(self, p: int) -> C.c_void_p:
        ctx = C.c_void_p()
        check(self._L.gossip_group_part(self._g, p, C.byref(ctx)), "gossip_group_part")
        return ctx

    # per-part measurement (each part's ctx times the kernels and exchanges issued on its stream)
    def enable_timing(self, on: bool = True) -> None:
        for p in range(self.n_parts):
            check(self._L.gossip_enable_timing(self.part_ctx(p), 1 if on else 0), "gossip_enable_timing")

    def kernel_time(self, p: int, name: str) -> tuple[float, int]:
        ms, n = C.c_double(), C.c_uint64()
        check(self._L.gossip_kernel_time(self.part_ctx(p), name.encode(), C.byref(ms), C.byref(n)),
              "gossip_kernel_time")
        return ms.value, n.value

    def kernel_bytes(self, p: int, name: str) -> float:
        b = C.c_double()
        check(self._L.gossip_kernel_bytes(self.part_ctx(p), name.encode(), C.byref(b)), "gossip_kernel_bytes")
        return b.value

    def coverage(self) -> np.ndarray:
        """Per-message coverage over all peers (the parts' counts summed)."""
        tot = np.zeros(self.n_msgs, dtype=np.uint64)
        for p in range(self.n_parts):
            out = np.zeros(self.n_msgs, dtype=np.uint64)
            check(self._L.gossip_read_coverage(self.part_ctx(p), _ptr(out, C.c_uint64)), "gossip_read_coverage")
            tot += out
        return tot

    def alive(self) -> np.ndarray:
        """Alive flags of all peers (every part keeps the same global bitset: churn is drawn redundantly)."""
        out = np.zeros(self.n_peers, dtype=np.uint8)
        check(self._L.gossip_read_alive(self.part_ctx(0), _ptr(out, C.c_uint8)), "gossip_read_alive")
        return out

    def registered(self) -> np.ndarray:
        """Seed-registry membership: a peer is gone once any part's reporter has reported it
        (each part clears the registry bits of its own reports)."""
        reg = None
        for p in range(self.n_parts):
            out = np.zeros(self.n_peers, dtype=np.uint8)
            check(self._L.gossip_read_registered(self.part_ctx(p), _ptr(out, C.c_uint8)), "gossip_read_registered")
            reg = out if reg is None else reg & out
        return reg

    def shape(self, p: int) -> dict:
        w, x, nl, ne = C.c_uint32(), C.c_uint32(), C.c_uint64(), C.c_uint64()
        check(self._L.gossip_get_shape(self.part_ctx(p), C.byref(w), C.byref(x), C.byref(nl), C.byref(ne)),
              "get_shape")
        return {"words": w.value, "exchange_words": x.value, "n_local": nl.value, "n_edges": ne.value}
