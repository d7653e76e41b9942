"""ctypes binding of oracle/libgossip_oracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the checker: tests compare libgossip_hip against it, never the
other way round, and nothing in the product imports this module.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

STAT_FIELDS = ("frontier", "traversals", "deliveries", "undelivered", "new_receipts", "duplicates", "injected",
               "died", "reports", "seed_removals", "digest", "covered", "reconnects", "rejoined")


class OStats(C.Structure):
    _fields_ = [("round", C.c_uint32), ("flags", C.c_uint32)] + [(f, C.c_uint64) for f in STAT_FIELDS]

    def as_dict(self):
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


class OCfg(C.Structure):
    _fields_ = [("n", C.c_uint64), ("n_msgs", C.c_uint32), ("seed", C.c_uint32), ("churn_threshold", C.c_uint32),
                ("ping_every", C.c_uint32), ("max_missed", C.c_uint32), ("max_rounds", C.c_uint32),
                ("min_rounds", C.c_uint32), ("threads", C.c_int), ("variant", C.c_int), ("extra_cap", C.c_uint32),
                ("list_len", C.c_uint32), ("n_started", C.c_uint64), ("rejoin_threshold", C.c_uint32),
                ("pad0", C.c_uint32)]


class OReport(C.Structure):
    _fields_ = [("round", C.c_uint32), ("reporter", C.c_uint32), ("dead", C.c_uint32)]


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


class Oracle:
    def __init__(self, so: Path):
        L = C.CDLL(str(so))
        L.oracle_threshold.restype = C.c_uint64
        L.oracle_skew_pick.restype = C.c_uint32
        L.oracle_started_under_cap.restype = C.c_uint64
        L.oracle_skew_pick.argtypes = [C.c_uint32, C.c_uint64]
        L.oracle_digest_weight.restype = C.c_uint64
        L.oracle_digest_weight.argtypes = [C.c_uint64]
        for name, t in (("oracle_hash_u64", C.c_uint64), ("oracle_hash_u32", C.c_uint32), ("oracle_hash_u8", C.c_uint8)):
            getattr(L, name).restype = C.c_uint64
            getattr(L, name).argtypes = [C.POINTER(t), C.c_uint64, C.c_int]
        L.oracle_sim_create.restype = C.c_void_p
        L.oracle_sim_reports.restype = C.c_uint64
        L.oracle_sim_sent_to_total.restype = C.c_uint64
        for name in ("oracle_sim_step", "oracle_sim_run", "oracle_sim_schedule"):
            getattr(L, name).restype = C.c_int
        self.L = L

    def philox(self, ctr, key):
        out = (C.c_uint32 * 4)()
        self.L.oracle_philox4x32_10((C.c_uint32 * 4)(*ctr), (C.c_uint32 * 2)(*key), out)
        return [int(x) for x in out]

    def hash(self, a, threads=8) -> int:
        """Fixture checksum: sum_i g(i) * a[i] mod 2^64 (g = the digest weights)."""
        a = np.ascontiguousarray(a).reshape(-1)
        fn, t = {8: (self.L.oracle_hash_u64, C.c_uint64), 4: (self.L.oracle_hash_u32, C.c_uint32),
                 1: (self.L.oracle_hash_u8, C.c_uint8)}[a.dtype.itemsize]
        return int(fn(_p(a, t), C.c_uint64(a.size), C.c_int(threads)))

    def threshold(self, j, L):
        return int(self.L.oracle_threshold(C.c_uint32(j), C.c_uint32(L)))

    def pick_origins(self, n, seed, count):
        out = (C.c_uint32 * max(count, 1))()
        self.L.oracle_pick_origins(C.c_uint64(n), C.c_uint32(seed), C.c_uint32(count), out)
        return np.array(list(out)[:count], dtype=np.uint32)

    def gen(self, kind, n, arg, seed, threads=8):
        rp = C.POINTER(C.c_uint64)()
        col = C.POINTER(C.c_uint32)()
        e = C.c_uint64()
        if kind == "ref_bootstrap":
            rc = self.L.oracle_gen_ref_bootstrap(C.c_uint32(n), C.c_uint32(arg), C.c_uint32(seed), C.byref(rp),
                                                 C.byref(col), C.byref(e))
        else:
            rc = self.L.oracle_gen_powerlaw(C.c_uint64(n), C.c_uint32(arg), C.c_uint32(seed), C.c_int(threads),
                                            C.byref(rp), C.byref(col), C.byref(e))
        assert rc == 0, "oracle generator failed"
        R = np.ctypeslib.as_array(rp, (n + 1,)).copy()
        Cc = np.ctypeslib.as_array(col, (max(e.value, 1),)).copy()[: e.value]
        self.L.oracle_free(C.cast(rp, C.c_void_p))
        self.L.oracle_free(C.cast(col, C.c_void_p))
        return R, Cc

    def gen_workload(self, w, threads=8):
        arg = w.n_seeds if w.graph == "ref_bootstrap" else w.list_len
        return self.gen(w.graph, w.n, arg, w.rng_seed, threads)

    def simulate(self, rp, col, n, n_msgs, origins, inject_rounds, *, seed=0, churn_threshold=0, ping_every=0,
                 max_missed=3, max_rounds=4096, min_rounds=0, kills=(), variant=0, threads=8, extra_cap=0,
                 list_len=6, n_started=0, rejoin_threshold=0):
        rp = np.ascontiguousarray(rp, dtype=np.uint64)
        col = np.ascontiguousarray(col if len(col) else np.zeros(1), dtype=np.uint32)
        cfg = OCfg(n, n_msgs, seed, churn_threshold, ping_every, max_missed, max_rounds, min_rounds, threads, variant,
                   extra_cap, list_len, n_started, rejoin_threshold)
        s = self.L.oracle_sim_create(C.byref(cfg), _p(rp, C.c_uint64), _p(col, C.c_uint32))
        assert s, "oracle_sim_create failed"
        s = C.c_void_p(s)
        try:
            o = np.ascontiguousarray(origins, dtype=np.uint32)
            r = np.ascontiguousarray(inject_rounds, dtype=np.uint32)
            kp = np.array([k[0] for k in kills] + [0], dtype=np.uint32)
            kr = np.array([k[1] for k in kills] + [0], dtype=np.uint32)
            assert self.L.oracle_sim_schedule(s, _p(o, C.c_uint32), _p(r, C.c_uint32), C.c_uint32(len(kills)),
                                              _p(kp, C.c_uint32), _p(kr, C.c_uint32)) == 0
            buf = (OStats * max_rounds)()
            nr = self.L.oracle_sim_run(s, buf, C.c_uint32(max_rounds))
            stats = [buf[i].as_dict() for i in range(nr)]
            W = (n_msgs + 63) // 64
            seen = np.zeros((n, W), dtype=np.uint64)
            self.L.oracle_sim_seen(s, _p(seen, C.c_uint64))
            cov = np.zeros(n_msgs, dtype=np.uint64)
            self.L.oracle_sim_coverage(s, _p(cov, C.c_uint64))
            nrep = int(self.L.oracle_sim_reports(s, None, C.c_uint64(0)))
            reps = np.zeros((max(nrep, 1), 3), dtype=np.uint32)
            self.L.oracle_sim_reports(s, reps.ctypes.data_as(C.POINTER(OReport)), C.c_uint64(nrep))
            reps = reps[:nrep]
            alive = np.zeros(n, dtype=np.uint8)
            self.L.oracle_sim_alive(s, _p(alive, C.c_uint8))
            reg = np.zeros(n, dtype=np.uint8)
            self.L.oracle_sim_registered(s, _p(reg, C.c_uint8))
            sent = int(self.L.oracle_sim_sent_to_total(s))
            ex_cnt = np.zeros(n, dtype=np.uint32)
            ex_col = np.zeros(max(n * extra_cap, 1), dtype=np.uint32)
            self.L.oracle_sim_extra(s, _p(ex_cnt, C.c_uint32), _p(ex_col, C.c_uint32))
            return dict(stats=stats, seen=seen, coverage=cov, reports=reps, alive=alive, registered=reg,
                        sent_to_total=sent, extra_counts=ex_cnt, extra_cols=ex_col[:n * extra_cap].reshape(n, extra_cap))
        finally:
            self.L.oracle_sim_destroy(s)

    def simulate_workload(self, w, rp, col, variant=0, threads=8, max_rounds=4096):
        return self.simulate(rp, col, w.n, w.n_msgs, w.origins, w.inject_rounds, seed=w.rng_seed,
                             churn_threshold=w.churn_threshold, ping_every=w.ping_every, max_missed=w.max_missed,
                             min_rounds=w.min_rounds, kills=w.kills, variant=variant, threads=threads,
                             max_rounds=max_rounds, extra_cap=w.extra_cap, list_len=w.list_len,
                             n_started=self.started_under_cap(w.n, w.list_cap) if w.graph == "ref_bootstrap" else 0,
                             rejoin_threshold=w.rejoin_threshold)

    def time_rounds(self, w, rp, col, threads=8, variant=0, repeats=5, max_rounds=4096):
        """CPU baseline: wall seconds of oracle_sim_run alone (the rounds; create,
        schedule and every read-back untimed), `repeats` fresh sims.  Returns
        (list of seconds, per-round stats of the last run)."""
        import time
        rp = np.ascontiguousarray(rp, dtype=np.uint64)
        col = np.ascontiguousarray(col if len(col) else np.zeros(1), dtype=np.uint32)
        cfg = OCfg(w.n, w.n_msgs, w.rng_seed, w.churn_threshold, w.ping_every, w.max_missed, max_rounds,
                   w.min_rounds, threads, variant, w.extra_cap, w.list_len,
                   self.started_under_cap(w.n, w.list_cap) if w.graph == "ref_bootstrap" else 0, w.rejoin_threshold)
        o = np.ascontiguousarray(w.origins, dtype=np.uint32)
        r = np.ascontiguousarray(w.inject_rounds, dtype=np.uint32)
        kp = np.array([k[0] for k in w.kills] + [0], dtype=np.uint32)
        kr = np.array([k[1] for k in w.kills] + [0], dtype=np.uint32)
        secs, stats = [], []
        for _ in range(repeats):
            s = C.c_void_p(self.L.oracle_sim_create(C.byref(cfg), _p(rp, C.c_uint64), _p(col, C.c_uint32)))
            assert s.value, "oracle_sim_create failed"
            try:
                assert self.L.oracle_sim_schedule(s, _p(o, C.c_uint32), _p(r, C.c_uint32), C.c_uint32(len(w.kills)),
                                                  _p(kp, C.c_uint32), _p(kr, C.c_uint32)) == 0
                buf = (OStats * max_rounds)()
                t0 = time.perf_counter()
                nr = self.L.oracle_sim_run(s, buf, C.c_uint32(max_rounds))
                secs.append(time.perf_counter() - t0)
                stats = [buf[i].as_dict() for i in range(nr)]
            finally:
                self.L.oracle_sim_destroy(s)
        return secs, stats

    def started_under_cap(self, n, list_cap):
        return int(self.L.oracle_started_under_cap(C.c_uint64(n), C.c_uint32(list_cap)))


class OraclePartition:
    """One rank's block of the oracle's partition emulation, with the same
    phase API the multi-rank driver (gossip_hip.distributed) drives on a
    libgossip_hip Engine.  CPU tests only."""

    def __init__(self, orc: Oracle, w, rp_global, col_global, begin, end, threads=1):
        L = orc.L
        L.oracle_part_create.restype = C.c_void_p
        L.oracle_part_reports.restype = C.c_uint64
        self.L, self.w = L, w
        self.begin, self.end = begin, end
        self.n_local = end - begin
        self.W = (w.n_msgs + 63) // 64
        base = int(rp_global[begin])
        self.rp = np.ascontiguousarray(rp_global[begin:end + 1] - np.uint64(base), dtype=np.uint64)
        self.col = np.ascontiguousarray(col_global[base:int(rp_global[end])], dtype=np.uint32)
        if self.col.size == 0:
            self.col = np.zeros(1, dtype=np.uint32)
        cfg = OCfg(w.n, w.n_msgs, w.rng_seed, w.churn_threshold, w.ping_every, w.max_missed, 4096, w.min_rounds,
                   threads, 0)
        self.p = C.c_void_p(L.oracle_part_create(C.byref(cfg), C.c_uint64(begin), C.c_uint64(end),
                                                  _p(self.rp, C.c_uint64), _p(self.col, C.c_uint32)))
        o = np.ascontiguousarray(w.origins, dtype=np.uint32)
        r = np.ascontiguousarray(w.inject_rounds, dtype=np.uint32)
        kp = np.array([k[0] for k in w.kills] + [0], dtype=np.uint32)
        kr = np.array([k[1] for k in w.kills] + [0], dtype=np.uint32)
        L.oracle_part_schedule(self.p, _p(o, C.c_uint32), _p(r, C.c_uint32), C.c_uint32(len(w.kills)),
                               _p(kp, C.c_uint32), _p(kr, C.c_uint32))
        self._send = self._recv = None
        self.world = 1

    def shape(self):
        return {"words": self.W, "exchange_words": self.W, "n_local": self.n_local, "n_edges": int(self.rp[-1])}

    def set_exchange(self, send_ptr, recv_ptr, part):
        self._send = C.cast(C.c_void_p(send_ptr), C.POINTER(C.c_uint64))
        self._recv = C.cast(C.c_void_p(recv_ptr), C.POINTER(C.c_uint64))
        self.world = len(part) - 1
        self._send_words = self.w.n * self.W

    def reset(self):
        self.L.oracle_part_reset(self.p)

    def set_gather(self, gather_ptr):
        self._gather = C.cast(C.c_void_p(gather_ptr), C.POINTER(C.c_uint64))

    def set_sparse(self, seg_ptr):
        self._seg = C.cast(C.c_void_p(seg_ptr), C.POINTER(C.c_uint64))
        self._counts = np.zeros(self.world, dtype=np.uint64)

    def round_begin(self, mode):
        self._pull = bool(self.L.oracle_part_begin(self.p, C.c_int(1 if mode in (1, 3) else 0)))
        self._sparse = (not self._pull) and mode == 2 and getattr(self, "_seg", None) is not None
        if self._pull:
            self.L.oracle_part_publish(self.p, self._gather)
        elif not self._sparse:
            C.memset(self._send, 0, self._send_words * 8)
        return (3 if mode == 3 else 1) if self._pull else (2 if self._sparse else 0)

    def round_compute(self):
        if self._pull:
            self.L.oracle_part_pull(self.p, self._gather)
        else:
            self.L.oracle_part_push_compute(self.p, self._send)
            if self._sparse:
                chunk = -(-self.w.n // self.world)
                self.L.oracle_part_compact(self.p, self._send, C.c_uint64(chunk), C.c_uint32(self.world),
                                           self._seg, _p(self._counts, C.c_uint64))

    def sparse_counts(self, world):
        return self._counts.copy()

    def round_finish_sparse(self, records_ptr, n_records):
        st = OStats()
        self.L.oracle_part_finish_records(self.p, C.cast(C.c_void_p(records_ptr), C.POINTER(C.c_uint64)),
                                          C.c_uint64(n_records), C.byref(st))
        return st.as_dict()

    def round_push(self):
        C.memset(self._send, 0, self._send_words * 8)
        self.L.oracle_part_push(self.p, self._send)

    def round_finish(self):
        st = OStats()
        self.L.oracle_part_finish(self.p, self._recv, C.c_uint32(self.world), C.byref(st))
        return st.as_dict()

    def round_commit(self, global_new_receipts):
        return bool(self.L.oracle_part_commit(self.p, C.c_uint64(global_new_receipts)))

    def read_seen(self):
        out = np.zeros((self.n_local, self.W), dtype=np.uint64)
        self.L.oracle_part_seen(self.p, _p(out, C.c_uint64))
        return out

    def reports(self):
        n = int(self.L.oracle_part_reports(self.p, None, C.c_uint64(0)))
        buf = (OReport * max(n, 1))()
        self.L.oracle_part_reports(self.p, buf, C.c_uint64(n))
        return np.array([(buf[i].round, buf[i].reporter, buf[i].dead) for i in range(n)],
                        dtype=np.uint32).reshape(n, 3)

    def close(self):
        if self.p:
            self.L.oracle_part_destroy(self.p)
            self.p = None
