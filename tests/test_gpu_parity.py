"""GPU parity: libgossip_hip (through its C-ABI) vs the CPU oracle on the
same seeded inputs -- bit-exact stats, seen sets, reports, alive/registry --
plus size-independent properties at BASELINE.json's full sizes."""
import dataclasses
import json
from pathlib import Path

import numpy as np
import pytest

from gossip_hip import Engine
from gossip_hip.workloads import _batches, config, run_engine

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"


def _engine(w, **kw):
    return Engine(w.n, w.n_msgs, **w.engine_kwargs(), **kw)


def _hand_csr(case):
    rows = case["rows"]
    rp = np.zeros(len(rows) + 1, dtype=np.uint64)
    rp[1:] = np.cumsum([len(r) for r in rows])
    return rp, np.array([c for r in rows for c in r], dtype=np.uint32)


@pytest.mark.parametrize("mode", ["push", "pull", "bin"])
@pytest.mark.parametrize("case", json.loads((GOLDEN / "hand_graphs.json").read_text())["cases"],
                         ids=lambda c: c["name"])
def test_hand_graphs(case, mode):
    fields = json.loads((GOLDEN / "hand_graphs.json").read_text())["fields"]
    with Engine(case["n"], len(case["origins"]), ping_every=case.get("ping_every", 0),
                max_missed=case.get("max_missed", 3), min_rounds=case.get("min_rounds", 0), mode=mode) as e:
        e.load_csr(*_hand_csr(case))
        e.inject(case["origins"], case["inject_rounds"])
        kills = case.get("kills", [])
        if kills:
            e.schedule_kills([k[0] for k in kills], [k[1] for k in kills])
        e.reset()
        stats = e.run()
        assert [[s[f] for f in fields] for s in stats] == case["expect"]
        assert e.coverage().tolist() == case["coverage"]
        assert e.reports().tolist() == case.get("reports", [])


@pytest.mark.parametrize("kind,n,arg,seed", [("ref_bootstrap", 8, 20, 0x5EED0001), ("ref_bootstrap", 300, 20, 5),
                                             ("powerlaw", 1 << 12, 6, 3), ("powerlaw", 1 << 18, 6, 0x5EED0002),
                                             ("powerlaw", 100_003, 11, 9)])
def test_overlay_generator_matches_oracle(oracle, kind, n, arg, seed):
    kw = dict(n_seeds=arg) if kind == "ref_bootstrap" else dict(list_len=arg)
    with Engine(n, 64, rng_seed=seed, graph=kind, **kw) as e:
        e.build_graph()
        rp, col = e.read_csr()
    orp, ocol = oracle.gen(kind, n, arg, seed)
    assert np.array_equal(rp, orp)
    assert np.array_equal(col, ocol)


def _compare(e, ref, w):
    got = e.run()
    assert len(got) == len(ref["stats"])
    for g, r in zip(got, ref["stats"]):
        assert g == r, (g, r)
    assert np.array_equal(e.read_seen(), ref["seen"])
    assert np.array_equal(e.coverage(), ref["coverage"])
    assert np.array_equal(e.reports(), ref["reports"])
    assert np.array_equal(e.alive(), ref["alive"])
    assert np.array_equal(e.registered(), ref["registered"])
    return got


@pytest.mark.parametrize("mode", ["auto", "push", "pull", "bin"])
@pytest.mark.parametrize("idx,n", [(1, None), (2, 1 << 16), (3, 1 << 18), (5, 1 << 16), (5, 50_000)])
def test_workload_parity(oracle, idx, n, mode):
    w = config(idx, n, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    with _engine(w, mode=mode) as e:
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        if w.kills:
            e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        e.reset()
        first = _compare(e, ref, w)
        e.reset()  # a second run from reset is identical
        assert e.run() == first


@pytest.mark.parametrize("blocked", ["force", "auto", "force_hubs", "auto_dense", "force_plain"])
@pytest.mark.parametrize("idx,n", [(2, 1 << 16), (3, 1 << 18), (5, 1 << 16), (5, 50_000), (3, 1 << 20)])
def test_blocked_push_parity(oracle, idx, n, blocked):
    """Propagation-blocked push rounds (gossip_blocked.hip): every push and binned
    round forced blocked, and the default schedule with its blocked rounds --
    against the oracle's per-round stats, seen sets, reports, alive and registry
    (broadcastMessage peer.cpp:310-316 -> handleClient peer.cpp:277-285; dead
    targets are undelivered sends, peer.cpp:312).  force_hubs: the leading tiles
    of in-degree > 1024 (twice the mean) take level 1's direct deliveries (at config 4's size only
    the real hubs do); auto_dense: the binned rounds under 30 % run blocked as at
    config 4's size; force_plain: without round 6's marked-tile level 1 of narrow rounds (the default
    wherever the frontier is under 5 % and the tile marks are kept)."""
    tuning = {}
    if blocked == "force_plain":
        tuning.update(blocked_marks=0)
    if blocked == "force_hubs":
        tuning["blocked_direct_in"] = 1024
    if blocked == "auto_dense":
        tuning["blocked_bin_slots"] = 0
    w = config(idx, n, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    with _engine(w, blocked=blocked.split("_")[0], tuning=tuning) as e:
        e.enable_timing(True)
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        if w.kills:
            e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        e.reset()
        first = _compare(e, ref, w)
        if blocked.startswith("force"):
            assert e.kernel_time("pb_apply")[1] > 0  # the blocked path ran
        e.reset()
        assert e.run() == first


@pytest.mark.parametrize("mode", ["push", "pull", "bin"])
@pytest.mark.parametrize("M", [65, 130, 300, 512])
def test_multiword_messages(oracle, M, mode):
    n = 1 << 14
    rng = np.random.default_rng(M)
    origins = rng.integers(0, n, M).astype(np.uint32)
    rounds = rng.integers(0, 4, M).astype(np.uint32)
    rp, col = oracle.gen("powerlaw", n, 6, 77)
    churn = 42949673 * 2   # dead peers: pull and binned rounds skip them as destinations
    ref = oracle.simulate(rp, col, n, M, origins, rounds, seed=77, churn_threshold=churn, ping_every=2,
                          max_missed=2)
    with Engine(n, M, rng_seed=77, churn_threshold=churn, ping_every=2, max_missed=2, mode=mode) as e:
        e.load_csr(rp, col)
        e.inject(origins, rounds)
        e.reset()
        _compare(e, ref, None)


@pytest.mark.parametrize("mode", ["auto", "bin"])
def test_coverage_history_last_row_is_final(oracle, mode):
    w = config(3, 1 << 14, pick=oracle.pick_origins)
    with _engine(w, coverage_history=True, mode=mode) as e:
        stats = run_engine(e, w)
        hist = e.coverage_history()
        assert hist.shape[0] == len(stats)
        assert np.array_equal(hist[-1], e.coverage())
        assert [int(h.sum()) for h in hist] == [s["covered"] for s in stats]


def _digest(seen):
    n, W = seen.shape
    idx = np.arange(n * W, dtype=np.uint64) + np.uint64(1)
    z = idx * np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = (z ^ (z >> np.uint64(31))) | np.uint64(1)
    return int(np.sum(z * seen.reshape(-1), dtype=np.uint64))


@pytest.mark.parametrize("idx,mode", [(3, "auto"), (3, "push"), (5, "auto"), (4, "auto")])
def test_full_size_properties(idx, mode):
    """BASELINE sizes (config 3: 2^24 peers; config 4: 2^28; config 5: 2^26
    with churn): checksum-of-state, conservation, push == pull, determinism."""
    w = config(idx)
    with _engine(w, mode=mode) as e:
        stats = run_engine(e, w)
        last = stats[-1]
        assert last["new_receipts"] == 0
        seen = e.read_seen()
        assert _digest(seen) == last["digest"]
        covered = int(np.bitwise_count(seen).sum())
        assert covered == last["covered"] == sum(s["new_receipts"] + s["injected"] for s in stats)
        assert int(e.coverage().sum()) == covered
        for s in stats:
            assert s["duplicates"] == s["deliveries"] - s["new_receipts"]
        if idx == 3:   # no churn: every message reaches its origin's whole component
            assert stats[0]["injected"] == 64
        else:
            alive = e.alive()
            assert int(alive.sum()) == w.n - sum(s["died"] for s in stats)
            reps = e.reports()
            assert len(reps) == sum(s["reports"] for s in stats)
            assert np.all(alive[reps[:, 2]] == 0)      # only dead peers are reported
            assert np.all(e.registered()[reps[:, 2]] == 0)
        e.reset()
        assert e.run() == stats


def test_push_equals_pull_at_full_size():
    """config 3 at its full 2^24 peers: the direction-optimised schedule, the
    gather-pull and binned schedules and the push-only schedule produce
    identical rounds and seen sets."""
    w = config(3)
    out = {}
    for mode in ("push", "auto", "pull", "bin"):
        with _engine(w, mode=mode) as e:
            out[mode] = (run_engine(e, w), e.read_seen())
    for mode in ("auto", "pull", "bin"):
        assert out["push"][0] == out[mode][0], mode
        assert np.array_equal(out["push"][1], out[mode][1]), mode


@pytest.mark.parametrize("n,cap", [(120, 4095), (300, 4095), (60, 1500), (50, 0)])
def test_f10_list_cap_parity(oracle, n, cap):
    """The F10 knob (list_cap): under the reference's 4 KB
    peer_list read, peers from the 77th on never start (registered, not
    alive); messages they would generate are never sent.  Engine == oracle on
    every round, with the config-1 kill and liveness schedule."""
    base = config(1)
    peers = np.array(sorted({0, 5, n // 3, 75 % n, 76 % n, n - 1}), dtype=np.uint32)
    o, r = _batches(peers, 10, 5)
    w = dataclasses.replace(base, n=n, n_msgs=int(o.size), origins=o, inject_rounds=r, list_cap=cap)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    started = oracle.started_under_cap(n, cap)
    assert int(ref["alive"][:started].sum()) >= started - 1 and not ref["alive"][started:].any()
    with _engine(w) as e:
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        e.reset()
        assert e.alive()[:started].all() and not e.alive()[started:].any()
        _compare(e, ref, w)


@pytest.mark.parametrize("idx,n,cap,mode", [(5, 1 << 14, 0, "auto"), (5, 1 << 14, 8, "auto"), (5, 50_000, 4, "push"),
                                            (5, 20_000, 0, "pull"), (1, None, 8, "auto"), (1, 40, 0, "auto")])
def test_rejoin_parity(oracle, idx, n, cap, mode):
    """Join churn (rejoin_threshold): restarted peers --
    re-registered, empty Message-List, dropped row, fresh out-edges in the
    overflow row -- bit-exact against the oracle, with and without
    re-bootstrap; digest and coverage lose the restarted peers' old words."""
    w = config(idx, n, pick=oracle.pick_origins, rebootstrap=cap)
    w = dataclasses.replace(w, rejoin_threshold=int((0.05 if idx == 5 else 0.3) * 2**32),
                            min_rounds=max(w.min_rounds, 30))
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    assert sum(s["rejoined"] for s in ref["stats"]) > 0
    with _engine(w, mode=mode) as e:
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        if w.kills:
            e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        e.reset()
        first = _compare(e, ref, w)
        cnt, ex = e.read_extra()
        if cap:
            assert np.array_equal(cnt, ref["extra_counts"])
            assert np.array_equal(ex, ref["extra_cols"])
        e.reset()
        assert e.run() == first


@pytest.mark.parametrize("idx,n,cap", [(5, 1 << 14, 4), (5, 50_000, 16), (1, None, 8), (1, 40, 3)])
def test_rebootstrap_parity(oracle, idx, n, cap):
    """Re-bootstrap after a death (handleDeadPeer
    peer.cpp:398-404): extra out-edges, their liveness and the pushes over
    them, bit-exact against the oracle."""
    w = config(idx, n, pick=oracle.pick_origins, rebootstrap=cap)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    with _engine(w) as e:
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        if w.kills:
            e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        e.reset()
        first = _compare(e, ref, w)
        cnt, ex = e.read_extra()
        assert np.array_equal(cnt, ref["extra_counts"])
        assert np.array_equal(ex, ref["extra_cols"])
        e.reset()
        assert e.run() == first


@pytest.mark.parametrize("max_missed,ping", [(3, 3), (1, 2), (2, 5)])
def test_closed_form_liveness_kills_and_hubs(oracle, max_missed, ping):
    """Closed-form liveness (single partition, symmetric overlay): the in-edges
    of a dead peer are visited through its own row at its max_missed-th ping
    round; hubs (heavy rows, chunked) and light peers killed at various
    rounds, with churn on top; bit-exact against the oracle's per-edge miss
    counters, and equal to the engine's own per-edge scan ("full_liveness")."""
    base = config(2, 1 << 14, pick=oracle.pick_origins)
    kills = [(0, 1), (1, 2), (5, 2), (100, 4), (7777, 0), (2, 6)]
    w = dataclasses.replace(base, kills=kills, ping_every=ping, max_missed=max_missed, min_rounds=24,
                            churn_threshold=int(0.01 * 2**32))
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    assert sum(s["reports"] for s in ref["stats"]) > 0
    runs = []
    for full in (0, 1):
        with _engine(w, tuning={"full_liveness": full}) as e:
            e.build_graph()
            e.inject(w.origins, w.inject_rounds)
            e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
            e.reset()
            runs.append(_compare(e, ref, w))
    assert runs[0] == runs[1]


def test_steps_right_after_build_graph(oracle):
    """create -> build_graph -> inject -> run with no explicit reset: the
    overlay install leaves the round-0 state (every peer alive, miss counters
    zero), so the run equals the oracle's."""
    w = config(5, 1 << 14, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    with _engine(w) as e:
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        _compare(e, ref, w)


@pytest.mark.parametrize("mode", ["auto", "push"])
def test_reload_overlay_with_kills(oracle, mode):
    """One ctx, the overlay loaded twice (a second load_csr after a run with
    deaths): the closed-form liveness state is rebuilt for the new overlay,
    so the ping rounds still mask and report exactly as the oracle does."""
    base = config(2, 1 << 13, pick=oracle.pick_origins)
    w = dataclasses.replace(base, kills=[(0, 1), (9, 2), (77, 3)], ping_every=2, max_missed=2, min_rounds=16,
                            churn_threshold=int(0.01 * 2**32))
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    assert sum(s["reports"] for s in ref["stats"]) > 0
    with _engine(w, mode=mode) as e:
        for _ in range(2):
            e.load_csr(rp, col)
            e.inject(w.origins, w.inject_rounds)
            e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
            _compare(e, ref, w)


_VARIANTS = {"defer_1": ({"defer_permille": 1}, {"blocked": "off"}), "stream": ({"bin_stream": 1}, {}),
             "slots": ({"bin_stream": 0}, {}), "no_first2": ({"pull_first2": 0}, {}),
             "no_flight": ({"in_flight": 0}, {}), "no_heavy_exit": ({"heavy_exit": 0}, {}),
             "small_bins": ({"bin_words": 4096, "bin_chunk": 2048}, {}), "apply_src": ({"src_stats": 0}, {}),
             "heavy_64": ({"heavy_degree": 64, "heavy_chunk": 128}, {}), "all_pull": ({}, {"bin_permille": 100000}),
             "blocked_wide": ({}, {"blocked_permille": 1000}), "pull_step_2": ({"pull_step": 2}, {}),
             "no_lists": ({"list_rounds": 0}, {}), "needy_test": ({"bin_needy_skip": 0}, {}),
             "stream_needy_test": ({"bin_stream": 1, "bin_needy_skip": 0}, {}),
             "apply_pipe_1": ({"apply_pipe": 1}, {}), "apply_pipe_2": ({"apply_pipe": 2}, {}),
             "apply_pipe_3": ({"apply_pipe": 3}, {}), "heavy_after_apply": ({"heavy_side": 0}, {}),
             # whole bins (the pipeline shapes only apply to them; overlays of <= 2^20 peers default to small bins)
             "whole_bins_pipe_2": ({"bin_words": 18432, "apply_pipe": 2}, {}),
             "whole_bins_pipe_4": ({"bin_words": 18432, "apply_pipe": 4}, {}),
             "whole_bins_pipe_5": ({"bin_words": 18432, "apply_pipe": 5}, {}),
             "whole_bins_pipe_6": ({"bin_words": 18432, "apply_pipe": 6}, {}),
             "whole_bins_pipe_7": ({"bin_words": 18432, "apply_pipe": 7}, {}),
             "whole_bins_pipe_8": ({"bin_words": 18432, "apply_pipe": 8}, {}),
             "whole_bins_pipe_9": ({"bin_words": 18432, "apply_pipe": 9}, {}),
             "whole_bins_pipe_10": ({"bin_words": 18432, "apply_pipe": 10}, {}),
             "half_bins": ({"bin_words": 9216}, {}),
             "zero_fill": ({"zero_fill": 1}, {}),
             "scatter_small": ({"scatter_small": 1}, {}),
             "small_kernels": ({"bin_words": 1024, "bin_chunk": 1024, "scatter_small": 1}, {}),
             "split_units": ({"scatter_units": 4096}, {}),
             "split_units_direct": ({"scatter_units": 4096, "scatter_split_direct": 1, "scatter_small": 1}, {}),
             "apply_wide": ({"bin_words": 2048, "apply_wide": 1}, {}),
             "apply_probe": ({"apply_probe": 1}, {}), "apply_one_per_bin": ({"apply_persist": 0}, {}), "slots_needy_test": ({"bin_stream": 0, "bin_needy_skip": 0}, {}),
             "blocked_dense": ({"blocked_bin_slots": 0}, {"blocked_permille": 1000}),
             "blocked_dense_pipe": ({"blocked_bin_slots": 0, "blocked_pipe": 1}, {"blocked_permille": 1000}),
             "blocked_unpiped": ({"blocked_pipe": 0}, {"blocked_permille": 1000}),
             "blocked_wide_pipe": ({"blocked_pipe": 1}, {"blocked_permille": 1000}),
             "blocked_dense_clear_peers": ({"blocked_bin_slots": 0, "blocked_clear_all": 0}, {"blocked_permille": 1000})}


@pytest.mark.parametrize("variant", sorted(_VARIANTS))
@pytest.mark.parametrize("idx,n,mode", [(2, 1 << 16, "auto"), (3, 1 << 18, "bin"), (5, 50_000, "auto"),
                                        (5, 1 << 16, "push"), (3, 1 << 18, "pull")])
def test_engine_variants_match_oracle(oracle, variant, idx, n, mode):
    """The A/B variants the engine keeps as explicit options (gossip_set_tuning,
    never the environment): the deferred seen update of wide push rounds, both
    binned layouts, the row pull's first-two-entries and in-flight tests, the
    heavy-row early exit and threshold, bin and chunk sizes, who books a binned
    round's source side, and the schedule switches -- all give the oracle's
    results."""
    tuning, kw = _VARIANTS[variant]
    w = config(idx, n, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    with _engine(w, mode=mode, tuning=tuning, **kw) as e:
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        if w.kills:
            e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        e.reset()
        _compare(e, ref, w)


def test_apply_probe_toggle(oracle):
    """apply_probe turned on, then off again, between runs of a streamed binned
    workload: the persistent apply's bin counters must survive the toggle (the
    probe-off branch once freed them and left the pointer dangling, so the next
    binned round took bins from freed memory)."""
    w = config(3, 1 << 18, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    with _engine(w, mode="bin") as e:
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        for probe in (1, 0, 1, 0):
            e.set_tuning("apply_probe", probe)
            e.reset()
            _compare(e, ref, w)


@pytest.mark.parametrize("variant", ["auto", "defer_10", "all_pull", "defer_10_all_pull", "defer_10_blocked",
                                     "defer_3_blocked"])
@pytest.mark.parametrize("stop", [3, 4, 5, 6, 7, 8])
def test_deferred_round_fold(oracle, variant, stop):
    """With blocked push rounds off, auto mode defers the seen update of the wide
    push round before the binned rounds (config 3 shape: round 2 here) and leaves
    the fold to the next round's apply or row-pull sweep.  A run stopped by
    max_rounds right after a deferred round, or after the fused fold, must still
    read the oracle's seen set and coverage; the explicit option forces the
    deferral (committed when the fold cannot be fused), and a huge binned
    threshold turns the binned rounds into pulls (push -> pull folds).  With
    blocked rounds on and the dense rounds blocked at this size
    (blocked_bin_slots 0), the fold rides on the blocked round's level-1
    sweep, whose hub deliveries test against seen | nw."""
    tuning = {}
    if "defer_10" in variant:
        tuning["defer_permille"] = 10
    if "defer_3" in variant:
        tuning["defer_permille"] = 3
    if "blocked" in variant:  # defer_3: hub tiles (in-degree > 1024) take direct deliveries
        tuning["blocked_bin_slots"] = 0
        tuning["blocked_direct_in"] = 1024 if "defer_3" in variant else -1
    kw = {"bin_permille": 100000} if "all_pull" in variant else {}
    w = config(3, 1 << 18, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col, max_rounds=stop)
    blocked = "auto" if "blocked" in variant else "off"
    with Engine(w.n, w.n_msgs, max_rounds=stop, blocked=blocked, tuning=tuning, **kw, **w.engine_kwargs()) as e:
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        e.reset()
        got = e.run()
        assert got == ref["stats"]
        assert np.array_equal(e.read_seen(), ref["seen"])
        assert np.array_equal(e.coverage(), ref["coverage"])


@pytest.mark.parametrize("variant", ["on", "off", "cap_small", "stop"])
@pytest.mark.parametrize("idx,n", [(2, 1 << 18), (3, 1 << 18), (3, 1 << 20), (2, 50_000)])
def test_needy_list_rounds(oracle, idx, n, variant):
    """Late pull rounds over needy lists (k_pull_list): the row pull after the
    dense rounds books the next round's source side at activation and lists
    the rows that still lack a bit; the rounds after it pull only those rows.
    Against the oracle's per-round stats, seen sets and coverage: on (the
    default), off, a list capacity of 64 (the lists overflow: the next round
    sweeps as a row pull whose source side is already booked), and runs cut by
    max_rounds inside the list chain (a reset clears the booking)."""
    tuning = {"list_rounds": 0} if variant == "off" else {"list_cap": 64} if variant == "cap_small" else {}
    w = config(idx, n, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    stops = [None] if variant != "stop" else [7, 8, 9, 10]
    with _engine(w, tuning=tuning) as e:
        e.enable_timing(True)
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        if w.kills:
            e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        for stop in stops:
            ref = oracle.simulate_workload(w, rp, col, **({"max_rounds": stop} if stop else {}))
            e.reset()
            got = []
            while True:
                st, fin = e.step()
                got.append(st)
                if fin or (stop and len(got) >= stop):
                    break
            assert got == ref["stats"][:len(got)]
            if stop is None:
                assert len(got) == len(ref["stats"])
                assert np.array_equal(e.read_seen(), ref["seen"])
                assert np.array_equal(e.coverage(), ref["coverage"])
        if variant == "on" and not w.kills:
            assert e.kernel_time("pull_list")[1] > 0  # the list rounds ran


@pytest.mark.parametrize("tiny", ["1", "0"])
@pytest.mark.parametrize("idx,n,max_rounds", [(1, None, 0), (1, 40, 0), (1, 40, 20), (2, 4096, 0), (3, 2048, 0),
                                               (5, 4096, 0), (5, 6000, 7), (5, 6000, 0)])
def test_small_overlay_one_launch_matches_oracle(oracle, tiny, idx, n, max_rounds):
    """Small overlays (<= 65,536 peers and edges) run whole in one launch
    (gossip_tiny.hip: kills, churn, liveness with reports and registry,
    injection, push, stats and termination on the device); the option runs
    them round by round ("tiny" = 0).  Both give the oracle's every round, seen set,
    coverage, reports, alive flags and registry, also when max_rounds cuts the
    run short; a second run from reset repeats the first."""
    w = config(idx, n, pick=oracle.pick_origins)
    kw = {"max_rounds": max_rounds} if max_rounds else {}
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col, **kw)
    with _engine(w, tuning={"tiny": int(tiny)}, **kw) as e:
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        if w.kills:
            e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        for _ in range(2):
            e.reset()
            _compare(e, ref, w)


def test_heavy_degree_is_a_layout_key(oracle):
    """"heavy_degree" set after the overlay is built takes effect only at the
    next build: the resident chunk list, bins and blocked segments keep the
    threshold they were laid out with (a row between the two thresholds
    would otherwise be skipped by the light kernels and covered by no chunk,
    losing its deliveries).  Then a rebuild applies it."""
    w = config(3, 1 << 18, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    with _engine(w) as e:
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        e.set_tuning("heavy_degree", 16)  # held back: the layout was built with 256
        e.reset()
        _compare(e, ref, w)
        e.build_graph()  # now rows > 16 are chunked
        e.reset()
        _compare(e, ref, w)


def test_list_cap_change_inside_a_list_chain(oracle):
    """"list_cap" changed while needy-list rounds are running must not
    reallocate the lists in flight (the next rounds read them and clear nx by
    them): the change waits for the next chain, and results stay the oracle's."""
    w = config(3, 1 << 18, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    with _engine(w) as e:
        e.enable_timing(True)
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        for rerun in range(2):
            e.reset()
            got, changed = [], False
            while True:
                st, fin = e.step()
                got.append(st)
                if not changed and e.kernel_time("pull_list")[1] > 0:
                    e.set_tuning("list_cap", 1 << 20 if rerun == 0 else 128)
                    changed = True
                if fin:
                    break
            assert changed
            assert got == ref["stats"]
            assert np.array_equal(e.read_seen(), ref["seen"])


def test_tuning_rejects_bad_values_and_huge_max_rounds_runs(oracle):
    """"pull_step" takes 1 or 2 only; a small overlay with a "no limit"
    max_rounds runs round by round instead of sizing the one-launch run's
    stats buffer by it, with the oracle's results."""
    from gossip_hip._abi import GossipError
    w = config(2, 4096, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    kw = w.engine_kwargs()
    kw["max_rounds"] = 1 << 30
    with Engine(w.n, w.n_msgs, **kw) as e:
        for bad in (0, -1, 3):
            with pytest.raises(GossipError):
                e.set_tuning("pull_step", bad)
        e.set_tuning("pull_step", 2)
        e.enable_timing(True)
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        e.reset()
        _compare(e, ref, w)
        assert e.kernel_time("tiny")[1] == 0


@pytest.mark.parametrize("idx,n", [(2, 1 << 18), (3, 1 << 18), (5, 1 << 16), (4, 1 << 18)])
def test_recorded_schedule_replay(oracle, idx, n):
    """gossip_run records the first run's per-round stats; a rerun from reset
    of the same inputs issues every round without waiting for its stats and
    checks the device's stats against the recording at the end.  Both runs
    give the oracle's results; a changed option drops the recording (the next
    run records again), and "replay" 0 never replays."""
    w = config(idx, n, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    with _engine(w) as e:
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        if w.kills:
            e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        for i in range(3):
            e.reset()
            _compare(e, ref, w)
            assert e.kernel_bytes("#replayed_runs") == i  # run 0 records, runs 1 and 2 replay
        e.set_tuning("pull_step", 2)  # drops the recording
        e.reset()
        _compare(e, ref, w)
        assert e.kernel_bytes("#replayed_runs") == 2
        e.reset()
        _compare(e, ref, w)
        assert e.kernel_bytes("#replayed_runs") == 3
        e.set_tuning("replay", 0)
        for _ in range(2):
            e.reset()
            _compare(e, ref, w)
        assert e.kernel_bytes("#replayed_runs") == 3
        # bench's timed steps: the run's stats left in a buffer kept across calls, read afterwards
        e.set_tuning("replay", 1)
        for _ in range(3):
            e.reset()
            assert e.run_into() == len(ref["stats"])
            assert e.last_stats() == ref["stats"]
        assert np.array_equal(e.read_seen(), ref["seen"])
