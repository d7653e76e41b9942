"""Library-driven multi-GPU rounds (gossip_dist.hip, RCCL inside
libgossip_hip) against the single-partition oracle run -- the partitioned
run must be bit-exact (P-invariance).

On one GPU: a group of P parts on the same device exchanges by device copies
(the C++ driver's schedule, the remote staging / record compaction /
remote-apply kernels and the report merge); a one-part group on device 0
(ncclCommInitAll) and an Engine joined with gossip_comm_init at world 1
(ncclCommInitRank) run the real RCCL calls (all-gather, send/recv all-to-all,
all-reduce, report all-gather)."""
import numpy as np
import pytest

from gossip_hip import Engine, Group, comm_unique_id, partition
from gossip_hip.workloads import config

pytestmark = pytest.mark.gpu


def _run_group(w, devices, **kw):
    with Group(w.n, w.n_msgs, devices, **w.engine_kwargs(), **kw) as g:
        g.build_graph()
        g.inject(w.origins, w.inject_rounds)
        if w.kills:
            g.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        g.reset()
        stats = g.run()
        seen, reps = g.read_seen(), g.reports()
        g.reset()
        again = g.run()
    return stats, seen, reps, again


@pytest.mark.parametrize("P", [2, 3, 4])
@pytest.mark.parametrize("idx,n", [(2, 1 << 15), (3, 100_000), (5, 1 << 15)])
def test_group_on_one_device_equals_oracle(oracle, idx, n, P):
    w = config(idx, n, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    stats, seen, reps, again = _run_group(w, [0] * P)
    assert stats == ref["stats"]
    assert np.array_equal(seen, ref["seen"])
    assert np.array_equal(reps, ref["reports"])
    assert again == stats


@pytest.mark.parametrize("gather", ["compact", "whole", "whole_1_stage", "whole_3_stages", "direct"])
@pytest.mark.parametrize("P", [2, 3, 5])
@pytest.mark.parametrize("idx,n", [(3, 100_003), (5, 1 << 15), (2, 40_000)])
def test_group_dense_exchange_forms_equal_oracle(oracle, idx, n, P, gather):
    """Dense rounds at P > 1 exchange either every block's whole slice of new
    words or, forced here for every dense round, the blocks' tile bitmaps and
    packed non-zero words (gossip_dist.hip compact_gather: bitmap all-gather,
    offsets from the tiles' popcount prefix, packed words as send / recv
    pairs, expansion into the gather buffer) -- on blocks that do not end on a
    tile boundary (n = 100,003) and a short last block (P = 3, 5).  Both forms
    give the oracle's run, as does the scatter reading other blocks' words
    straight from the gather buffer ("direct": scatter_direct).  A binned
    round's whole-slice exchange goes out in stages of source segments, the
    scatter of each stage's chunks waiting for its event (4 by default; 1 =
    one piece; 3 does not divide the 64 segments evenly)."""
    w = config(idx, n, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    tuning = {"gather_permille": 0 if gather.startswith("whole") else 1000}
    if gather == "whole_1_stage":
        tuning["exchange_stages"] = 1
    if gather == "whole_3_stages":
        tuning["exchange_stages"] = 3
    if gather == "direct":
        tuning["scatter_direct"] = 1
    stats, seen, reps, again = _run_group(w, [0] * P, tuning=tuning)
    assert stats == ref["stats"]
    assert np.array_equal(seen, ref["seen"])
    assert np.array_equal(reps, ref["reports"])
    assert again == stats


@pytest.mark.parametrize("px", ["all", "off", "append"])
@pytest.mark.parametrize("P", [2, 3, 4])
@pytest.mark.parametrize("idx,n", [(3, 100_003), (5, 1 << 15), (2, 40_000)])
def test_group_record_push_equals_oracle(oracle, idx, n, P, px):
    """Sparse push rounds at P > 1 as records per destination block
    (gossip_blocked.hip build_px / k_px_pack: level 1 of a blocked round with
    the destination blocks as its bins, the own block delivered at once, the
    records packed per block and exchanged as {peer, word}) -- forced for
    every sparse round ("all": px_permille 0), the push appending its remote
    deliveries as records itself, one counter atomic per wave and destination
    ("append": every sparse round under the record push's frontier), and the
    staging push with its compaction ("off") -- all give the oracle's run,
    with dead peers and masked edges (config 5) and short last blocks."""
    w = config(idx, n, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    pm = {"all": 0, "off": -1, "append": 1 << 30}[px]
    stats, seen, reps, again = _run_group(w, [0] * P, tuning={"px_permille": pm})
    assert stats == ref["stats"]
    assert np.array_equal(seen, ref["seen"])
    assert np.array_equal(reps, ref["reports"])
    assert again == stats


@pytest.mark.parametrize("idx,n", [(2, 1 << 15), (5, 1 << 15)])
def test_group_one_part_rccl_equals_oracle(oracle, idx, n):
    """ncclCommInitAll over device 0: every collective of the driver through RCCL."""
    w = config(idx, n, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    stats, seen, reps, again = _run_group(w, [0])
    assert stats == ref["stats"]
    assert np.array_equal(seen, ref["seen"])
    assert np.array_equal(reps, ref["reports"])


@pytest.mark.parametrize("idx,n", [(3, 1 << 16), (5, 1 << 15)])
def test_comm_init_world1_equals_oracle(oracle, idx, n):
    """One process per GPU path (bench --gpus N): ncclCommInitRank at world 1,
    gossip_run issuing the collectives, gossip_comm_finalize gathering reports."""
    w = config(idx, n, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    part = partition(w.n, 1)
    with Engine(w.n, w.n_msgs, part=(part[0], part[1]), **w.engine_kwargs()) as e:
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        e.comm_init(comm_unique_id(), 1, 0)
        e.reset()
        stats = e.run()
        reps = e.comm_finalize(stats)
        modes = e.comm_modes()
        assert stats == ref["stats"]
        assert np.array_equal(e.read_seen(), ref["seen"])
        assert np.array_equal(reps, ref["reports"])
        assert len(modes) == len(stats)


def test_group_rejects_mixed_devices():
    from gossip_hip import GossipError
    with pytest.raises(GossipError):
        Group(1 << 12, 64, [0, 0, 1])


def test_group_run_into_keeps_stats_in_a_reused_buffer(oracle):
    """Group.run_into (bench's timed steps): gossip_group_run into a buffer kept
    across calls, the per-round stats read after the run -- the oracle's rounds,
    run after run."""
    w = config(2, 1 << 15, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    with Group(w.n, w.n_msgs, [0, 0], **w.engine_kwargs()) as g:
        g.build_graph()
        g.inject(w.origins, w.inject_rounds)
        for _ in range(2):
            g.reset()
            assert g.run_into() == len(ref["stats"])
            assert g.last_stats() == ref["stats"]
        assert np.array_equal(g.read_seen(), ref["seen"])


def _ref_bootstrap_workload(n):
    """The literal bootstrap overlay (config 1's model, n <= 4096) at n peers: 64 messages from peers spread over
    the ids at round 0, peer 3 killed at round 12, pings every 15 rounds -- config 1 sends 10 messages per peer,
    more than 512 at n > 51."""
    from dataclasses import replace
    w = config(1, 8)
    o = (np.arange(64, dtype=np.uint32) * (n // 64)).astype(np.uint32)
    return replace(w, n=n, n_msgs=64, origins=o, inject_rounds=np.zeros(64, dtype=np.uint32),
                   name=f"ref_bootstrap_{n}")


@pytest.mark.parametrize("n,P", [(4000, 2), (1001, 3)])
def test_group_ref_bootstrap_blocks_round_up_to_tiles(oracle, n, P):
    """gossip_group_create on an overlay other than powerlaw cuts ceil(n/P) blocks rounded up to whole 64-peer
    tiles (gossip_group_create_parts takes only tile-aligned blocks; round 5 returned EINVAL here):
    the literal bootstrap DAG at a peer count off a tile boundary gives the oracle's run."""
    import ctypes as C
    w = _ref_bootstrap_workload(n)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    rp = np.asarray(rp, dtype=np.uint64)
    col = np.asarray(col, dtype=np.uint32)
    with Group(w.n, w.n_msgs, [0] * P, **w.engine_kwargs()) as g:
        # the literal DAG is generated single-partition only: each block loads its rows (gossip_load_csr)
        b = [0]
        for p in range(P):
            b.append(b[-1] + g.shape(p)["n_local"])
        assert all(x % 64 == 0 for x in b[:-1]) and b[-1] == n
        for p in range(P):
            lrp = np.ascontiguousarray(rp[b[p]:b[p + 1] + 1] - rp[b[p]])
            lcol = np.ascontiguousarray(col[rp[b[p]]:rp[b[p + 1]]])
            st = g._L.gossip_load_csr(g.part_ctx(p), lrp.ctypes.data_as(C.POINTER(C.c_uint64)),
                                      lcol.ctypes.data_as(C.POINTER(C.c_uint32)), lrp.size - 1, int(lrp[-1]))
            assert st == 0, g._L.gossip_last_error().decode()
        g.inject(w.origins, w.inject_rounds)
        g.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        g.reset()
        stats = g.run()
        assert stats == ref["stats"]
        assert np.array_equal(g.read_seen(), ref["seen"])
        assert np.array_equal(g.reports(), ref["reports"])


def test_group_uniform_partition_rounds_up_to_tiles(oracle):
    """GOSSIP_FLAG_UNIFORM_PARTITION with ceil(n/P) off a tile (100,003 / 3 = 33,335): tile-aligned blocks, the
    oracle's run."""
    w = config(3, 100_003, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    stats, seen, reps, again = _run_group(w, [0] * 3, uniform_partition=True)
    assert stats == ref["stats"]
    assert np.array_equal(seen, ref["seen"])
    assert again == stats


def test_group_too_small_for_whole_tiles_is_einval():
    from gossip_hip import GossipError
    with pytest.raises(GossipError, match="64-peer tiles"):
        Group(100, 64, [0, 0, 0], graph="ref_bootstrap")  # 64-peer blocks: [0, 64, 100, 100]
