"""gossip_partition_edges (host code of libgossip_hip, no GPU): blocks of
about equal work for the powerlaw overlay -- contiguous, whole 64-peer tiles,
covering [0, n) -- checked against the oracle's own overlay: every block's
edges plus 2 edge-equivalents per peer within a few per cent of the mean,
where blocks of ceil(n/P) peers put 2.5x the mean edges on the first one."""
import numpy as np
import pytest

from gossip_hip import partition, partition_edges
from gossip_hip.workloads import config


@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
def test_blocks_are_contiguous_tiles(P):
    n = 1 << 20
    b = partition_edges(n, 64, P)
    assert b[0] == 0 and b[-1] == n and len(b) == P + 1
    assert all(b[q + 1] > b[q] for q in range(P))
    assert all(x % 64 == 0 for x in b[:-1])


@pytest.mark.parametrize("n,P", [(191, 2), (200, 3), (1000, 8), (4097, 4), (1 << 14 | 5, 8)])
def test_small_blocks_off_a_tile_stay_whole_tiles(n, P):
    """n % 64 != 0: the room kept for the blocks after a boundary is a whole number of tiles too (round 5
    capped a boundary at n - 64 (P - q), off a tile -- [0, 127, 191] -- which gossip_group_create_parts rejects)."""
    b = partition_edges(n, 64, P)
    assert b[0] == 0 and b[-1] == n and all(b[q + 1] > b[q] for q in range(P))
    if n >= 64 * P:
        assert all(x % 64 == 0 for x in b[:-1]), b


def test_other_overlays_and_tiny_ones_get_uniform_blocks():
    assert partition_edges(4096, 64, 4, graph="ref_bootstrap") == partition(4096, 4)
    assert partition_edges(100, 64, 3) == partition(100, 3)  # fewer than 64 peers per block


@pytest.mark.parametrize("P", [2, 4, 8])
def test_blocks_balance_the_oracles_overlay(oracle, P):
    w = config(4, 1 << 20, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    rp = np.asarray(rp, dtype=np.int64)

    def costs(b):
        return np.array([rp[b[q + 1]] - rp[b[q]] + 2 * (b[q + 1] - b[q]) for q in range(P)], dtype=np.float64)

    bal = costs(partition_edges(w.n, w.n_msgs, P, **w.engine_kwargs()))
    uni = costs(partition(w.n, P))
    assert bal.max() / bal.mean() < 1.05
    assert uni.max() / uni.mean() > 1.2  # what the uniform blocks did


@pytest.mark.parametrize("begins", [[1, 64, 128], [0, 64, 100], [0, 100, 128], [0, 64, 64, 128]])
def test_group_create_parts_rejects_bad_blocks(begins):
    """gossip_group_create_parts checks the caller's partition before touching a device: blocks must cover
    [0, n_peers), be non-empty and start on whole 64-peer tiles."""
    from gossip_hip import Group
    from gossip_hip._abi import GossipError
    with pytest.raises(GossipError, match="part"):
        Group(128, 64, [0] * (len(begins) - 1), begins=begins)
