"""Partitioned engine on one GPU: P vertex blocks (one gossip_ctx each) in
one process, the all-to-all done by device copies.  Exercises the remote
staging (push) and apply_remote kernels and the partitioned overlay
generator against the single-partition oracle run (P-invariance)."""
import numpy as np
import pytest

from gossip_hip import Engine
from gossip_hip._abi import STAT_FIELDS
from gossip_hip.distributed import MASK64, partition
from gossip_hip.workloads import config

pytestmark = pytest.mark.gpu


def run_partitioned(w, P, pull=True, sparse=False, binned=False):
    """Mirror of gossip_hip.distributed.PartitionedRun with the collectives done
    by device copies: all-gather for pull rounds, all-to-all for push rounds."""
    import torch
    part = partition(w.n, P)
    chunk = part[1]
    engines = [Engine(w.n, w.n_msgs, part=(part[p], part[p + 1]), device=0, **w.engine_kwargs()) for p in range(P)]
    stream = torch.cuda.current_stream().cuda_stream
    for e in engines:
        e.build_graph()
        e.inject(w.origins, w.inject_rounds)
        if w.kills:
            e.schedule_kills([k[0] for k in w.kills], [k[1] for k in w.kills])
        e.reset()
        e.set_stream(stream)
    X = engines[0].shape()["exchange_words"]
    nl = [part[p + 1] - part[p] for p in range(P)]
    sends = [torch.zeros(w.n * X, dtype=torch.int64, device="cuda") for _ in range(P)]
    recvs = [torch.zeros(P * nl[q] * X, dtype=torch.int64, device="cuda") for q in range(P)]
    gathers = [torch.zeros(P * chunk * X, dtype=torch.int64, device="cuda") for _ in range(P)]
    R = 1 + X
    segs = [torch.zeros(P * chunk * R, dtype=torch.int64, device="cuda") for _ in range(P)]
    rec_in = [torch.zeros(P * nl[q] * R, dtype=torch.int64, device="cuda") for q in range(P)]
    for p, e in enumerate(engines):
        e.set_exchange(sends[p].data_ptr(), recvs[p].data_ptr(), part)
        e.set_gather(gathers[p].data_ptr())
        e.set_sparse(segs[p].data_ptr())
    rounds, modes, dig, cov, prev_new = [], [], 0, 0, 0
    while True:
        want = (3 if binned else 1) if pull and prev_new * 1000 >= 50 * w.n else (2 if sparse else 0)
        got = {e.round_begin(want) for e in engines}
        assert len(got) == 1
        mode = got.pop()
        modes.append(mode)
        if mode in (1, 3):   # all-gather of every block's new words
            for q in range(P):
                for p in range(P):
                    gathers[q][p * chunk * X:(p + 1) * chunk * X].copy_(gathers[p][p * chunk * X:(p + 1) * chunk * X])
        for e in engines:
            e.round_compute()
        if mode == 0:   # all-to-all of the remote masks
            for q in range(P):
                for p in range(P):
                    recvs[q][p * nl[q] * X:(p + 1) * nl[q] * X].copy_(sends[p][part[q] * X:part[q + 1] * X])
        if mode == 2:   # counts, then the records of every sender, in sender order
            counts = [e.sparse_counts(P) for e in engines]
            loc = []
            for q, e in enumerate(engines):
                off = 0
                for p in range(P):
                    c = int(counts[p][q])
                    rec_in[q][off * R:(off + c) * R].copy_(segs[p][q * chunk * R:(q * chunk + c) * R])
                    off += c
                loc.append(e.round_finish_sparse(rec_in[q].data_ptr(), off))
            assert all(not torch.any(sd) for sd in sends)   # compaction left the staging buffers clear
        else:
            loc = [e.round_finish() for e in engines]
        g = {f: sum(l[f] for l in loc) for f in STAT_FIELDS}
        dig = (dig + g["digest"]) & MASK64
        cov += g["covered"]
        g.update(round=loc[0]["round"], flags=loc[0]["flags"], digest=dig, covered=cov,
                 duplicates=g["deliveries"] - g["new_receipts"])
        prev_new = g["new_receipts"]
        fins = {e.round_commit(g["new_receipts"]) for e in engines}
        assert len(fins) == 1
        rounds.append(g)
        if fins.pop():
            break
    reps = np.concatenate([e.reports() for e in engines])
    reps = np.array(sorted(map(tuple, reps.tolist())), dtype=np.uint32).reshape(-1, 3)
    first = {}
    for r, _, v in reps.tolist():
        first.setdefault(v, r)
    for st in rounds:
        st["seed_removals"] = sum(1 for r in first.values() if r == st["round"])
    seen = np.concatenate([e.read_seen() for e in engines])
    csrs = [e.read_csr() for e in engines]
    for e in engines:
        e.close()
    return rounds, seen, reps, csrs, part, modes


@pytest.mark.parametrize("pull,sparse,binned", [(True, True, False), (True, False, False), (False, True, False),
                                               (True, True, True)])
@pytest.mark.parametrize("P", [2, 3, 4])
@pytest.mark.parametrize("idx,n", [(2, 1 << 15), (3, 100_000), (5, 1 << 15)])
def test_partitioned_gpu_equals_oracle(oracle, idx, n, P, pull, sparse, binned):
    w = config(idx, n, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    rounds, seen, reps, csrs, part, modes = run_partitioned(w, P, pull, sparse, binned)
    if pull and idx != 5:
        assert (3 if binned else 1) in modes
    if sparse:
        assert 2 in modes
    for p, (lrp, lcol) in enumerate(csrs):   # partitioned generator = slices of the global overlay
        base = int(rp[part[p]])
        assert np.array_equal(lrp, rp[part[p]:part[p + 1] + 1] - np.uint64(base))
        assert np.array_equal(lcol & np.uint32(0x7FFFFFFF), col[base:int(rp[part[p + 1]])])
    assert rounds == ref["stats"]
    assert np.array_equal(seen, ref["seen"])
    assert np.array_equal(reps, ref["reports"])


@pytest.mark.parametrize("P", [2, 3])
def test_partitioned_rebootstrap_equals_oracle(oracle, P):
    """Re-bootstrap is per reporter, so a vertex-partitioned run adds the same
    edges as the single-partition oracle."""
    w = config(5, 1 << 15, pick=oracle.pick_origins, rebootstrap=8)
    rp, col = oracle.gen_workload(w)
    ref = oracle.simulate_workload(w, rp, col)
    rounds, seen, reps, csrs, part, modes = run_partitioned(w, P, True, True)
    assert rounds == ref["stats"]
    assert np.array_equal(seen, ref["seen"])
    assert np.array_equal(reps, ref["reports"])
    assert sum(r["reconnects"] for r in rounds) > 0
