"""bench.py's host-side accounting on CPU, with a scripted stand-in for the
engine: SURVEY 8(d)'s per-round bytes (32 B per frontier peer, 20 B per
traversal, plus the liveness term of a ping round), the round's mode from the
kernels that ran, and how per-part device times combine -- the max over the
parts when each has its own GPU, the sum when P parts share one GPU."""
import importlib.util
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", REPO / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules["bench_under_test"] = mod
    spec.loader.exec_module(mod)
    return mod


class FakeRun:
    """Rounds scripted as (stats, {part: {kernel: ms}}, {counter: value}); ktime/kbytes are cumulative."""

    def __init__(self, parts, n_gpus, rounds):
        self.parts, self.n_gpus, self.rounds = parts, n_gpus, rounds
        self.i = 0
        self.t = [dict() for _ in range(parts)]
        self.b = [dict() for _ in range(parts)]

    def reset(self):
        self.i = 0

    def timing(self, on):
        pass

    def ktime(self, p, k):
        return (self.t[p].get(k, 0.0), 1)

    def kbytes(self, p, k):
        return self.b[p].get(k, 0.0)

    def round_step(self):
        st, times, counters = self.rounds[self.i]
        for p in range(self.parts):
            for k, v in times.get(p, {}).items():
                self.t[p][k] = self.t[p].get(k, 0.0) + v
            for k, v in counters.get(p, {}).items():
                self.b[p][k] = self.b[p].get(k, 0.0) + v
        self.i += 1
        return st, self.i == len(self.rounds)


def _rounds(parts):
    return [
        ({"round": 0, "frontier": 10, "traversals": 100},
         {p: {"push_light": 0.5, "push_heavy": 0.25} for p in range(parts)}, {}),
        ({"round": 1, "frontier": 1000, "traversals": 50_000},
         {p: {"bin_scatter": 1.0, "bin_apply": 2.0, "pull_heavy": 0.5 + p, "all_gather": 0.25} for p in range(parts)},
         {p: {"#pings": 800.0, "#pinging_peers": 100.0, "bin_scatter": 1e7} for p in range(parts)}),
        ({"round": 2, "frontier": 900, "traversals": 40_000},
         {p: {"pull_light": 3.0} for p in range(parts)}, {}),
    ]


@pytest.mark.parametrize("parts,n_gpus", [(1, 1), (4, 4), (4, 1)])
def test_per_round_profile_bytes_modes_and_part_times(parts, n_gpus):
    b = _bench()
    rows = b.per_round_profile(FakeRun(parts, n_gpus, _rounds(parts)), n_peers=10_000)
    assert [r["mode"] for r in rows] == ["push", "bin", "pull"]
    assert [r["work_avoiding"] for r in rows] == [False, False, True]
    # 8(d): 32 B per frontier peer + 20 B per traversal; the ping round adds 6.125 B per ping and 16 B per
    # pinging peer, summed over the parts
    live = parts * (6.125 * 800 + 16 * 100)
    assert rows[0]["alg_bytes"] == 32 * 10 + 20 * 100
    assert rows[1]["alg_bytes"] == round(32 * 1000 + 20 * 50_000 + live)
    assert rows[1]["liveness_bytes"] == round(live)
    assert rows[1]["design_bytes"] == parts * 1e7
    # device time: max over the parts on their own GPUs, their sum when they share one
    per_part = [1.0 + 2.0 + 0.5 + p for p in range(parts)]
    want = max(per_part) if parts == n_gpus else sum(per_part)
    assert rows[1]["kernel_ms"] == pytest.approx(want)
    assert rows[1]["exchange_ms"] == pytest.approx(0.25 if parts == n_gpus else 0.25 * parts)
    assert rows[1]["dense_ms"] == pytest.approx(want)
    frac = rows[1]["alg_bytes"] / (want / 1e3) / 1e9 / b.HBM_PEAK_GBS
    assert rows[1]["frac"] == pytest.approx(frac, abs=1e-4)


def test_part_agg():
    b = _bench()
    assert b.part_agg(FakeRun(1, 1, [])) is max
    assert b.part_agg(FakeRun(8, 8, [])) is max
    assert b.part_agg(FakeRun(8, 1, [])) is sum


def test_liveness_round_is_flagged():
    """A ping round whose kernels move fewer bytes than 8(d)'s liveness term
    charges (the closed-form liveness walks only the dying peers' rows) is
    marked work_avoiding ("liveness"); a binned ping round whose design bytes
    exceed its 8(d) bytes is not."""
    b = _bench()
    rounds = _rounds(1) + [
        ({"round": 3, "frontier": 10, "traversals": 100},
         {0: {"push_light": 0.01, "liveness": 0.01}}, {0: {"#pings": 1e9, "#pinging_peers": 1e8, "push_light": 2320.0}}),
    ]
    rows = b.per_round_profile(FakeRun(1, 1, rounds), n_peers=10_000)
    assert [r["avoided"] for r in rows] == [None, None, "pull", "liveness"]
    assert rows[3]["work_avoiding"] and rows[3]["frac"] > 1


def test_link_projection():
    """exchange_link_ms: the bytes the busiest rank receives per step over its
    P - 1 links; the projected P-GPU step adds it to the slowest part's kernels."""
    from gossip_hip.engine import EXCHANGES, KERNELS
    b = _bench()
    run = FakeRun(4, 1, [])
    k_ms = [{k: (0.0, 0) for k in KERNELS + EXCHANGES} for _ in range(4)]
    k_b = [{k: 0.0 for k in KERNELS + EXCHANGES} for _ in range(4)]
    for p in range(4):
        k_ms[p]["bin_scatter"] = (2.0 * (p + 1), 2)  # 2 timed steps
        k_b[p]["all_gather"] = 2 * 459e6 * (p + 1)
    out = b.link_projection(run, k_ms, k_b, 2, None)
    link = 4 * 459e6 / (3 * b.XGMI_LINK_GBS * 1e9) * 1e3
    assert out["exchange_link_ms_per_step"] == pytest.approx(link, abs=1e-3)
    assert out["part_kernel_ms_per_step"] == [1.0, 2.0, 3.0, 4.0]
    assert out["projected_ms_per_step"] == pytest.approx(4.0 + link, abs=1e-3)
    # the other reading of AMD's 153.6 GB/s a link (both ways together): twice the link time
    assert out["exchange_link_ms_per_step_half_rate"] == pytest.approx(2 * link, abs=2e-3)
    assert out["projected_ms_per_step_half_rate"] == pytest.approx(4.0 + 2 * link, abs=2e-3)
    assert b.link_projection(FakeRun(1, 1, []), k_ms[:1], k_b[:1], 2, None) == {}


def test_critical_path_of_side_stream_kernels():
    """A round's critical-path device time: the heavy rows' pull beside a binned round's scatter counts only when
    the round has no heavy_commit (whose timer covers the join)."""
    b = _bench()
    from gossip_hip.engine import KERNELS
    binned = {"bin_scatter": 5.0, "bin_apply": 6.0, "pull_heavy": 4.0, "heavy_commit": 0.1}
    assert b.critical(binned, KERNELS) == pytest.approx(11.1)
    assert b.critical({"bin_scatter": 5.0, "bin_apply": 6.0, "pull_heavy": 0.4}, KERNELS) == pytest.approx(11.4)
    assert b.critical({"push_light": 0.2, "push_heavy": 0.1, "churn": 0.1}, KERNELS) == pytest.approx(0.4)
