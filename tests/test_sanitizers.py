"""Host code under sanitizers, CPU only: the drop-in
surface under ThreadSanitizer and Address+UB sanitizers (concurrent seed
registrations / dead-node reports / stop() as the reference's
thread-per-connection seed and signal handler would issue them), the oracle's
drivers under Address+UB sanitizers, and the real-socket loopback harness
built with Address+UB sanitizers on a loopback workload."""
import os
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
SAN = REPO / "tests" / "sanitize"
OUT = SAN / "_build"


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-C", str(SAN), "all", "-j4"], check=True, capture_output=True)
    return OUT


def _run(exe, env_extra, *args):
    env = dict(os.environ, **env_extra)
    p = subprocess.run([str(exe), *args], cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "Sanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-4000:]
    return p.stdout


def test_surface_threadsanitizer(built):
    out = _run(built / "surface_tsan", {"TSAN_OPTIONS": "halt_on_error=1"}, "tests/golden/network.txt")
    assert "0 bad replies" in out


def test_surface_address_ub_sanitizer(built):
    out = _run(built / "surface_asan", {"ASAN_OPTIONS": "detect_leaks=1"}, "tests/golden/network.txt")
    assert "0 bad replies" in out


def test_oracle_address_ub_sanitizer(built):
    out = _run(built / "oracle_asan", {"ASAN_OPTIONS": "detect_leaks=1", "OMP_NUM_THREADS": "4"})
    assert "0 failure(s)" in out


def test_loopback_address_ub_sanitizer(built, oracle, monkeypatch):
    """The harness binary under ASan/UBSan on a config-2 style run (real TCP on 127.0.0.1)."""
    import numpy as np

    from gossip_hip import loopback
    from gossip_hip.workloads import config
    monkeypatch.setattr(loopback, "BINARY", built / "gossip_loopback_asan")
    w = config(2, 60, pick=oracle.pick_origins)
    rp, col = oracle.gen_workload(w)
    env = {"ASAN_OPTIONS": "detect_leaks=1"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        got = loopback.run_loopback(rp, col, w.origins, w.inject_rounds, n_seeds=w.n_seeds)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    ref = oracle.simulate_workload(w, rp, col)
    assert got["errors"] == 0
    assert sum(len(v) for v in got["seen"].values()) == int(np.bitwise_count(ref["seen"]).sum())
