"""CPU tests of the boundary: libgossip_hip loads, exports every symbol the
header declares, and fails loudly (never falls back) without a gfx950 GPU."""
import ctypes as C

import numpy as np
import pytest

from gossip_hip import _abi
from gossip_hip.engine import pick_origins
from gossip_hip.workloads import config, ping_every_rounds


def test_every_declared_symbol_is_exported(hip_lib):
    names = _abi.declared_symbols()
    assert len(names) >= 25
    for name in names:
        assert hasattr(hip_lib, name), name


def test_library_is_gfx950_code_object():
    data = _abi.LIB_PATH.read_bytes()
    assert b"gfx950" in data


def test_strerror_table(hip_lib):
    assert hip_lib.gossip_strerror(0) == b"ok"
    assert hip_lib.gossip_strerror(_abi.GOSSIP_ENODEV) == b"no gfx950 device"


def test_create_rejects_bad_config(hip_lib):
    cfg = _abi.GossipConfig()
    cfg.n_peers = 0
    cfg.n_msgs = 1
    ctx = C.c_void_p()
    assert hip_lib.gossip_create(C.byref(cfg), C.byref(ctx)) == _abi.GOSSIP_EINVAL
    cfg.n_peers = 10
    cfg.n_msgs = 513
    assert hip_lib.gossip_create(C.byref(cfg), C.byref(ctx)) == _abi.GOSSIP_EINVAL
    cfg.n_peers, cfg.n_msgs, cfg.part_begin, cfg.part_end, cfg.rejoin_threshold = 64, 8, 0, 32, 1000
    assert hip_lib.gossip_create(C.byref(cfg), C.byref(ctx)) == _abi.GOSSIP_EINVAL  # rejoin: single partition only


def test_pick_origins_matches_oracle(oracle):
    for n, seed, k in [(1 << 20, 0x5EED0002, 6), (1 << 24, 0x5EED0003, 64), (100, 9, 64)]:
        assert np.array_equal(pick_origins(n, seed, k), oracle.pick_origins(n, seed, k))


def test_ping_period_matches_reference_loop():
    # 5 s tick (peer.cpp:353) gated by lastPing >= 13 s (peer.cpp:329-330) -> every 15 s
    assert ping_every_rounds(13, 5) == 15
    assert ping_every_rounds(5, 5) == 5


def test_workload_shapes(oracle):
    w1 = config(1, pick=oracle.pick_origins)
    assert w1.n == 8 and w1.n_msgs == 80 and w1.graph == "ref_bootstrap"
    assert sorted(set(w1.inject_rounds.tolist())) == list(range(0, 50, 5))
    w2 = config(2, pick=oracle.pick_origins)
    assert w2.n == 1 << 20 and w2.n_msgs == 60
    w5 = config(5, 1 << 10, pick=oracle.pick_origins)
    assert w5.churn_threshold == 42949673 and w5.ping_every == 3


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="checks the no-GPU failure path")
def test_engine_fails_loudly_without_gpu():
    from gossip_hip import Engine, GossipError
    with pytest.raises(GossipError) as ei:
        Engine(1024, 64)
    assert ei.value.status == _abi.GOSSIP_ENODEV


def test_ctypes_layouts_match_header(tmp_path):
    """The ctypes mirrors of gossip_config / gossip_round_stats have the C header's size and field offsets."""
    import subprocess

    structs = {"gossip_config": _abi.GossipConfig, "gossip_round_stats": _abi.RoundStats}
    lines = []
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "gossip/gossip.h"\nint main(void) {\n'
                   + "\n".join(lines) + "\nreturn 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", str(_abi.REPO_ROOT / "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    for row in filter(None, out):
        cname, field, value = row.split()
        py = structs[cname]
        got = C.sizeof(py) if field == "size" else getattr(py, field).offset
        assert got == int(value), (cname, field)
