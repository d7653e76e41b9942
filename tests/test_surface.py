"""CPU tests of the drop-in C++ surface: NetworkConfig against the real
reference's outputs (tests/golden/config_cases.json, produced by the
reference's own config.cpp), and the wire/log formats of Appendix A."""
import ctypes as C
import hashlib
import json
import subprocess
import time
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
BUILD = REPO / "p2p-gossipprotocol_amd" / "build"
GOLDEN = REPO / "tests" / "golden"


@pytest.fixture(scope="module")
def surf():
    L = C.CDLL(str(BUILD / "libgossip_surface.so"))
    for name in ("gossip_surface_netcfg", "gossip_surface_message", "gossip_surface_hash", "gossip_surface_register",
                 "gossip_surface_dead_node", "gossip_surface_log", "gossip_surface_seed"):
        getattr(L, name).restype = C.c_int
    return L


def _call(fn, *args):
    buf = C.create_string_buffer(1 << 16)
    assert fn(*args, buf, C.c_size_t(len(buf))) == 0
    return buf.value.decode()


@pytest.mark.parametrize("case", json.loads((GOLDEN / "config_cases.json").read_text())["cases"],
                         ids=lambda c: c["name"])
def test_network_config_matches_reference(surf, tmp_path, case):
    if case["text"] is None:
        path = str(tmp_path / "does_not_exist.txt")
    else:
        path = str(tmp_path / "cfg.txt")
        Path(path).write_bytes(case["text"].encode())
    got = json.loads(_call(surf.gossip_surface_netcfg, path.encode()))
    want = dict(case["result"])
    if case["text"] is None:
        got["what"] = got["what"].replace(path, "<PATH>")
    assert got == want


def test_reference_network_txt(surf):
    got = json.loads(_call(surf.gossip_surface_netcfg, str(GOLDEN / "network.txt").encode()))
    assert got["ok"] and len(got["seeds"]) == 20 and got["min_seeds"] == 11
    assert got["seeds"][0] == "192.168.1.100:8000" and got["seeds"][-1] == "192.168.1.119:8019"


def test_message_hash_vectors(surf):
    for v in json.loads((GOLDEN / "sha256_kat.json").read_text())["vectors"]:
        h = _call(surf.gossip_surface_hash, v["content"].encode(), v["timestamp"].encode(), v["source_ip"].encode())
        assert h == v["hash"]


def test_gossip_json_is_nlohmann_compact_sorted(surf):
    # peer.cpp:298-307 built with nlohmann::json (std::map -> sorted keys), dump() compact
    js = _call(surf.gossip_surface_message, b"192.168.99.96", 5000, 0, 0)
    obj = json.loads(js)
    assert js == json.dumps(obj, sort_keys=True, separators=(",", ":"))
    assert obj["content"] == "Message from 192.168.99.96:5000"
    assert obj["timestamp"] == "1740441600000000000"
    assert obj["hash"] == "22bc21fe3ddbe90113181a0082839106688897e8c500bfdd73cf16ddf1346459"
    assert len(js) == 231
    assert _call(surf.gossip_surface_register, b"192.168.99.96", 5000) == \
        '{"ip":"192.168.99.96","port":5000,"type":"register"}'
    assert _call(surf.gossip_surface_dead_node, b"127.0.0.1", 5003) == \
        '{"dead_ip":"127.0.0.1","dead_port":5003,"type":"dead_node"}'


def test_log_lines(surf):
    t = 1740441600 + 45
    ct = time.strftime("%a %b %e %H:%M:%S %Y", time.gmtime(t)) + "\n"
    assert _call(surf.gossip_surface_log, 0, C.c_longlong(t), b"Peer disconnected: 127.0.0.1:5003") == \
        ct + ": Peer disconnected: 127.0.0.1:5003\n"                      # peer.cpp:131
    assert _call(surf.gossip_surface_log, 1, C.c_longlong(t), b"Removed dead peer: 127.0.0.1:5003") == \
        ct + "Removed dead peer: 127.0.0.1:5003\n"                        # seed.cpp:185


def test_cli_config_error_and_usage(tmp_path):
    exe = str(BUILD / "gossip_peer_network")
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 1 and "Error: Invalid number of arguments" in r.stderr and "Usage:" in r.stdout
    bad = tmp_path / "bad.txt"
    bad.write_text("10.0.0.1:1\nping_interval=0\n")
    r = subprocess.run([exe, str(bad)], capture_output=True, text=True)
    assert r.returncode == 1
    assert "Configuration error: Configuration Error: Ping interval must be positive" in r.stderr
    r = subprocess.run([exe, str(tmp_path / "nope.txt")], capture_output=True, text=True)
    assert r.returncode == 1 and "Unable to open config file" in r.stderr


@pytest.mark.skipif(not Path("/root/reference/main.cpp").exists(), reason="reference sources only in the build container")
def test_reference_main_compiles_against_dropin_headers(tmp_path):
    """The reference's own main.cpp (read from /root/reference, fed on stdin so
    its directory's headers are not picked up) compiles unchanged against
    include/gossip/*.hpp and links with libgossip_surface."""
    exe = tmp_path / "peer_network"
    src = Path("/root/reference/main.cpp").read_bytes()
    r = subprocess.run(["g++", "-std=c++17", f"-I{REPO / 'include'}", f"-I{REPO / 'include' / 'gossip'}", "-x", "c++",
                        "-", "-x", "none", f"-L{BUILD}", "-lgossip_surface", "-lgossip_hip",
                        f"-Wl,-rpath,{BUILD}", "-o", str(exe)], input=src, capture_output=True)
    assert r.returncode == 0, r.stderr.decode()
    assert exe.exists()


def test_seed_registry_first_insert_lastseen_and_removal_print(surf, capfd):
    """SeedNode as seed.cpp:109-178 has it: peerList is a map keyed by
    (ip, port), so a repeated registration keeps the key -- and the key's
    lastSeen, which getPeerList reports -- from the first insertion
    (seed.cpp:155,173-175); a dead_node report erases the key and prints
    "Removed dead peer" to stdout unconditionally (seed.cpp:164); a later
    registration inserts it afresh."""
    a, b = json.dumps({"ip": "127.0.0.1", "port": 5001, "type": "register"}), \
        json.dumps({"ip": "127.0.0.1", "port": 5002, "type": "register"})
    dead = json.dumps({"dead_ip": "127.0.0.1", "dead_port": 5001, "type": "dead_node"})
    ops = f"100 {a}\n105 {b}\n110 {a}\n115 {dead}\n120 {a}\n"
    out = _call(surf.gossip_surface_seed, ops.encode()).split("\n")
    lists = [json.loads(x)["peers"] for x in out if x.startswith("{")]
    assert lists[0] == [{"ip": "127.0.0.1", "lastSeen": 100, "port": 5001}]
    assert lists[1] == [{"ip": "127.0.0.1", "lastSeen": 100, "port": 5001},
                        {"ip": "127.0.0.1", "lastSeen": 105, "port": 5002}]
    assert lists[2] == lists[1]  # re-registration at 110: the key (and its lastSeen) stays
    assert out[3] == ""          # dead_node: no response
    assert lists[3] == [{"ip": "127.0.0.1", "lastSeen": 105, "port": 5002},
                        {"ip": "127.0.0.1", "lastSeen": 120, "port": 5001}]
    assert "Removed dead peer: 127.0.0.1:5001" in capfd.readouterr().out
