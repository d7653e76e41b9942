"""pytest configuration: the `gpu` marker, import paths, prebuilt artefacts."""
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
PKG = REPO / "p2p-gossipprotocol_amd"
for p in (str(PKG), str(REPO / "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle():
    """ctypes binding of the CPU restatement (test infrastructure only)."""
    so = REPO / "oracle" / "_build" / "libgossip_oracle.so"
    if not so.exists():  # CPU-side convenience; on the GPU box the prebuilt .so travels
        subprocess.run(["make", "-C", str(REPO / "oracle"), "all"], check=True, capture_output=True)
    import oracle_ref
    return oracle_ref.Oracle(so)


@pytest.fixture(scope="session")
def hip_lib():
    from gossip_hip import _abi
    return _abi.lib()
