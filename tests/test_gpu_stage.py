"""The LDS record-staging protocol of the propagation-blocked rounds
(p2p-gossipprotocol_amd/csrc/gossip_stage.hpp) on the GPU, through
tests/gpu_support/stage_selftest.hip: every record staged by every wave of
every workgroup must arrive exactly once, in its own bin's segment, with the
segments' lengths equal to their whole generations -- in both geometries the
blocked kernels use (level 1: 32 records per generation, two buffers per
bin, 32-bit destinations, up to 160 bins; level 2: 64 records, two buffers
per bin, 16-bit destinations, up to 100 bins) and a third (16 records), on
spread and on
contended bins (7 of 8 records into one bin, every wave at once: the case
whose lost records and hang round 3 traced to a reservation that wrapped its
counter), and on the 96/128-bin tables the kernels
size their LDS for.  A wave that gave up waiting (bit 4, GOSSIP_ESTALL in the
engine) fails the case."""
import ctypes as C
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
LIB = Path(__file__).resolve().parent / "gpu_support" / "libstage_selftest.so"


@pytest.fixture(scope="module")
def stage_lib():
    if not LIB.exists():
        pytest.fail(f"{LIB} is not built (__graft_entry__.build() / make -C tests/gpu_support)")
    L = C.CDLL(str(LIB))
    L.stage_selftest.restype = C.c_int
    L.stage_selftest.argtypes = [C.c_uint32] * 5 + [C.POINTER(C.c_uint64)]
    return L


@pytest.mark.parametrize("kb", [16, 32, 64])
@pytest.mark.parametrize("nb,per_wg,skew,grid", [(1, 20000, 0, 512), (3, 576, 1, 512), (57, 20000, 0, 512),
                                                 (96, 9000, 1, 256), (96, 20000, 0, 256), (160, 3000, 0, 1024),
                                                 (7, 100, 1, 2048)])
def test_stage_every_record_once(stage_lib, kb, nb, per_wg, skew, grid):
    nb = min(nb, 100) if kb == 64 else nb  # level 2's LDS holds 100 bins of two 64-record buffers
    out = (C.c_uint64 * 8)()
    assert stage_lib.stage_selftest(nb, per_wg, skew, grid, kb, out) == 0
    ok, got, total, bad, dup, err, seg_len, want_len = list(out)
    assert err == 0, f"error flags {err:#x} (4: a staging wave stalled, 2: a segment overflowed)"
    assert (got, bad, dup) == (total, 0, 0)
    assert seg_len == want_len
    assert ok == 1
