"""ctypes binding of libgossip_hip's C-ABI (include/gossip/gossip.h).

Plumbing only: every computation happens in the HIP library.  Loading fails
loudly if the library is missing -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent          # p2p-gossipprotocol_amd/
REPO_ROOT = PKG_ROOT.parent
LIB_PATH = Path(os.environ.get("GOSSIP_HIP_LIB", PKG_ROOT / "build" / "libgossip_hip.so"))
HEADER = REPO_ROOT / "include" / "gossip" / "gossip.h"

GOSSIP_OK = 0
GOSSIP_EINVAL = -1
GOSSIP_ENOMEM = -2
GOSSIP_EHIP = -3
GOSSIP_ESTATE = -4
GOSSIP_ENODEV = -5
GOSSIP_EOVERFLOW = -6
GOSSIP_ECOMM = -7
GOSSIP_ESTALL = -8
COMM_ID_BYTES = 128

GRAPH_POWERLAW = 1
GRAPH_REF_BOOTSTRAP = 2
FLAG_COVERAGE_HISTORY = 1
FLAG_FORCE_PUSH = 2
FLAG_FORCE_PULL = 4
FLAG_NO_BIN = 8
FLAG_FORCE_BIN = 16
FLAG_NO_BLOCKED = 32
FLAG_FORCE_BLOCKED = 64
FLAG_UNIFORM_PARTITION = 128
MODE_AUTO = -1
MODE_PUSH = 0
MODE_PULL = 1
MODE_PUSH_SPARSE = 2
MODE_BIN = 3
MODE_BLOCKED = 4


class GossipConfig(C.Structure):
    _fields_ = [
        ("n_peers", C.c_uint64),
        ("part_begin", C.c_uint64),
        ("part_end", C.c_uint64),
        ("n_msgs", C.c_uint32),
        ("rng_seed", C.c_uint32),
        ("graph_model", C.c_uint32),
        ("list_len", C.c_uint32),
        ("n_seeds", C.c_uint32),
        ("churn_threshold", C.c_uint32),
        ("ping_every", C.c_uint32),
        ("max_missed", C.c_uint32),
        ("max_rounds", C.c_uint32),
        ("min_rounds", C.c_uint32),
        ("device", C.c_int32),
        ("flags", C.c_uint32),
        ("report_capacity", C.c_uint64),
        ("pull_permille", C.c_uint32),
        ("front_permille", C.c_uint32),
        ("bin_permille", C.c_uint32),
        ("extra_cap", C.c_uint32),
        ("list_cap", C.c_uint32),
        ("rejoin_threshold", C.c_uint32),
        ("blocked_permille", C.c_uint32),
    ]


STAT_FIELDS = ("frontier", "traversals", "deliveries", "undelivered", "new_receipts", "duplicates", "injected",
               "died", "reports", "seed_removals", "digest", "covered", "reconnects", "rejoined")


class RoundStats(C.Structure):
    _fields_ = [("round", C.c_uint32), ("flags", C.c_uint32)] + [(f, C.c_uint64) for f in STAT_FIELDS]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


class DeadReport(C.Structure):
    _fields_ = [("round", C.c_uint32), ("reporter", C.c_uint32), ("dead", C.c_uint32)]


class GossipError(RuntimeError):
    def __init__(self, status: int, where: str, detail: str):
        super().__init__(f"{where}: status {status}: {detail}")
        self.status = status


_lib = None


def lib() -> C.CDLL:
    """Load libgossip_hip.so once; raise if it is absent (no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(f"libgossip_hip.so not found at {LIB_PATH}; run __graft_entry__.build() "
                          f"(make -C p2p-gossipprotocol_amd)")
    L = C.CDLL(str(LIB_PATH))
    P, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
    pu32, pu64, pu8 = C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), C.POINTER(C.c_uint8)
    sigs = {
        "gossip_create": (i32, [C.POINTER(GossipConfig), C.POINTER(P)]),
        "gossip_destroy": (None, [P]),
        "gossip_strerror": (C.c_char_p, [i32]),
        "gossip_last_error": (C.c_char_p, []),
        "gossip_set_stream": (i32, [P, P]),
        "gossip_get_shape": (i32, [P, pu32, pu32, pu64, pu64]),
        "gossip_build_graph": (i32, [P]),
        "gossip_load_csr": (i32, [P, pu64, pu32, u64, u64]),
        "gossip_read_csr": (i32, [P, pu64, pu32]),
        "gossip_read_extra": (i32, [P, pu32, pu32]),
        "gossip_inject": (i32, [P, pu32, pu32, u32]),
        "gossip_schedule_kills": (i32, [P, pu32, pu32, u32]),
        "gossip_pick_origins": (i32, [u64, u32, u32, pu32]),
        "gossip_device_count": (i32, [C.POINTER(C.c_int32)]),
        "gossip_reset": (i32, [P]),
        "gossip_step": (i32, [P, C.POINTER(RoundStats)]),
        "gossip_run": (i32, [P, C.POINTER(RoundStats), u32, pu32]),
        "gossip_set_exchange": (i32, [P, P, P, u32, pu64]),
        "gossip_round_push": (i32, [P]),
        "gossip_set_gather": (i32, [P, P]),
        "gossip_round_begin": (i32, [P, i32, C.POINTER(C.c_int)]),
        "gossip_round_compute": (i32, [P]),
        "gossip_set_sparse": (i32, [P, P]),
        "gossip_sparse_counts": (i32, [P, pu64]),
        "gossip_round_finish_sparse": (i32, [P, P, u64, C.POINTER(RoundStats)]),
        "gossip_round_finish": (i32, [P, C.POINTER(RoundStats)]),
        "gossip_round_commit": (i32, [P, u64, C.POINTER(C.c_int)]),
        "gossip_read_seen": (i32, [P, pu64]),
        "gossip_read_coverage": (i32, [P, pu64]),
        "gossip_read_coverage_history": (i32, [P, pu64, u32, pu32]),
        "gossip_read_reports": (i32, [P, C.POINTER(DeadReport), u64, pu64]),
        "gossip_read_alive": (i32, [P, pu8]),
        "gossip_read_registered": (i32, [P, pu8]),
        "gossip_enable_timing": (i32, [P, i32]),
        "gossip_kernel_time": (i32, [P, C.c_char_p, C.POINTER(C.c_double), pu64]),
        "gossip_kernel_bytes": (i32, [P, C.c_char_p, C.POINTER(C.c_double)]),
        "gossip_set_tuning": (i32, [P, C.c_char_p, C.c_int64]),
        # library-driven multi-GPU rounds (gossip_dist.hip)
        "gossip_partition": (i32, [u64, u32, pu64]),
        "gossip_partition_edges": (i32, [C.POINTER(GossipConfig), u32, pu64]),
        "gossip_comm_unique_id": (i32, [pu8]),
        "gossip_comm_init": (i32, [P, pu8, u32, u32]),
        "gossip_comm_finalize": (i32, [P, C.POINTER(RoundStats), u32, C.POINTER(DeadReport), u64, pu64]),
        "gossip_comm_modes": (i32, [P, C.POINTER(C.c_int32), u32, pu32]),
        "gossip_group_create": (i32, [C.POINTER(GossipConfig), u32, C.POINTER(C.c_int32), C.POINTER(P)]),
        "gossip_group_create_parts": (i32, [C.POINTER(GossipConfig), u32, C.POINTER(C.c_int32),
                                            C.POINTER(C.c_uint64), C.POINTER(P)]),
        "gossip_group_destroy": (None, [P]),
        "gossip_group_part": (i32, [P, u32, C.POINTER(P)]),
        "gossip_group_build_graph": (i32, [P]),
        "gossip_group_inject": (i32, [P, pu32, pu32, u32]),
        "gossip_group_schedule_kills": (i32, [P, pu32, pu32, u32]),
        "gossip_group_reset": (i32, [P]),
        "gossip_group_step": (i32, [P, C.POINTER(RoundStats)]),
        "gossip_group_run": (i32, [P, C.POINTER(RoundStats), u32, pu32]),
        "gossip_group_read_seen": (i32, [P, pu64]),
        "gossip_group_read_reports": (i32, [P, C.POINTER(DeadReport), u64, pu64]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(status: int, where: str) -> int:
    if status < 0:
        L = lib()
        raise GossipError(status, where, f"{L.gossip_strerror(status).decode()}: {L.gossip_last_error().decode()}")
    return status


def declared_symbols() -> list[str]:
    """Function names declared in include/gossip/gossip.h."""
    import re
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:gossip_status|void|const char\*)\s+(gossip_\w+)\s*\(", text, re.M)))
