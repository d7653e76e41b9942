"""gossip_hip -- host package of the MI355X gossip-propagation engine.

The compute path is libgossip_hip.so (HIP kernels for gfx950); this package
is the ctypes binding plus the multi-rank driver (torch.distributed/RCCL).
"""
from ._abi import GossipError, declared_symbols, lib  # noqa: F401
from .engine import KERNELS, Engine, pick_origins  # noqa: F401
from .workloads import Workload, config, ping_every_rounds, run_engine  # noqa: F401
