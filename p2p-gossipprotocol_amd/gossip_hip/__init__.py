"""gossip_hip -- host package of the MI355X gossip-propagation engine.

The compute path is libgossip_hip.so (HIP kernels for gfx950); this package
is the ctypes binding.  Multi-GPU rounds are driven by the library itself
over RCCL (Engine.comm_init, Group); distributed.py is the torch.distributed
mirror of the same driver, kept as the gloo test harness.
"""
from ._abi import GossipError, declared_symbols, lib  # noqa: F401
from .engine import EXCHANGES, KERNELS, Engine, Group, comm_unique_id, device_count, partition, partition_edges, pick_origins  # noqa: F401
from .workloads import Workload, config, ping_every_rounds, run_engine  # noqa: F401
