"""minips_amd: an MI355X-native parameter-server training framework.

Capabilities of Distributed-Deep-Learning/MiniPs (KV push/pull API, BSP/SSP/ASP consistency,
range-sharded tables, checkpoint/rollback, heartbeat failure detection) re-designed for one
process per MI355X GPU: a native C++ runtime (``minips_amd._runtime``), hand-written gfx950
HIP kernels (``minips_amd._kernels``) and RCCL collectives over xGMI (``minips_amd.ps``).
"""
__version__ = "0.1.0"

from . import ops  # noqa: F401
