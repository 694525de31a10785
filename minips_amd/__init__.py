"""minips_amd: an MI355X-native parameter-server training framework.

Capabilities of Distributed-Deep-Learning/MiniPs (KV push/pull API, BSP/SSP/ASP consistency,
range-sharded tables, checkpoint/rollback, heartbeat failure detection) re-designed for one
process per MI355X GPU: a native C++ runtime (``minips_amd._runtime``), hand-written gfx950
HIP kernels (``minips_amd._kernels``) and RCCL collectives over xGMI (``minips_amd.ps``).
"""
__version__ = "0.1.0"

import os as _os

# HIP multiplexes a process's streams onto GPU_MAX_HW_QUEUES hardware queues (default 4). A
# training step here runs up to 6-7 streams (compute, weight-gradient side stream, planning,
# clock pipelines, default): with 4 queues two of them share one and serialise -- the W&D SSP
# step ran its dgrad chain and weight gradients on one queue (0.513 vs 0.444 ms/step with 8;
# BSP unchanged, profiles/r4/ab_hw_queues.txt). The HIP runtime reads it when it is loaded (with
# torch), so this default only takes effect when minips_amd is imported before torch (the
# ``python -m minips_amd.*`` entry points; bench.py and tools/bench_models.py set it themselves
# before importing torch); a setting other than HIP's default 4 wins; MINIPS_HW_QUEUES picks ours.
if _os.environ.get("GPU_MAX_HW_QUEUES", "4") == "4":  # unset or HIP's default (the GPU box exports 4)
    _os.environ["GPU_MAX_HW_QUEUES"] = _os.environ.get("MINIPS_HW_QUEUES", "8")

from . import ops  # noqa: F401
