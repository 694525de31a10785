#!/bin/bash
# kernel traces (collective BSP headline, one-sided SSP) + roctx marker traces of both
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
bash tools/gpu_runs/r4/r4_prof.sh
bash tools/gpu_runs/r4/r4_markers.sh
