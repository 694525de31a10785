#!/bin/bash
# kernel traces (collective BSP headline, one-sided SSP) + roctx marker traces of both
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
bash tools/r4_prof.sh
bash tools/r4_markers.sh
