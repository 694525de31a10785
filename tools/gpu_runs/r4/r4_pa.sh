#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for i in 1 2 3; do
  for cfg in "MINIPS_PLAN_AT=start" "MINIPS_PLAN_AT=head MINIPS_COMPUTE_PRIORITY=1" "MINIPS_COMPUTE_PRIORITY=1"; do
    env $cfg timeout -k 10 200 python bench.py --steps 400 --warmup 20 > gpurun_out/r4/bp.log 2>&1
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bp.log)"
  done
done
