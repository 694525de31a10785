#!/bin/bash
# W&D weight-gradient split-K after the slice-major XCD mapping: workgroup target / rows per split
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for i in 1 2; do
  for cfg in "MINIPS_WD_WGRAD_BLOCKS=320" "MINIPS_WD_WGRAD_BLOCKS=512" "MINIPS_WGRAD_MIN_ROWS_OVERLAP=512" "MINIPS_WD_WGRAD_BLOCKS=512 MINIPS_WGRAD_MIN_ROWS_OVERLAP=512" "MINIPS_WD_WGRAD_BLOCKS=256"; do
    env $cfg timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4/bench_k.log 2>&1
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_k.log)"
  done
done
