#!/bin/bash
# W&D headline: re-measure the step's existing knobs at the round-4 tree (interleaved, 2 rounds)
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for i in 1 2; do
  for cfg in "MINIPS_X=0" "MINIPS_WD_WGRAD_BLOCKS=256" "MINIPS_WD_WGRAD_BLOCKS=192" "MINIPS_WD_K1_ALIGN=8" "MINIPS_WGRAD_MIN_ROWS_OVERLAP=2048" "MINIPS_WGRAD_MIN_ROWS_OVERLAP=512" "MINIPS_WGRAD_DEFER=0"; do
    env $cfg timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4/bench_knob.log 2>&1
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_knob.log)"
  done
done
