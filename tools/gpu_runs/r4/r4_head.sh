#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for i in 1 2; do
  for cfg in "MINIPS_HEAD_BLOCKS=128" "MINIPS_HEAD_BLOCKS=256" "MINIPS_HEAD_BLOCKS=64"; do
    env $cfg timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4/bench_h.log 2>&1
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_h.log)"
  done
done
