#!/bin/bash
# GPT-2 knobs at 8 HW queues + slice-major split-K map
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for i in 1 2; do
  for cfg in "MINIPS_WGRAD_BLOCKS=512" "MINIPS_WGRAD_BLOCKS=256" "MINIPS_WGRAD_BLOCKS=768" "MINIPS_WGRAD_MIN_ROWS_OVERLAP=512" "MINIPS_GPT2_OVERLAP_W1=0" "MINIPS_COMPUTE_PRIORITY=1"; do
    env $cfg timeout -k 10 300 python tools/bench_models.py --model gpt2 --steps 40 --warmup 8 > gpurun_out/r4/g.log 2>&1
    echo "$cfg $(grep -o '"value": [0-9.]*' gpurun_out/r4/g.log | tail -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/g.log | tail -1)"
  done
done
