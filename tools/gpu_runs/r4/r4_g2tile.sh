#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for i in 1 2; do
  for cfg in "MINIPS_GEMM_TILE=0" "MINIPS_GEMM_TILE=256" "MINIPS_GEMM_TILE=128" "MINIPS_GEMM_V4=3"; do
    env $cfg timeout -k 10 300 python tools/bench_models.py --model gpt2 --steps 40 --warmup 8 > gpurun_out/r4/g.log 2>&1
    echo "gpt2 $cfg $(grep -o '"value": [0-9.]*' gpurun_out/r4/g.log | tail -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/g.log | tail -1)"
  done
done
