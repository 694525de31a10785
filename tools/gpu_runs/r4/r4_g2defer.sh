#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for i in 1 2 3; do
  for cfg in "MINIPS_GPT2_WGRAD_DEFER=0" "MINIPS_GPT2_WGRAD_DEFER=1"; do
    env $cfg timeout -k 10 300 python tools/bench_models.py --model gpt2 --steps 60 --warmup 10 > gpurun_out/r4/g.log 2>&1
    echo "gpt2 $cfg $(grep -o '"value": [0-9.]*' gpurun_out/r4/g.log | tail -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/g.log | tail -1)"
  done
done
