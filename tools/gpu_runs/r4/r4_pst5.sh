#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for i in 1 2; do
  for cfg in "MINIPS_PS_PUSH_STREAM=0" "MINIPS_PS_PUSH_STREAM=1 MINIPS_FAST_PLAN_EVENTS=0"; do
    env $cfg timeout -k 10 300 python tools/bench_models.py --model widedeep-ssp --transport onesided --steps 200 --warmup 20 > gpurun_out/r4/w.log 2>&1
    echo "wd-ssp-os $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/w.log | tail -1)"
    env $cfg timeout -k 10 400 python tools/bench_models.py --model dlrm-10b --steps 100 --warmup 20 > gpurun_out/r4/d.log 2>&1
    echo "dlrm-10b $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/d.log | tail -1)"
  done
done
