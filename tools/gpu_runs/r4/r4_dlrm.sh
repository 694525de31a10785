#!/bin/bash
# DLRM-10B vs round 3 (0.650 ms): HW queues / fast events; W&D default-flip candidates
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for cfg in "MINIPS_HW_QUEUES=8" "MINIPS_HW_QUEUES=4" "MINIPS_FAST_EVENTS=0" "MINIPS_HW_QUEUES=4 MINIPS_FAST_EVENTS=0"; do
  env $cfg timeout -k 10 400 python tools/bench_models.py --model dlrm-10b --steps 200 --warmup 20 > gpurun_out/r4/d10.log 2>&1 || { echo "$cfg FAILED"; tail -3 gpurun_out/r4/d10.log; continue; }
  echo "dlrm-10b $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/d10.log | tail -1) $(grep -o '"transport": "[a-z]*"' gpurun_out/r4/d10.log | tail -1) $(grep -o '"consistency": "[a-z0-9]*"' gpurun_out/r4/d10.log | tail -1)"
done
for i in 1 2; do
  for cfg in "MINIPS_PLAN_AT=start" "MINIPS_PLAN_AT=head MINIPS_COMPUTE_PRIORITY=1" "MINIPS_PLAN_AT=head"; do
    env $cfg timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4/bench_k.log 2>&1
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_k.log)"
  done
done
