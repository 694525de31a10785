#!/bin/bash
# HW queue count vs the step's stream count (streams beyond the HW queues share one and serialise)
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for i in 1 2; do
  for q in 4 8; do
    for t in onesided collective; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python tools/bench_models.py --model widedeep-ssp --transport $t --steps 200 --warmup 20 > gpurun_out/r4/wd_ssp.log 2>&1
      echo "hwq=$q ssp $t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/wd_ssp.log)"
    done
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4/bench_q.log 2>&1
    echo "hwq=$q bsp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_q.log)"
  done
done
