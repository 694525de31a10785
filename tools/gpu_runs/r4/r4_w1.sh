#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_widedeep_gpu.py tests/test_nn_gpu.py -x -q -m gpu --timeout 280 --timeout-method thread > gpurun_out/r4/w1_tests.log 2>&1 || { tail -40 gpurun_out/r4/w1_tests.log; exit 1; }
tail -2 gpurun_out/r4/w1_tests.log
for i in 1 2; do
  for cfg in "MINIPS_WD_W1_LATE=0" "MINIPS_WD_W1_LATE=1" "MINIPS_WGRAD_STREAM=0"; do
    env $cfg timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4/bench_w.log 2>&1
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_w.log)"
  done
done
