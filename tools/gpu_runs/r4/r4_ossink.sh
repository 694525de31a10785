#!/bin/bash
# one-sided dense push folding the split-K wgrad planes vs reduce kernels; SSP transports
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_onesided.py tests/test_gpt2.py tests/test_widedeep_gpu.py -x -q -m gpu --timeout 280 --timeout-method thread > gpurun_out/r4/oss_tests.log 2>&1 || { tail -40 gpurun_out/r4/oss_tests.log; exit 1; }
tail -2 gpurun_out/r4/oss_tests.log
for i in 1 2; do
  for cfg in "MINIPS_WGRAD_DEFER=1" "MINIPS_WGRAD_DEFER=0"; do
    for t in onesided collective; do
      env $cfg timeout -k 10 300 python tools/bench_models.py --model widedeep-ssp --transport $t --steps 200 --warmup 20 > gpurun_out/r4/w.log 2>&1
      echo "wd-ssp $t $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/w.log | tail -1)"
    done
  done
done
timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4/b.log 2>&1 && echo "bsp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/b.log)"
