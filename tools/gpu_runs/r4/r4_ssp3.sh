#!/bin/bash
# one-sided dense clock on the side stream; 8 HW queues by default (minips_amd/__init__.py)
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_onesided.py tests/test_widedeep_gpu.py tests/test_multirank_gpu.py -x -q --timeout 280 --timeout-method thread > gpurun_out/r4/ssp3_tests.log 2>&1 || { tail -40 gpurun_out/r4/ssp3_tests.log; exit 1; }
tail -2 gpurun_out/r4/ssp3_tests.log
for i in 1 2; do
  for t in onesided collective; do
    timeout -k 10 200 python tools/bench_models.py --model widedeep-ssp --transport $t --steps 200 --warmup 20 > gpurun_out/r4/wd_ssp_$t.log 2>&1
    echo "ssp $t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/wd_ssp_$t.log)"
  done
  MINIPS_DENSE_ON_SIDE=0 timeout -k 10 200 python tools/bench_models.py --model widedeep-ssp --transport onesided --steps 200 --warmup 20 > gpurun_out/r4/wd_ssp_os0.log 2>&1
  echo "ssp onesided dense-on-main $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/wd_ssp_os0.log)"
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4/bench_b.log 2>&1
  echo "bsp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_b.log)"
done
