#!/bin/bash
# W&D headline: re-measure the step's existing knobs at the round-4 tree (interleaved, 2 rounds)
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_widedeep_gpu.py tests/test_multirank_gpu.py -x -q -m gpu -k "head or widedeep" --timeout 280 --timeout-method thread > gpurun_out/r4/knob_tests.log 2>&1 || { tail -40 gpurun_out/r4/knob_tests.log; exit 1; }
tail -2 gpurun_out/r4/knob_tests.log
for i in 1 2; do
  for cfg in "MINIPS_WD_FUSED_HEAD=1" "MINIPS_WD_FUSED_HEAD=0"; do
    env $cfg timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4/bench_knob.log 2>&1
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_knob.log)"
  done
done
