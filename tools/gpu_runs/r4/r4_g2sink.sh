#!/bin/bash
# GPT-2 / W&D SSP: split-K wgrad planes folded by the (bucket) Adam vs reduce kernels
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_gpt2.py tests/test_widedeep_gpu.py tests/test_multirank_gpu.py tests/test_checkpoint_scale.py -x -q -m gpu --timeout 280 --timeout-method thread > gpurun_out/r4/g2s_tests.log 2>&1 || { tail -40 gpurun_out/r4/g2s_tests.log; exit 1; }
tail -2 gpurun_out/r4/g2s_tests.log
for i in 1 2; do
  for cfg in "MINIPS_WGRAD_DEFER=1" "MINIPS_WGRAD_DEFER=0"; do
    env $cfg timeout -k 10 300 python tools/bench_models.py --model gpt2 --steps 40 --warmup 8 > gpurun_out/r4/g.log 2>&1
    echo "gpt2 $cfg $(grep -o '"value": [0-9.]*' gpurun_out/r4/g.log | tail -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/g.log | tail -1)"
    env $cfg timeout -k 10 300 python tools/bench_models.py --model widedeep-ssp --transport collective --steps 200 --warmup 20 > gpurun_out/r4/w.log 2>&1
    echo "wd-ssp-coll $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/w.log | tail -1)"
  done
done
