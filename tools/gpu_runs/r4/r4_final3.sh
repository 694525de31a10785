#!/bin/bash
# GPU suite with the one-sided push stream on by default; SSP bench lines; GPT-2 tile A/B
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r4/final3_tests.log 2>&1 || { tail -60 gpurun_out/r4/final3_tests.log; exit 1; }
tail -2 gpurun_out/r4/final3_tests.log
for t in onesided collective; do
  timeout -k 10 300 python tools/bench_models.py --model widedeep-ssp --transport $t --steps 200 --warmup 20 > gpurun_out/r4/fw_$t.log 2>&1 && echo "wd-ssp $t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/fw_$t.log | tail -1)"
done
bash tools/gpu_runs/r4/r4_g2tile.sh
