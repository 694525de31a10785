#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "mlp or graph" --timeout 280 --timeout-method thread > gpurun_out/r4/mls_tests.log 2>&1 || { tail -40 gpurun_out/r4/mls_tests.log; exit 1; }
tail -2 gpurun_out/r4/mls_tests.log
for i in 1 2; do
  for cfg in "MINIPS_WGRAD_DEFER=1" "MINIPS_WGRAD_DEFER=0"; do
    env $cfg timeout -k 10 400 python tools/bench_models.py --model mlp --steps 300 --warmup 30 > gpurun_out/r4/m.log 2>&1
    echo "mlp $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/m.log | tail -1)"
  done
done
