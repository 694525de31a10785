#!/bin/bash
# wgrad kernel variants: standalone shapes and the W&D step.
set -eo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in v1 v2 v3; do
  echo "== MINIPS_GEMM_WGRAD=$v"
  timeout -k 10 120 env MINIPS_GEMM_WGRAD=$v python tools/bench_gemm.py 2>&1 | grep wgrad
  for rows in 1024 2048 4096; do
    echo -n "step rows_overlap=$rows: "
    timeout -k 10 120 env MINIPS_GEMM_WGRAD=$v MINIPS_WGRAD_MIN_ROWS_OVERLAP=$rows python bench.py --steps 200 --warmup 5 | python -c "import json,sys; print(json.loads(sys.stdin.readlines()[-1])['ms_per_step'])"
  done
done
for s in 0 1; do
  echo -n "slab=$s v2 step: "
  timeout -k 10 120 env MINIPS_SPLITK_SLAB=$s MINIPS_GEMM_WGRAD=v2 python bench.py --steps 200 --warmup 5 | python -c "import json,sys; print(json.loads(sys.stdin.readlines()[-1])['ms_per_step'])"
done
