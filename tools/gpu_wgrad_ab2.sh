#!/bin/bash
set -eo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
st() { timeout -k 10 120 env "$@" python bench.py --steps 300 --warmup 5 | python -c "import json,sys; print(json.loads(sys.stdin.readlines()[-1])['ms_per_step'])"; }
for v in v1 v2; do for slab in 0 1; do for rows in 384 512 768 1024; do
  echo -n "wgrad=$v slab=$slab rows=$rows: "; st MINIPS_GEMM_WGRAD=$v MINIPS_SPLITK_SLAB=$slab MINIPS_WGRAD_MIN_ROWS_OVERLAP=$rows
done; done; done
