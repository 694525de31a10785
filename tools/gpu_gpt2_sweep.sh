#!/bin/bash
# GPT-2 (config 4) 1-GPU throughput under the weight-gradient GEMM knobs (ops/__init__.py).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  local tag="$1"; shift
  env "$@" timeout -k 10 200 python tools/bench_models.py --model gpt2 --steps 10 --warmup 3 > gpurun_out/sw.log 2>&1 || { echo "$tag FAILED"; tail -5 gpurun_out/sw.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/sw.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
run base MINIPS_X=0
run v3 MINIPS_GEMM_WGRAD=v3
run v2_blocks256 MINIPS_WGRAD_BLOCKS=256
run v2_blocks1024 MINIPS_WGRAD_BLOCKS=1024
run v2_rows2048 MINIPS_WGRAD_MIN_ROWS_OVERLAP=2048
run v2_rows512 MINIPS_WGRAD_MIN_ROWS_OVERLAP=512
run v1 MINIPS_GEMM_WGRAD=v1
run slab0 MINIPS_SPLITK_SLAB=0
run tile128 MINIPS_GEMM_TILE=128
run tile128_slab0 MINIPS_GEMM_TILE=128 MINIPS_SPLITK_SLAB=0
run rows2048_slab0 MINIPS_WGRAD_MIN_ROWS_OVERLAP=2048 MINIPS_SPLITK_SLAB=0
