#!/bin/bash
# Generic A/B of environment knobs on the GPU box (one script for every knob sweep; the earlier
# per-experiment scripts were folded into it, e.g. the GPT-2 wgrad sweep is
# CMD='python tools/bench_models.py --model gpt2 --steps 10 --warmup 3' AB='...'). Variants are ';'-separated env lists:
#   AB='MINIPS_GEMM_WGRAD=v1;MINIPS_GEMM_WGRAD=v2 MINIPS_SPLITK_SLAB=0' bash tools/gpu_ab.sh
#   RUNS=3 STEPS=300 BENCH_ARGS='--batch 8192' AB='...' bash tools/gpu_ab.sh
#   CMD='python tools/bench_kernels.py kscan --Ks 848' AB='MINIPS_GEMM_TILE=128;MINIPS_GEMM_TILE=256' bash tools/gpu_ab.sh
# With the default CMD (bench.py) it prints ms/step per run; otherwise the command's output tail.
set -eo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
IFS=';' read -ra VARIANTS <<< "${AB:-MINIPS_AB_BASELINE=1}"
for v in "${VARIANTS[@]}"; do
  for i in $(seq "${RUNS:-2}"); do
    if [[ -z "${CMD}" ]]; then
      env $v timeout -k 10 240 python bench.py --steps "${STEPS:-200}" --warmup 5 ${BENCH_ARGS} > gpurun_out/ab.log 2>&1
      python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'])"
    else
      echo "== $v (run $i)"
      env $v timeout -k 10 240 ${CMD} 2>&1 | tail -${TAIL:-20}
    fi
  done
done
