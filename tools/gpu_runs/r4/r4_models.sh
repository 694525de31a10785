#!/bin/bash
# W&D knobs at 8 HW queues (planning placement, compute-stream priority), then every model's bench line
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for i in 1 2; do
  for cfg in "MINIPS_PLAN_AT=start" "MINIPS_PLAN_AT=head" "MINIPS_PLAN_AT=dgrad" "MINIPS_COMPUTE_PRIORITY=1"; do
    env $cfg timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4/bench_k.log 2>&1
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_k.log)"
  done
done
: > gpurun_out/r4/models_1gpu_r4.jsonl
for m in gpt2 mlp dlrm dlrm-10b widedeep-ssp; do
  timeout -k 10 400 python tools/bench_models.py --model $m --steps 50 --warmup 10 > gpurun_out/r4/model_$m.log 2>&1 || { echo "$m FAILED"; tail -5 gpurun_out/r4/model_$m.log; continue; }
  tail -1 gpurun_out/r4/model_$m.log >> gpurun_out/r4/models_1gpu_r4.jsonl
  echo "$m $(grep -o '"value": [0-9.]*' gpurun_out/r4/model_$m.log | tail -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/model_$m.log | tail -1)"
done
timeout -k 10 400 python tools/bench_models.py --model widedeep-ssp --transport onesided --steps 200 --warmup 20 > gpurun_out/r4/model_wdos.log 2>&1 && tail -1 gpurun_out/r4/model_wdos.log >> gpurun_out/r4/models_1gpu_r4.jsonl
timeout -k 10 400 python tools/bench_models.py --model dlrm-10b --consistency asp --steps 50 --warmup 10 > gpurun_out/r4/model_d10.log 2>&1 && tail -1 gpurun_out/r4/model_d10.log >> gpurun_out/r4/models_1gpu_r4.jsonl
