#!/bin/bash
# final-tree model bench lines
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
: > gpurun_out/r4/models_final.jsonl
for m in mlp dlrm dlrm-10b gpt2; do
  timeout -k 10 400 python tools/bench_models.py --model $m --steps 100 --warmup 20 > gpurun_out/r4/mf_$m.log 2>&1 && tail -1 gpurun_out/r4/mf_$m.log >> gpurun_out/r4/models_final.jsonl
done
for t in onesided collective; do
  timeout -k 10 400 python tools/bench_models.py --model widedeep-ssp --transport $t --steps 200 --warmup 20 > gpurun_out/r4/mf_wd_$t.log 2>&1 && tail -1 gpurun_out/r4/mf_wd_$t.log >> gpurun_out/r4/models_final.jsonl
done
grep -o '"metric": "[^"]*"\|"ms_per_step": [0-9.]*\|"value": [0-9.]*' gpurun_out/r4/models_final.jsonl | paste - - -
