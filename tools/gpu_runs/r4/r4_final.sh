#!/bin/bash
# final-tree GPU pass: whole GPU suite, smoke, headline bench (driver defaults and 300 steps), models
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r4/final_tests.log 2>&1 || { tail -60 gpurun_out/r4/final_tests.log; exit 1; }
tail -2 gpurun_out/r4/final_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/final_smoke.log 2>&1 && tail -1 gpurun_out/r4/final_smoke.log
timeout -k 10 200 python bench.py > gpurun_out/r4/final_bench_default.log 2>&1 && tail -1 gpurun_out/r4/final_bench_default.log
timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4/final_bench_300.log 2>&1 && tail -1 gpurun_out/r4/final_bench_300.log
: > gpurun_out/r4/final_models.jsonl
for m in gpt2 widedeep-ssp; do
  timeout -k 10 400 python tools/bench_models.py --model $m --steps 100 --warmup 20 > gpurun_out/r4/fm_$m.log 2>&1 && tail -1 gpurun_out/r4/fm_$m.log >> gpurun_out/r4/final_models.jsonl
done
timeout -k 10 400 python tools/bench_models.py --model widedeep-ssp --transport onesided --steps 200 --warmup 20 > gpurun_out/r4/fm_wdos.log 2>&1 && tail -1 gpurun_out/r4/fm_wdos.log >> gpurun_out/r4/final_models.jsonl
timeout -k 10 400 python tools/bench_models.py --model widedeep-ssp --transport collective --steps 200 --warmup 20 > gpurun_out/r4/fm_wdc.log 2>&1 && tail -1 gpurun_out/r4/fm_wdc.log >> gpurun_out/r4/final_models.jsonl
grep -o '"metric": "[^"]*"\|"ms_per_step": [0-9.]*\|"value": [0-9.]*' gpurun_out/r4/final_models.jsonl | paste - - -
