#!/bin/bash
# Paired bf16 epilogue stores: the full GPU test suite first (GEMM numerics vs fp32 references),
# then W&D bench x3 and the GPT-2 model bench.
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_epi.log 2>&1 || { tail -40 gpurun_out/pytest_epi.log; exit 1; }
tail -1 gpurun_out/pytest_epi.log
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 > gpurun_out/epi_$rep.log 2>&1 || { tail -20 gpurun_out/epi_$rep.log; exit 1; }
  tail -1 gpurun_out/epi_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('wd', d['ms_per_step'], d['value'], d['loss_last'])"
done
timeout -k 10 300 python tools/bench_models.py --model gpt2 --steps 10 --warmup 3 > gpurun_out/epi_gpt2.log 2>&1 || { tail -20 gpurun_out/epi_gpt2.log; exit 1; }
tail -1 gpurun_out/epi_gpt2.log
timeout -k 10 300 python tools/bench_models.py --model mlp --steps 10 --warmup 3 > gpurun_out/epi_mlp.log 2>&1 || { tail -20 gpurun_out/epi_mlp.log; exit 1; }
tail -1 gpurun_out/epi_mlp.log
