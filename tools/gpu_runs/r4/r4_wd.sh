#!/bin/bash
# round-4 W&D pass: kernel numerics of the row-parallel embedding apply, the one-sided GPU tests
# (coarse shards + explicit release / acquire), then A/B bench lines
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_onesided_consistency.py tests/test_onesided.py -x -v -m gpu -k "rows_emb or fused_emb or onesided or torn or bf16_rows or basic_map or async or owner_apply" --timeout 240 --timeout-method thread > gpurun_out/r4/wd_tests.log 2>&1 || { tail -60 gpurun_out/r4/wd_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4/wd_tests.log | tail -3
for i in 1 2; do
  for v in 1 0; do
    MINIPS_ROWS_ADAGRAD=$v timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/r4/bench_rows$v.log 2>&1
    echo "rows_adagrad=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_rows$v.log)"
  done
done
for e in "MINIPS_PS_SHARD_MEM=0" "MINIPS_PS_SHARD_MEM=1" "MINIPS_PS_LOCKS=0"; do
  env $e timeout -k 10 200 python tools/bench_models.py --model widedeep-ssp --transport onesided --steps 50 --warmup 10 > gpurun_out/r4/wd_os.log 2>&1
  echo "onesided $e $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/wd_os.log)"
done
