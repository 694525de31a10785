#!/bin/bash
# round-4 W&D pass 2: row-parallel embedding apply in lookup order (the default path now), the
# one-sided fences moved into one 64-workgroup kernel, inbox memory A/B; then kernel traces
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_onesided_consistency.py tests/test_onesided.py tests/test_widedeep_gpu.py -x -v -m gpu -k "rows_emb or fused_emb or onesided or torn or bf16_rows or basic_map or async or owner_apply or widedeep" --timeout 240 --timeout-method thread > gpurun_out/r4/wd2_tests.log 2>&1 || { tail -60 gpurun_out/r4/wd2_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4/wd2_tests.log | tail -3
for i in 1 2; do
  for v in 1 0; do
    MINIPS_ROWS_ADAGRAD=$v timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/r4/bench_rows$v.log 2>&1
    echo "rows_adagrad=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_rows$v.log)"
  done
done
for e in "MINIPS_PS_INBOX_MEM=2" "MINIPS_PS_INBOX_MEM=0" "MINIPS_PS_INBOX_MEM=1"; do
  env $e timeout -k 10 200 python tools/bench_models.py --model widedeep-ssp --transport onesided --steps 50 --warmup 10 > gpurun_out/r4/wd_os.log 2>&1
  echo "onesided $e $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/wd_os.log)"
done
timeout -k 10 200 python tools/bench_models.py --model widedeep-ssp --steps 50 --warmup 10 > gpurun_out/r4/wd_coll.log 2>&1
echo "collective ssp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/wd_coll.log)"
bash tools/gpu_runs/r4/r4_prof.sh
bash tools/gpu_runs/r4/r4_markers.sh
timeout -k 10 500 python tools/bench_models.py --model dlrm-10b --steps 30 --warmup 5 > gpurun_out/r4/dlrm10b_os.log 2>&1
echo "dlrm-10b onesided: $(tail -1 gpurun_out/r4/dlrm10b_os.log)"
