#!/bin/bash
# round-4 W&D pass 3: numerics of the row-parallel embedding apply (both layouts) and the split-K
# fold, then the headline step A/B: rows apply on/off x fold on/off (interleaved, 2 rounds)
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_widedeep_gpu.py tests/test_onesided.py tests/test_onesided_consistency.py -x -q -m gpu -k "widedeep or adagrad or emb or onesided or torn or lazy" --timeout 280 --timeout-method thread > gpurun_out/r4/wd3_tests.log 2>&1 || { tail -60 gpurun_out/r4/wd3_tests.log; exit 1; }
tail -2 gpurun_out/r4/wd3_tests.log
for i in 1 2; do
  for cfg in "MINIPS_PERSIST_PUSH=1" "MINIPS_PERSIST_PUSH=0"; do
    env $cfg timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4/bench_ab.log 2>&1
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_ab.log)"
  done
done
for e in "MINIPS_PS_INBOX_MEM=2" "MINIPS_PS_INBOX_MEM=0"; do
  env $e timeout -k 10 200 python tools/bench_models.py --model widedeep-ssp --transport onesided --steps 100 --warmup 10 > gpurun_out/r4/wd_os.log 2>&1
  echo "onesided ssp $e $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/wd_os.log)"
done
timeout -k 10 200 python tools/bench_models.py --model widedeep-ssp --steps 100 --warmup 10 > gpurun_out/r4/wd_coll.log 2>&1
echo "collective ssp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/wd_coll.log)"
