#!/bin/bash
# v5 (ping-pong 256x256) GEMM: correctness (every layout, tails, split-K, batched), then v2 vs v5
# vs hipBLASLt on the W&D and GPT-2 shapes, then the W&D step with v5 where the 256 tile is picked
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gemm_tiles_gpu.py -x -q -k "env0" --timeout 280 > gpurun_out/r4/v5_test.log 2>&1 || { tail -30 gpurun_out/r4/v5_test.log; exit 1; }
tail -2 gpurun_out/r4/v5_test.log
timeout -k 10 300 python tools/bench_kernels.py gemm --set wd --v4 0,4 > gpurun_out/r4/gemm_wd_v5.txt 2>&1
cat gpurun_out/r4/gemm_wd_v5.txt
timeout -k 10 400 python tools/bench_kernels.py gemm --set gpt2 --v4 0,4 > gpurun_out/r4/gemm_gpt2_v5.txt 2>&1
cat gpurun_out/r4/gemm_gpt2_v5.txt
for m in 0 3 4; do
  MINIPS_GEMM_V4=$m timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/r4/bench_v5_$m.log 2>&1
  echo "v4mode=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_v5_$m.log)"
done
