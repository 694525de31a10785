#!/bin/bash
# round-4 GEMM v4 check: correctness (every layout, tails, split-K, batched), then v2 vs v4 vs hipBLASLt
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gemm_tiles_gpu.py -x -q -k "env0" --timeout 280 > gpurun_out/r4/v4_test.log 2>&1 || { tail -30 gpurun_out/r4/v4_test.log; exit 1; }
tail -2 gpurun_out/r4/v4_test.log
timeout -k 10 300 python tools/bench_kernels.py gemm --set wd --v4 0,2 > gpurun_out/r4/gemm_wd_v4.txt 2>&1
cat gpurun_out/r4/gemm_wd_v4.txt
timeout -k 10 400 python tools/bench_kernels.py gemm --set gpt2 --v4 0,2 > gpurun_out/r4/gemm_gpt2_v4.txt 2>&1
cat gpurun_out/r4/gemm_gpt2_v4.txt
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/r4/bench_base.log 2>&1
tail -1 gpurun_out/r4/bench_base.log
MINIPS_GEMM_V4=1 timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/r4/bench_v4.log 2>&1
tail -1 gpurun_out/r4/bench_v4.log
