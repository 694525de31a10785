#!/bin/bash
# GEMM correctness (GPU tests of every layout / epilogue / tile) then the shape benchmarks.
set -eo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_tiles_gpu.py tests/test_kernels_gpu.py tests/test_nn_gpu.py tests/test_gpt2.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 || { tail -40 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
timeout -k 10 120 env MINIPS_GEMM_TILE=256 python tools/gemm_kscan.py --tag v2-256 --Ks 128,512,848,1024,4096
timeout -k 10 120 python tools/bench_gemm.py
timeout -k 10 120 python bench.py --steps 200 --warmup 5 | tail -1
