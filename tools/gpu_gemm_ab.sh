#!/bin/bash
# bench_gemm for the current build and (if present) an alternative kernel .so, interleaved lines.
set -eo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/gemm_a.log 2>&1
if [ -f build/alt_kernels.so ]; then
  cp minips_amd/_kernels.cpython-310-x86_64-linux-gnu.so /tmp/cur.so
  cp build/alt_kernels.so minips_amd/_kernels.cpython-310-x86_64-linux-gnu.so
  timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/gemm_b.log 2>&1
  cp /tmp/cur.so minips_amd/_kernels.cpython-310-x86_64-linux-gnu.so
  paste -d'\n' gpurun_out/gemm_a.log gpurun_out/gemm_b.log | grep -v amdgpu
else
  grep -v amdgpu gpurun_out/gemm_a.log
fi
