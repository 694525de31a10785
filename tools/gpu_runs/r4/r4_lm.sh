#!/bin/bash
# LM-head GEMMs: v2 vs v5 vs hipBLASLt at several K splits (the dgrad is K = 50304)
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for sp in 4 8 12; do
  timeout -k 10 300 python tools/bench_kernels.py gemm --shapes "g.lm.d:8192:768:50304:nn" --split $sp --v4 0,4 2>&1 | grep -v amdgpu.ids | sed "s/^/split $sp /"
done
timeout -k 10 300 python tools/bench_kernels.py gemm --shapes "g.lm.f:8192:50304:768:nt,g.fc2.d:8192:3072:768:nn,g.qkv.d:8192:768:2304:nn" --split 1 --v4 0,4 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python tools/bench_kernels.py gemm --shapes "g.qkv.d:8192:768:2304:nn,g.fc.d:8192:768:3072:nn" --split 3 --v4 0,4 2>&1 | grep -v amdgpu.ids | sed "s/^/split 3 /"
