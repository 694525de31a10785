#!/bin/bash
# round 5: new deterministic reductions + owner apply tests, emulated N-rank step, v6 GEMM A/B
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_widedeep_gpu.py -x -q --timeout 120 --timeout-method thread -k "embedding_backward or owner_rows or device_counts or dgrad_permuted or widedeep or wd_ or colsum" > gpurun_out/r5/t_seg.log 2>&1 || { tail -40 gpurun_out/r5/t_seg.log; exit 1; }
tail -3 gpurun_out/r5/t_seg.log
timeout -k 10 300 python tools/bench_kernels.py gemm --set gpt2 --v4 0,6 > gpurun_out/r5/gemm_gpt2_v6.txt 2>&1 || { tail -30 gpurun_out/r5/gemm_gpt2_v6.txt; exit 1; }
cat gpurun_out/r5/gemm_gpt2_v6.txt
timeout -k 10 300 python tools/bench_kernels.py gemm --set wd --v4 0,6 --no-lib > gpurun_out/r5/gemm_wd_v6.txt 2>&1 || { tail -30 gpurun_out/r5/gemm_wd_v6.txt; exit 1; }
cat gpurun_out/r5/gemm_wd_v6.txt
bash tools/gpu_round.sh emu
