#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_round4_gpu.py tests/test_kernels_gpu.py -x -q -m gpu -k "round4 or plan or chunked or multi_copy or clock or push" --timeout 200 --timeout-method thread > gpurun_out/r4/new_tests.log 2>&1 || { tail -40 gpurun_out/r4/new_tests.log; exit 1; }
tail -2 gpurun_out/r4/new_tests.log
bash tools/gpu_runs/r4/r4_g2tile.sh
