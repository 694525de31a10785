#!/bin/bash
# round-4 one-sided PS check on one MI355X: the GPU tests of the asynchronous tables (two processes
# share the card), then W&D SSP over the one-sided vs the collective transport
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_onesided_consistency.py tests/test_onesided.py -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r4/onesided_gpu.log 2>&1 || { tail -60 gpurun_out/r4/onesided_gpu.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r4/onesided_gpu.log | tail -20
timeout -k 10 200 python tools/bench_models.py --model widedeep-ssp --transport onesided --steps 50 --warmup 10 > gpurun_out/r4/wd_ssp_onesided.log 2>&1
grep "^{" gpurun_out/r4/wd_ssp_onesided.log | cut -c1-200
timeout -k 10 200 python tools/bench_models.py --model widedeep-ssp --transport collective --steps 50 --warmup 10 > gpurun_out/r4/wd_ssp_coll.log 2>&1
grep "^{" gpurun_out/r4/wd_ssp_coll.log | cut -c1-200
