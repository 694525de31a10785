#!/bin/bash
# push-stream loss spike: with fence-free vs system-fence events
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
MINIPS_PS_PUSH_STREAM=1 MINIPS_FAST_EVENTS=0 timeout -k 10 300 python -u -m pytest tests/test_multirank_gpu.py -x -q -k "ssp_world4" --timeout 280 --timeout-method thread > gpurun_out/r4/pst_dbg1.log 2>&1; echo "push stream + torch events: rc=$?"; tail -3 gpurun_out/r4/pst_dbg1.log | cut -c1-300
MINIPS_PS_PUSH_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_multirank_gpu.py -x -q -k "ssp_world4" --timeout 280 --timeout-method thread > gpurun_out/r4/pst_dbg2.log 2>&1; echo "push stream + fast events: rc=$?"; tail -3 gpurun_out/r4/pst_dbg2.log | cut -c1-300
