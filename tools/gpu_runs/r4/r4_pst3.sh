#!/bin/bash
# which fence-free hand-off the push stream depends on: planning-stream events vs the rest
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
MINIPS_PS_PUSH_STREAM=1 MINIPS_FAST_PLAN_EVENTS=0 timeout -k 10 300 python -u -m pytest tests/test_multirank_gpu.py -x -q -k "ssp_world4" --timeout 280 --timeout-method thread > gpurun_out/r4/pst3.log 2>&1; echo "push stream + system-fence plan/feeder events: rc=$?"; tail -2 gpurun_out/r4/pst3.log | cut -c1-200
