#!/bin/bash
# is the depth-lookahead loss drift float-atomic order (bias-vector column sums) or a race?
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for b in ext vec; do
  MINIPS_WD_BIAS=$b timeout -k 10 300 python -u -m pytest tests/test_widedeep_gpu.py -x -q -k "lookahead_depth" --timeout 280 --timeout-method thread > gpurun_out/r4/det_$b.log 2>&1 && echo "bias=$b pass" || { echo "bias=$b FAIL"; grep -o "assert 0.000[0-9]* < 0.0001" gpurun_out/r4/det_$b.log | head -2; }
done
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u -m pytest tests/test_widedeep_gpu.py -x -q -k "lookahead_depth" --timeout 280 --timeout-method thread > gpurun_out/r4/det_q$q.log 2>&1 && echo "hwq=$q pass" || { echo "hwq=$q FAIL"; grep -o "assert 0.000[0-9]* < 0.0001" gpurun_out/r4/det_q$q.log | head -2; }
done
