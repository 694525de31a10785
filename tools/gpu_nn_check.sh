#!/bin/bash
# NN-kernel GPU tests, then the MLP / DLRM / DLRM-10B model benches (one JSON line each).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py tests/test_models_cpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_nn.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_nn.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_nn.log | head -20; exit $rc; }
for m in ${MODELS:-mlp dlrm dlrm-10b}; do
  timeout -k 10 300 python tools/bench_models.py --model $m --steps 30 --warmup 5 > gpurun_out/bench_$m.log 2>&1 || { tail -20 gpurun_out/bench_$m.log; exit 1; }
  grep "^{" gpurun_out/bench_$m.log | cut -c1-240
done
