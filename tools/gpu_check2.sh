#!/bin/bash
# Fused Adam grad-clear: kernel + W&D tests, then interleaved bench A/B against the pre-change
# numbers (same call), then the full GPU test suite and smoke.
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_widedeep_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_c2.log 2>&1 || { tail -30 gpurun_out/pytest_c2.log; exit 1; }
tail -1 gpurun_out/pytest_c2.log
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 > gpurun_out/c2_$rep.log 2>&1 || { tail -20 gpurun_out/c2_$rep.log; exit 1; }
  tail -1 gpurun_out/c2_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['value'], d['loss_last'])"
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
