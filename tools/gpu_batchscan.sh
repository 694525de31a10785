#!/bin/bash
# Host- vs GPU-bound check for the W&D step: bench.py at several per-GPU batches (a flat ms/step
# as the batch shrinks means the host issue rate is the limit), then the new GPU tests.
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for b in 4096 8192 16384 32768; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --batch $b > gpurun_out/scan_$b.log 2>&1 || { tail -20 gpurun_out/scan_$b.log; exit 1; }
  tail -1 gpurun_out/scan_$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($b, d['ms_per_step'], d['value'])"
done
timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -k kmeans -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_km.log 2>&1 || { tail -30 gpurun_out/pytest_km.log; exit 1; }
tail -2 gpurun_out/pytest_km.log
