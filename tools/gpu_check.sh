#!/bin/bash
# Quick GPU pass after a change: GPU tests (one process, per-test timeout), then bench A/B.
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
MINIPS_OVERLAP=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_nooverlap.log 2>&1 || { tail -30 gpurun_out/bench_nooverlap.log; exit 1; }
tail -1 gpurun_out/bench_nooverlap.log
