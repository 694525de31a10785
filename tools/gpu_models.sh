#!/bin/bash
# Throughput of every model on one GPU (tools/bench_models.py); each run has its own time limit.
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for m in ${MODELS:-mlp gpt2 dlrm dlrm-10b lr kmeans widedeep-ssp}; do
  timeout -k 10 300 python tools/bench_models.py --model $m --steps ${STEPS:-10} --warmup 3 > gpurun_out/bench_$m.log 2>&1 || { tail -30 gpurun_out/bench_$m.log; exit 1; }
  tail -1 gpurun_out/bench_$m.log
done
