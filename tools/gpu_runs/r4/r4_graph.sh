#!/bin/bash
# HIP-graph replay of the whole W&D step vs eager issue, under the runtime's graph execution knobs
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r4/graph_tests.log 2>&1 || { tail -40 gpurun_out/r4/graph_tests.log; exit 1; }
tail -2 gpurun_out/r4/graph_tests.log
for i in 1 2; do
  for cfg in "MINIPS_GRAPH=0" "MINIPS_GRAPH=1"; do
    env $cfg timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4/bench_graph.log 2>&1 || { echo "$cfg FAILED"; tail -5 gpurun_out/r4/bench_graph.log; continue; }
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_graph.log)"
  done
done
bash tools/gpu_runs/r4/r4_graph_trace.sh
