#!/bin/bash
# Kernel traces of the one-rank W&D bench, eager vs HIP-graph replay, with the steady-state step
# breakdown (tools/trace_steps.py: wall vs GPU-busy union, per-queue busy, kernels by time).
set -eo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for g in ${MODES:-0 1}; do
  d=gpurun_out/trace_g$g
  rm -rf $d
  (cd /tmp && export TMPDIR=/tmp; cd - >/dev/null
   MINIPS_GRAPH=$g timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python bench.py --steps 30 --warmup 5 ${BENCH_ARGS} > $d.log 2>&1)
  f=$(find $d -name "*kernel_trace.csv" | head -1)
  echo "=== MINIPS_GRAPH=$g ($f)"
  python tools/trace_steps.py "$f" --anchor adam_kernel --skip 8 --top ${TOP:-30} | tee $d.summary.txt
done
