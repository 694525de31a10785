#!/bin/bash
# One GPU-box pass: smoke, GPU tests, short bench, rocprofv3 kernel stats / trace, host-sync audit.
#   bash tools/gpu_round.sh [all|smoke|test|bench|prof|trace|audit]
# Every GPU step has its own time limit; any failure stops the script (set -e + &&).
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
STAGE=${1:-all}
if [[ $STAGE == all || $STAGE == smoke ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  tail -3 gpurun_out/smoke.log
fi
if [[ $STAGE == all || $STAGE == test ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q ${PYTEST_ARGS} --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
  tail -2 gpurun_out/bench.log
fi
if [[ $STAGE == all || $STAGE == prof ]]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*kernel_stats.csv" | head -3
fi
if [[ $STAGE == trace ]]; then  # per-queue kernel timeline of the default step (tools/trace_steps.py)
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o run -- python bench.py --steps 30 --warmup 5 ${BENCH_ARGS} > gpurun_out/trace.log 2>&1 || { tail -30 gpurun_out/trace.log; exit 1; }
fi
if [[ $STAGE == audit ]]; then  # host issue time + host syncs per step at world 1 (the real path) and 4 / 8 (gloo, one card)
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --sync-audit 50 > gpurun_out/audit_w1.txt 2>&1
  for w in 4 8; do
    MINIPS_SHARE_DEVICE=1 MINIPS_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $w --master-addr 127.0.0.1 --master-port 2950$w bench.py --gpus $w --steps 10 --warmup 3 \
      --batch 4096 --sync-audit 10 > gpurun_out/audit_w$w.txt 2>&1
  done
fi
