#!/bin/bash
# A/B: dense clock on a side stream at one rank (MINIPS_OVERLAP_W1=dense), issued from the wgrad
# side stream (MINIPS_DENSE_CLOCK_ON_SIDE=1) or behind the sparse push (=0); then the W&D and
# multi-rank GPU tests (world 2 runs the async dense clock on the new path).
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "none 1" "dense 1" "dense 0"; do
    set -- $cfg
    MINIPS_OVERLAP_W1=$1 MINIPS_DENSE_CLOCK_ON_SIDE=$2 timeout -k 10 200 python bench.py --steps 40 --warmup 5 > gpurun_out/ds.log 2>&1 || { tail -20 gpurun_out/ds.log; exit 1; }
    tail -1 gpurun_out/ds.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('w1=$1 side=$2', d['ms_per_step'], d['value'], d['loss_last'])"
  done
done
MINIPS_OVERLAP_W1=dense timeout -k 10 400 python -u -m pytest tests/test_widedeep_gpu.py tests/test_multirank_gpu.py tests/test_checkpoint_gpu_tables.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ds.log 2>&1 || { tail -30 gpurun_out/pytest_ds.log; exit 1; }
tail -1 gpurun_out/pytest_ds.log
