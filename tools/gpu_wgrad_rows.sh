#!/bin/bash
# A/B of MINIPS_WGRAD_MIN_ROWS_OVERLAP (reduction rows per split of side-stream wgrads), interleaved.
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2 3; do
  for mb in 2048 4096 8192; do
    MINIPS_WGRAD_MIN_ROWS_OVERLAP=$mb timeout -k 10 200 python bench.py --steps 40 --warmup 5 > gpurun_out/wb_$mb.log 2>&1 || { tail -20 gpurun_out/wb_$mb.log; exit 1; }
    tail -1 gpurun_out/wb_$mb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('min_rows $mb', d['ms_per_step'], d['value'], d['loss_last'])"
  done
done
