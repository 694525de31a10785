#!/bin/bash
# A/B of MINIPS_OVERLAP_W1 (table kinds whose BSP clock runs on a side stream on one rank).
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2; do
  for k in none dense sparse dense,sparse; do
    MINIPS_OVERLAP_W1=$k timeout -k 10 200 python bench.py --steps 40 --warmup 5 > gpurun_out/ow_$rep.log 2>&1 || { tail -20 gpurun_out/ow_$rep.log; exit 1; }
    tail -1 gpurun_out/ow_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('overlap_w1 $k', d['ms_per_step'], d['value'], d['loss_last'])"
  done
done
