#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
SH="wd.wgrad3:256:512:16384:tn,wd.wgrad2:512:1024:16384:tn,wd.wgrad1:1024:896:16384:tn"
for t in 0 256; do
  for b in 320 256 512; do
    MINIPS_WGRAD_TILE=$t MINIPS_WGRAD_BLOCKS=$b timeout -k 10 200 python tools/bench_kernels.py gemm --no-lib --shapes "$SH" > gpurun_out/r4/wt.txt 2>&1
    echo "tile=$t blocks=$b $(grep -o 'sum: .*' gpurun_out/r4/wt.txt)"; grep "wd.wgrad" gpurun_out/r4/wt.txt
  done
done
for i in 1 2; do
  for cfg in "MINIPS_WGRAD_TILE=0" "MINIPS_WGRAD_TILE=256" "MINIPS_WGRAD_TILE=256 MINIPS_WD_WGRAD_BLOCKS=256"; do
    env $cfg timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4/bt.log 2>&1
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bt.log)"
  done
done
