#!/bin/bash
# whole GPU suite at 8 HW queues, smoke, SSP transports (8 vs 4 queues), headline bench
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r4/full2_tests.log 2>&1 || { tail -60 gpurun_out/r4/full2_tests.log; exit 1; }
tail -2 gpurun_out/r4/full2_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke2.log 2>&1 && tail -1 gpurun_out/r4/smoke2.log
for q in 8 4; do
  for t in onesided collective; do
    MINIPS_HW_QUEUES=$q timeout -k 10 200 python tools/bench_models.py --model widedeep-ssp --transport $t --steps 200 --warmup 20 > gpurun_out/r4/wd_ssp_$t.log 2>&1
    echo "q=$q ssp $t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/wd_ssp_$t.log)"
  done
  MINIPS_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4/bench_q$q.log 2>&1
  echo "q=$q bsp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_q$q.log)"
done
timeout -k 10 200 python bench.py > gpurun_out/r4/bench_default.log 2>&1
tail -1 gpurun_out/r4/bench_default.log
