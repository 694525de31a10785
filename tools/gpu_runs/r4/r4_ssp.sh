#!/bin/bash
# fast events everywhere on the step path; one-sided vs collective SSP through the look-ahead feeder
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 500 python -u -m pytest tests/test_widedeep_gpu.py tests/test_graph_gpu.py tests/test_multirank_gpu.py tests/test_kernels_gpu.py -x -q -m gpu -k "widedeep or graph or multirank or onesided or ps_" --timeout 280 --timeout-method thread > gpurun_out/r4/ssp_tests.log 2>&1 || { tail -40 gpurun_out/r4/ssp_tests.log; exit 1; }
tail -2 gpurun_out/r4/ssp_tests.log
for i in 1 2; do
  for cfg in "MINIPS_FAST_EVENTS=1" "MINIPS_FAST_EVENTS=0"; do
    env $cfg timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4/bench_ev.log 2>&1
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_ev.log)"
  done
  for t in onesided collective; do
    timeout -k 10 200 python tools/bench_models.py --model widedeep-ssp --transport $t --steps 200 --warmup 20 > gpurun_out/r4/wd_ssp_$t.log 2>&1
    echo "ssp $t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/wd_ssp_$t.log)"
  done
done
STEPS=300 timeout -k 10 120 python tools/step_probe.py issue > gpurun_out/r4/issue3.txt 2>&1
grep rep gpurun_out/r4/issue3.txt
