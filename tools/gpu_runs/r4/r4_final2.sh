#!/bin/bash
# closing GPU pass: whole GPU suite (incl. the round-4 kernel tests), smoke, headline bench,
# then the one-sided push-stream A/B
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r4/final2_tests.log 2>&1 || { tail -60 gpurun_out/r4/final2_tests.log; exit 1; }
tail -2 gpurun_out/r4/final2_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/final2_smoke.log 2>&1 && tail -1 gpurun_out/r4/final2_smoke.log
timeout -k 10 200 python bench.py > gpurun_out/r4/final2_bench_default.log 2>&1 && tail -1 gpurun_out/r4/final2_bench_default.log
timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4/final2_bench_300.log 2>&1 && tail -1 gpurun_out/r4/final2_bench_300.log
STEPS=300 timeout -k 10 120 python tools/step_probe.py issue > gpurun_out/r4/final2_issue.txt 2>&1 && grep rep gpurun_out/r4/final2_issue.txt
MINIPS_PS_PUSH_STREAM=1 timeout -k 10 600 python -u -m pytest tests/test_onesided.py tests/test_onesided_consistency.py -x -q -m gpu --timeout 280 --timeout-method thread > gpurun_out/r4/pst_tests.log 2>&1 || { tail -40 gpurun_out/r4/pst_tests.log; exit 1; }
tail -2 gpurun_out/r4/pst_tests.log
for i in 1 2; do
  for cfg in "MINIPS_PS_PUSH_STREAM=0" "MINIPS_PS_PUSH_STREAM=1"; do
    env $cfg timeout -k 10 300 python tools/bench_models.py --model widedeep-ssp --transport onesided --steps 200 --warmup 20 > gpurun_out/r4/w.log 2>&1
    echo "wd-ssp-os $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/w.log | tail -1)"
    env $cfg timeout -k 10 400 python tools/bench_models.py --model dlrm-10b --steps 100 --warmup 20 > gpurun_out/r4/d.log 2>&1
    echo "dlrm-10b $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/d.log | tail -1)"
  done
done
