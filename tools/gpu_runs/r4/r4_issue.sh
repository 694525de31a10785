#!/bin/bash
# host issue after the stream-helper changes: tests, issue probe, bench
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_widedeep_gpu.py tests/test_graph_gpu.py tests/test_multirank_gpu.py -x -q -m gpu --timeout 280 --timeout-method thread > gpurun_out/r4/issue_tests.log 2>&1 || { tail -40 gpurun_out/r4/issue_tests.log; exit 1; }
tail -2 gpurun_out/r4/issue_tests.log
STEPS=300 timeout -k 10 120 python tools/step_probe.py issue > gpurun_out/r4/issue2.txt 2>&1
grep rep gpurun_out/r4/issue2.txt
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4/bench_issue.log 2>&1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_issue.log
done
SORT=tottime STEPS=300 TOP=40 timeout -k 10 120 python tools/step_probe.py cprofile > gpurun_out/r4/cprof3.txt 2>&1
