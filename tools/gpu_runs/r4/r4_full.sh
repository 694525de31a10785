#!/bin/bash
# round-4 full GPU pass: every GPU test, smoke, the headline bench, the DLRM-10B one-sided line
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r4/full_tests.log 2>&1 || { tail -60 gpurun_out/r4/full_tests.log; exit 1; }
tail -3 gpurun_out/r4/full_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.log 2>&1 && echo smoke ok
timeout -k 10 300 python bench.py > gpurun_out/r4/bench_default.log 2>&1
tail -1 gpurun_out/r4/bench_default.log
timeout -k 10 500 python tools/bench_models.py --model dlrm-10b --steps 30 --warmup 5 > gpurun_out/r4/dlrm10b_os.log 2>&1
tail -1 gpurun_out/r4/dlrm10b_os.log
