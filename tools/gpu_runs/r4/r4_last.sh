#!/bin/bash
# last GPU pass of the round: whole GPU suite, smoke, default bench
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r4/last_tests.log 2>&1 || { tail -60 gpurun_out/r4/last_tests.log | cut -c1-300; exit 1; }
tail -2 gpurun_out/r4/last_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/last_smoke.log 2>&1 && tail -1 gpurun_out/r4/last_smoke.log
timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4/last_bench.log 2>&1 && grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/last_bench.log
