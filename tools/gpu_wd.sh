#!/bin/bash
# W&D 1-GPU: bench x3 (run-to-run spread) + rocprofv3 kernel stats summary.
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 ${BENCH_ARGS} > gpurun_out/bench_$i.log 2>&1
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$i.log').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wd -o run -- python bench.py --steps 20 --warmup 3 > gpurun_out/prof_wd.log 2>&1
python tools/prof_summary.py gpurun_out/prof_wd/run_kernel_stats.csv 13 > gpurun_out/prof_wd/summary.txt
python tools/trace_steps.py gpurun_out/prof_wd/run_kernel_trace.csv --top 45 > gpurun_out/prof_wd/steps.txt
cat gpurun_out/prof_wd/steps.txt
