#!/bin/bash
# rocprofv3 kernel stats of bench.py (W&D) and of one model bench; summaries into gpurun_out/.
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wd -o run -- python bench.py --steps 10 --warmup 3 > gpurun_out/prof_wd.log 2>&1
python tools/prof_summary.py gpurun_out/prof_wd/run_kernel_stats.csv 13 > gpurun_out/prof_wd/summary.txt
for m in ${PROF_MODELS:-gpt2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$m -o run -- python tools/bench_models.py --model $m --steps 3 --warmup 1 > gpurun_out/prof_$m.log 2>&1
  python tools/prof_summary.py gpurun_out/prof_$m/run_kernel_stats.csv 4 > gpurun_out/prof_$m/summary.txt
done
