#!/bin/bash
# kernel stats + timeline of the final tree's W&D step
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/r4/prof_final
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python bench.py --steps 60 --warmup 10 > $d.log 2>&1
python tools/prof_summary.py stats $d/run_kernel_stats.csv 70 --top 30 > gpurun_out/r4/prof_final_stats.txt
python tools/prof_summary.py trace $d/run_kernel_trace.csv --anchor adam_kernel --skip 8 --timeline > gpurun_out/r4/prof_final_trace.txt
head -40 gpurun_out/r4/prof_final_stats.txt
