#!/bin/bash
# kernel traces of the W&D step (collective BSP, the headline) and of one-sided SSP, with the
# steady-state step breakdown and one step's timeline
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
d=gpurun_out/r4/tr_bsp; rm -rf $d
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python bench.py --steps 30 --warmup 5 > $d.log 2>&1
f=$(find $d -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py trace "$f" --anchor adam_kernel --skip 8 --top 30 --timeline > gpurun_out/r4/tr_bsp.txt
head -40 gpurun_out/r4/tr_bsp.txt
d=gpurun_out/r4/tr_os; rm -rf $d
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python tools/bench_models.py --model widedeep-ssp --transport onesided --steps 30 --warmup 5 > $d.log 2>&1
f=$(find $d -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py trace "$f" --anchor wd_assemble --skip 8 --top 40 --timeline > gpurun_out/r4/tr_os.txt
head -50 gpurun_out/r4/tr_os.txt
