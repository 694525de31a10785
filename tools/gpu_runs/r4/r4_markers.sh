#!/bin/bash
# roctx ranges (MINIPS_ROCTX=1) of the W&D step under rocprofv3 --marker-trace: collective BSP (the
# headline) and one-sided SSP (the owner's apply batches from the native server thread)
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
d=gpurun_out/r4/mk_bsp; rm -rf $d
MINIPS_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $d -o run -- python bench.py --steps 30 --warmup 5 > $d.log 2>&1
f=$(find $d -name "*marker_api_trace.csv" | head -1)
head -2 "$f" > gpurun_out/r4/mk_bsp_head.txt
python tools/prof_summary.py markers "$f" --steps 35 > gpurun_out/r4/mk_bsp.txt
cat gpurun_out/r4/mk_bsp.txt
d=gpurun_out/r4/mk_os; rm -rf $d
MINIPS_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $d -o run -- python tools/bench_models.py --model widedeep-ssp --transport onesided --steps 30 --warmup 5 > $d.log 2>&1
f=$(find $d -name "*marker_api_trace.csv" | head -1)
python tools/prof_summary.py markers "$f" --steps 35 > gpurun_out/r4/mk_os.txt
cat gpurun_out/r4/mk_os.txt
