#!/bin/bash
# SSP (s=1) one-sided vs collective under both drivers; traces of the collective/lookahead case;
# refreshed headline roofline (kernel trace of bench.py)
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for i in 1 2; do
  for fd in lookahead inline; do
    for t in onesided collective; do
      timeout -k 10 200 python tools/bench_models.py --model widedeep-ssp --transport $t --feeder $fd --steps 200 --warmup 20 > gpurun_out/r4/wd_ssp.log 2>&1
      echo "ssp $t $fd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/wd_ssp.log)"
    done
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/r4/tr_ssp_coll
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python tools/bench_models.py --model widedeep-ssp --transport collective --steps 30 --warmup 5 > $d.log 2>&1
python tools/prof_summary.py trace $d/run_kernel_trace.csv --anchor adam_kernel --skip 8 --timeline > gpurun_out/r4/tr_ssp_coll.txt
d=gpurun_out/r4/tr_ssp_os
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python tools/bench_models.py --model widedeep-ssp --transport onesided --steps 30 --warmup 5 > $d.log 2>&1
python tools/prof_summary.py trace $d/run_kernel_trace.csv --anchor wd_assemble --skip 8 --timeline > gpurun_out/r4/tr_ssp_os.txt
timeout -k 10 120 python tools/kernel_roofline.py --measure-U > gpurun_out/r4/U.txt 2>&1
cat gpurun_out/r4/U.txt
d=gpurun_out/r4/tr_head
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python bench.py --steps 60 --warmup 10 > $d.log 2>&1
U=$(grep -o "U mean [0-9]*" gpurun_out/r4/U.txt | grep -o "[0-9]*$")
python tools/kernel_roofline.py $d/run_kernel_trace.csv --U $U > gpurun_out/r4/roofline.md
python tools/prof_summary.py trace $d/run_kernel_trace.csv --anchor adam_kernel --skip 8 --timeline > gpurun_out/r4/tr_head.txt
cat gpurun_out/r4/roofline.md
