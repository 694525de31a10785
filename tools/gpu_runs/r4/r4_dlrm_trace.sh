#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for t in onesided collective; do
  d=gpurun_out/r4/tr_d10_$t
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python tools/bench_models.py --model dlrm-10b --transport $t --steps 30 --warmup 5 > $d.log 2>&1
  grep -o '"ms_per_step": [0-9.]*' $d.log | tail -1
  python tools/prof_summary.py trace $d/run_kernel_trace.csv --anchor interact --skip 8 --timeline > gpurun_out/r4/tr_d10_$t.txt 2>&1 || python tools/prof_summary.py trace $d/run_kernel_trace.csv --anchor adam --skip 8 --timeline > gpurun_out/r4/tr_d10_$t.txt
  head -70 gpurun_out/r4/tr_d10_$t.txt
done
