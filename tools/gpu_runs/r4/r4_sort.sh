#!/bin/bash
# chunked planning sort (F x 4 workgroups) vs one workgroup per column; then the LN backward A/B
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_widedeep_gpu.py -x -q -m gpu -k "plan or widedeep" --timeout 280 --timeout-method thread > gpurun_out/r4/sort_tests.log 2>&1 || { tail -40 gpurun_out/r4/sort_tests.log; exit 1; }
tail -2 gpurun_out/r4/sort_tests.log
for i in 1 2; do
  for cfg in "MINIPS_PLAN_SORT=4" "MINIPS_PLAN_SORT=1"; do
    env $cfg timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4/bench_s.log 2>&1
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_s.log)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/psort -o run -- python bench.py --steps 40 --warmup 10 > gpurun_out/r4/psort.log 2>&1
python tools/prof_summary.py stats gpurun_out/r4/psort/run_kernel_stats.csv 50 --top 30 > gpurun_out/r4/psort_stats.txt
grep -i "plan\|gemm_v2_kernel<256, 256, false, false" gpurun_out/r4/psort_stats.txt
cd "$GRAFT_REPO_ROOT" && bash tools/gpu_runs/r4/r4_ln.sh
