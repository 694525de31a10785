#!/bin/bash
# rocprofv3 kernel stats of the MLP (config 2) and DLRM (config 5) 1-GPU steps.
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for m in ${MODELS:-mlp dlrm}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$m -o run -- python tools/bench_models.py --model $m --steps 20 --warmup 5 > gpurun_out/prof_$m.log 2>&1
  f=$(find gpurun_out/prof_$m -name "*kernel_stats.csv" | head -1)
  python tools/prof_summary.py $f 25 > gpurun_out/${m}_kernels.txt
  grep -v amdgpu.ids gpurun_out/prof_$m.log | tail -1 | cut -c1-200
  head -22 gpurun_out/${m}_kernels.txt
done
