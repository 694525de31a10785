#!/bin/bash
# LayerNorm backward: one-wave LDS-free variant vs the 4-wave LDS-combining kernel, in GPT-2's step
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
MINIPS_LN_BWD_WAVE=1 timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py tests/test_kernels_gpu.py -x -q -k "layernorm or gpt2" --timeout 280 --timeout-method thread > gpurun_out/r4/ln_tests.log 2>&1 || { tail -40 gpurun_out/r4/ln_tests.log; exit 1; }
tail -2 gpurun_out/r4/ln_tests.log
for i in 1 2; do
  for cfg in "MINIPS_LN_BWD_WAVE=0" "MINIPS_LN_BWD_WAVE=1 MINIPS_LN_BWD_WROWS=8" "MINIPS_LN_BWD_WAVE=1 MINIPS_LN_BWD_WROWS=16" "MINIPS_LN_BWD_WAVE=1 MINIPS_LN_BWD_WROWS=32"; do
    env $cfg timeout -k 10 300 python tools/bench_models.py --model gpt2 --steps 30 --warmup 5 > gpurun_out/r4/g.log 2>&1
    echo "$cfg $(grep -o '"value": [0-9.]*' gpurun_out/r4/g.log | tail -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/g.log | tail -1)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MINIPS_LN_BWD_WAVE=1 MINIPS_LN_BWD_WROWS=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/gln -o run -- python tools/bench_models.py --model gpt2 --steps 6 --warmup 2 > gpurun_out/r4/gln.log 2>&1
python tools/prof_summary.py stats gpurun_out/r4/gln/run_kernel_stats.csv 8 --top 20 > gpurun_out/r4/gpt2_ln_wave.txt
cat gpurun_out/r4/gpt2_ln_wave.txt
