set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/r4/bench_base.log 2>&1
tail -1 gpurun_out/r4/bench_base.log
timeout -k 10 300 python tools/bench_kernels.py gemm --set wd > gpurun_out/r4/gemm_wd_base.txt 2>&1
cat gpurun_out/r4/gemm_wd_base.txt
timeout -k 10 300 python tools/bench_kernels.py gemm --set gpt2 > gpurun_out/r4/gemm_gpt2_base.txt 2>&1
cat gpurun_out/r4/gemm_gpt2_base.txt
