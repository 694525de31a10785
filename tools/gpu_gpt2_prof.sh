set -eo pipefail
cd /root/repo
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python tools/bench_models.py --model gpt2 --steps 10 --warmup 3 > gpurun_out/gpt2_bench.log 2>&1
tail -1 gpurun_out/gpt2_bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd /root/repo
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gpt2 -o run -- python tools/bench_models.py --model gpt2 --steps 4 --warmup 2 > gpurun_out/prof_gpt2.log 2>&1
f=$(find gpurun_out/prof_gpt2 -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py $f 6 > gpurun_out/gpt2_kernels.txt
head -30 gpurun_out/gpt2_kernels.txt
