set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 -k "kmeans" > gpurun_out/km_test.log 2>&1 || { tail -40 gpurun_out/km_test.log; exit 1; }
tail -2 gpurun_out/km_test.log
timeout -k 10 300 python tools/bench_models.py --model kmeans --steps 10 --warmup 3 2>&1 | grep '^{'
timeout -k 10 300 python tools/bench_models.py --model dlrm-10b --steps 10 --warmup 3 2>&1 | tail -3
timeout -k 10 300 python tools/bench_models.py --model dlrm --steps 10 --warmup 3 2>&1 | grep '^{'
