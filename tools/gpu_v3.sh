set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
MINIPS_GEMM_V3_EARLY=0 timeout -k 10 400 python -u -m pytest tests/test_gemm_tiles_gpu.py -x -v --timeout 300 -k "env0" > gpurun_out/v3_test.log 2>&1 || { tail -40 gpurun_out/v3_test.log; exit 1; }
tail -2 gpurun_out/v3_test.log
MINIPS_GEMM_V3_EARLY=0 timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/bench_gemm_v3b.log 2>&1
MINIPS_GEMM_V3=0 timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/bench_gemm_v2.log 2>&1
paste -d'\n' gpurun_out/bench_gemm_v3b.log gpurun_out/bench_gemm_v2.log | grep -v amdgpu
MINIPS_GEMM_V3_EARLY=0 SPLITS=1,8,16 TAG=v3b timeout -k 10 200 python tools/sweep_wgrad.py 2>&1 | grep -v amdgpu
