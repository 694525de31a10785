set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
TAG=v1 timeout -k 10 200 python tools/sweep_wgrad.py > gpurun_out/sweep_v1.log 2>&1
TAG=v2t128 MINIPS_GEMM_WGRAD_V2=1 MINIPS_GEMM_TILE=128 timeout -k 10 200 python tools/sweep_wgrad.py > gpurun_out/sweep_v2a.log 2>&1
TAG=v2t256 MINIPS_GEMM_WGRAD_V2=1 MINIPS_GEMM_TILE=256 timeout -k 10 200 python tools/sweep_wgrad.py > gpurun_out/sweep_v2b.log 2>&1
cat gpurun_out/sweep_v*.log | grep -v amdgpu.ids
