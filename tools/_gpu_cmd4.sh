set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for m in gpt2 mlp dlrm; do for v in 0 256 0 256; do echo "== $m MINIPS_GEMM_TILE=$v" ; MINIPS_GEMM_TILE=$v timeout -k 10 300 python tools/bench_models.py --model $m --steps 40 --warmup 5 > gpurun_out/g3.log 2>&1 || { tail -20 gpurun_out/g3.log; exit 1; }; grep '^{' gpurun_out/g3.log | cut -c 1-150; done; done
