set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do for v in 256 0; do echo "== MINIPS_GPT2_LM_TILE=$v" ; MINIPS_GPT2_LM_TILE=$v timeout -k 10 300 python tools/bench_models.py --model gpt2 --steps 40 --warmup 5 > gpurun_out/g2.log 2>&1 || { tail -20 gpurun_out/g2.log; exit 1; }; grep '^{' gpurun_out/g2.log | cut -c 1-180; done; done
