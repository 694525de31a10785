set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -m gpu -x -q -k "attention or lm_head" --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 || { tail -40 gpurun_out/pytest_sel.log; exit 1; }
tail -1 gpurun_out/pytest_sel.log
for o in "2,1" "3,2" "2,2"; do echo "occ $o: $(MINIPS_ATTN_OCC=$o timeout -k 10 120 python tools/bench_kernels.py attn | grep ours)"; done | tee gpurun_out/attn_occ.txt
timeout -k 10 200 python tools/bench_kernels.py nn > gpurun_out/micro_nn.txt 2>&1; cat gpurun_out/micro_nn.txt
for v in "MINIPS_LM_GEMM=ours MINIPS_GPT2_XENT=stats" "MINIPS_LM_GEMM=ours MINIPS_GPT2_XENT=rowwise" "MINIPS_LM_GEMM=lib" "MINIPS_LM_GEMM=lib MINIPS_ATTN_OCC=2,1"; do
  echo "$v $(env $v timeout -k 10 300 python tools/bench_models.py --model gpt2 --steps 10 --warmup 3 2>&1 | grep '^{' | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("last"))')"
done | tee gpurun_out/gpt2_lm_ab.txt
