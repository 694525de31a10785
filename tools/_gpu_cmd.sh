set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2 3; do for v in mm addmm; do echo "gpt2 $v $(MINIPS_LM_WGRAD=$v timeout -k 10 300 python tools/bench_models.py --model gpt2 --steps 10 --warmup 3 2>&1 | grep '^{' | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; done; done
