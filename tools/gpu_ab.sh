#!/bin/bash
# A/B of env knobs on the 1-GPU W&D bench: each variant 2 runs, ms/step printed.
set -eo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
IFS=';' read -ra VARIANTS <<< "${AB:-X=0}"
for v in "${VARIANTS[@]}"; do
  for i in 1 2; do
    env $v timeout -k 10 200 python bench.py --steps 50 --warmup 10 ${BENCH_ARGS} > gpurun_out/ab.log 2>&1
    python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'])"
  done
done
