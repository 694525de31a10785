#!/bin/bash
# Interleaved A/B of env knobs on the 1-GPU W&D bench: ROUNDS rounds over all variants, so slow
# drift of the box hits every variant alike; prints each run and the per-variant median.
set -eo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
IFS=';' read -ra VARIANTS <<< "${AB:-X=0}"
: > gpurun_out/ab3.txt
for r in $(seq ${ROUNDS:-3}); do
  for v in "${VARIANTS[@]}"; do
    env $v timeout -k 10 200 python bench.py --steps ${STEPS:-50} --warmup 10 ${BENCH_ARGS} > gpurun_out/ab.log 2>&1
    python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'])" | tee -a gpurun_out/ab3.txt
  done
done
python - <<'PY'
import collections, statistics
d = collections.defaultdict(list)
for line in open("gpurun_out/ab3.txt"):
    k, v = line.rsplit(" ", 1)
    d[k].append(float(v))
for k, vs in d.items():
    print(f"median {statistics.median(vs):.4f}  {k}  ({' '.join(f'{x:.4f}' for x in vs)})")
PY
