#!/bin/bash
# A/B of the bench's batch/plan lookahead depth (MINIPS_LOOKAHEAD), interleaved runs, then the
# multi-rank GPU tests (bench.py under torchrun) and the W&D GPU tests.
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2; do
  for la in 1 2 3; do
    MINIPS_LOOKAHEAD=$la timeout -k 10 200 python bench.py --steps 40 --warmup 5 > gpurun_out/la_$la.log 2>&1 || { tail -20 gpurun_out/la_$la.log; exit 1; }
    tail -1 gpurun_out/la_$la.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lookahead $la', d['ms_per_step'], d['value'], d['loss_last'])"
  done
done
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py tests/test_widedeep_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_la.log 2>&1 || { tail -30 gpurun_out/pytest_la.log; exit 1; }
tail -2 gpurun_out/pytest_la.log
