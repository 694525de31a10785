#!/bin/bash
# PMC pass: v2 vs v5 on an nn GEMM (g.qkv.d) and an nt GEMM (g.lm.f slice): MFMA busy, LDS bank conflicts
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4/pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
C="SQ_WAVES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS"
for m in 0 4; do
  for sh in "g.lm.d:8192:768:50304:nn"; do
    d=gpurun_out/r4/pmc/m${m}_${sh%%:*}
    MINIPS_GEMM_V4=$m timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $d -o run -- python tools/bench_kernels.py one --shape $sh --reps 5 --split 8 > $d.log 2>&1 || { echo "pmc failed m=$m $sh"; tail -5 $d.log; exit 1; }
    f=$(find $d -name "*counter_collection.csv" | head -1)
    echo "== v4mode=$m $sh"
    python tools/prof_summary.py pmc "$f" | grep -A8 "gemm_v\|splitk"
  done
done
