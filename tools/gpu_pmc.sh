#!/bin/bash
# PMC passes (each its own run, <= 8 SQ counters) over tools/gemm_pmc.py; summaries under gpurun_out/pmc.
set -eo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_MFMA --output-format csv -d gpurun_out/pmc/p1 -o run -- python tools/gemm_pmc.py > gpurun_out/pmc/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_LDS_ADDR_CONFLICT SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc/p2 -o run -- python tools/gemm_pmc.py > gpurun_out/pmc/p2.log 2>&1
python tools/pmc_summary.py $(find gpurun_out/pmc -name "*counter_collection.csv")
