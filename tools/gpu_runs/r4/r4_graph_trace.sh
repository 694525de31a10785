#!/bin/bash
# kernel timeline of HIP-graph replays of the W&D step (MINIPS_GRAPH=1)
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/r4/tr_graph
MINIPS_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python bench.py --steps 30 --warmup 5 > $d.log 2>&1
python tools/prof_summary.py trace $d/run_kernel_trace.csv --anchor adam_kernel --skip 8 --timeline > gpurun_out/r4/tr_graph.txt
cat gpurun_out/r4/tr_graph.txt
