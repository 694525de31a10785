#!/bin/bash
# A/B of the HIP-graph runtime knobs on the one-rank W&D step (bench.py, graph replay).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { echo "== $*"; env "$@" timeout -k 10 120 python bench.py --steps 200 --warmup 5 | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d['ms_per_step'], d['config']['hip_graph'])" || exit 1; }
run MINIPS_GRAPH=0
run MINIPS_GRAPH=1
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run DEBUG_HIP_FORCE_GRAPH_QUEUES=1
run DEBUG_HIP_FORCE_GRAPH_QUEUES=2
run DEBUG_HIP_FORCE_GRAPH_QUEUES=4
run DEBUG_HIP_FORCE_GRAPH_QUEUES=8
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
