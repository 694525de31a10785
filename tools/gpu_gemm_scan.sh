#!/bin/bash
# K-scans of the W&D forward GEMM (M=16384, N=1024) per tile / kernel variant.
set -eo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10 120"
$T env MINIPS_GEMM_TILE=256 python tools/gemm_kscan.py --tag v2-256
$T env MINIPS_GEMM_TILE=128 python tools/gemm_kscan.py --tag v2-128
$T env MINIPS_GEMM_TILE=200 python tools/gemm_kscan.py --tag v2-256x128
$T env MINIPS_GEMM_TILE=256 MINIPS_GEMM_V3=1 python tools/gemm_kscan.py --tag v3
$T env MINIPS_GEMM_TILE=256 python tools/gemm_kscan.py --tag v2-256-nn --layout nn
$T env MINIPS_GEMM_TILE=256 python tools/gemm_kscan.py --tag v2-256-M4k --M 4096 --N 4096
