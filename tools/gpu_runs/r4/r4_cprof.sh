#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
STEPS=300 timeout -k 10 120 python tools/step_probe.py issue > gpurun_out/r4/issue.txt 2>&1
cat gpurun_out/r4/issue.txt
SORT=cumulative STEPS=300 TOP=70 CALLERS="current_stream|_get_device_index|__enter__" timeout -k 10 120 python tools/step_probe.py cprofile > gpurun_out/r4/cprof_cum.txt 2>&1
