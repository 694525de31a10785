#!/bin/bash
# early-step curve: host-proximity test (GPU work queued before step 0), and the host-issue profile
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
: > gpurun_out/r4/curve2.txt
for pre in 0 30; do
  PRELOAD_MS=$pre REPEAT=2 PAUSE_S=0.5 STEPS=600 timeout -k 10 120 python tools/step_probe.py curve >> gpurun_out/r4/curve2.txt 2>&1
done
cat gpurun_out/r4/curve2.txt
STEPS=300 TOP=60 timeout -k 10 120 python tools/step_probe.py cprofile > gpurun_out/r4/cprof.txt 2>&1
head -90 gpurun_out/r4/cprof.txt
