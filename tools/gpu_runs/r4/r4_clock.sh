#!/bin/bash
# early-step curve with the in-kernel clock probe after every step
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
: > gpurun_out/r4/curve_clock.txt
CLOCK_PROBE=1 REPEAT=2 PAUSE_S=0.01 STEPS=300 timeout -k 10 120 python tools/step_probe.py curve >> gpurun_out/r4/curve_clock.txt 2>&1
CLOCK_PROBE=1 REPEAT=2 PAUSE_S=1.0 STEPS=300 timeout -k 10 120 python tools/step_probe.py curve >> gpurun_out/r4/curve_clock.txt 2>&1
CLOCK_PROBE=1 SPIN_MS=300 STEPS=300 timeout -k 10 120 python tools/step_probe.py curve >> gpurun_out/r4/curve_clock.txt 2>&1
grep -v amdgpu.ids gpurun_out/r4/curve_clock.txt
