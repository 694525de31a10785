#!/bin/bash
# which kernels carry the slow early steps: kernel trace of two 300-step curves 0.5 s apart
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
REPEAT=2 PAUSE_S=0.5 STEPS=300 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4/early -o run -- python tools/step_probe.py curve > gpurun_out/r4/early.log 2>&1 || { tail -20 gpurun_out/r4/early.log; exit 1; }
grep steps gpurun_out/r4/early.log
f=gpurun_out/r4/early/run_kernel_trace.csv
python tools/prof_summary.py early $f --windows 2-10,10-30,30-60,150-290,302-310,310-330,330-360,450-590 --top 30 > gpurun_out/r4/early.txt
cat gpurun_out/r4/early.txt
: > gpurun_out/r4/curve3.txt
for p in 0.01 0.1 1.0; do
  echo "pause $p" >> gpurun_out/r4/curve3.txt
  REPEAT=2 PAUSE_S=$p STEPS=200 timeout -k 10 120 python tools/step_probe.py curve >> gpurun_out/r4/curve3.txt 2>&1
done
cat gpurun_out/r4/curve3.txt
