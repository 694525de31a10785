#!/bin/bash
# split-K XCD mapping (MINIPS_GEMM_ZMAP): correctness, wgrad microbench, W&D step A/B; then the
# early-step curve with a compute-bound vs memory-bound pre-load and the DPM clock levels sampled
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_gemm_tiles_gpu.py tests/test_kernels_gpu.py tests/test_widedeep_gpu.py -x -q -m gpu -k "gemm or wgrad or widedeep or fold" --timeout 280 --timeout-method thread > gpurun_out/r4/zmap_tests.log 2>&1 || { tail -40 gpurun_out/r4/zmap_tests.log; exit 1; }
tail -2 gpurun_out/r4/zmap_tests.log
SH="wd.wgrad3:256:512:16384:tn,wd.wgrad2:512:1024:16384:tn,wd.wgrad1:1024:896:16384:tn,g.wgrad.fc:3072:768:8192:tn,g.wgrad.qkv:2304:768:8192:tn"
for z in 0 1; do
  MINIPS_GEMM_ZMAP=$z timeout -k 10 200 python tools/bench_kernels.py gemm --no-lib --shapes "$SH" > gpurun_out/r4/zmap_gemm_$z.txt 2>&1
  echo "ZMAP=$z"; cat gpurun_out/r4/zmap_gemm_$z.txt
done
for i in 1 2; do
  for z in 1 0; do
    MINIPS_GEMM_ZMAP=$z timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4/bench_zmap.log 2>&1
    echo "ZMAP=$z $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4/bench_zmap.log)"
  done
done
# DPM levels every ~20 ms during the curves (all cards; ours is the one that moves)
( for i in $(seq 1 400); do
    echo "t $(date +%s.%N)"
    for f in /sys/class/drm/card*/device/pp_dpm_sclk /sys/class/drm/card*/device/pp_dpm_mclk /sys/class/drm/card*/device/pp_dpm_fclk; do
      [ -r "$f" ] && echo "$f $(tr '\n' ' ' < "$f")"
    done
    sleep 0.02
  done ) > gpurun_out/r4/dpm.txt 2>&1 &
SAMPLER=$!
echo "curve start $(date +%s.%N)" > gpurun_out/r4/curve.txt
STEPS=1500 timeout -k 10 120 python tools/step_probe.py curve >> gpurun_out/r4/curve.txt 2>&1
echo "curve gemm-spin start $(date +%s.%N)" >> gpurun_out/r4/curve.txt
SPIN_MS=300 SPIN_KIND=gemm STEPS=1500 timeout -k 10 120 python tools/step_probe.py curve >> gpurun_out/r4/curve.txt 2>&1
echo "curve mem-spin start $(date +%s.%N)" >> gpurun_out/r4/curve.txt
SPIN_MS=300 SPIN_KIND=mem STEPS=1500 timeout -k 10 120 python tools/step_probe.py curve >> gpurun_out/r4/curve.txt 2>&1
echo "curve end $(date +%s.%N)" >> gpurun_out/r4/curve.txt
kill $SAMPLER 2>/dev/null || true
cat gpurun_out/r4/curve.txt
