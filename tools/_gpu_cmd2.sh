set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/lm_tiles.txt
: > $o
timeout -k 10 200 python tools/bench_kernels.py gemm --shapes g.lm.f:8192:50304:768:nt,g.lm.w:50304:768:8192:tn,g.lm.d:8192:768:50304:nn --split 8 >> $o 2>&1 || { tail -20 $o; exit 1; }
for T in 0 256 200 128; do echo "== tile $T (lm.f, lm.w)" >> $o; MINIPS_GEMM_TILE=$T timeout -k 10 200 python tools/bench_kernels.py gemm --no-lib --shapes g.lm.f:8192:50304:768:nt,g.lm.w:50304:768:8192:tn >> $o 2>&1 || { tail -20 $o; exit 1; }; done
for T in 0 200; do for S in 4 6 8; do echo "== tile $T split $S (lm.d)" >> $o; MINIPS_GEMM_TILE=$T timeout -k 10 200 python tools/bench_kernels.py gemm --no-lib --shapes g.lm.d:8192:768:50304:nn --split $S >> $o 2>&1 || { tail -20 $o; exit 1; }; done; done
grep -v amdgpu.ids $o
