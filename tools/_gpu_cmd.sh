set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in 0 1; do
  d=gpurun_out/trace_fh$v; rm -rf $d
  MINIPS_WD_TRIM=0 MINIPS_WD_FUSED_HEAD=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python bench.py --steps 30 --warmup 5 > $d.log 2>&1
  f=$(find $d -name "*kernel_trace.csv" | head -1)
  echo "=== FUSED_HEAD=$v"; python tools/prof_summary.py trace "$f" --anchor adam_kernel --skip 8 --top 24
done
