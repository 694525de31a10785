#!/bin/bash
# One GPU-box pass; every GPU step has its own time limit and any failure stops the script.
#   bash tools/gpu_round.sh STAGE [STAGE ...]     (stages run in the order given; default: all)
#     all          smoke + GPU tests + short bench + rocprofv3 kernel stats of the bench
#     trace        kernel trace of the W&D bench (BENCH_ARGS), with the steady-state step breakdown and
#                  one step's timeline (tools/prof_summary.py trace; ANCHOR: the kernel a step starts at)
#     lag          host launch return vs GPU start of every kernel of a steady step (tools/prof_summary.py lag)
#     audit        host issue time + host syncs per step at world 1 (the real path) and 4 / 8 (gloo, one card)
#     micro        isolated GPT-2 kernels: every GEMM shape vs hipBLASLt, memory-bound kernels, attention
#     models       bench lines of the other BASELINE configs (MODELS, default "mlp dlrm dlrm-10b gpt2")
#     models-prof  rocprofv3 kernel stats of those model steps (MODELS)
#     emu          bench.py --emulate-world N (EMU_WORLDS, default "2 8") next to N=1, kernel trace of N=EMU_PROF
#     ab           interleaved A/B: variants are ';'-separated env lists in AB, each run RUNS times (default 2)
#                  round-robin (`base`: no env; `args=<bench flags>`: extra bench.py flags); a variant may start
#                  with `tree=<dir>` to run another built tree (e.g. the
#                  previous round's, checked out and built in-tree under ab_old/). With the default CMD
#                  (bench.py, STEPS default 300) it prints ms/step per run, else the command's output tail:
#                    AB='tree=ab_old;base' bash tools/gpu_round.sh ab         (previous round vs this tree)
#                    CMD='python tools/bench_kernels.py kscan --Ks 848' AB='MINIPS_GEMM_TILE=128;MINIPS_GEMM_TILE=256'
#     host         per-phase host issue time (bench.py --host-phases) at world 1 and emulated EMU_PROF (8), and
#                  the host cost per call of c10d collectives / bindings / events (bench_kernels.py issue)
#     race         the 4-rank SSP one-sided test with the push stream on, once per MINIPS_STREAM_DEBUG variant in
#                  RACE_VARIANTS (';'-separated; a failing test goes on to the next variant, a crash stops)
#     pytest       one pytest selection: PYTEST_SEL (e.g. 'tests/test_multirank_gpu.py -k ssp'), env PYTEST_ENV
#     pmc          hardware counters of the W&D step (BENCH_ARGS), one rocprofv3 --pmc pass per counter group
#                  (8 SQ counters; FETCH_SIZE and WRITE_SIZE each alone -- one run holds at most 4 TCC
#                  counters), merged per kernel by tools/prof_summary.py pmctable (MATCH: kernel regex)
# Knobs: STEPS, BENCH_ARGS, PYTEST_ARGS, MODELS, ANCHOR, AB, RUNS, CMD, TAIL, PYTEST_SEL, PYTEST_ENV, MATCH.
# This one runner replaces the per-experiment command files of rounds 1-4 (git history keeps them).
set -eo pipefail
cd "$(dirname "$0")/.."
ROOT=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
prof_env() { cd /tmp && export TMPDIR=/tmp && cd - > /dev/null; }
for STAGE in "${@:-all}"; do
if [[ $STAGE == all || $STAGE == smoke ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  tail -3 gpurun_out/smoke.log
fi
if [[ $STAGE == all || $STAGE == test ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q ${PYTEST_ARGS} --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
  tail -2 gpurun_out/bench.log
fi
if [[ $STAGE == all || $STAGE == prof ]]; then
  prof_env
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*kernel_stats.csv" | head -3
fi
if [[ $STAGE == trace ]]; then
  prof_env
  for g in 0; do
    d=gpurun_out/trace_g$g
    rm -rf $d
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python bench.py --steps 30 --warmup 5 ${BENCH_ARGS} > $d.log 2>&1 || { tail -30 $d.log; exit 1; }
    f=$(find $d -name "*kernel_trace.csv" | head -1)
    echo "=== trace ($f)"
    python tools/prof_summary.py trace "$f" --anchor ${ANCHOR:-wd_head_kernel} --skip 8 --top ${TOP:-30} --timeline | tee $d.summary.txt
  done
fi
if [[ $STAGE == lag ]]; then
  # host launch time vs GPU start per kernel (runtime tracing adds host cost per HIP call: an upper
  # bound on how host-bound the step is)
  prof_env
  d=gpurun_out/lag
  rm -rf $d
  timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $d -o run -- python bench.py --steps 40 --warmup 5 ${BENCH_ARGS} > $d.log 2>&1 || { tail -30 $d.log; exit 1; }
  python tools/prof_summary.py lag "$(find $d -name "*kernel_trace.csv" | head -1)" "$(find $d -name "*hip_api_trace.csv" | head -1)" --anchor ${ANCHOR:-wd_head_kernel} > $d.summary.txt
  head -60 $d.summary.txt
  rm -rf $d
fi
if [[ $STAGE == audit ]]; then
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --sync-audit 50 > gpurun_out/audit_w1.txt 2>&1
  for w in 4 8; do
    MINIPS_SHARE_DEVICE=1 MINIPS_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $w --master-addr 127.0.0.1 --master-port 2950$w bench.py --gpus $w --steps 10 --warmup 3 \
      --batch 4096 --sync-audit 10 > gpurun_out/audit_w$w.txt 2>&1
  done
fi
if [[ $STAGE == micro ]]; then
  timeout -k 10 300 python tools/bench_kernels.py gemm --set gpt2 > gpurun_out/micro_gemm_gpt2.txt 2>&1
  timeout -k 10 200 python tools/bench_kernels.py nn > gpurun_out/micro_nn.txt 2>&1
  timeout -k 10 200 python tools/bench_kernels.py attn > gpurun_out/micro_attn.txt 2>&1
fi
if [[ $STAGE == models ]]; then
  for m in ${MODELS:-mlp dlrm dlrm-10b gpt2}; do
    timeout -k 10 300 python tools/bench_models.py --model $m --steps ${STEPS:-30} --warmup 5 > gpurun_out/bench_$m.log 2>&1 || { tail -20 gpurun_out/bench_$m.log; exit 1; }
    grep "^{" gpurun_out/bench_$m.log | cut -c1-300
  done
fi
if [[ $STAGE == models-prof ]]; then
  prof_env
  for m in ${MODELS:-mlp dlrm gpt2}; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$m -o run -- python tools/bench_models.py --model $m --steps 6 --warmup 2 > gpurun_out/prof_$m.log 2>&1 || { tail -20 gpurun_out/prof_$m.log; exit 1; }
    f=$(find gpurun_out/prof_$m -name "*kernel_stats.csv" | head -1)
    python tools/prof_summary.py stats $f 8 > gpurun_out/${m}_kernels.txt
    head -25 gpurun_out/${m}_kernels.txt
  done
fi
if [[ $STAGE == emu ]]; then
  # the per-rank program of an N-rank step on this one GPU (bench.py --emulate-world: loopback
  # collectives, wire time excluded) next to the one-rank step, then a kernel trace of the largest N
  timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 10 ${BENCH_ARGS} > gpurun_out/emu_w1.log 2>&1 || { tail -30 gpurun_out/emu_w1.log; exit 1; }
  grep "^{" gpurun_out/emu_w1.log | cut -c1-200
  for w in ${EMU_WORLDS:-2 8}; do
    timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 10 --emulate-world $w ${BENCH_ARGS} > gpurun_out/emu_w$w.log 2>&1 || { tail -30 gpurun_out/emu_w$w.log; exit 1; }
    grep "^{" gpurun_out/emu_w$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('emulated', $w, d['ms_per_step'], 'ms/step', json.dumps(d.get('diag')))"
  done
  prof_env
  w=${EMU_PROF:-8}
  d=gpurun_out/emu_prof_w$w
  rm -rf $d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python bench.py --steps 40 --warmup 10 --emulate-world $w --diag-steps 0 ${BENCH_ARGS} > $d.log 2>&1 || { tail -30 $d.log; exit 1; }
  python tools/prof_summary.py stats $d/run_kernel_stats.csv 50 --top 40 > $d.stats.txt
  python tools/prof_summary.py trace $d/run_kernel_trace.csv --anchor wd_head_kernel --skip 8 --top 40 > $d.trace.txt
  head -60 $d.trace.txt
fi
if [[ $STAGE == ab ]]; then
  IFS=';' read -ra VARIANTS <<< "${AB:-base}"
  for i in $(seq "${RUNS:-2}"); do
    for v in "${VARIANTS[@]}"; do
      dir=$ROOT; envs=$v; extra=""; [[ $v == base ]] && envs=""
      if [[ $v == tree=* ]]; then dir=$ROOT/${v%% *}; dir=${dir/tree=/}; envs=${v#* }; [[ $envs == tree=* ]] && envs=""; fi
      if [[ $v == args=* ]]; then extra=${v#args=}; envs=""; fi
      if [[ -z "${CMD}" ]]; then
        (cd "$dir" && env $envs timeout -k 10 300 python bench.py --steps "${STEPS:-300}" --warmup 10 ${BENCH_ARGS} $extra > $ROOT/gpurun_out/ab.log 2>&1) || { tail -20 gpurun_out/ab.log; exit 1; }
        python -c "import json; d=json.loads([l for l in open('gpurun_out/ab.log') if l.startswith('{')][-1]); print('[$v]', d['ms_per_step'])"
      else
        echo "== [$v] (run $i)"
        (cd "$dir" && env $envs timeout -k 10 300 ${CMD} > $ROOT/gpurun_out/ab.log 2>&1) || { tail -20 gpurun_out/ab.log; exit 1; }
        tail -${TAIL:-20} gpurun_out/ab.log
      fi
    done
  done
fi
if [[ $STAGE == pmc ]]; then
  prof_env
  files=()
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES" FETCH_SIZE WRITE_SIZE; do
    tag=${grp%% *}; d=gpurun_out/pmc_$tag
    rm -rf $d
    timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d $d -o run -- python bench.py --steps 6 --warmup 2 ${BENCH_ARGS} > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
    files+=("$(find $d -name "*counter_collection.csv" | head -1)")
  done
  python tools/prof_summary.py pmctable "${files[@]}" --match "${MATCH:-}" | tee gpurun_out/pmc_table.txt
fi
if [[ $STAGE == host ]]; then
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --host-phases 100 ${BENCH_ARGS} > gpurun_out/host_w1.log 2>&1 || { tail -30 gpurun_out/host_w1.log; exit 1; }
  grep "host-phases" gpurun_out/host_w1.log | head -40
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --emulate-world ${EMU_PROF:-8} --diag-steps 0 --host-phases 100 ${BENCH_ARGS} > gpurun_out/host_emu.log 2>&1 || { tail -30 gpurun_out/host_emu.log; exit 1; }
  grep "host-phases" gpurun_out/host_emu.log | head -40
  timeout -k 10 200 python tools/bench_kernels.py issue > gpurun_out/host_issue_calls.txt 2>&1 || { tail -30 gpurun_out/host_issue_calls.txt; exit 1; }
  cat gpurun_out/host_issue_calls.txt
fi
if [[ $STAGE == race ]]; then
  IFS=';' read -ra RV <<< "${RACE_VARIANTS:-none;delay=300;delay=300,where=use;delay=300,where=fork}"
  sel='tests/test_multirank_gpu.py::test_widedeep_ssp_world4_tracks_one_rank_bsp[onesided]'
  for v in "${RV[@]}"; do
    dbg=$v; [[ $v == none ]] && dbg=""
    rc=0
    MINIPS_PS_PUSH_STREAM=${PUSH:-1} MINIPS_STREAM_DEBUG="$dbg" timeout -k 10 300 python -u -m pytest "$sel" -x -q \
      --timeout 240 --timeout-method thread > gpurun_out/race.log 2>&1 || rc=$?
    echo "[race] push=${PUSH:-1} debug='$v' rc=$rc $(grep -Eo '[0-9]+ (passed|failed)[^=]*' gpurun_out/race.log | tail -1)"
    grep -Eo "AssertionError: \(.{0,200}" gpurun_out/race.log | head -2 || true
    if [[ $rc -ne 0 && $rc -ne 1 ]]; then tail -20 gpurun_out/race.log; exit 1; fi
  done
fi
if [[ $STAGE == pytest ]]; then
  env ${PYTEST_ENV} timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest ${PYTEST_SEL:-tests -m gpu} -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 || { tail -40 gpurun_out/pytest_sel.log; exit 1; }
  tail -5 gpurun_out/pytest_sel.log
fi
done
