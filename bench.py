#!/usr/bin/env python3
"""Headline benchmark: samples/sec (whole node) of Criteo-shaped Wide&Deep under BSP on the
MI355X parameter server (BASELINE.json metric), one process per GPU.

    python bench.py --gpus 1 --steps 50 --warmup 10
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 50 --warmup 10

Per-GPU batch is fixed (weak scaling). Every timed step does the full PS superstep: synthetic
batch generation on the GPU, sparse Get (dedupe + all-to-all), deep-tower forward/backward,
sparse + dense Add, and the Clock (all-to-all of gradient rows + row-wise Adagrad on the
owner shards, reduce-scatter + Adam + all-gather of the dense tower). Rank 0 prints one JSON
line; `value` is the whole-job throughput and the time is the max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# 8 HIP hardware queues (the step's 6-7 streams otherwise share 4 and serialise; see
# minips_amd/__init__.py): HIP reads this when torch loads it, so before the torch import
if "--host-phases" in sys.argv:  # before the package import: metrics reads it once
    os.environ["MINIPS_ROCTX"] = "host"
if os.environ.get("GPU_MAX_HW_QUEUES", "4") == "4":  # unset or HIP's default (the GPU box exports 4)
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("MINIPS_HW_QUEUES", "8")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "samples/sec (whole node) Criteo-shaped Wide&Deep BSP at 1/2/4/8 MI355X"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16384, help="per-GPU batch (weak scaling)")
    ap.add_argument("--consistency", default="bsp", choices=["bsp", "ssp", "asp"])
    ap.add_argument("--staleness", type=int, default=0)
    ap.add_argument("--test-cards", default="", help=argparse.SUPPRESS)
    ap.add_argument("--profile-steps", type=int, default=0,
                    help="after the timed run: host issue time per step and a cProfile of N more steps (stderr)")
    ap.add_argument("--bucket_mb", type=float, default=0.0,
                    help="several ranks: dense-clock bucket size in MB (layers merged from the last one; 0 = one "
                         "reduce-scatter + all-gather after the backward)")
    ap.add_argument("--host-phases", type=int, default=0,
                    help="after the timed region: this many steps with per-phase host issue time (stderr)")
    ap.add_argument("--diag-steps", type=int, default=None,
                    help="after the timed run: N more steps with per-collective timing and the host-sync audit, "
                         "reported in the JSON line under 'diag' (default 10 with several ranks, else 0)")
    ap.add_argument("--nccl-algo", default=None,
                    help="RCCL algorithm selection passed through as NCCL_ALGO (e.g. Ring, Tree; "
                         "tools/bench_kernels.py rccl measures the choices against the 7-link bound)")
    ap.add_argument("--nccl-proto", default=None, help="RCCL protocol passed through as NCCL_PROTO (Simple, LL, LL128)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="one process emulates rank --emulate-rank of an N-rank job: tables sized and routed as "
                         "that rank, every world > 1 code path, collectives replaced by loopback copies of the "
                         "same bytes (ps.comm.LoopbackComm; wire time excluded). Reports per-rank throughput")
    ap.add_argument("--emulate-rank", type=int, default=0)
    ap.add_argument("--emu-wire", default=None, choices=["none", "ring", "direct"],
                    help="emulated world: model each collective's link time (LoopbackComm wire model, SURVEY "
                         "§5.8: 7 xGMI links of --emu-link-gbps; RS/AG ring or direct) as a device spin")
    ap.add_argument("--emu-link-gbps", type=float, default=None)
    ap.add_argument("--lookahead", type=int, default=0,
                    help="batches generated + key-planned ahead (0: feeder.default_depth, 2)")
    ap.add_argument("--sync-audit", type=int, default=0,
                    help="after the timed run: N more steps under minips_amd.utils.syncaudit (host issue time, "
                         "host syncs per step and their call sites; one '[sync-audit] {json}' line per rank, stderr)")
    args = ap.parse_args()

    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig
    from minips_amd.ps.comm import init_distributed

    for k, v in (("NCCL_ALGO", args.nccl_algo), ("NCCL_PROTO", args.nccl_proto)):
        if v:  # read by RCCL when the communicator is created
            os.environ[k] = v
    if args.emulate_world > 1:
        from minips_amd.ps.comm import LoopbackComm

        init_distributed()  # (one process: device selection only)
        comm = LoopbackComm(args.emulate_world, args.emulate_rank, wire=args.emu_wire, link_gbps=args.emu_link_gbps)
    else:
        comm = init_distributed()
    n = comm.world
    emulated = comm.emulated
    if n != args.gpus and comm.rank == 0 and not emulated:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {n}", file=sys.stderr)
    dev = comm.device

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    cfg = WideDeepConfig(consistency=args.consistency, staleness=args.staleness, bucket_mb=args.bucket_mb)
    if args.test_cards:  # CPU/gloo plumbing tests only: a small table, NOT the benchmark config
        cfg.cards = [int(c) for c in args.test_cards.split(",")]
    model = WideDeep(cfg, comm)
    data = CriteoSynth(args.batch, cards=cfg.cards, device=dev, seed=1000 + comm.rank)

    # the step runs on its own stream; batches are generated (and their keys routed) on the
    # planning stream, LOOKAHEAD steps ahead (minips_amd/models/feeder.py)
    from minips_amd.models.feeder import LookaheadFeeder
    from minips_amd.models.layers import compute_priority

    if dev.type == "cuda":
        main_stream = torch.cuda.Stream(device=dev, priority=compute_priority())
        main_stream.wait_stream(torch.cuda.default_stream(dev))  # model init ran on the default stream
        torch.cuda.set_stream(main_stream)
    feeder = LookaheadFeeder(model, data, comm, depth=args.lookahead or None)
    step = feeder.step
    loss0 = None
    for i in range(args.warmup):
        l = step()
        if i == 0:
            loss0 = float(l.item()) / args.batch
    model.drain()
    sync()
    comm.barrier()
    sync()
    wire0 = getattr(comm, "wire_us", 0.0)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        l = step()
    model.drain()
    sync()
    comm.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if n > 1 and comm.initialized:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    loss_last = float(l.item()) / args.batch
    samples = args.batch * (1 if emulated else n) * args.steps
    value = samples / elapsed
    # diagnostics AFTER the timed region (the timed steps ran without any of this): bytes and
    # achieved GB/s per collective kind, host issue time and host syncs per step -- so a multi-GPU
    # run explains its own number (comm-bound vs host-bound vs compute-bound)
    diag_steps = args.diag_steps if args.diag_steps is not None else (10 if n > 1 else 0)
    diag = None
    if diag_steps > 0:
        from minips_amd.utils.syncaudit import SyncAudit

        comm.timing = []
        t1 = time.perf_counter()
        with SyncAudit() as audit:
            for _ in range(diag_steps):
                audit.step_begin()
                step()
                audit.step_end()
        model.drain()
        sync()
        wall = time.perf_counter() - t1
        rep = audit.report(wall)
        diag = dict(steps=diag_steps, wall_ms_per_step=rep["wall_ms_per_step"],
                    host_issue_ms_per_step=rep["host_issue_ms_median"], host_syncs_per_step=rep["syncs_per_step"],
                    collectives=comm.timing_report(diag_steps))
        comm.timing = None
        if n > 1 and comm.initialized:  # rank 0 reports the slowest rank's host issue time
            hi = torch.tensor([rep["host_issue_ms_median"]], dtype=torch.float64, device=dev)
            dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            diag["host_issue_ms_per_step_max_rank"] = round(float(hi.item()), 4)
    if emulated:
        wire = ("wire time excluded" if comm.wire == "none" else
                f"modelled wire time: {comm.wire} RS/AG, {comm.link_gbps:g} GB/s links, {comm.latency_us:g} us latency")
        parallelism = (f"EMULATED rank {comm.rank} of ps-dp{n} ({args.consistency}; one process, loopback "
                       f"collectives: the per-rank program of an N-rank step, {wire})")
    elif n == 1:
        # one rank owns every shard: Get/Add/Clock are local gathers/applies, no collective runs
        parallelism = f"ps-dp1 ({args.consistency}; single rank: local shards, no collectives)"
    else:
        parallelism = (f"ps-dp{n} ({args.consistency}" + (f" s={args.staleness}" if args.consistency != "bsp" else "")
                       + f" over {comm.backend}: a2a sparse rows, RS/AG dense)")
    if comm.rank == 0 or emulated:
        out = {
            "metric": METRIC if not emulated else
            f"samples/sec of ONE emulated rank of a {n}-rank Wide&Deep BSP step (loopback collectives)",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": 1 if emulated else n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (Criteo-Kaggle cardinalities, Zipf-like ids, 13 dense N(0,1)); random-init weights",
            "config": {
                "model": ("PLUMBING TEST (small tables, not the benchmark) " if args.test_cards else "")
                + "Wide&Deep: 26 sparse (33.76M rows, emb 32 + wide 1, row-wise Adagrad) + 13 dense; "
                "deep MLP 845-1024-512-256-1 (Adam; layer-1 bias folded, K padded to 896)",
                "global_batch": args.batch * (1 if emulated else n),
                "seq_len": None,
                "parallelism": parallelism,
                "per_gpu_batch": args.batch,
                "consistency": args.consistency,
                "world_size": comm.world,
                "backend": comm.backend,
                "bucket_mb": args.bucket_mb if n > 1 else None,
                "lookahead": feeder.depth,
                **({k.lower(): os.environ[k] for k in ("NCCL_ALGO", "NCCL_PROTO") if os.environ.get(k)}),
                **({"emulated_world": n, "emulated_rank": comm.rank, "emu_wire": comm.wire,
                    "emu_wire_us_per_step": round((comm.wire_us - wire0) / args.steps, 2)}
                   if emulated else {}),
            },
            "loss_first": round(loss0, 5) if loss0 is not None else None,
            "loss_last": round(loss_last, 5),
        }
        if diag is not None:
            out["diag"] = diag
        print(json.dumps(out), flush=True)
    if args.sync_audit > 0:  # after the timed region: host issue time + host waits per step
        from minips_amd.utils.syncaudit import SyncAudit

        t1 = time.perf_counter()
        with SyncAudit() as audit:  # the steps only: the drain + synchronize below are not step syncs
            for _ in range(args.sync_audit):
                audit.step_begin()
                step()
                audit.step_end()
        model.drain()
        sync()
        wall = time.perf_counter() - t1
        rep = dict(rank=comm.rank, world=n, backend=comm.backend, **audit.report(wall))
        print("[sync-audit] " + json.dumps(rep), file=sys.stderr, flush=True)
    if args.profile_steps > 0:  # after the timed region: host issue time per step + host hot spots
        import cProfile
        import pstats

        issue = []
        pr = cProfile.Profile()
        t1 = time.perf_counter()
        for _ in range(args.profile_steps):
            a = time.perf_counter()
            pr.enable()
            step()
            pr.disable()
            issue.append(time.perf_counter() - a)
        model.drain()
        sync()
        wall = (time.perf_counter() - t1) / args.profile_steps
        issue.sort()
        print(f"[profile] wall {wall * 1e3:.3f} ms/step (cProfile on), host issue median "
              f"{issue[len(issue) // 2] * 1e3:.3f} ms, min {issue[0] * 1e3:.3f}, max {issue[-1] * 1e3:.3f}",
              file=sys.stderr, flush=True)
        pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(25)
        pstats.Stats(pr, stream=sys.stderr).sort_stats("cumulative").print_stats(40)
    if args.host_phases > 0:  # after the timed region: inclusive host time per phase, per step
        from minips_amd.utils import metrics

        metrics.host_times_reset()
        t1 = time.perf_counter()
        for _ in range(args.host_phases):
            with metrics.phase("step"):
                step()
        issue = (time.perf_counter() - t1) / args.host_phases
        model.drain()
        sync()
        wall = (time.perf_counter() - t1) / args.host_phases
        rows = sorted(metrics.HOST_TIMES.items(), key=lambda kv: -kv[1][0])
        print(f"[host-phases] issue {issue * 1e3:.4f} ms/step, wall {wall * 1e3:.4f} ms/step "
              f"(world {n}{' emulated' if emulated else ''})", file=sys.stderr)
        for name, (ns, calls) in rows:
            print(f"[host-phases] {ns / 1e3 / args.host_phases:9.1f} us/step {calls / args.host_phases:6.2f} "
                  f"calls/step  {name}", file=sys.stderr)
        sys.stderr.flush()
    if n > 1 and comm.initialized:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
