#!/usr/bin/env python3
"""Throughput of the other BASELINE configurations on the GPU parameter server, with the same
timing discipline as bench.py (W untimed warmup steps, exactly K timed steps bracketed by
barrier + synchronize, max over ranks, whole-job value, one JSON line on rank 0).

    python tools/bench_models.py --model gpt2 --steps 10 --warmup 3
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_models.py --model dlrm

models: mlp (config 2, samples/s), gpt2 (config 4, tokens/s), dlrm (config 5, samples/s),
        dlrm-10b (config 5 at its per-GPU shard: 1.25B rows x 64 bf16 per GPU, ASP), lr (config 1 on GPUs,
        samples/s), kmeans (samples/s), widedeep-ssp (config 3).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# 8 HIP hardware queues (the step's 6-7 streams otherwise share 4 and serialise; see
# minips_amd/__init__.py): HIP reads this when torch loads it, so before the torch import
if os.environ.get("GPU_MAX_HW_QUEUES", "4") == "4":  # unset or HIP's default (the GPU box exports 4)
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("MINIPS_HW_QUEUES", "8")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(args, comm):
    dev = comm.device
    r = comm.rank
    if args.model == "mlp":
        from minips_amd.data.synthetic import MnistSynth
        from minips_amd.models.mlp import MLP, MLPConfig

        B = args.batch or 8192
        m = MLP(MLPConfig(consistency=args.consistency, staleness=args.staleness), comm)
        data = MnistSynth(B, device=dev, seed=r)
        use_graph = bool(args.graph) and comm.world == 1 and args.consistency == "bsp"
        if use_graph:  # launch-bound model: one HIP-graph launch per step
            from minips_amd.utils.graph import GraphedStep

            step = GraphedStep(lambda x, y: m.train_step(x, y)[0], data.next(), tables=[m.table])
            return m, (lambda: step(*data.next())), B, "samples/s", \
                dict(model="MLP 784-512-512-10 (Adam, dense PS table)", seq_len=None, hip_graph=True)
        return m, (lambda: m.train_step(*data.next())[0]), B, "samples/s", \
            dict(model="MLP 784-512-512-10 (Adam, dense PS table)", seq_len=None, hip_graph=False)
    if args.model == "gpt2":
        from minips_amd.data.synthetic import TokenSynth
        from minips_amd.models.gpt2 import GPT2, GPT2Config

        B, T = args.batch or 8, args.seq
        m = GPT2(GPT2Config(consistency=args.consistency, staleness=args.staleness), comm)
        data = TokenSynth(B, T, device=dev, seed=r)
        return m, (lambda: m.train_step(*data.next())), B * T, "tokens/s", \
            dict(model="GPT-2 small 124M (12L/768d/12H, vocab 50257), dense params sharded over PS ranks",
                 seq_len=T, batch_per_gpu=B)
    if args.model in ("dlrm", "dlrm-10b"):
        from minips_amd.models.dlrm import DLRM, DLRMConfig

        B = args.batch or 16384
        if args.model == "dlrm-10b":
            # BASELINE config 5: a 10B-row table over 8 GPUs = 1.25B rows (x 16 fp32 + row-wise
            # Adagrad state = 85 GB) per GPU; weak scaling keeps the per-GPU shard fixed
            rows = args.rows_per_gpu * comm.world
            cfg = DLRMConfig(num_rows=rows, D=args.dim, consistency=args.consistency if args.consistency != "bsp"
                             else "asp", staleness=args.staleness, transport=args.transport, max_batch=B)
        else:
            cfg = DLRMConfig(num_rows=args.rows, consistency=args.consistency, staleness=args.staleness,
                             transport=args.transport, max_batch=B)
        m = DLRM(cfg, comm)
        from minips_amd.data.synthetic import DLRMSynth

        gen = DLRMSynth(B, cfg.F, cfg.num_rows, cfg.n_dense, device=dev, seed=r)

        def batch():
            return gen.next()

        state = {"cur": batch()}

        def step():  # next batch generated one step ahead: lookahead key planning
            nxt = batch()
            cur, state["cur"] = state["cur"], nxt
            return m.train_step(*cur, next_keys=nxt[1])

        return m, step, B, "samples/s", dict(model=f"DLRM {cfg.num_rows} rows x {cfg.D} {cfg.emb_dtype} "
                                                   f"(26 sparse + 13 dense), "
                                                   f"{cfg.consistency}, {cfg.transport}", seq_len=None,
                                             rows_per_gpu=cfg.num_rows // comm.world, consistency=cfg.consistency)
    if args.model == "lr":
        from minips_amd.data.synthetic import SparseLRSynth
        from minips_amd.models.lr import SparseLR, SparseLRConfig

        B = args.batch or 65536
        vdt = getattr(torch, args.value_dtype)
        m = SparseLR(SparseLRConfig(consistency=args.consistency, staleness=args.staleness, value_dtype=vdt), comm)
        data = SparseLRSynth(B, nnz=64, device=dev, seed=r)
        return m, (lambda: m.train_step(*data.next())), B, "samples/s", \
            dict(model=f"sparse LR, 16.6M features, 64 nnz/row, {args.value_dtype} table", seq_len=None)
    if args.model == "kmeans":
        from minips_amd.models.kmeans import KMeans, KMeansConfig

        B = args.batch or 65536
        cfg = KMeansConfig(K=1000, dims=128, consistency=args.consistency, staleness=args.staleness)
        m = KMeans(cfg, comm)
        g = torch.Generator(device=dev)
        g.manual_seed(r)
        return m, (lambda: m.train_step(torch.randn(B, cfg.dims, generator=g, device=dev))), B, "samples/s", \
            dict(model="mini-batch K-Means K=1000 D=128", seq_len=None)
    if args.model == "widedeep-ssp":
        from minips_amd.data.synthetic import CriteoSynth
        from minips_amd.models.widedeep import WideDeep, WideDeepConfig

        B = args.batch or 16384
        cfg = WideDeepConfig(consistency="ssp", staleness=max(1, args.staleness), transport=args.transport,
                             max_batch=B)
        m = WideDeep(cfg, comm)
        data = CriteoSynth(B, cards=cfg.cards, device=dev, seed=1000 + r)
        if args.feeder == "inline":  # the next batch generated on the compute stream at step start
            state = {"cur": data.next()}

            def step():
                nxt = data.next()
                cur, state["cur"] = state["cur"], nxt
                return m.train_step(*cur, next_keys=nxt[1])

            return m, step, B, "samples/s", dict(model=f"Wide&Deep Criteo SSP ({args.transport})", seq_len=None,
                                                 consistency=f"ssp{cfg.staleness}", transport=args.transport,
                                                 feeder="inline")
        # bench.py's driver: the step on its own stream, the next batch generated and planned on
        # the planning stream a step ahead (LookaheadFeeder), for either transport
        from minips_amd.models.feeder import LookaheadFeeder
        from minips_amd.models.layers import compute_priority

        if dev.type == "cuda":
            main = torch.cuda.Stream(device=dev, priority=compute_priority())
            main.wait_stream(torch.cuda.default_stream(dev))
            torch.cuda.set_stream(main)
        feeder = LookaheadFeeder(m, data, comm)
        return m, feeder.step, B, "samples/s", dict(model=f"Wide&Deep Criteo SSP ({args.transport})", seq_len=None,
                                             consistency=f"ssp{cfg.staleness}", transport=args.transport,
                                             feeder="lookahead")
    raise SystemExit(f"unknown model {args.model}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2", choices=["mlp", "gpt2", "dlrm", "dlrm-10b", "lr", "kmeans",
                                                         "widedeep-ssp"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (samples or sequences)")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--rows", type=int, default=100_000_000, help="DLRM embedding rows (whole table)")
    ap.add_argument("--rows-per-gpu", type=int, default=1_250_000_000, help="dlrm-10b: rows per GPU shard")
    ap.add_argument("--dim", type=int, default=64, help="dlrm-10b: embedding width (bf16 rows: 64 fits 288 GB)")
    ap.add_argument("--consistency", default="bsp")
    ap.add_argument("--graph", type=lambda v: v.lower() in ("1", "true", "yes"), default=None,
                    help="mlp: capture the step in a HIP graph (one rank, BSP; off by default: at batch 8192 the "
                         "step is GPU-bound, 0.364 vs 0.350 ms measured)")
    ap.add_argument("--staleness", type=int, default=0)
    ap.add_argument("--feeder", default="lookahead", choices=["lookahead", "inline"],
                    help="widedeep-ssp: next batch generated + planned a step ahead on the planning stream "
                         "(bench.py's LookaheadFeeder) or generated inline at the step start")
    ap.add_argument("--transport", default="auto", choices=["auto", "collective", "onesided"],
                    help="widedeep-ssp / dlrm: RCCL collectives or the asynchronous PS (ps/onesided.py); auto = "
                         "the model's default (DLRM SSP/ASP: onesided; widedeep-ssp: collective)")
    ap.add_argument("--value-dtype", default="float32", choices=["float32", "float64"],
                    help="lr: table precision (float64 = the reference's CreateTable<double>)")
    args = ap.parse_args()
    if args.transport == "auto" and not args.model.startswith("dlrm"):
        args.transport = "collective"
    from minips_amd.ps.comm import init_distributed

    comm = init_distributed()
    dev = comm.device
    model, step, per_step, unit, cfg = build(args, comm)
    for _ in range(args.warmup):
        step()
    model.drain()
    torch.cuda.synchronize(dev)
    comm.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    model.drain()
    torch.cuda.synchronize(dev)
    comm.barrier()
    torch.cuda.synchronize(dev)
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if comm.world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t)
    if comm.rank == 0:
        print(json.dumps({
            "metric": f"{unit.split('/')[0]}/sec (whole job) {args.model} {cfg.pop('consistency', args.consistency)}",
            "value": round(per_step * comm.world * args.steps / el, 1), "unit": unit, "n_gpus": comm.world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1000 * el / args.steps, 3),
            "higher_is_better": True, "scaling": "weak",
            "dtype": ("bf16" if args.model in ("mlp", "gpt2", "dlrm", "dlrm-10b", "widedeep-ssp")
                      else ("fp64" if args.value_dtype == "float64" and args.model == "lr" else "fp32")),
            "data": "synthetic", "last": float(out.float().sum()) if torch.is_tensor(out) else None,
            "config": dict(cfg, parallelism=f"ps-dp{comm.world}"),
        }), flush=True)
    if comm.world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
