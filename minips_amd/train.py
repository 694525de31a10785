"""Training driver of one PS rank (one process per GPU; torchrun / minips_amd.elastic set the env).

    python -m minips_amd.train --model widedeep --steps 100 --checkpoint_toggle=1 \
        --checkpoint_file_prefix=/tmp/ck/ --checkpoint_every 20

Flags keep the reference names where the reference has them (lr_example.cpp:20-56, §5.6):
checkpoint_toggle, checkpoint_file_prefix, use_weight_file, heartbeat_interval, report_prefix,
report_interval, with_injected_straggler, kModelType (= --consistency), kStaleness, batch_size,
num_iters (= --steps), alpha (LR). Extra: --fail_rank/--fail_step fault injection, --metrics_dir.
On --use_weight_file the tables restore from the checkpoint and training resumes at the saved
iteration with the data stream advanced to the same position, so a restarted run ends with the
same parameters as an uninterrupted one (BSP).
The last line on rank 0 is a JSON summary (losses, final iteration, parameter checksum).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


import torch
import torch.distributed as dist


def _flag_bool(v):
    return str(v).lower() in ("1", "true", "yes", "on")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="widedeep", choices=["widedeep", "mlp", "dlrm", "gpt2", "lr", "kmeans"])
    ap.add_argument("--steps", "--num_iters", dest="steps", type=int, default=20)
    ap.add_argument("--batch", "--batch_size", dest="batch", type=int, default=0)
    ap.add_argument("--consistency", "--kModelType", dest="consistency", default="bsp", type=str.lower)
    ap.add_argument("--staleness", "--kStaleness", dest="staleness", type=int, default=0)
    ap.add_argument("--small", type=_flag_bool, default=False, help="tiny shapes (CPU tests)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--checkpoint_toggle", type=_flag_bool, default=False)
    ap.add_argument("--checkpoint_file_prefix", default="/tmp/minips_ckpt/")
    ap.add_argument("--checkpoint_every", type=int, default=100)
    ap.add_argument("--use_weight_file", type=_flag_bool, default=False)
    ap.add_argument("--heartbeat_interval", type=float, default=0.0)
    ap.add_argument("--heartbeat_dir", default="")
    ap.add_argument("--fail_rank", type=int, default=-1)
    ap.add_argument("--fail_step", type=int, default=-1)
    ap.add_argument("--fail_mode", default="exit", choices=["exit", "hang"])
    ap.add_argument("--checkpoint_commit", default="eager", choices=["eager", "async"],
                    help="eager: publish a checkpoint at the next step (waits for its files); async: "
                         "publish once every rank's writer finished (training never waits for the disk)")
    ap.add_argument("--with_injected_straggler", type=_flag_bool, default=False)
    ap.add_argument("--kStorageType", default="Vector", type=str.lower, choices=["vector", "map"],
                    help="LR parameter storage: Vector (key range) or Map (GPU hash table, MapStorage)")
    ap.add_argument("--K", type=int, default=0, help="K-Means centres (0: model default)")
    ap.add_argument("--kmeans_init_mode", default="", choices=["", "random", "kmeans++", "kmeans_parallel"],
                    help="K-Means seeding from a batch of local data (reference kmeans.cpp:154-192); "
                         "empty: N(0,1) centres")
    ap.add_argument("--report_prefix", default="")
    ap.add_argument("--report_interval", type=int, default=10)
    ap.add_argument("--metrics_dir", default="")
    ap.add_argument("--timing_skip", type=int, default=0,
                    help="iterations excluded from steady_ms_per_iter (first-launch / warm-up costs)")
    ap.add_argument("--alpha", type=float, default=0.05)
    ap.add_argument("--input", default="", help="libsvm file / directory / comma list (LR; reference --input)")
    ap.add_argument("--num_dims", type=int, default=0, help="feature count (reference flag; 0: infer / default)")
    return ap.parse_args(argv)


SMALL_CARDS = [50, 7, 300, 20, 5, 60, 90, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27,
               28]


def build(args, comm):
    """-> (model, tables {id: table}, data stream with next()/skip(), step fn(batch) -> loss, samples/step)."""
    dev = comm.device
    r = comm.rank
    seed = args.seed * 1000 + r
    if args.model == "widedeep":
        from .data.synthetic import CriteoSynth
        from .models.widedeep import WideDeep, WideDeepConfig

        cfg = WideDeepConfig(consistency=args.consistency, staleness=args.staleness,
                             **({"cards": SMALL_CARDS} if args.small else {}))
        m = WideDeep(cfg, comm)
        B = args.batch or (64 if args.small else 16384)
        data = CriteoSynth(B, cards=cfg.cards, device=dev, seed=seed)
        return m, {0: m.emb, 1: m.dense}, data, (lambda b: m.train_step(*b)), B
    if args.model == "mlp":
        from .data.synthetic import MnistSynth
        from .models.mlp import MLP, MLPConfig

        m = MLP(MLPConfig(consistency=args.consistency, staleness=args.staleness), comm)
        B = args.batch or (64 if args.small else 8192)
        data = _Skippable(MnistSynth(B, device=dev, seed=seed))
        return m, {0: m.table}, data, (lambda b: m.train_step(*b)[0]), B
    if args.model == "dlrm":
        from .models.dlrm import DLRM, DLRMConfig

        cfg = DLRMConfig(num_rows=20000 if args.small else 100_000_000, consistency=args.consistency,
                         staleness=args.staleness)
        m = DLRM(cfg, comm)
        B = args.batch or (64 if args.small else 16384)
        data = _Skippable(_DLRMData(B, cfg, dev, seed))
        return m, {0: m.emb, 1: m.dense}, data, (lambda b: m.train_step(*b)), B
    if args.model == "gpt2":
        from .data.synthetic import TokenSynth
        from .models.gpt2 import GPT2, GPT2Config

        kw = dict(vocab=500, n_ctx=64, d=128, n_layer=2, n_head=2) if args.small else {}
        cfg = GPT2Config(consistency=args.consistency, staleness=args.staleness, **kw)
        m = GPT2(cfg, comm)
        B = args.batch or (2 if args.small else 8)
        data = _Skippable(TokenSynth(B, cfg.n_ctx, vocab=cfg.vocab, device=dev, seed=seed))
        return m, {0: m.table}, data, (lambda b: m.train_step(*b)), B * cfg.n_ctx
    if args.model == "lr" and args.input:
        # reference LR on a libsvm file (lr_example.cpp --input): this rank's shard is loaded by the
        # native block assigner / mmap reader and kept resident in HBM; batches are consecutive
        # rows from a random start (lib/batch_data_sampler.cpp), cut on the device
        from .data.loader import LibsvmData
        from .models.lr import SparseLR, SparseLRConfig

        shard = LibsvmData(args.input, r, comm.world).to(dev)
        nd = args.num_dims
        if not nd:  # every rank must size the table alike: max feature id over all shards
            t = torch.tensor([float(shard.cols.max()) + 1 if shard.cols.numel() else 1.0], device=dev)
            comm.all_reduce_(t, op=dist.ReduceOp.MAX)
            nd = int(t.item())
        m = SparseLR(SparseLRConfig(num_dims=nd, alpha=args.alpha, consistency=args.consistency,
                                    staleness=args.staleness, storage=args.kStorageType), comm)
        B = args.batch or 1024
        return m, {0: m.table}, _Skippable(_Batches(shard, B, seed)), (lambda b: -m.train_step(*b)), B
    if args.model == "lr":
        from .data.synthetic import SparseLRSynth
        from .models.lr import SparseLR, SparseLRConfig

        nd = args.num_dims or (5000 if args.small else 16_609_143)
        m = SparseLR(SparseLRConfig(num_dims=nd, alpha=args.alpha, consistency=args.consistency,
                                    staleness=args.staleness, storage=args.kStorageType), comm)
        B = args.batch or (128 if args.small else 65536)
        data = _Skippable(SparseLRSynth(B, num_dims=nd, nnz=16 if args.small else 64, device=dev, seed=seed))
        return m, {0: m.table}, data, (lambda b: -m.train_step(*b)), B
    if args.model == "kmeans":
        from .models.kmeans import KMeans, KMeansConfig

        cfg = KMeansConfig(K=args.K or (8 if args.small else 1000), dims=16 if args.small else 128,
                           consistency=args.consistency, staleness=args.staleness,
                           init_mode=args.kmeans_init_mode or "random", seed=seed)
        B = args.batch or (256 if args.small else 65536)
        # seeding reads its own batch of local data (rank 0's seeds are broadcast)
        init = _GaussData(max(B, cfg.K), cfg.dims, dev, seed + 7919).next() if args.kmeans_init_mode else None
        m = KMeans(cfg, comm, init_data=init)
        data = _Skippable(_GaussData(B, cfg.dims, dev, seed))
        return m, {0: m.table}, data, (lambda b: m.train_step(b)), B
    raise ValueError(args.model)


class _Skippable:
    def __init__(self, inner):
        self.inner = inner

    def next(self):
        return self.inner.next()

    def skip(self, n):
        for _ in range(n):
            self.inner.next()


class _Batches:
    def __init__(self, shard, B, seed):
        self.it = shard.batches(B, seed=seed)

    def next(self):
        return next(self.it)


class _DLRMData:
    def __init__(self, B, cfg, dev, seed):
        self.B, self.cfg, self.dev = B, cfg, dev
        self.g = torch.Generator(device=dev)
        self.g.manual_seed(seed)

    def next(self):
        dense = torch.randn(self.B, self.cfg.n_dense, generator=self.g, device=self.dev)
        keys = torch.randint(0, self.cfg.num_rows, (self.B, self.cfg.F), generator=self.g, device=self.dev)
        return dense, keys, (dense[:, 0] > 0).float()


class _GaussData:
    def __init__(self, B, D, dev, seed):
        self.B, self.D, self.dev = B, D, dev
        self.g = torch.Generator(device=dev)
        self.g.manual_seed(seed)

    def next(self):
        return torch.randn(self.B, self.D, generator=self.g, device=self.dev)


def main(argv=None):
    args = parse(argv)
    from .ps.checkpoint import Checkpointer
    from .ps.comm import init_distributed
    from .ps.fault import FaultInjector, Heartbeat
    from .utils import metrics

    if args.metrics_dir:
        os.environ["MINIPS_METRICS_DIR"] = args.metrics_dir
    comm = init_distributed()
    rank = comm.rank
    hb = Heartbeat(args.heartbeat_dir, rank, args.heartbeat_interval) \
        if args.heartbeat_interval > 0 and args.heartbeat_dir else None
    model, tables, data, step_fn, per_step = build(args, comm)
    ck = Checkpointer(comm, args.checkpoint_file_prefix)
    start = 0
    if args.use_weight_file:
        start = ck.load(tables)
        data.skip(start)
        failed = int(os.environ.get("MINIPS_FAILED_RANK", "-1"))
        metrics.fault_tolerance_phase(4 if rank == failed else 5, f"rank {rank} restored iteration {start}")
    inj = FaultInjector(rank, args.fail_rank, args.fail_step, args.with_injected_straggler, args.seed,
                        mode=args.fail_mode, heartbeat=hb)
    log = metrics.get_logger()
    losses = []
    report = open(args.report_prefix + f"report_{rank}", "a") if args.report_prefix else None
    t_start = time.perf_counter()
    t_steady, n_steady = None, 0
    for it in range(start, args.steps):
        if it == start + args.timing_skip:
            if comm.device.type == "cuda":
                torch.cuda.synchronize(comm.device)
            t_steady, n_steady = time.perf_counter(), args.steps - it
        if args.checkpoint_commit == "async":
            ck.try_commit()  # publishes an in-flight checkpoint once every rank's files are written
        else:
            ck.commit()  # publishes the checkpoint issued after the previous step (no-op otherwise)
        inj.step(it)
        t0 = time.perf_counter()
        with metrics.range(f"step {it}"):
            loss = step_fn(data.next())
        if (it + 1) % 10 == 0 or it + 1 == args.steps:
            lv = float(loss.float().sum()) / per_step
            losses.append((it, lv))
            log.step(it, per_step, time.perf_counter() - t0, comm.stats, loss=lv)
            if rank == 0:
                print(f"Current iteration={it + 1} on node={rank} loss={lv:.5f}", flush=True)
        if report and (it + 1) % args.report_interval == 0:
            report.write(f"{it + 1}\t{(time.perf_counter() - t_start) * 1e3:.1f}\n")
            report.flush()
        if args.checkpoint_toggle and args.checkpoint_every > 0 and (it + 1) % args.checkpoint_every == 0 \
                and it + 1 < args.steps:
            ck.save(tables, iteration=it + 1)
    model.drain()
    if comm.device.type == "cuda":
        torch.cuda.synchronize(comm.device)
    steady_ms = (time.perf_counter() - t_steady) * 1e3 / n_steady if t_steady is not None and n_steady else None
    ck.commit()
    # parameter checksum over every table (identical on all ranks): the parameter values only
    # (hash tables also export their keys, which are not parameters)
    def _param_sum(t):
        arrays = t.shard_state()[1]
        a = arrays.get("params", arrays.get("master", arrays.get("rows")))
        if a is None:
            a = next(iter(arrays.values()))
        return float(a.double().sum())

    sums = torch.tensor([_param_sum(t) for t in tables.values()], dtype=torch.float64, device=comm.device)
    comm.all_reduce_(sums)
    if comm.device.type == "cuda":
        torch.cuda.synchronize(comm.device)
    if hb:
        hb.stop()
    if rank == 0:
        print(json.dumps(dict(model=args.model, steps=args.steps, start=start, losses=losses,
                              checksum=[round(float(x), 6) for x in sums.cpu()],
                              total_ms=round((time.perf_counter() - t_start) * 1e3, 1),
                              steady_ms_per_iter=round(steady_ms, 4) if steady_ms is not None else None)),
              flush=True)
    if comm.world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
