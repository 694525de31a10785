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
    ap.add_argument("--checkpoint_text_limit", type=int, default=1 << 22,
                    help="write the reference text file (<idx>:<val>) for shards of up to this many values "
                    "(-1: every shard, streamed); the binary sidecar is always written")
    ap.add_argument("--checkpoint_every", type=int, default=100)
    ap.add_argument("--use_weight_file", type=_flag_bool, default=False)
    ap.add_argument("--heartbeat_interval", type=float, default=0.0)
    ap.add_argument("--heartbeat_dir", default="")
    ap.add_argument("--fail_rank", type=int, default=-1)
    ap.add_argument("--fail_step", type=int, default=-1)
    ap.add_argument("--fail_mode", default="exit", choices=["exit", "hang", "hang_in_step"])
    ap.add_argument("--scale_check_every", type=int, default=10,
                    help="steps between checks for a supervisor scale directive (a max all-reduce of the "
                         "directive generation the ranks saw; minips_amd.elastic scale)")
    ap.add_argument("--recovery", default="inplace", choices=["inplace", "restart"],
                    help="inplace: after a peer failure the survivors roll back in their processes and "
                         "the supervisor relaunches only the failed rank; restart: the whole rank set")
    ap.add_argument("--value_dtype", default="float32", choices=["float32", "float64"],
                    help="LR table precision; float64 = the reference's CreateTable<double> (lr_example.cpp:182)")
    ap.add_argument("--transport", default="auto", choices=["auto", "collective", "onesided"],
                    help="W&D / DLRM SSP/ASP data path: RCCL collectives, or the asynchronous PS "
                         "(one-sided row reads, inbox pushes, owner-side optimizer apply; ps/onesided.py); "
                         "auto = the model's default (DLRM SSP/ASP: onesided, otherwise collective)")
    ap.add_argument("--asp_bound", type=int, default=-1,
                    help="ASP on the one-sided transport: >= 0 bounds how far a Get may run ahead of the "
                         "owners' applies (the SSP gate); -1 (default): unbounded, the reference ASP")
    ap.add_argument("--asp_depth", type=int, default=2,
                    help="ASP on the collective transport: clocks in flight before a Get waits (pipelining)")
    ap.add_argument("--force_quit_rank", type=int, default=-1,
                    help="(LR --input) treat this rank's shard as empty: it ForceQuits, the others continue")
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
    ap.add_argument("--num_workers_per_node", type=int, default=1,
                    help="LR: logical workers per rank, each with its own sampler and batch_size (reference flag); "
                    "their batches of a clock go out as one fused Get/Add")
    ap.add_argument("--input", default="", help="libsvm file / directory / comma list (LR; reference --input); "
                    "local, webhdfs://nn:port/path or hdfs://nn:port/path")
    ap.add_argument("--hdfs_namenode", default="", help="read a bare --input path from this HDFS namenode")
    ap.add_argument("--hdfs_namenode_port", type=int, default=9000)
    ap.add_argument("--hdfs_http_port", type=int, default=0, help="> 0: read HDFS through WebHDFS on this port")
    ap.add_argument("--assigner_master_port", type=int, default=0,
                    help="> 0: rank 0 serves locality-aware block assignment (HDFSBlockAssigner) on this port")
    ap.add_argument("--num_dims", type=int, default=0, help="feature count (reference flag; 0: infer / default)")
    args = ap.parse_args(argv)
    if args.transport == "auto":  # SSP / ASP run on the asynchronous one-sided PS (W&D, DLRM), BSP on collectives
        args.transport = ("onesided" if args.model in ("dlrm", "widedeep") and args.consistency in ("ssp", "asp")
                          else "collective")
    return args


def _load_input(args, comm):
    """This rank's libsvm shard: static byte-range blocks, or blocks handed out by the locality-aware
    assigner that rank 0 serves (reference HDFSManager: node 0 runs the HDFSBlockAssigner)."""
    from ._native import runtime
    from .data.loader import LibsvmData

    url = args.input
    if args.hdfs_namenode and "://" not in url:
        auth = (f"webhdfs://{args.hdfs_namenode}:{args.hdfs_http_port}" if args.hdfs_http_port > 0
                else f"hdfs://{args.hdfs_namenode}:{args.hdfs_namenode_port}")
        url = auth + ("" if url.startswith("/") else "/") + url
    if args.assigner_master_port <= 0:
        return LibsvmData(url, comm.rank, comm.world)
    srv = None
    if comm.rank == 0:
        srv = runtime().BlockAssignerServer(args.assigner_master_port)
        srv.start()
    master = os.environ.get("MASTER_ADDR", "127.0.0.1")
    data = LibsvmData(url, comm.rank, comm.world, assigner=f"{master}:{args.assigner_master_port}",
                      host=runtime().local_host_name())
    if srv is not None:  # serve until every loader thread of every rank has exited (kExit)
        srv.wait_done(600.0)
        print(f"[rank 0] block assigner: {srv.local_served} local / {srv.remote_served} remote blocks", flush=True)
        srv.stop()
    return data


SMALL_CARDS = [50, 7, 300, 20, 5, 60, 90, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27,
               28]


def build(args, comm):
    """-> (model, tables {id: table}, make_data() -> a fresh data stream with next()/skip(), step
    fn(batch) -> loss, samples/step). A fresh stream + skip(k) repositions the data at iteration k
    (restart and in-place rollback)."""
    dev = comm.device
    r = comm.rank
    seed = args.seed * 1000 + r
    if args.model == "widedeep":
        from .data.synthetic import CriteoSynth
        from .models.widedeep import WideDeep, WideDeepConfig

        B = args.batch or (64 if args.small else 16384)
        cfg = WideDeepConfig(consistency=args.consistency, staleness=args.staleness, transport=args.transport,
                             max_batch=B, **({"cards": SMALL_CARDS} if args.small else {}))
        m = WideDeep(cfg, comm)
        return m, {0: m.emb, 1: m.dense}, (lambda: CriteoSynth(B, cards=cfg.cards, device=dev, seed=seed)), \
            (lambda b: m.train_step(*b)), B
    if args.model == "mlp":
        from .data.synthetic import MnistSynth
        from .models.mlp import MLP, MLPConfig

        m = MLP(MLPConfig(consistency=args.consistency, staleness=args.staleness), comm)
        B = args.batch or (64 if args.small else 8192)
        return m, {0: m.table}, (lambda: _Skippable(MnistSynth(B, device=dev, seed=seed))), \
            (lambda b: m.train_step(*b)[0]), B
    if args.model == "dlrm":
        from .models.dlrm import DLRM, DLRMConfig

        B = args.batch or (64 if args.small else 16384)
        cfg = DLRMConfig(num_rows=20000 if args.small else 100_000_000, consistency=args.consistency,
                         staleness=args.staleness, transport=args.transport, max_batch=B)
        m = DLRM(cfg, comm)
        return m, {0: m.emb, 1: m.dense}, (lambda: _Skippable(_DLRMData(B, cfg, dev, seed))), \
            (lambda b: m.train_step(*b)), B
    if args.model == "gpt2":
        from .data.synthetic import TokenSynth
        from .models.gpt2 import GPT2, GPT2Config

        kw = dict(vocab=500, n_ctx=64, d=128, n_layer=2, n_head=2) if args.small else {}
        cfg = GPT2Config(consistency=args.consistency, staleness=args.staleness, **kw)
        m = GPT2(cfg, comm)
        B = args.batch or (2 if args.small else 8)
        return m, {0: m.table}, (lambda: _Skippable(TokenSynth(B, cfg.n_ctx, vocab=cfg.vocab, device=dev,             \
                                                               seed=seed))),                                          \
            (lambda b: m.train_step(*b)), B * cfg.n_ctx
    if args.model == "lr" and args.input:
        # reference LR on a libsvm file (lr_example.cpp --input): this rank's shard is loaded by the
        # native block assigner / mmap reader and kept resident in HBM; batches are consecutive
        # rows from a random start (lib/batch_data_sampler.cpp), cut on the device
        from .models.lr import SparseLR, SparseLRConfig

        shard = args._shard.to(dev)
        nd = args.num_dims
        if not nd:  # every rank must size the table alike: max feature id over all shards
            t = torch.tensor([float(shard.cols.max()) + 1 if shard.cols.numel() else 1.0], device=dev)
            comm.all_reduce_(t, op=dist.ReduceOp.MAX)
            nd = int(t.item())
        m = SparseLR(SparseLRConfig(num_dims=nd, alpha=args.alpha, consistency=args.consistency,
                                    staleness=args.staleness, storage=args.kStorageType,
                                    value_dtype=getattr(torch, args.value_dtype)), comm)
        B = args.batch or 1024
        W = max(1, args.num_workers_per_node)
        return m, {0: m.table}, (lambda: _Skippable(_WorkerGroup([_Batches(shard, B, seed + _WSEED * w)
                                                                  for w in range(W)]))), \
            (lambda b: -m.train_step(*b)), B * W
    if args.model == "lr":
        from .data.synthetic import SparseLRSynth
        from .models.lr import SparseLR, SparseLRConfig

        nd = args.num_dims or (5000 if args.small else 16_609_143)
        m = SparseLR(SparseLRConfig(num_dims=nd, alpha=args.alpha, consistency=args.consistency,
                                    staleness=args.staleness, storage=args.kStorageType,
                                    value_dtype=getattr(torch, args.value_dtype)), comm)
        B = args.batch or (128 if args.small else 65536)
        W = max(1, args.num_workers_per_node)
        return m, {0: m.table}, \
            (lambda: _Skippable(_WorkerGroup([SparseLRSynth(B, num_dims=nd, nnz=16 if args.small else 64, device=dev,
                                                            seed=seed + _WSEED * w) for w in range(W)]))), \
            (lambda b: -m.train_step(*b)), B * W
    if args.model == "kmeans" and args.input:
        # the reference K-Means input: sparse libsvm points (kmeans.cpp reads --input); the
        # shard stays resident in HBM and batches are consecutive rows, cut on the device
        from .models.kmeans import KMeans, KMeansConfig

        shard = args._shard.to(dev)
        nd = args.num_dims
        if not nd:  # every rank must size the table alike: max feature id over all shards
            t = torch.tensor([float(shard.cols.max()) + 1 if shard.cols.numel() else 1.0], device=dev)
            comm.all_reduce_(t, op=dist.ReduceOp.MAX)
            nd = int(t.item())
        cfg = KMeansConfig(K=args.K or 8, dims=nd, consistency=args.consistency, staleness=args.staleness,
                           init_mode=args.kmeans_init_mode or "random", seed=seed)
        B = args.batch or 256
        init = None
        if args.kmeans_init_mode:
            rp, c, v, _ = shard.batch(0, max(B, cfg.K))
            init = torch.zeros(rp.numel() - 1, nd, dtype=torch.float32, device=dev)
            row = torch.repeat_interleave(torch.arange(rp.numel() - 1, device=dev), rp[1:] - rp[:-1])
            ok = c < nd
            init.index_put_((row[ok], c[ok]), v[ok], accumulate=True)  # densify the seeding batch only
        m = KMeans(cfg, comm, init_data=init)
        return m, {0: m.table}, (lambda: _Skippable(_Batches(shard, B, seed))), \
            (lambda b: m.train_step_csr(b[0], b[1], b[2])), B
    if args.model == "kmeans":
        from .models.kmeans import KMeans, KMeansConfig

        cfg = KMeansConfig(K=args.K or (8 if args.small else 1000), dims=16 if args.small else 128,
                           consistency=args.consistency, staleness=args.staleness,
                           init_mode=args.kmeans_init_mode or "random", seed=seed)
        B = args.batch or (256 if args.small else 65536)
        # seeding reads its own batch of local data (rank 0's seeds are broadcast)
        init = _GaussData(max(B, cfg.K), cfg.dims, dev, seed + 7919).next() if args.kmeans_init_mode else None
        m = KMeans(cfg, comm, init_data=init)
        return m, {0: m.table}, (lambda: _Skippable(_GaussData(B, cfg.dims, dev, seed))), (lambda b: m.train_step(b)), B
    raise ValueError(args.model)


_WSEED = 104729


class _WorkerGroup:
    """``--num_workers_per_node`` logical workers on one GPU rank (the reference runs that many
    worker threads per process over the node's data, driver/engine.cpp:266-288, lr_example.cpp:
    203-207): each worker keeps its own sampler (own start point / seed, its own batch_size), and
    the W CSR batches of a clock are concatenated into ONE Get / Add / Clock -- one set of launches
    instead of W. Under BSP this is exactly the reference's result: all W workers read the clock-c
    parameters and the server sums their pushes (VectorStorage::SubAdd is additive); under SSP/ASP
    the workers of a rank advance together, a schedule both models admit."""

    def __init__(self, its):
        self.its = its

    def next(self):
        parts = [it.next() for it in self.its]
        if len(parts) == 1:
            return parts[0]
        rps, off = [], 0
        for i, (rp, c, _, _) in enumerate(parts):
            rps.append((rp if i == 0 else rp[1:]) + off)
            off += c.numel()
        return (torch.cat(rps), torch.cat([p[1] for p in parts]), torch.cat([p[2] for p in parts]),
                torch.cat([p[3] for p in parts]))


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
        from .data.synthetic import DLRMSynth

        self.gen = DLRMSynth(B, cfg.F, cfg.num_rows, cfg.n_dense, device=dev, seed=seed)

    def next(self):
        return self.gen.next()


class _GaussData:
    def __init__(self, B, D, dev, seed):
        self.B, self.D, self.dev = B, D, dev
        self.g = torch.Generator(device=dev)
        self.g.manual_seed(seed)

    def next(self):
        return torch.randn(self.B, self.D, generator=self.g, device=self.dev)


def _is_comm_failure(e: BaseException) -> bool:
    """A collective failed because a peer died or the communicator was aborted -- by type, not by
    message: RCCL (TORCH_NCCL_ASYNC_ERROR_HANDLING=2: an aborted / timed-out communicator) and the
    c10d store raise the torch.distributed error classes (DistBackendError, DistNetworkError,
    DistStoreError); gloo's transport raises a RuntimeError tagged with its gloo source location
    ("[.../gloo/transport/tcp/pair.cc:547] Connection closed by peer"). Errors of this process's
    own code (a failed kernel, the async PS server) are not peer failures and propagate."""
    if isinstance(e, dist.DistError):
        return True
    head = str(e).split("]", 1)[0]
    return isinstance(e, RuntimeError) and head.startswith("[") and "/gloo/" in head


def _force_quit(comm, has_data: bool, rank: int):
    """Graceful degradation (reference lr_example.cpp:145-152, mailbox.cpp:159-171): a rank with
    no data leaves and the others continue among themselves. Every rank learns every rank's flag
    (one all-gather), the survivors form a sub-group (collective over the full group); a quitting
    rank returns None. Survivors get a Comm over their group: the tables are built on it, so
    they are sharded over the survivors only."""
    from .ps.comm import Comm
    from .utils import metrics

    if comm.world == 1:
        return comm
    flags = torch.empty(comm.world, dtype=torch.float32, device=comm.device)
    comm.all_gather(flags, torch.tensor([1.0 if has_data else 0.0], device=comm.device))
    survivors = [r for r, f in enumerate(flags.tolist()) if f > 0]
    if len(survivors) == comm.world:
        return comm
    if not survivors:
        raise RuntimeError("no rank has any data")
    quitters = sorted(set(range(comm.world)) - set(survivors))
    if rank == survivors[0]:
        metrics.fault_tolerance_phase(2, f"kForceQuit from ranks {quitters} (no data); {len(survivors)} ranks continue")
    group = dist.new_group(survivors)
    if not has_data:
        print(f"[rank {rank}] kForceQuit: no data, leaving the job", file=sys.stderr, flush=True)
        return None
    return Comm(group=group, device=comm.device)


class _ckpt_state:
    """Heartbeat state "ckpt" while a checkpoint is written / committed: a multi-GB shard write
    advances no step, and the supervisor gives that state its own (long) limit instead of the
    stuck-in-a-step progress timeout."""

    def __init__(self, hb):
        self.hb = hb

    def __enter__(self):
        if self.hb is not None:
            self.prev, self.hb.state = self.hb.state, "ckpt"

    def __exit__(self, *exc):
        if self.hb is not None:
            self.hb.state = self.prev


def _scale_directive(hb_dir: str, generation: int) -> dict | None:
    """A supervisor scale directive newer than ``generation`` (None: none, or a failure rollback)."""
    try:
        d = json.loads(open(os.path.join(hb_dir, "rollback.json")).read())
    except (OSError, ValueError):
        return None
    return d if d.get("kind") == "scale" and int(d.get("generation", -1)) > generation else None


def _wait_directive(hb_dir: str, generation: int, timeout: float = 300.0) -> dict:
    """Rollback directive of the supervisor (minips_amd.elastic): a newer generation with the
    rendezvous port of the re-formed group (the reference's kRollBack, mailbox.cpp:172-191)."""
    path = os.path.join(hb_dir, "rollback.json")
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            d = json.loads(open(path).read())
            if int(d["generation"]) > generation:
                return d
        except (OSError, ValueError, KeyError):
            pass
        time.sleep(0.05)
    raise TimeoutError("no rollback directive from the supervisor")


def main(argv=None):
    args = parse(argv)
    from .ps.checkpoint import Checkpointer
    from .ps.comm import init_distributed
    from .ps.fault import FaultInjector, Heartbeat
    from .utils import metrics

    if args.metrics_dir:
        os.environ["MINIPS_METRICS_DIR"] = args.metrics_dir
    os.environ["MINIPS_ASP_DEPTH"] = str(max(0, args.asp_depth))
    if args.asp_bound >= 0:
        os.environ["MINIPS_ASP_BOUND"] = str(args.asp_bound)
    # the asynchronous tables' peers hold IPC mappings of every shard and a shared board: a lost
    # rank restarts the whole set from the checkpoint, never an in-place rollback
    inplace = args.recovery == "inplace" and bool(args.heartbeat_dir) and args.transport != "onesided"
    if inplace:  # RCCL: a dead peer aborts the communicator and raises, instead of killing us
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
    comm = init_distributed()
    rank = comm.rank
    generation = int(os.environ.get("MINIPS_GENERATION", "0"))
    hb = Heartbeat(args.heartbeat_dir, rank, args.heartbeat_interval, state_fn=lambda: comm.state()) \
        if args.heartbeat_interval > 0 and args.heartbeat_dir else None
    if hb is not None:
        # what this rank can recover from: the supervisor takes the in-place branch only if EVERY
        # rank can roll back in its process (the one-sided tables cannot: peers hold IPC mappings of
        # the dead rank's shards and a shared progress board -- the whole set restarts instead)
        hb.write_caps(inplace=inplace, transport=args.transport)
    if args.model in ("lr", "kmeans") and args.input:
        from .data.loader import LibsvmData

        args._shard = _load_input(args, comm)
        sub = _force_quit(comm, args._shard.n > 0 and args.force_quit_rank != rank, rank)
        if sub is None:
            if hb:
                hb.stop()
            dist.destroy_process_group()
            return 0
        if sub is not comm:
            comm = sub
            inplace = False  # a sub-group job restarts as a whole (its ranks are a subset)
    model, tables, make_data, step_fn, per_step = build(args, comm)
    data = make_data()
    ck = Checkpointer(comm, args.checkpoint_file_prefix, text_limit=args.checkpoint_text_limit)
    start = 0
    if args.use_weight_file and not ck.exists():
        # a restart before the first committed checkpoint (or with checkpoint_toggle off): there
        # is nothing to roll back to, so the relaunched job starts over
        print(f"[rank {rank}] --use_weight_file but no committed checkpoint under "
              f"{args.checkpoint_file_prefix!r}: starting from iteration 0", file=sys.stderr, flush=True)
    elif args.use_weight_file:
        start = ck.load(tables)
        data.skip(start)
        failed = int(os.environ.get("MINIPS_FAILED_RANK", "-1"))
        metrics.fault_tolerance_phase(4 if rank == failed else 5, f"rank {rank} restored iteration {start}")
    if hb:
        hb.progress(start - 1)
    inj = FaultInjector(rank, args.fail_rank, args.fail_step, args.with_injected_straggler, args.seed,
                        mode=args.fail_mode, heartbeat=hb)
    log = metrics.get_logger()
    losses = []
    report = open(args.report_prefix + f"report_{rank}", "a") if args.report_prefix else None
    t_start = time.perf_counter()
    t_steady, n_steady = None, 0

    def rollback():
        """Survivor side of an in-place recovery (reference: mailbox.cpp:172-191 kRollBack ->
        RollBackServer / RollBackWorker): drop the broken communicator, join the re-formed group
        on the supervisor's new rendezvous, restore every table from the last committed
        checkpoint and reposition the data; the relaunched rank restores the same iteration."""
        nonlocal generation, data, losses
        hb.state = "recover"
        ck.abandon()
        try:
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001 - the group is already broken
            pass
        d = _wait_directive(args.heartbeat_dir, generation)
        generation = int(d["generation"])
        os.environ["MASTER_PORT"] = str(d["port"])
        os.environ["MINIPS_GENERATION"] = str(generation)
        dist.destroy_process_group() if dist.is_initialized() else None
        init_distributed()
        comm.refresh()
        for t in tables.values():
            t.reset_after_rollback()
        if hasattr(model, "_pending_plans"):
            model._pending_plans = []  # planned on the broken communicator
        if not ck.exists():
            raise RuntimeError("in-place rollback needs a committed checkpoint")
        it0 = ck.load(tables)
        data = make_data()
        data.skip(it0)
        losses = [x for x in losses if x[0] < it0]
        metrics.fault_tolerance_phase(5, f"rank {rank} rolled back in place to iteration {it0} "
                                         f"(failed rank {d.get('failed_rank')}, generation {generation})")
        hb.state = "run"
        hb.progress(it0 - 1)
        return it0

    def scale(it_now: int):
        """Live rescale at a step boundary (the reference's kScaleRollback): every rank of the old
        group checkpoints iteration ``it_now``, leaves the group; ranks < the new world re-form it
        in this process, rebuild their tables on the new shard ranges and restore (reshard) that
        checkpoint; the others retire. Returns the iteration to continue from, or None (retired)."""
        nonlocal generation, data, losses, model, tables, make_data, step_fn, per_step, ck
        hb.state = "recover"
        model.drain()
        with _ckpt_state(hb):
            ck.save(tables, iteration=it_now, blocking=True)
            ck.commit()
        d = _wait_directive(args.heartbeat_dir, generation)
        generation, world = int(d["generation"]), int(d["world"])
        comm.barrier()
        ps = getattr(comm, "_async_ps", None)
        if ps is not None:
            # one-sided tables: stop this owner's server thread (it holds raw pointers to the shards
            # and inboxes freed below) and drop the board; build() makes a fresh AsyncPS on the new
            # group, whose ranks (new ones included) all join its rendezvous
            ps.close()
            comm._async_ps = None
        dist.destroy_process_group()
        if rank >= world:
            metrics.fault_tolerance_phase(5, f"rank {rank} retired by the scale to {world} ranks at iteration {it_now}")
            hb.stop()
            return None
        os.environ.update(MASTER_PORT=str(d["port"]), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                          MINIPS_GENERATION=str(generation))
        model = tables = step_fn = None  # free the old shards before the new ones are allocated
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        init_distributed()
        comm.refresh()
        model, tables, make_data, step_fn, per_step = build(args, comm)
        ck = Checkpointer(comm, args.checkpoint_file_prefix, text_limit=args.checkpoint_text_limit)
        it0 = ck.load(tables)
        data = make_data()
        data.skip(it0)
        losses = [x for x in losses if x[0] < it0]
        metrics.fault_tolerance_phase(5, f"rank {rank} rescaled in place to {world} ranks at iteration {it0} "
                                         f"(generation {generation})")
        hb.state = "run"
        hb.progress(it0 - 1)
        return it0

    it = start
    while it < args.steps:
        # (the rule depends on ``it`` only: ranks started by a scale-out resume at the same
        # iteration as the survivors and must take part in the same checks)
        if hb is not None and args.scale_check_every > 0 and it % args.scale_check_every == 0:
            # do the ranks agree that a scale directive is pending? (all of them act at THIS step)
            d = _scale_directive(args.heartbeat_dir, generation)
            flag = torch.tensor([float(d["generation"]) if d else 0.0], device=comm.device)
            comm.all_reduce_(flag, op=dist.ReduceOp.MAX)
            if float(flag) > generation:
                nxt = scale(it)
                if nxt is None:
                    return 0
                it = nxt
                t_steady = None
                continue
        try:
            if it == start + args.timing_skip and t_steady is None:
                if comm.device.type == "cuda":
                    torch.cuda.synchronize(comm.device)
                t_steady, n_steady = time.perf_counter(), args.steps - it
            with _ckpt_state(hb):  # checkpoint phases are not steps: their own heartbeat state
                if args.checkpoint_commit == "async":
                    ck.try_commit()  # publishes an in-flight checkpoint once every rank's files are written
                else:
                    ck.commit()  # publishes the checkpoint issued after the previous step (no-op otherwise)
            inj.step(it)
            t0 = time.perf_counter()
            with metrics.range(f"step {it}"):
                batch = data.next()
                inj.in_step(it)
                loss = step_fn(batch)
            if (it + 1) % 10 == 0 or it + 1 == args.steps:
                with comm.waiting():
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
                with _ckpt_state(hb):
                    ck.save(tables, iteration=it + 1)
            if hb:
                hb.progress(it)
            it += 1
        except Exception as e:  # noqa: BLE001
            if not (inplace and hb is not None and comm.world > 1 and _is_comm_failure(e)):
                raise
            print(f"[rank {rank}] collective failed at iteration {it} ({type(e).__name__}): rolling back in place",
                  file=sys.stderr, flush=True)
            it = rollback()
            t_steady = None
    model.drain()
    if comm.device.type == "cuda":
        torch.cuda.synchronize(comm.device)
    steady_ms = (time.perf_counter() - t_steady) * 1e3 / n_steady if t_steady is not None and n_steady else None
    with _ckpt_state(hb):
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
    if comm.rank == 0:
        print(json.dumps(dict(model=args.model, steps=args.steps, start=start, losses=losses,
                              checksum=[round(float(x), 6) for x in sums.cpu()],
                              total_ms=round((time.perf_counter() - t_start) * 1e3, 1),
                              steady_ms_per_iter=round(steady_ms, 4) if steady_ms is not None else None,
                              world=comm.world, generation=generation)),
              flush=True)
    if comm.world > 1:
        comm.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
