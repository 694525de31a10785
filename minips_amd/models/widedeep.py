"""Wide&Deep on Criteo-shaped data over the GPU parameter server (BASELINE config 3 and the
north-star benchmark).

Parameters
  sparse table  one row per categorical id (sum of the 26 cardinalities, 33.8M rows):
                [32-dim deep embedding | 1 wide weight | 3 pad], row-wise Adagrad with a
                separate accumulator for the deep part and for the wide weight.
  dense table   deep tower Linear(845->1024)->ReLU->Linear(1024->512)->ReLU->
                Linear(512->256)->ReLU->Linear(256->1), one flat fp32 master vector, Adam;
                biases are folded into the weight matrices (constant-1 input column).
Step (every kernel is a gfx950 HIP kernel; comm is RCCL):
  sparse Get -> wd_assemble (lookup + dense concat + wide sum) -> 3 MFMA GEMMs (bias+ReLU
  fused) -> wd_head (last layer + BCE fwd/bwd fused) -> per layer wgrad GEMM (split-K, the
  bias gradient falls out of the ones column) + dgrad GEMM (ReLU mask fused) -> wd_emb_backward (segment sum into unique
  rows) -> sparse Add + dense Add -> Clock (all-to-all / reduce-scatter, fused optimizers,
  all-gather).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from .. import ops
from ..ps.comm import Comm
from ..utils import streams
from ..utils.metrics import phase, traced
from .layers import Replayer, SideStream
from .feeder import LookaheadPlans


@dataclass
class WideDeepConfig:
    cards: list = field(default_factory=lambda: list(__import__(
        "minips_amd.data.synthetic", fromlist=["CRITEO_KAGGLE_CARDS"]).CRITEO_KAGGLE_CARDS))
    n_dense: int = 13
    emb_dim: int = 32
    row_width: int = 36          # 32 deep + 1 wide + 3 pad (16-byte rows)
    hidden: tuple = (1024, 512, 256)
    lr_dense: float = 1e-3
    lr_sparse: float = 0.02
    consistency: str = "bsp"
    staleness: int = 0
    # "collective": SparseTable / DenseTable over RCCL; "onesided": SSP / ASP with no collective on
    # the data path -- rows pulled one-sidedly from the owners' HBM, gradients pushed into the
    # owners' inboxes, row-wise Adagrad / Adam applied by each owner's server thread (ps/onesided.py);
    # "auto" (default): one-sided for SSP / ASP (the reference's asynchronous servers; on one MI355X
    # 0.404 vs 0.400 ms/step, profiles/r6/ssp_onesided_vs_collective.txt -- no collective rendezvous
    # at N > 1), collective for BSP
    transport: str = "auto"
    dense_transport: str | None = None  # (None: ``transport``) the dense table's, when it differs
    max_batch: int = 16384       # onesided: inbox slots hold max_batch * F gradient rows
    seed: int = 0
    # several ranks: the dense clock runs per bucket of >= bucket_mb MB of gradient (layers merged
    # from the last one), a bucket's reduce-scatter + Adam + all-gather issued as soon as its
    # layers' weight gradients exist -- beside the remaining backward (0: one clock at the end).
    # The 6.3 MB of W&D gradients: one reduce-scatter + all-gather after the backward measured
    # 6 % faster than two buckets at 8 emulated ranks (0.475-0.503 vs 0.517-0.530 ms/step: half
    # the collective calls and clock issue on the host-bound step; profiles/r5/ab_dense_buckets.txt),
    # and no worse with modelled xGMI wire time either (ring RS/AG 0.498 vs 0.505, direct 0.487 vs
    # 0.517 ms/step, 8 emulated ranks; profiles/r6/ab_buckets_wire.txt)
    bucket_mb: float = 0.0

    def __post_init__(self):
        if self.transport == "auto":
            self.transport = "onesided" if self.consistency in ("ssp", "asp") else "collective"
        if self.dense_transport is None:
            self.dense_transport = self.transport

    @property
    def F(self):
        return len(self.cards)

    @property
    def in_dim(self):
        k = self.F * self.emb_dim + self.n_dense + 1  # + constant-1 bias column
        return (k + 7) // 8 * 8


# where train_step issues the next batch's planning (dedupe, CSR, count exchange) and, with a
# callable next_keys, its generation: "start" | "head" (after the forward) | "dgrad" (after the
# dgrad chain, beside the memory-bound embedding backward) | "push" (after the sparse clock), per
# world size {1: one rank, 2: several}: "dgrad" with the feeder's plan wait (the GPU starts the
# planning there; feeder.LookaheadFeeder.plan_wait); one rank "head" / "push" measured 0.389 /
# 0.371 vs 0.352 ms/step, 8 emulated ranks 0.436-0.452 / 0.437-0.449 vs 0.427-0.441
# (profiles/r5/ab_plan_wait.txt)
_PLAN_AT = {1: "dgrad", 2: "dgrad"}
# issue an async dense clock from the weight-gradient side stream (see train_step). Measured
# slower on one MI355X (OVERLAP_W1=dense: 0.525-0.529 -> 0.544-0.549 ms/step: Adam then
# competes with the memory-bound embedding backward; tools/gpu_round.sh ab), so off by default.
_DENSE_CLOCK_ON_SIDE = False


# Dense layout (see WideDeep.__init__): layer-1 K padding, and bias handling of layers 2/3:
# "ext" (folded, K = 1032 / 520) or "vec" (bias vectors, K = 1024 / 512, colsum bias gradients).
# In the whole W&D step on one MI355X (tools/gpu_round.sh ab, ms/step): ext/8 0.453, ext/64 0.451,
# vec/8 0.460, vec/64 0.457 -- the isolated GEMM gains of "vec" (fwd2 -7 us, W2 wgrad -10 us)
# do not survive the 3-stream overlap (its W2 weight gradient switches to 512 128x128 blocks,
# which crowd the dgrad chain), so "ext" with a 64-aligned layer-1 K was the default through round 3.
# Round 4 (split-K planes folded by Adam, fence-free forks, the rest of this round's step): vec
# 0.3879 / 0.3882 vs ext 0.4016 / 0.4021 ms/step (profiles/r4/ab_wd_knobs.txt) -- "vec" only since
# round 5 (layer 1 keeps its bias folded into column k_in of the padded input).
_K1_ALIGN = 64
# split-K workgroup target of the three weight gradients (ops.linear_wgrad blocks): W&D 0.402 ms at
# 320 vs 0.409-0.412 at the default 512 (GPT-2 keeps 512: 12.90 vs 13.18 ms at 256), ab_wd_r3.txt;
# round 5 (planning mid-step): 0.349-0.351 vs 0.357-0.359 at 192, 0.360-0.361 at 512 (ab_wd_r5.txt)
# round 6 (head fold off the chain, side-stream Adam after the embedding dgrad): 256 -- W1 / W2 / W3 in
# 5 / 8 / 16 slices instead of 6 / 10 / 16, fewer planes for the Adam to fold -- 0.3384-0.3407 vs
# 0.3395-0.3454 at 320, 0.346-0.351 at 192 / 224, 0.351-0.353 at 384 / 448 (ab_wd_r6.txt)
_WGRAD_BLOCKS = 256


# DENSE_ON_SIDE off: one rank's dense Adam on the main stream at the step end (joined)
_DENSE_ON_SIDE = True
# WD_W1_LATE on: fork the layer-1 weight gradient after the embedding dgrad (beside the
# embedding backward rather than beside the dgrad: two big GEMMs at once only share the CUs);
# round 3 measured it 5 % slower (profiles/r3/ab_wd_r3.txt)
# (round 6, the planning mid-step: 0.363 vs 0.342-0.344 ms/step, profiles/r6/ab_wd_r6.txt)
_W1_LATE = False
# the one-rank side-stream Adam waits for the compute stream only up to the embedding dgrad (the
# last reader of W), not up to the end of the step's issue (off: the round-5 fork at the end):
# 0.3514-0.3553 vs 0.3564-0.3568 ms/step (profiles/r6/ab_wd_r6.txt)
_ADAM_AFTER_DGRAD = True
# ROWIDX off: the input assembly follows inv -> uniq instead of the planner's per-lookup rows
_ROWIDX = True
# the dense forward and the backward GEMM chain up to the embedding dgrad, recorded once per set of
# buffers and replayed from a native launch list (layers.Replayer): ~25 binding calls per step leave
# the host path -- wd.bwd_dense host 71 -> 53 us at one rank; step time unchanged there (GPU-bound:
# 0.368-0.370 either way) and at 8 emulated ranks (0.491-0.499 vs 0.488-0.502 ms), where the step
# waits on the planning's count exchange instead (profiles/r5/host_issue.txt). False: op by op.
_REPLAY = True
# the head's batch sums (last-layer weight/bias gradient, layer-3 bias gradient, loss) folded by a
# separate kernel on the weight-gradient stream instead of by the head's last blocks: the two ticketed
# fold levels leave the dgrad chain (head 17 -> 11 us in-step): 0.335-0.339 vs 0.344-0.345 ms/step
# (profiles/r6/ab_wd_r6.txt). False: the round-5 in-kernel fold.
_HEAD_DEFER = True
# (the dgrads beside the weight-gradient stream keep the launcher's 256x256 tile: forcing 128x128 on
# the dH1 / dX dgrad, which shares CUs with the wgrads' 128x128 workgroups, measured 0.336-0.339 /
# 0.344-0.345, both 0.347-0.353, 256x128 0.376-0.379 vs 0.336-0.339 ms; profiles/r6/ab_wd_r6.txt)


# (round 6: per-layer split-K of the weight gradients instead of the workgroup target -- isolated,
# the target's 6 / 10 / 16 splits of W1 / W2 / W3 run 50.6 / 33.9 / 17.7 us against 42.0 / 26.8 /
# 17.7 at 8 / 16 / 16 (profiles/r6/wgrad_split_sweep.txt) -- but in the step the faster, wider
# splits crowd the dgrad chain: 0.363-0.366 ms at 8,16,16 vs 0.354-0.355 at the target, 6,16,16
# 0.352-0.355 (profiles/r6/ab_wd_r6.txt); the knob was removed)
def _wgrad(dH, H, Gw, sink=None):
    # (round 4: the hipBLASLt alternative, WD_WGRAD=lib, measured slower and removed)
    return ops.linear_wgrad(dH, H, Gw, blocks=_WGRAD_BLOCKS, defer=sink)


def _align(n, a=8):
    return (n + a - 1) // a * a


def _table_maker(comm, engine):
    from ..engine import create_table

    if engine is not None:
        return lambda kind, **kw: engine.table(engine.create_table(kind, **kw))
    ids = iter(range(1 << 20))
    return lambda kind, **kw: create_table(comm, kind, table_id=next(ids), **kw)


class WideDeep(LookaheadPlans):
    def __init__(self, cfg: WideDeepConfig, comm: Comm, engine=None):
        self.cfg = cfg
        self.comm = comm
        dev = comm.device
        F, D = cfg.F, cfg.emb_dim
        self.num_rows = int(sum(cfg.cards))
        bases = [sum(cfg.cards[:f]) for f in range(F)]  # feature f's ids start at its offset
        # tables through the Engine factory (minips_amd.engine.create_table): an Engine given here
        # owns them (its create_table / checkpoint / run), otherwise they are built on ``comm``
        make = _table_maker(comm, engine)
        onesided = cfg.transport == "onesided"
        self.emb = make("sparse", num_rows=self.num_rows, width=cfg.row_width, optimizer="rowwise_adagrad",
                        lr=cfg.lr_sparse, model=cfg.consistency, staleness=cfg.staleness, transport=cfg.transport,
                        split=D, init_std=0.01, seed=cfg.seed, columns=(bases, cfg.cards), pull_dtype=torch.bfloat16,
                        **({"max_keys": cfg.max_batch * F} if onesided else {}))
        # wide weights start at zero (columns >= D)
        self.emb.shard[:, D:].zero_()
        # Dense layout: layer 1 is stored as W_ext [n_out, k_pad] with the bias in column k_in; its
        # input carries a constant-1 column at k_in, so the forward GEMM adds the bias and the
        # weight-gradient GEMM yields its gradient (no bias epilogue, no column-sum atomics).
        # Layer 1's k_pad is a multiple of 64: whole 64-deep K-steps and 128-byte rows for the
        # LDS-DMA (K = 896: the 16384x1024 forward takes 30.7 us vs 38.8 us at align8's 848;
        # tools/bench_kernels.py gemm). Layers 2/3 have bias vectors: dH3's column sums come from
        # wd_head, dH2's from a column-sum kernel.
        self.k_in = [cfg.F * cfg.emb_dim + cfg.n_dense, *cfg.hidden[:-1]]
        self.k_pad = [_align(self.k_in[0] + 1, _K1_ALIGN),
                      *self.k_in[1:]]
        self.layout = {}
        off = 0
        for i, n_out in enumerate(cfg.hidden):
            self.layout[f"W{i + 1}"] = (off, (n_out, self.k_pad[i]))
            off += _align(n_out * self.k_pad[i], 64)
            if i > 0:
                self.layout[f"b{i + 1}"] = (off, (n_out,))
                off += _align(n_out, 64)
        self.layout["w4"] = (off, (cfg.hidden[-1] + 8,))  # [w4 | b4 | pad]
        off += cfg.hidden[-1] + 8
        self.n_params = off
        starts = [self.layout[f"W{i + 1}"][0] for i in range(len(cfg.hidden))]
        bucketed = cfg.bucket_mb > 0 and cfg.dense_transport == "collective" and comm.world > 1
        self.dense = make("dense", n_params=self.n_params, optimizer="adam", lr=cfg.lr_dense, model=cfg.consistency,
                          staleness=cfg.staleness, transport=cfg.dense_transport,
                          **(dict(buckets=starts, bucket_mb=cfg.bucket_mb) if bucketed else {}))
        # the bucket each layer's weight gradient completes (None: one clock at the end)
        self._wbucket = [self.dense.bucket_for_layer(x) for x in starts] if bucketed else None
        self.dense.load_full(self._init_dense(dev))
        self._bufs = {}
        self._side = SideStream(dev)
        self._replay = Replayer(self._side) if self._side.stream is not None else None

    def _init_dense(self, dev):
        g = torch.Generator(device="cpu")
        g.manual_seed(self.cfg.seed + 17)
        full = torch.zeros(self.n_params, dtype=torch.float32)
        for i in range(len(self.cfg.hidden)):
            w = self.view(full, f"W{i + 1}")
            ops.kaiming_uniform_(w[:, : self.k_in[i]], self.k_in[i], g)
            w[:, self.k_in[i]:] = 0  # bias column and padding start at zero
        h = self.cfg.hidden[-1]
        ops.kaiming_uniform_(self.view(full, "w4")[:h], h, g)
        return full.to(dev)

    def view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        # ~15 views of the persistent parameter / gradient buffers per step: cached by address
        # (a live cached view keeps its storage, so no other buffer can take that address)
        key = (buf.data_ptr(), buf.dtype, name)
        views = self.__dict__.setdefault("_views", {})
        v = views.get(key)
        if v is None:
            off, shape = self.layout[name]
            n = 1
            for s in shape:
                n *= s
            v = buf[off: off + n].view(shape)
            if buf.is_cuda:
                if len(views) > 256:
                    views.clear()
                views[key] = v
        return v

    def _buffers(self, B):
        if B not in self._bufs:
            dev, cfg = self.comm.device, self.cfg
            bf = dict(dtype=torch.bfloat16, device=dev)
            h1, h2, h3 = cfg.hidden

            X = torch.zeros(B, self.k_pad[0], **bf)  # constant-1 column at k_in (layer-1 bias), zero pad
            X[:, self.k_in[0]] = 1.0

            self._bufs[B] = dict(
                X=X, H1=torch.empty(B, h1, **bf), H2=torch.empty(B, h2, **bf),
                H3=torch.empty(B, h3, **bf), dH3=torch.empty(B, h3, **bf), dH2=torch.empty(B, h2, **bf),
                dH1=torch.empty(B, h1, **bf),
                dX=torch.empty(B, cfg.F * cfg.emb_dim, **bf),  # bf16: half the bytes of the emb backward
                wide=torch.empty(B, dtype=torch.float32, device=dev),
                dwide=torch.empty(B, dtype=torch.float32, device=dev),
                loss=torch.zeros(1, dtype=torch.float32, device=dev),
            )
        return self._bufs[B]

    def _forward(self, b, P):
        ops.linear_fwd(b["X"], self.view(P, "W1"), None, "relu", out=b["H1"])
        ops.linear_fwd(b["H1"], self.view(P, "W2"), self.view(P, "b2"), "relu", out=b["H2"])
        ops.linear_fwd(b["H2"], self.view(P, "W3"), self.view(P, "b3"), "relu", out=b["H3"])

    def forward(self, dense, keys, rows, plan):
        """Forward only (eval): returns logits [B] fp32."""
        B = dense.shape[0]
        b = self._buffers(B)
        pend_side = self.__dict__.pop("_side_pending", None)
        if pend_side is not None:  # the last train step's Adam (side stream) before W is read
            streams.current(self.comm.device).wait_event(pend_side[1])
        P = self.dense.get()
        F, D = self.cfg.F, self.cfg.emb_dim
        ops.wd_assemble(dense, rows, plan.inv, F, D, b["X"], b["wide"], ones_col=self.k_in[0])
        self._forward(b, P)
        h = self.cfg.hidden[-1]
        w4 = self.view(P, "w4").float()
        return b["H3"].float() @ w4[:h] + w4[h] + b["wide"]

    @traced("wd.train_step")
    def train_step(self, dense, keys, labels, next_keys=None, next_on_plan_stream: bool = False) -> torch.Tensor:
        """One BSP superstep: Get, forward, backward, Add, Clock. Returns the summed loss
        (a device tensor; no host sync).

        Ordering for overlap (MI355X: RCCL on side streams, one communicator lane each):
          sparse Get (gather + rows all-to-all) -> assemble -> dense Get (waits for the previous
          dense Clock only here) -> forward -> head -> dgrad chain -> embedding backward ->
          sparse Add+Clock (all-to-all of gradient rows + row-wise Adagrad on the push lane,
          overlapping the weight-gradient GEMMs) -> wgrad GEMMs -> dense Add+Clock
          (reduce-scatter + Adam + all-gather on the dense lane, overlapping the next step's
          sparse Get). ``next_keys`` starts the next batch's key planning right away
          (``next_on_plan_stream``: that batch was generated on the planning stream itself)."""
        cfg = self.cfg
        B = dense.shape[0]
        F, D = cfg.F, cfg.emb_dim
        h = cfg.hidden[-1]
        b = self._buffers(B)
        plan = self._take_plan(keys)  # issued ahead (LookaheadPlans.prefetch) or planned now

        def issue_next(point):
            # next_keys may be a callable that produces the next batch (on the planning stream)
            # when called: the planning work then starts at _PLAN_AT, not at the step start
            if next_keys is not None and point == _PLAN_AT[min(2, self.comm.world)]:
                nk = next_keys() if callable(next_keys) else next_keys
                self.prefetch(nk, keys_on_plan_stream=next_on_plan_stream)

        with phase("wd.plan_next"):
            issue_next("start")
        pend_side = self.__dict__.pop("_side_pending", None)
        if pend_side is not None and pend_side[0] is not None:  # the previous step's weight gradients
            streams.current(self.comm.device).wait_event(pend_side[0])  # read X: done before it is rewritten
        ph = phase("wd.get_assemble")
        ph.__enter__()
        src = self.emb.get_source(keys, plan=plan)  # one rank: the rows are read in place
        if src is not None:
            plan, table, index, base = src
            # (members, memrow, positions, rowstart, rowidx): the planner's per-lookup rows
            rowidx = plan.csr[4] if plan.csr is not None and len(plan.csr) >= 5 and _ROWIDX else None
            ops.wd_assemble_tab(dense, table, index, base, plan.inv, F, D, b["X"], b["wide"], ones_col=self.k_in[0],
                                zero=b["loss"], rowidx=rowidx)
        else:
            rows, plan = self.emb.get(keys, plan=plan)
            ops.wd_assemble(dense, rows, plan.inv, F, D, b["X"], b["wide"], ones_col=self.k_in[0], zero=b["loss"])
        if pend_side is not None:  # ... and its dense Adam ran (side stream) before the forward reads W
            streams.current(self.comm.device).wait_event(pend_side[1])
        ph.__exit__(None, None, None)
        ph = phase("wd.fwd_head")
        ph.__enter__()
        G = self.dense.grad
        P = self.dense.get()
        scale = 1.0 / (B * self.comm.world)
        w4, gw4 = self.view(P, "w4"), self.view(G, "w4")
        sink = self.dense.slab_sink() if hasattr(self.dense, "slab_sink") else None
        side = self._side
        defer = _HEAD_DEFER and side.stream is not None
        rp = self._replay if (self._replay is not None and _REPLAY and self._wbucket is None
                              and streams.DELAY_US <= 0 and not torch.cuda.is_current_stream_capturing()) else None
        key = (B, P.data_ptr(), G.data_ptr(), sink is not None, defer)
        if rp is not None:
            rp(("fwd",) + key, lambda: self._forward(b, P))
        else:
            self._forward(b, P)
        # the head also sums dH3 over the batch (per-block partials): the layer-3 bias gradient
        ops.wd_head(b["H3"], w4[:h], w4[h:h + 1], b["wide"], labels, b["dH3"], gw4[:h], gw4[h:h + 1],
                    b["dwide"], b["loss"], self.view(G, "b3"), scale, defer_fold=defer)
        ph.__exit__(None, None, None)
        ph = phase("wd.bwd_dense")
        ph.__enter__()
        issue_next("head")
        # weight gradients fork onto a second stream as soon as their inputs exist, beside the
        # dgrad chain (their split-K tails and reduces fill the gaps of the dependent chain).
        # Each fork records an event on the compute stream (~2-4 us queue bubble on MI355X), but
        # fewer, later forks lose more overlap than they save: W3+W2 forked together 0.431-0.438,
        # all three after dgrad1 0.446 vs 0.418-0.421 ms/step (profiles/r3/ab_wd_forks.txt)
        # one rank: the weight gradients' split-K slices are folded by the dense table's Adam (sink)
        fold = (B, h, gw4[:h], gw4[h:h + 1], b["loss"], self.view(G, "b3")) if defer else None
        if rp is not None:
            rp(("bwd",) + key, lambda: self._backward_chain(b, P, G, sink, side, fold))
        else:
            self._backward_chain(b, P, G, sink, side, fold)
        # the embedding gradient leaves the dgrad GEMM already in the planner's row-sorted order
        # (one 64-byte row per lookup, grouped by unique key), so the embedding backward reads one
        # contiguous stream instead of gathering 64-byte pieces of [B, F*D] rows
        # (members, memrow, positions or None[, rowstart]): positions -> the dgrad writes the rows sorted
        sorted_rows = plan.csr is not None and len(plan.csr) >= 3 and plan.csr[2] is not None
        if sorted_rows:
            ops.linear_dgrad(b["dH1"], self.view(P, "W1"), n_cols=F * D, out=b["dX"].view(B * F, D),
                             perm=plan.csr[2], seg=D)
        else:
            ops.linear_dgrad(b["dH1"], self.view(P, "W1"), n_cols=F * D, out=b["dX"])
        # W's last reader of the step is issued: a side-stream dense Adam may start after this point
        w_read = side.point() if _ADAM_AFTER_DGRAD and self.comm.world == 1 else None
        if _W1_LATE:  # the layer-1 weight gradient beside the memory-bound embedding backward instead
            with side.fork():
                _wgrad(b["dH1"], b["X"], self.view(G, "W1"), sink)
        # an async dense clock (its own stream) needs only the weight gradients: issued from the
        # side stream it starts as soon as the last wgrad ends, beside the embedding backward and
        # the sparse push, instead of behind them
        pipe = getattr(self.dense, "pipe", None)  # (collective tables only)
        dense_early = _DENSE_CLOCK_ON_SIDE and pipe is not None and pipe.async_ and side.stream is not None
        if dense_early:  # (side.fork: the clock's Adam rewrites W after the embedding dgrad read it)
            with side.fork():
                self.dense.add()
                self.dense.clock()
        issue_next("dgrad")
        ph.__exit__(None, None, None)
        ph = phase("wd.emb_push")
        ph.__enter__()
        dXe = b["dX"].view(B * F, D) if sorted_rows else b["dX"]
        self.emb.add_lookup_grads(plan, dXe, b["dwide"], F, D, sorted_rows=sorted_rows)  # the table reduces
        self.emb.clock()
        issue_next("push")
        ph.__exit__(None, None, None)
        ph = phase("wd.dense_clock")
        ph.__enter__()
        capturing = side.stream is not None and torch.cuda.is_current_stream_capturing()
        dense_side = (_DENSE_ON_SIDE and not dense_early and side.stream is not None and self.comm.world == 1
                      and pipe is not None and not pipe.async_ and not capturing)
        # the one-sided dense table (ps/onesided.py): its clock -- the push into the owners' inboxes
        # -- only needs the weight gradients, and the next step's reads are SSP-stale anyway, so it
        # goes on the side stream too (the next step's Get and assembly overlap the wgrad tail)
        dense_side = dense_side or (_DENSE_ON_SIDE and side.stream is not None and pipe is None
                                    and getattr(self.dense, "side_clock_ok", False) and not capturing)
        if dense_side:
            # one rank, synchronous clock: the dense Adam runs on the side stream right behind the
            # last weight gradient, and the main stream does not join here -- the next step waits
            # for the weight gradients before its assembly rewrites X and for the Adam (or the
            # one-sided push, which reads and clears the gradient buffer) before its forward reads W
            # and its head writes gradients, so the clock overlaps the next step's input assembly
            # The Adam rewrites W, which this step's embedding dgrad (issued on the compute stream
            # after the last weight-gradient fork) still reads: the side stream first waits for the
            # compute stream (side.fork) -- a missing edge by construction. With the edge, repeated
            # op-by-op runs stopped varying at the 4th decimal (profiles/r5/race_dgrad_adam.txt)
            ev_x = side.mark()
            if defer:  # the returned loss is folded on the side stream: final on the compute stream
                side.wait(ev_x)  # (the next step's assembly waited for this point anyway)
            with side.fork(after=w_read):
                self.dense.add()
                self.dense.clock()
            self._side_pending = (None if defer else ev_x, side.mark())
            if hasattr(self.dense, "hold"):  # a checkpoint (drain) waits for this Adam too
                self.dense.hold(self._side_pending[1])
        else:
            side.join()
            if not dense_early:
                self.dense.add()
                self.dense.clock()
        ph.__exit__(None, None, None)
        with phase("wd.advance_plans"):
            self._advance_next_plan()
        return b["loss"]

    def _backward_chain(self, b, P, G, sink, side, fold=None):
        """dgrad chain down to dH1 with the three weight gradients (and the layer-2 bias gradient)
        forked beside it: GEMM-family ops and forks only (replayable, see layers.Replayer).
        ``fold``: wd_head_fold's arguments (the head deferred its batch sums), run first on the
        side stream."""
        k3 = self.k_in[2]
        with side.fork():
            if fold is not None:
                ops.wd_head_fold(*fold)
            _wgrad(b["dH3"], b["H2"], self.view(G, "W3"), sink)
        ops.linear_dgrad(b["dH3"], self.view(P, "W3"), mask=b["H2"], n_cols=k3, out=b["dH2"])
        with side.fork():
            ops.colsum_add(b["dH2"], self.view(G, "b2"))  # the layer-2 bias gradient
            _wgrad(b["dH2"], b["H1"], self.view(G, "W2"), sink)
        ops.linear_dgrad(b["dH2"], self.view(P, "W2"), mask=b["H1"], n_cols=self.k_in[1], out=b["dH1"])
        self._bucket_done(1, side)  # (layers 2, 3 and the head: their weight gradients are issued)
        if not _W1_LATE:
            with side.fork():
                _wgrad(b["dH1"], b["X"], self.view(G, "W1"), sink)

    def _bucket_done(self, layer: int, side):
        """Every layer >= ``layer`` has its weight gradient issued (on the side stream): the buckets
        starting at or above layer ``layer``'s offset go out now (several ranks, bucketed clocks)."""
        if self._wbucket is None:
            return
        k = self._wbucket[layer]
        if k is not None and all(b is None or b >= k for b in self._wbucket[layer:]):
            for j in sorted({b for b in self._wbucket[layer:] if b is not None}, reverse=True):
                self.dense.bucket_ready(j, events=(side.mark(),))

    def drain(self):
        pend_side = self.__dict__.pop("_side_pending", None)
        if pend_side is not None:
            streams.current(self.comm.device).wait_event(pend_side[1])
        self.emb.drain()
        self.dense.drain()
