"""DLRM-style model with a (up to) 10B-row embedding table sharded over the PS ranks
(BASELINE config 5), asynchronous SGD by default.

  sparse: one SparseTable row per categorical id, width D (default 64), 64-bit keys, row-wise
          Adagrad (1 float of optimizer state per row), bf16 rows by default: 10B rows x 64 bf16 =
          1.28 TB of weights + 40 GB of state over 8 x 288 GB (fp32 rows would be 2.56 TB).
  dense:  bottom MLP 13 -> 512 -> 256 -> D, dot interaction of the D-vector with the 26
          embeddings (351 pairs + D), top MLP 416 -> 512 -> 256 -> 1, BCE. One DenseTable.
Consistency "asp" on the collective transport runs every Clock's exchange (all-to-all-v over
RCCL point-to-point send/recv + apply) on a side stream, gating the next Gets at a 2-clock
pipelining depth; transport "onesided" is the unbounded asynchronous PS (ps/onesided.py).
"bsp"/"ssp" are available as for the other models.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from .. import ops
from ..ps.comm import Comm
from .widedeep import _table_maker
from .layers import SideStream, Linear, ParamLayout, align, ext_activation
from .feeder import LookaheadPlans


@dataclass
class DLRMConfig:
    num_rows: int = 10_000_000_000
    F: int = 26
    n_dense: int = 13
    D: int = 64
    bottom: tuple = (512, 256)
    top: tuple = (512, 256)
    lr_dense: float = 1e-3
    lr_sparse: float = 0.02
    consistency: str = "asp"
    staleness: int = 0
    p2p: bool = True
    # "collective": SparseTable / DenseTable over RCCL (all-to-all-v / RS+AG, gated per consistency);
    # "onesided": SSP / ASP with NO collective on the data path -- rows read from the owners'
    # IPC-mapped HBM over xGMI, gradients pushed into the owners' inboxes, row-wise Adagrad / Adam
    # applied by each owner's server thread with its own state (ps/onesided.py);
    # "auto" (default): onesided for SSP / ASP (the asynchronous PS is what those models mean),
    # collective for BSP
    transport: str = "auto"
    max_batch: int = 16384       # onesided: inbox slots hold max_batch * F gradient rows
    # embedding rows in bf16 (fp32 row-wise Adagrad state, stochastically rounded applies): the
    # default 10B x 64 table is 1.28 TB of rows + 40 GB of state = 8 x 165 GB, inside 8 x 288 GB
    # (fp32 rows would need 2.56 TB). Both transports store them so (the one-sided owners apply
    # in fp32 and round back stochastically, csrc/kernels/onesided.hip).
    emb_dtype: str = "bfloat16"
    seed: int = 0
    cards: list = field(default_factory=list)  # optional per-feature cardinalities (sum <= num_rows)

    def __post_init__(self):
        if self.transport == "auto":
            self.transport = "onesided" if self.consistency in ("ssp", "asp") else "collective"


class DLRM(LookaheadPlans):
    def __init__(self, cfg: DLRMConfig, comm: Comm, engine=None):
        self.cfg, self.comm = cfg, comm
        D, F = cfg.D, cfg.F
        self.NV = F + 1
        make = _table_maker(comm, engine)
        onesided = cfg.transport == "onesided"
        self.emb = make("sparse", num_rows=cfg.num_rows, width=D, optimizer="rowwise_adagrad", lr=cfg.lr_sparse,
                        model=cfg.consistency, staleness=cfg.staleness, transport=cfg.transport, init_std=0.01,
                        seed=cfg.seed, pull_dtype=torch.bfloat16,
                        value_dtype=getattr(torch, cfg.emb_dtype),
                        **({"max_keys": cfg.max_batch * F} if onesided else {"p2p": cfg.p2p}))
        self.layout = ParamLayout()
        dims = [cfg.n_dense, *cfg.bottom, D]
        self.bottom = [Linear(self.layout, f"bot{i}", dims[i], dims[i + 1]) for i in range(len(dims) - 1)]
        self.n_int = D + self.NV * (self.NV - 1) // 2
        tdims = [self.n_int, *cfg.top]
        self.top = [Linear(self.layout, f"top{i}", tdims[i], tdims[i + 1]) for i in range(len(tdims) - 1)]
        self.layout.add("head", (cfg.top[-1] + 8,))
        self.dense = make("dense", n_params=self.layout.size, optimizer="adam", lr=cfg.lr_dense, model=cfg.consistency,
                          staleness=cfg.staleness, transport=cfg.transport, **({} if onesided else {"p2p": False}))
        g = torch.Generator().manual_seed(cfg.seed + 3)
        full = torch.zeros(self.layout.size)
        for l in self.bottom + self.top:
            l.init(full, g)
        h = self.layout.view(full, "head")
        h[: cfg.top[-1]].uniform_(-cfg.top[-1] ** -0.5, cfg.top[-1] ** -0.5, generator=g)
        self.dense.load_full(full)
        self._bufs = {}
        # weight gradients inline by default: with the round-2 MFMA interaction the dgrad chain is
        # short and the side stream's contention costs more than the overlap gains (1 GPU: 0.686
        # inline vs 0.714 ms/step forked); DLRM_WGRAD_STREAM on forks them
        self._side = SideStream(comm.device, False)

    def _buffers(self, B):
        if B not in self._bufs:
            dev, cfg = self.comm.device, self.cfg
            bf = dict(dtype=torch.bfloat16, device=dev)
            bdims = [cfg.n_dense, *cfg.bottom]
            self._bufs[B] = dict(
                bacts=[ext_activation(B, d, dev) for d in bdims],
                bgrads=[torch.empty(B, d, **bf) for d in cfg.bottom],
                V=torch.zeros(B, self.NV * cfg.D, **bf),
                tacts=[ext_activation(B, self.n_int, dev)] + [ext_activation(B, d, dev) for d in cfg.top[:-1]],
                H=torch.empty(B, cfg.top[-1], **bf), dH=torch.empty(B, cfg.top[-1], **bf),
                tgrads=[torch.empty(B, d, **bf) for d in cfg.top[:-1]],
                dI=torch.zeros(B, align(self.n_int), **bf),
                # bf16 interaction gradient: half the bytes the embedding backward gathers
                # (the MFMA interaction kernel writes it directly; fp32 only off the MFMA shapes)
                dV=torch.empty(B, self.NV * cfg.D, dtype=torch.bfloat16 if self.NV <= 32 and cfg.D in (16, 32, 64)
                               and dev.type == "cuda" else torch.float32, device=dev),
                dbot=torch.empty(B, cfg.D, **bf),
                zero=torch.zeros(B, dtype=torch.float32, device=dev),
                dwide=torch.empty(B, dtype=torch.float32, device=dev),
                loss=torch.zeros(1, device=dev),
            )
        return self._bufs[B]

    def train_step(self, dense, keys, labels, next_keys=None, next_on_plan_stream: bool = False):
        cfg = self.cfg
        B, F, D = dense.shape[0], cfg.F, cfg.D
        b = self._buffers(B)
        plan = self._take_plan(keys)
        if next_keys is not None:
            nk = next_keys() if callable(next_keys) else next_keys
            self.prefetch(nk, keys_on_plan_stream=next_on_plan_stream)
        rows, plan = self.emb.get(keys, plan=plan)
        G = self.dense.grad
        # V = [emb_0 .. emb_{F-1} | bottom(dense)]  (the dense vector is the last one)
        ops.lookup_rows(rows, plan.inv, F, D, b["V"])
        P = self.dense.get()
        ba = b["bacts"]
        ba[0][:, : cfg.n_dense].copy_(dense)
        for i, l in enumerate(self.bottom):
            out = ba[i + 1] if i + 1 < len(self.bottom) else b["V"][:, F * D:]
            l.forward(P, ba[i], out, "relu")
        ta = b["tacts"]
        ops.dlrm_interact_fwd(b["V"], self.NV, D, ta[0], dense_idx=F)
        for i, l in enumerate(self.top):
            out = ta[i + 1] if i + 1 < len(self.top) else b["H"]
            l.forward(P, ta[i], out, "relu")
        hw = self.layout.view(P, "head")
        hg = self.layout.view(G, "head")
        h = cfg.top[-1]
        b["loss"].zero_()
        ops.wd_head(b["H"], hw[:h], hw[h:h + 1], b["zero"], labels, b["dH"], hg[:h], hg[h:h + 1], b["dwide"],
                    b["loss"], None, 1.0 / (B * self.comm.world))
        # dgrad chain first (top MLP -> interaction), then the embedding gradient goes out on the
        # sparse push lane while the weight-gradient GEMMs run on the compute stream
        dy = b["dH"]
        side = self._side
        # split-K weight-gradient planes summed by the dense update (the Adam, or the one-sided push)
        # instead of reduce kernels (up to 4 regions: the top MLP's, issued first)
        sink = self.dense.slab_sink() if hasattr(self.dense, "slab_sink") else None
        for i in range(len(self.top) - 1, -1, -1):
            l = self.top[i]
            with side.fork():  # weight gradients beside the dgrad chain (per-layer buffers: no reuse)
                l.wgrad(G, dy, ta[i], sink)
            if i > 0:
                dx = b["tgrads"][i - 1]
                l.dgrad(P, dy, dx, mask=ta[i])
            else:
                dx = b["dI"]
                l.dgrad(P, dy, dx)
            dy = dx
        ops.dlrm_interact_bwd(b["V"], self.NV, D, b["dI"], b["dV"], b["dbot"], dense_idx=F)
        self.emb.add_lookup_grads(plan, b["dV"], None, F, D)
        self.emb.clock()
        dy = b["dbot"]
        for i in range(len(self.bottom) - 1, -1, -1):
            l = self.bottom[i]
            with side.fork():
                l.wgrad(G, dy, ba[i], sink)
            if i > 0:
                dx = b["bgrads"][i - 1]
                l.dgrad(P, dy, dx, mask=ba[i])
                dy = dx
        side.join()
        self.dense.add()
        self.dense.clock()
        self._advance_next_plan()
        return b["loss"]

    def drain(self):
        self.emb.drain()
        self.dense.drain()
