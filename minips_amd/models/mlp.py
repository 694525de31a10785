"""3-layer MLP on MNIST-shaped synthetic data with dense push/pull under BSP (BASELINE
config 2): 784 -> 512 -> 512 -> 10, ReLU, softmax cross-entropy; all parameters in one
DenseTable (reduce-scatter of gradients, fused Adam on the owned shard, all-gather pull).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .. import ops
from ..ps.comm import Comm
from ..ps.tables import DenseTable
from .layers import Linear, ParamLayout, SideStream, align, ext_activation


@dataclass
class MLPConfig:
    in_dim: int = 784
    hidden: tuple = (512, 512)
    classes: int = 10
    lr: float = 1e-3
    optimizer: str = "adam"
    consistency: str = "bsp"
    staleness: int = 0
    seed: int = 0


class MLP:
    def __init__(self, cfg: MLPConfig, comm: Comm):
        self.cfg, self.comm = cfg, comm
        self.layout = ParamLayout()
        dims = [cfg.in_dim, *cfg.hidden]
        self.layers = [Linear(self.layout, f"fc{i}", dims[i], dims[i + 1]) for i in range(len(cfg.hidden))]
        self.cpad = align(cfg.classes)
        self.layers.append(Linear(self.layout, "out", dims[-1], cfg.classes, n_pad=self.cpad))
        self.table = DenseTable(comm, self.layout.size, optimizer=cfg.optimizer, lr=cfg.lr,
                                consistency=cfg.consistency, staleness=cfg.staleness)
        g = torch.Generator().manual_seed(cfg.seed)
        full = torch.zeros(self.layout.size)
        for l in self.layers:
            l.init(full, g)
        self.table.load_full(full)
        self._bufs = {}
        # weight gradients inline by default: this step is too small for a side stream to pay
        # (measured 0.424 vs 0.350 ms per step at batch 8192); MLP_WGRAD_STREAM on forks them
        self._side = SideStream(comm.device, False)

    def _buffers(self, B):
        if B not in self._bufs:
            dev = self.comm.device
            acts = [ext_activation(B, self.cfg.in_dim, dev)] + [ext_activation(B, h, dev) for h in self.cfg.hidden]
            grads = [torch.empty(B, h, dtype=torch.bfloat16, device=dev) for h in self.cfg.hidden]
            self._bufs[B] = dict(acts=acts, grads=grads,
                                 logits=torch.zeros(B, self.cpad, dtype=torch.bfloat16, device=dev),
                                 loss=torch.zeros(1, device=dev), correct=torch.zeros(1, device=dev))
        return self._bufs[B]

    def train_step(self, x, y):
        """x [B, 784] fp32, y [B] int64. Returns (loss_sum, correct) device tensors."""
        B = x.shape[0]
        b = self._buffers(B)
        acts = b["acts"]
        acts[0][:, : self.cfg.in_dim].copy_(x)
        P = self.table.get()
        G = self.table.grad
        for i, l in enumerate(self.layers[:-1]):
            l.forward(P, acts[i], acts[i + 1], "relu")
        logits = b["logits"]
        self.layers[-1].forward(P, acts[-1], logits, "none")
        b["loss"].zero_()
        b["correct"].zero_()
        ops.softmax_xent(logits, self.cfg.classes, y, 1.0 / (B * self.comm.world), b["loss"], b["correct"])
        dy = logits  # in place: (softmax - onehot) / global batch, zero padding columns
        side = self._side
        # split-K weight-gradient planes summed by the table's Adam (no reduce kernels; None for
        # other optimizers / several ranks)
        sink = self.table.slab_sink()
        for i in range(len(self.layers) - 1, -1, -1):
            l = self.layers[i]
            with side.fork():
                l.wgrad(G, dy, acts[i], sink)
            if i > 0:
                dx = b["grads"][i - 1]
                l.dgrad(P, dy, dx, mask=acts[i])
                dy = dx
        side.join()
        self.table.add()
        self.table.clock()
        return b["loss"], b["correct"]

    def drain(self):
        self.table.drain()
