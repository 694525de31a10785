"""Mini-batch K-Means on the GPU parameter server (reference examples/kmeans_example.cpp):
the K x D centres and the K member counts live in one DenseTable with the plain ``add`` apply.
Each Clock a worker assigns its batch to the nearest centres (fused ``kmeans_assign`` kernel),
accumulates per-centre sums/counts (scatter-add), and pushes
    dC_k = (sum_k - n_k C_k) / (N_k + n_k_global)      dN_k = n_k
i.e. the learning rate 1/count of the reference's per-point update, applied per batch.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .. import ops
from ..ps.comm import Comm
from ..ps.tables import DenseTable


@dataclass
class KMeansConfig:
    K: int = 100
    dims: int = 128
    consistency: str = "bsp"
    staleness: int = 0
    seed: int = 0


class KMeans:
    def __init__(self, cfg: KMeansConfig, comm: Comm, init_centres: torch.Tensor | None = None):
        self.cfg, self.comm = cfg, comm
        K, D = cfg.K, cfg.dims
        self.table = DenseTable(comm, K * D + K, optimizer="add", pull_dtype=torch.float32,
                                consistency=cfg.consistency, staleness=cfg.staleness)
        full = torch.zeros(K * D + K)
        if init_centres is None:
            g = torch.Generator().manual_seed(cfg.seed)
            init_centres = torch.randn(K, D, generator=g)
        full[: K * D] = init_centres.reshape(-1).float()
        self.table.load_full(full)

    def centres(self):
        K, D = self.cfg.K, self.cfg.dims
        return self.table.get()[: K * D].view(K, D)

    def train_step(self, X):
        """X [B, D] fp32. Returns the batch's summed squared distance (before the update)."""
        K, D = self.cfg.K, self.cfg.dims
        dev = self.comm.device
        P = self.table.get()
        C = P[: K * D].view(K, D)
        N = P[K * D: K * D + K]
        dist = torch.empty(X.shape[0], dtype=torch.float32, device=dev)
        assign = ops.kmeans_assign(X, C, dist=dist)
        idx = assign.to(torch.int64)
        sums = torch.zeros(K, D, dtype=torch.float32, device=dev)
        ops.scatter_add_rows(X.contiguous(), idx, sums)
        n = torch.bincount(idx, minlength=K).to(torch.float32)
        n_glob = self.comm.all_reduce_(n.clone())
        denom = (N + n_glob).clamp_min(1.0)
        G = self.table.grad
        G[: K * D].view(K, D).copy_((sums - n[:, None] * C) / denom[:, None])
        G[K * D: K * D + K].copy_(n)
        self.table.add()
        self.table.clock()
        return dist.sum()

    def drain(self):
        self.table.drain()
