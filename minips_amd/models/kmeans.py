"""Mini-batch K-Means on the GPU parameter server (reference apps/kmeans/kmeans.cpp), on dense
points (train_step) or sparse libsvm/CSR points (train_step_csr, the reference's input):
the K x D centres and the K member counts live in one DenseTable with the plain ``add`` apply.
Each Clock a worker assigns its batch to the nearest centres (fused ``kmeans_assign`` kernel),
accumulates per-centre sums/counts (scatter-add), and pushes
    dC_k = (sum_k - n_k C_k) / (N_k + n_k_global)      dN_k = n_k
i.e. the learning rate 1/count of the reference's per-point update, applied per batch.

Centre seeding (reference apps/kmeans/kmeans_helper.hpp:68-207, run by worker 0 in
apps/kmeans/kmeans.cpp:154-192): ``init_centres`` does random / kmeans++ / kmeans_parallel on
the GPU -- every D^2 step is one ``kmeans_assign`` distance pass (MFMA form once the candidate
set is large), sampling stays on the device (``torch.multinomial``), and with several ranks
rank 0 seeds from its local data and the result is broadcast (sum all-reduce of a zeroed
buffer), so every rank loads the same table.
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
    init_mode: str = "random"  # random / kmeans++ / kmeans_parallel (used with init_data)


def _min_sqdist(X, C):
    dist = torch.empty(X.shape[0], dtype=torch.float32, device=X.device)
    ops.kmeans_assign(X, C, dist=dist)
    return dist.clamp_min_(0.0)


def _d2_sample(P, K, gen, weights=None, first=None):
    """k-means++ D^2 sampling of K rows of P (optionally weighted); stays on the device."""
    n = P.shape[0]
    w = torch.ones(n, dtype=torch.float32, device=P.device) if weights is None else weights.float()
    i0 = torch.multinomial(w, 1, generator=gen) if first is None else first
    idx = [i0]
    d = _min_sqdist(P, P[i0])
    for _ in range(1, K):
        p = d * w
        # all mass on already-chosen points (duplicates): fall back to the weights
        p = torch.where(p.sum() > 0, p, w)
        i = torch.multinomial(p, 1, generator=gen)
        idx.append(i)
        d = torch.minimum(d, _min_sqdist(P, P[i]))
    return P[torch.cat(idx)].clone()


def init_centres(X, K, mode="kmeans++", seed=0, comm: Comm | None = None, rounds=5, oversample=None):
    """Seed K centres from the local data X [n, D] fp32 (reference kmeans_helper.hpp:68-207).

    random          : K distinct rows chosen uniformly.
    kmeans++        : D^2 sampling, one new centre per distance pass.
    kmeans_parallel : k-means|| -- ``rounds`` passes each keeping every point with probability
                      l*d(x)/sum d (l = oversample, default 2K), candidates weighted by the
                      points they attract, then weighted k-means++ down to K.
    With ``comm`` over several ranks rank 0 seeds and the centres are broadcast."""
    X = X.float().contiguous()
    dev = X.device
    K = int(K)
    if comm is not None and comm.world > 1 and comm.rank != 0:
        C = torch.zeros(K, X.shape[1], dtype=torch.float32, device=dev)
        return comm.all_reduce_(C)
    gen = torch.Generator(device=dev).manual_seed(int(seed))
    n = X.shape[0]
    if n < K:
        raise ValueError(f"need at least K={K} points to seed, got {n}")
    if mode == "random":
        C = X[torch.randperm(n, generator=gen, device=dev)[:K]].clone()
    elif mode == "kmeans++":
        C = _d2_sample(X, K, gen)
    elif mode == "kmeans_parallel":
        l = float(oversample or 2 * K)
        i0 = torch.randint(0, n, (1,), generator=gen, device=dev)
        cand = [X[i0]]
        d = _min_sqdist(X, cand[0])
        for _ in range(int(rounds)):
            tot = d.sum()
            keep = torch.rand(n, generator=gen, device=dev) < (l * d / tot.clamp_min(1e-30))
            new = X[keep]
            if new.shape[0] == 0:
                continue
            cand.append(new)
            d = torch.minimum(d, _min_sqdist(X, new))
        Cand = torch.cat(cand)
        if Cand.shape[0] < K:  # too few candidates: top up with random points
            extra = X[torch.randperm(n, generator=gen, device=dev)[: K - Cand.shape[0]]]
            Cand = torch.cat([Cand, extra])
        a = ops.kmeans_assign(X, Cand).to(torch.int64)
        w = torch.bincount(a, minlength=Cand.shape[0]).float().clamp_min_(1e-3)
        C = _d2_sample(Cand, K, gen, weights=w)
    else:
        raise ValueError(f"unknown kmeans init mode {mode!r}")
    if comm is not None and comm.world > 1:
        comm.all_reduce_(C)
    return C


_seed_centres = init_centres  # KMeans.__init__'s ``init_centres`` argument shadows the name


def sampled_sse(X, C, n=50, seed=0):
    """Mean squared distance of ``n`` sampled points to their nearest centre (the reference's
    report worker, kmeans_helper.hpp:235-266)."""
    g = torch.Generator(device=X.device).manual_seed(int(seed))
    idx = torch.randint(0, X.shape[0], (min(n, X.shape[0]),), generator=g, device=X.device)
    return float(_min_sqdist(X[idx].float().contiguous(), C.float().contiguous()).mean())


class KMeans:
    def __init__(self, cfg: KMeansConfig, comm: Comm, init_centres: torch.Tensor | None = None,
                 init_data: torch.Tensor | None = None):
        self.cfg, self.comm = cfg, comm
        K, D = cfg.K, cfg.dims
        self.table = DenseTable(comm, K * D + K, optimizer="add", pull_dtype=torch.float32,
                                consistency=cfg.consistency, staleness=cfg.staleness)
        full = torch.zeros(K * D + K)
        if init_centres is None and init_data is not None:
            init_centres = _seed_centres(init_data, K, cfg.init_mode, cfg.seed, comm).cpu()
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

    def train_step_csr(self, rowptr, cols, vals):
        """Sparse points (CSR batch; the reference clusters libsvm rows, kmeans_helper.hpp:45-66,
        kmeans.cpp:238-267) against the dense centres: the same batched 1/count update as
        train_step. Returns the batch's summed squared distance (before the update)."""
        K, D = self.cfg.K, self.cfg.dims
        dev = self.comm.device
        P = self.table.get()
        C = P[: K * D].view(K, D)
        N = P[K * D: K * D + K]
        n_pts = rowptr.numel() - 1
        dist = torch.empty(n_pts, dtype=torch.float32, device=dev)
        assign = ops.kmeans_assign_csr(rowptr, cols, vals, C, dist=dist)
        sums = torch.zeros(K, D, dtype=torch.float32, device=dev)
        ops.kmeans_csr_accum(rowptr, cols, vals, assign, sums)
        n = torch.bincount(assign.to(torch.int64), minlength=K).to(torch.float32)
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
