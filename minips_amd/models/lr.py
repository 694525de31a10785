"""Sparse logistic regression on the GPU parameter server (BASELINE config 1, reference
examples/lr_example.cpp): one width-1 fp32 SparseTable row per feature, the server apply is the
reference's plain ``w += delta`` ("add"), and the worker computes
delta[col] = alpha * sum_rows x * (y - sigmoid(w . x)) for the features present in its batch
(lr_example.cpp:291-312) with the fused ``lr_sparse_step`` kernel over the pulled rows.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .. import ops
from ..ps.comm import Comm
from ..ps.tables import HashSparseTable, SparseTable


@dataclass
class SparseLRConfig:
    num_dims: int = 16_609_143  # webspam trigram feature count (reference default num_dims)
    alpha: float = 0.1
    consistency: str = "bsp"
    staleness: int = 0
    storage: str = "vector"  # reference kStorageType: "vector" (dense key range) or "map" (hash)
    value_dtype: torch.dtype = torch.float32  # float64: the reference's CreateTable<double>


class SparseLR:
    def __init__(self, cfg: SparseLRConfig, comm: Comm):
        self.cfg, self.comm = cfg, comm
        if cfg.storage.lower() == "map":  # MapStorage: rows created on first touch, zero-initialised
            self.table = HashSparseTable(comm, 1, optimizer="add", pull_dtype=torch.float32, init_std=0.0,
                                         consistency=cfg.consistency, staleness=cfg.staleness)
        elif cfg.storage.lower() == "vector":
            self.table = SparseTable(comm, cfg.num_dims, 1, optimizer="add", pull_dtype=torch.float32, init_std=0.0,
                                     consistency=cfg.consistency, staleness=cfg.staleness,
                                     value_dtype=cfg.value_dtype)
        else:
            raise ValueError(f"kStorageType {cfg.storage!r}: Map or Vector")

    def train_step(self, rowptr, cols, vals, labels):
        """CSR batch (rowptr [B+1], cols/vals [nnz], labels [B] in {0,1} or {-1,1}).
        Returns the number of correctly classified rows (before the update)."""
        dev = self.comm.device
        rows, plan = self.table.get(cols)
        delta = torch.zeros(max(plan.cap, 1), dtype=rows.dtype, device=dev)
        correct = torch.zeros(1, dtype=torch.float32, device=dev)
        if plan.cap:
            ops.lr_sparse_step(rowptr, plan.inv, vals, labels, rows.view(-1)[: plan.cap], self.cfg.alpha,
                               delta[: plan.cap], correct)
            self.table.add(plan, delta.view(-1, 1))
        self.table.clock()
        return correct

    def evaluate(self, rowptr, cols, vals, labels):
        w = self.table.get_rows(cols).view(-1)
        correct = torch.zeros(1, dtype=torch.float32, device=self.comm.device)
        idx = torch.arange(cols.numel(), device=cols.device)
        ops.lr_sparse_step(rowptr, idx, vals, labels, w, 0.0, None, correct)
        return correct

    def drain(self):
        self.table.drain()
