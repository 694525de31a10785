"""Synthetic data generators shaped like the BASELINE configs (no datasets are downloadable).

* Criteo-shaped click logs (Wide&Deep / DLRM): 13 dense features ~ N(0,1), 26 categorical
  features with the Criteo-Kaggle cardinalities; ids are drawn log-uniformly (a Zipf(1)-like
  head: P(id <= k) = ln(k+1)/ln(card)) and scattered by a bijective multiplicative hash so the
  hot ids spread over all server shards. Labels are a noisy function of the features, so the
  loss decreases during training.
* MNIST-shaped dense batches (784 -> 10 classes), GPT-2 token batches, webspam-shaped sparse
  LR batches (16.6M feature ids, libsvm-like nnz per row).
All generation happens on the target device with a torch.Generator (deterministic per rank).
"""
from __future__ import annotations

import math

import torch

# Criteo Kaggle (display advertising challenge) per-feature cardinalities.
CRITEO_KAGGLE_CARDS = [
    1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593, 3194, 27, 14992,
    5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105, 142572,
]
_HASH_PRIME = 2654435761  # prime: multiplication mod card is a bijection unless card % prime == 0


class CriteoSynth:
    def __init__(self, batch: int, cards=None, n_dense: int = 13, device="cpu", seed: int = 0,
                 hot_alpha: float = 1.0):
        self.batch = batch
        self.cards = list(cards or CRITEO_KAGGLE_CARDS)
        self.F = len(self.cards)
        self.n_dense = n_dense
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self.offsets = torch.tensor([0] + list(_cumsum(self.cards))[:-1], dtype=torch.int64, device=self.device)
        self.card_t = torch.tensor(self.cards, dtype=torch.int64, device=self.device)
        self.log_card = torch.log(self.card_t.to(torch.float64) + 1.0)
        self.num_rows = int(sum(self.cards))
        self.hot_alpha = hot_alpha
        self.w_dense = torch.randn(n_dense, generator=self.gen, device=self.device) / math.sqrt(n_dense)

    def next(self):
        B, F = self.batch, self.F
        if self.device.type == "cuda":
            # one fused gfx950 launch (csrc/kernels/data.hip) instead of ~15 torch kernels
            from .._native import kernels

            self._init_gpu()
            self._host_step += 1
            dense = torch.empty(B, self.n_dense, device=self.device)
            keys = torch.empty(B, F, dtype=torch.int64, device=self.device)
            labels = torch.empty(B, device=self.device)
            if torch.cuda.is_current_stream_capturing():
                # a captured step draws a fresh batch on every replay: the counter advances on the
                # device (graph_prepare set it from the host count before the capture)
                self._step_dev.add_(1)
                kernels().criteo_synth(self._seed, 0, self._step_dev, self.card_t, self.offsets, self.w_dense,
                                       dense, keys, labels)
            else:
                kernels().criteo_synth(self._seed, self._host_step, None, self.card_t, self.offsets, self.w_dense,
                                       dense, keys, labels)
            return dense, keys, labels
        u = torch.rand(B, F, generator=self.gen, device=self.device, dtype=torch.float64)
        raw = torch.floor(torch.exp(u * self.log_card) - 1.0).to(torch.int64)
        raw = torch.minimum(raw, self.card_t - 1).clamp_min(0)
        ids = (raw * _HASH_PRIME) % self.card_t
        keys = ids + self.offsets
        dense = torch.randn(B, self.n_dense, generator=self.gen, device=self.device)
        logit = dense @ self.w_dense + 0.5 * ((raw[:, :4] % 2).sum(1).float() - 1.0)
        noise = torch.rand(B, generator=self.gen, device=self.device)
        labels = (torch.sigmoid(2.0 * logit) > noise).float()
        return dense, keys, labels

    def _init_gpu(self):
        if not hasattr(self, "_seed"):
            self._seed = int(torch.randint(0, 2**62, (1,), generator=self.gen, device=self.device).item())
            self._host_step = 0
            # device twin of the step counter, used inside HIP-graph captures only
            self._step_dev = torch.zeros(1, dtype=torch.int64, device=self.device)

    def graph_prepare(self):
        """Before capturing a step that draws batches: the device counter = the host count."""
        if self.device.type == "cuda":
            self._init_gpu()
            self._step_dev.fill_(self._host_step)

    def graph_replayed(self, n: int = 1):
        """A captured step was replayed ``n`` times: the host count follows the device's."""
        self._host_step += n

    def skip(self, n: int):
        """Advance past ``n`` batches (resume from a checkpoint at the same data position)."""
        if self.device.type == "cuda":
            self._init_gpu()
            self._host_step += n
        else:
            for _ in range(n):
                self.next()


def _cumsum(xs):
    s = 0
    for x in xs:
        s += x
        yield s


class DLRMSynth:
    """DLRM batches (BASELINE config 5): F keys per sample uniform over the whole table, n_dense
    N(0,1) features, label = dense[:, 0] > 0. On the GPU one fused launch (csrc/kernels/data.hip
    uniform_synth, counter-based RNG) per batch; on the CPU the torch generator."""

    def __init__(self, batch: int, F: int, num_rows: int, n_dense: int = 13, device="cpu", seed: int = 0):
        self.batch, self.F, self.num_rows, self.n_dense = batch, F, int(num_rows), n_dense
        self.device = torch.device(device)
        self.seed = int(seed)
        self._step = 0
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)

    def next(self):
        B = self.batch
        if self.device.type == "cuda":
            from .._native import kernels

            dense = torch.empty(B, self.n_dense, device=self.device)
            keys = torch.empty(B, self.F, dtype=torch.int64, device=self.device)
            labels = torch.empty(B, device=self.device)
            kernels().uniform_synth(self.seed, self._step, self.num_rows, dense, keys, labels)
            self._step += 1
            return dense, keys, labels
        dense = torch.randn(B, self.n_dense, generator=self.gen, device=self.device)
        keys = torch.randint(0, self.num_rows, (B, self.F), generator=self.gen, device=self.device)
        return dense, keys, (dense[:, 0] > 0).float()


class MnistSynth:
    """784-dim inputs in [0,1) and 10-class labels from a fixed random linear teacher."""

    def __init__(self, batch: int, device="cpu", seed: int = 0, dim: int = 784, classes: int = 10):
        self.batch, self.dim, self.classes = batch, dim, classes
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self.teacher = torch.randn(dim, classes, generator=self.gen, device=self.device)

    def next(self):
        x = torch.rand(self.batch, self.dim, generator=self.gen, device=self.device)
        y = torch.argmax(x @ self.teacher, dim=1)
        return x, y


class TokenSynth:
    """GPT-2 token batches: [B, T+1] uniform ids (inputs = [:, :-1], targets = [:, 1:])."""

    def __init__(self, batch: int, seq: int, vocab: int = 50257, device="cpu", seed: int = 0):
        self.batch, self.seq, self.vocab = batch, seq, vocab
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)

    def next(self):
        t = torch.randint(0, self.vocab, (self.batch, self.seq + 1), generator=self.gen, device=self.device)
        return t[:, :-1].contiguous(), t[:, 1:].contiguous()


class SparseLRSynth:
    """webspam-shaped sparse LR: `num_dims` features, ~nnz ids per row, linear teacher labels."""

    def __init__(self, batch: int, num_dims: int = 16_609_143, nnz: int = 64, device="cpu", seed: int = 0):
        self.batch, self.num_dims, self.nnz = batch, num_dims, nnz
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)

    def next(self):
        B, k = self.batch, self.nnz
        cols = torch.randint(0, self.num_dims, (B, k), generator=self.gen, device=self.device)
        vals = torch.rand(B, k, generator=self.gen, device=self.device)
        teacher = ((cols * _HASH_PRIME) % 7).float() - 3.0
        y = ((teacher * vals).sum(1) > 0).float()
        rowptr = torch.arange(0, (B + 1) * k, k, device=self.device, dtype=torch.int64)
        return rowptr, cols.reshape(-1), vals.reshape(-1), y
