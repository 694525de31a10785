"""File ingest (SURVEY.md §2.6 io/, §2.7 lib/): libsvm shards through the native block assigner +
mmap line reader cover every line exactly once across ranks, and a file-fed sparse LR learns
through the prefetching loader."""
import random

import torch

from minips_amd.data.loader import LibsvmData, PrefetchToDevice


def _write_libsvm(path, n=600, dims=300, seed=0):
    rng = random.Random(seed)
    w = [rng.uniform(-1, 1) for _ in range(dims)]
    with open(path, "w") as f:
        for _ in range(n):
            feats = sorted(rng.sample(range(dims), 12))
            vals = [rng.random() for _ in feats]
            y = 1 if sum(w[j] * v for j, v in zip(feats, vals)) > 0 else -1
            f.write(f"{y} " + " ".join(f"{j + 1}:{v:.4f}" for j, v in zip(feats, vals)) + "\n")


def test_libsvm_shards_cover_file(tmp_path):
    p = tmp_path / "train.libsvm"
    _write_libsvm(p)
    full = LibsvmData(str(p))
    assert len(full) == 600 and int(full.cols.min()) >= 0 and int(full.cols.max()) < 300  # 1-based -> 0-based
    parts = [LibsvmData(str(p), r, 3, threads=2) for r in range(3)]
    assert sum(len(x) for x in parts) == 600
    assert sorted(torch.cat([x.labels for x in parts]).tolist()) == sorted(full.labels.tolist())


def test_file_fed_sparse_lr_learns(tmp_path):
    from minips_amd.models.lr import SparseLR, SparseLRConfig
    from minips_amd.ps.comm import Comm

    p = tmp_path / "train.libsvm"
    _write_libsvm(p, n=2000)
    data = LibsvmData(str(p))
    m = SparseLR(SparseLRConfig(num_dims=300, alpha=0.1), Comm(device=torch.device("cpu")))
    it = PrefetchToDevice(data.batches(100), "cpu")
    accs = [float(m.train_step(*next(it))) / 100 for _ in range(60)]
    it.close()
    assert sum(accs[-10:]) / 10 > 0.8, accs
