"""File ingest (SURVEY.md §2.6 io/, §2.7 lib/): libsvm shards through the native block assigner +
mmap line reader cover every line exactly once across ranks, and a file-fed sparse LR learns
through the prefetching loader."""
import pytest
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


def test_batch_slices_match_rowwise_reference(tmp_path):
    """Vectorised CSR batch cutting (incl. wrap-around and batches longer than the shard) equals a
    row-by-row reference."""
    p = tmp_path / "small.libsvm"
    _write_libsvm(p, n=37, dims=50)
    d = LibsvmData(str(p))
    for start, size in [(0, 5), (30, 12), (36, 1), (10, 80)]:
        rp, cols, vals, y = d.batch(start, size)
        idx = [(start + i) % 37 for i in range(size)]
        ref_cols = torch.cat([d.cols[int(d.rowptr[i]): int(d.rowptr[i + 1])] for i in idx])
        ref_lens = torch.tensor([int(d.rowptr[i + 1] - d.rowptr[i]) for i in idx])
        assert torch.equal(cols, ref_cols) and torch.equal(y, d.labels[idx])
        assert torch.equal(rp[1:] - rp[:-1], ref_lens) and int(rp[0]) == 0 and vals.numel() == cols.numel()


def test_train_driver_file_input(tmp_path):
    """python -m minips_amd.train --model lr --input <libsvm>: the reference LR app's file-fed path."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = tmp_path / "train.libsvm"
    _write_libsvm(p, n=3000)
    r = subprocess.run([sys.executable, "-m", "minips_amd.train", "--model", "lr", "--input", str(p), "--batch", "100",
                        "--steps", "150", "--alpha", "0.1"], cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    accs = [-v for _, v in out["losses"]]
    assert sum(accs[-5:]) / 5 > 0.85, accs


@pytest.mark.parametrize("mode", ["kmeans++", "kmeans_parallel"])
def test_train_driver_kmeans_init_flags(mode):
    """--K / --kmeans_init_mode (the reference K-Means app's flags, kmeans.cpp:18-52)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "minips_amd.train", "--model", "kmeans", "--small=1", "--steps", "4",
                        "--K", "6", "--kmeans_init_mode", mode], cwd=root, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["model"] == "kmeans" and all(v == v for _, v in out["losses"])


def test_train_driver_lr_map_storage_matches_vector():
    """--kStorageType Map (GPU hash-table MapStorage) trains exactly like Vector storage (the
    reference LR app's kStorageType flag; both start from zero rows)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for st in ("Vector", "Map"):
        r = subprocess.run([sys.executable, "-m", "minips_amd.train", "--model", "lr", "--small=1", "--steps", "20",
                            "--kStorageType", st], cwd=root, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
        res[st] = (out["losses"], out["checksum"])
    # same training and the same parameter sum; on a GPU the delta sums use fp32 atomics and the
    # two storages order their unique keys differently, so compare with a float tolerance
    (lm, cm), (lv, cv) = res["Map"], res["Vector"]
    assert [i for i, _ in lm] == [i for i, _ in lv]
    for (_, a), (_, b) in zip(lm, lv):
        assert abs(a - b) <= 1e-4 * max(1.0, abs(b)), res
    for a, b in zip(cm, cv):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(b)), res


def _clustered_libsvm(path, n=800, seed=0):
    """4 sparse clusters in 32 features: a point of cluster c has 6 of the 8 features
    [8c, 8c+8) set to ~1 (libsvm, 1-based). Best SSE/point ~1.5; one centre ~4.9."""
    import random

    rng = random.Random(seed)
    with open(path, "w") as f:
        for _ in range(n):
            c = rng.randrange(4)
            feats = sorted(rng.sample(range(8 * c, 8 * c + 8), 6))
            f.write("1" + "".join(f" {j + 1}:{1.0 + 0.05 * rng.uniform(-1, 1):.4f}" for j in feats) + "\n")


def _kmeans_parity(tmp_path, device_env):
    import json
    import os
    import subprocess
    import sys

    from _util import ensure_built, write_hostfile
    from minips_amd import launch

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    data = str(tmp_path / "pts.svm")
    _clustered_libsvm(data)
    ensure_built("runtime", "apps")
    hf = write_hostfile(str(tmp_path / "hosts"), 1)
    rcs = launch.launch_nodes("kmeans", hf, [f"--input={data}", "--K=4", "--num_dims=32", "--num_iters=60",
                                             "--batch_size=40", "--kmeans_init_mode=kmeans++",
                                             "--num_workers_per_node=2", "--report_interval=10"],
                              log_dir=str(tmp_path / "logs"), timeout=120)
    assert rcs == [0], rcs
    native = json.loads([l for l in open(tmp_path / "logs" / "node_0.log") if l.startswith("{")][-1])
    native_pp = native["sampled_sse"] / 50.0
    r = subprocess.run([sys.executable, "-m", "minips_amd.train", "--model", "kmeans", "--input", data, "--K", "4",
                        "--num_dims", "32", "--kmeans_init_mode", "kmeans++", "--steps", "60", "--batch", "128"],
                       cwd=root, capture_output=True, text=True, timeout=300, env=dict(os.environ, **device_env))
    assert r.returncode == 0, r.stderr[-3000:]
    ours = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    ours_pp = ours["losses"][-1][1]
    return native_pp, ours_pp


def test_kmeans_csr_matches_native_app(tmp_path):
    """Sparse (libsvm) K-Means: the PS K-Means on CSR batches reaches the clustering quality of
    the native C++ app (per-point updates, reference kmeans.cpp) on the same file (SSE/point
    near the 1.5 optimum, far below the 4.9 of one centre). Parity unpinned beyond that:
    batched vs per-point updates and different sampling."""
    native_pp, ours_pp = _kmeans_parity(tmp_path, {"CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
    # both well below one centre's 4.9; ours (batched 1/count steps) at least as good as the
    # native per-point updates, which may leave two clusters under one centre (~3)
    assert native_pp < 4.0 and ours_pp < 2.5, (native_pp, ours_pp)
    assert ours_pp <= native_pp + 0.5, (native_pp, ours_pp)


@pytest.mark.gpu
def test_kmeans_csr_gpu_matches_native_app(dev, tmp_path):
    """The same with the gfx950 CSR kernels (kmeans_assign_csr / kmeans_csr_accum)."""
    native_pp, ours_pp = _kmeans_parity(tmp_path, {})
    assert native_pp < 4.0 and ours_pp < 2.5, (native_pp, ours_pp)
    assert ours_pp <= native_pp + 0.5, (native_pp, ours_pp)
