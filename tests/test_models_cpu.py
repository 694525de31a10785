"""CPU (torch reference ops) tests of the dense-tower models: each learns on synthetic data,
and a 2-rank gloo run of the same global batch matches the 1-rank run (BSP) -- SURVEY.md §4
items 3/5 (multi-worker semantics, end-to-end convergence)."""
import pytest
import torch

from test_ps_gloo import run_world


def _mlp_run(rank, world, steps=5, per_rank=64):
    from minips_amd.data.synthetic import MnistSynth
    from minips_amd.models.mlp import MLP, MLPConfig
    from minips_amd.ps.comm import Comm

    comm = Comm(device=torch.device("cpu"))
    m = MLP(MLPConfig(), comm)
    data = MnistSynth(per_rank * 2, device="cpu", seed=3)
    losses = []
    for _ in range(steps):
        x, y = data.next()
        lo, hi = (rank * per_rank, (rank + 1) * per_rank) if world > 1 else (0, 2 * per_rank)
        loss, _ = m.train_step(x[lo:hi], y[lo:hi])
        t = loss.clone()
        comm.all_reduce_(t)
        losses.append(float(t) / (2 * per_rank))
    return losses, m.table.full_master()[:4000].tolist()


def _mlp_fn(rank, world):
    return _mlp_run(rank, world)


def test_mlp_learns_cpu():
    losses, _ = _mlp_run(0, 1, steps=12)
    assert losses[-1] < 0.7 * losses[0], losses


def test_mlp_two_ranks_match_one():
    two = run_world(_mlp_fn)
    one_l, one_m = _mlp_run(0, 1)
    assert two[0][0] == two[1][0]
    for a, b in zip(two[0][0], one_l):
        assert abs(a - b) < 2e-3, (two[0][0], one_l)
    assert max(abs(a - b) for a, b in zip(two[0][1], one_m)) < 2e-3


def _dlrm_run(rank, world, steps=5, per_rank=64, consistency="bsp", p2p=True):
    from minips_amd.models.dlrm import DLRM, DLRMConfig
    from minips_amd.ps.comm import Comm

    comm = Comm(device=torch.device("cpu"))
    cfg = DLRMConfig(num_rows=5000, consistency=consistency, p2p=p2p)
    m = DLRM(cfg, comm)
    g = torch.Generator().manual_seed(9)
    full = torch.randn(cfg.num_rows, cfg.D, generator=g) * 0.05
    m.emb.shard.copy_(full[m.emb.base: m.emb.base + m.emb.rows_local])
    dg = torch.Generator().manual_seed(4)
    losses = []
    for _ in range(steps):
        dense = torch.randn(2 * per_rank, cfg.n_dense, generator=dg)
        keys = torch.randint(0, cfg.num_rows, (2 * per_rank, cfg.F), generator=dg)
        y = (dense[:, 0] + 0.3 * (keys[:, 0] % 2).float() > 0).float()
        lo, hi = (rank * per_rank, (rank + 1) * per_rank) if world > 1 else (0, 2 * per_rank)
        loss = m.train_step(dense[lo:hi], keys[lo:hi], y[lo:hi])
        m.drain()
        t = loss.clone()
        comm.all_reduce_(t)
        losses.append(float(t) / (2 * per_rank))
    return losses, m.dense.full_master()[:4000].tolist()


def _dlrm_fn(rank, world):
    return _dlrm_run(rank, world)


def _dlrm_asp_fn(rank, world):
    return _dlrm_run(rank, world, steps=8, consistency="asp")


def test_dlrm_learns_cpu():
    losses, _ = _dlrm_run(0, 1, steps=15)
    assert losses[-1] < losses[0], losses


def test_dlrm_two_ranks_p2p_match_one():
    two = run_world(_dlrm_fn)
    one_l, one_m = _dlrm_run(0, 1)
    assert two[0][0] == two[1][0]
    for a, b in zip(two[0][0], one_l):
        assert abs(a - b) < 2e-3, (two[0][0], one_l)
    assert max(abs(a - b) for a, b in zip(two[0][1], one_m)) < 2e-3


def test_dlrm_asp_two_ranks_runs():
    out = run_world(_dlrm_asp_fn)
    for r in (0, 1):
        losses = out[r][0]
        assert all(l == l for l in losses) and losses[-1] < 1.0


# ------------------------------------------------------------------------------ LR / K-Means
def _lr_run(rank, world, steps=25):
    from minips_amd.data.synthetic import SparseLRSynth
    from minips_amd.models.lr import SparseLR, SparseLRConfig
    from minips_amd.ps.comm import Comm

    comm = Comm(device=torch.device("cpu"))
    m = SparseLR(SparseLRConfig(num_dims=4000, alpha=0.05), comm)
    data = SparseLRSynth(256, num_dims=4000, nnz=16, seed=7 + rank)
    accs = []
    for _ in range(steps):
        accs.append(float(m.train_step(*data.next())) / 256)
    return accs, m.table.shard[:50].reshape(-1).tolist()


def _lr_fn(rank, world):
    return _lr_run(rank, world)


def test_sparse_lr_learns_cpu():
    accs, _ = _lr_run(0, 1)
    assert sum(accs[-5:]) / 5 > 0.7, accs


def test_sparse_lr_two_ranks():
    out = run_world(_lr_fn)
    for r in (0, 1):
        assert sum(out[r][0][-5:]) / 5 > 0.7, out[r][0]


def test_lr_worker_group_equals_separate_worker_pushes():
    """--num_workers_per_node W on one rank: the fused Get/Add of the W workers' batches gives the
    same table as W reference workers that each Get the clock-c rows, push their own deltas, and
    share one Clock (server sums the pushes, vector_storage.hpp:28-38)."""
    from minips_amd import ops
    from minips_amd.data.synthetic import SparseLRSynth
    from minips_amd.models.lr import SparseLR, SparseLRConfig
    from minips_amd.ps.comm import Comm
    from minips_amd.train import _WorkerGroup

    cfg = SparseLRConfig(num_dims=3000, alpha=0.05, value_dtype=torch.float64)
    fused = SparseLR(cfg, Comm(device=torch.device("cpu")))
    sep = SparseLR(cfg, Comm(device=torch.device("cpu")))
    mk = lambda: [SparseLRSynth(64, num_dims=3000, nnz=12, seed=s) for s in (5, 6, 7)]  # noqa: E731
    group, solo = _WorkerGroup(mk()), mk()
    for _ in range(6):
        fused.train_step(*group.next())
        batches = [w.next() for w in solo]
        pulled = [sep.table.get(b[1]) for b in batches]  # every worker reads clock-c parameters
        for (rp, cols, vals, y), (rows, plan) in zip(batches, pulled):
            delta = torch.zeros(max(plan.cap, 1), dtype=rows.dtype)
            ops.lr_sparse_step(rp, plan.inv, vals, y, rows.view(-1)[: plan.cap], cfg.alpha, delta[: plan.cap],
                               torch.zeros(1))
            sep.table.add(plan, delta.view(-1, 1))
        sep.table.clock()
    torch.testing.assert_close(fused.table.shard, sep.table.shard, rtol=0, atol=1e-12)
    assert float(fused.table.shard.abs().sum()) > 0


def _km_run(rank, world, steps=8):
    from minips_amd.models.kmeans import KMeans, KMeansConfig
    from minips_amd.ps.comm import Comm

    comm = Comm(device=torch.device("cpu"))
    g = torch.Generator().manual_seed(0)
    true = torch.randn(6, 12, generator=g) * 5
    km = KMeans(KMeansConfig(K=6, dims=12), comm, init_centres=true + torch.randn(6, 12, generator=g))
    dg = torch.Generator().manual_seed(100 + rank)
    sse = []
    for _ in range(steps):
        X = true[torch.randint(0, 6, (512,), generator=dg)] + torch.randn(512, 12, generator=dg) * 0.5
        sse.append(float(km.train_step(X)) / 512)
    return sse, km.centres().reshape(-1).tolist()


def _km_fn(rank, world):
    return _km_run(rank, world)


def test_kmeans_converges_two_ranks():
    out = run_world(_km_fn)
    assert out[0][1] == out[1][1]  # both ranks pull the same centres
    for r in (0, 1):
        assert out[r][0][-1] < 12 * 0.25 * 1.3, out[r][0]


def _blobs(K=8, D=16, n=4000, seed=0):
    g = torch.Generator().manual_seed(seed)
    true = torch.randn(K, D, generator=g) * 6
    X = true[torch.randint(0, K, (n,), generator=g)] + torch.randn(n, D, generator=g) * 0.3
    return true, X


@pytest.mark.parametrize("mode", ["random", "kmeans++", "kmeans_parallel"])
def test_kmeans_init_modes(mode):
    """Seeding modes of the reference's init_task (kmeans_helper.hpp:68-207): D^2 seeding
    covers every well-separated blob; all modes return K rows drawn from the data."""
    from minips_amd.models.kmeans import init_centres, sampled_sse

    true, X = _blobs()
    C = init_centres(X, 8, mode, seed=3)
    assert C.shape == (8, 16)
    # every centre is a data point (k-means|| candidates are data points too)
    assert (torch.cdist(C, X, compute_mode="donot_use_mm_for_euclid_dist").min(1).values < 1e-4).all()
    if mode != "random":
        hit = torch.cdist(true, C).argmin(0).unique().numel()
        assert hit == 8, hit
        assert sampled_sse(X, C, n=200) < 16 * 0.3 ** 2 * 4
    with pytest.raises(ValueError):
        init_centres(X, 8, "bogus")


def _km_init_fn(rank, world):
    from minips_amd.models.kmeans import KMeans, KMeansConfig
    from minips_amd.ps.comm import Comm

    _, X = _blobs(seed=10 + rank)  # different local data per rank
    km = KMeans(KMeansConfig(K=8, dims=16, init_mode="kmeans++", seed=1), Comm(device=torch.device("cpu")),
                init_data=X)
    return km.centres().reshape(-1).tolist()


def test_kmeans_init_broadcast_two_ranks():
    out = run_world(_km_init_fn)
    assert out[0] == out[1]  # rank 0 seeds, every rank loads the same centres


def test_bitmap_plan_cpu_reference_and_dlrm_synth_cpu():
    """CPU paths of the round-2 planner / generator: ops.bitmap_plan is the sorted-unique plan (the
    GPU kernel is checked against it in test_kernels_gpu.py), DLRMSynth draws in-range keys with
    labels = dense[:, 0] > 0."""
    from minips_amd import ops
    from minips_amd.data.synthetic import DLRMSynth

    keys = torch.tensor([7, 3, 7, 99, 0, 3, 50])
    bounds = torch.tensor([0, 40, 100])
    u, inv, counts, U = ops.bitmap_plan(keys, bounds, 100)
    n = int(U.reshape(-1)[0])
    assert u[:n].tolist() == [0, 3, 7, 50, 99]
    assert torch.equal(u[:n][inv], keys)
    assert counts.tolist() == [3, 2]
    d = DLRMSynth(64, 26, 1000, 13, device="cpu", seed=1)
    dense, k, lab = d.next()
    assert k.shape == (64, 26) and int(k.min()) >= 0 and int(k.max()) < 1000
    assert torch.equal(lab, (dense[:, 0] > 0).float())
