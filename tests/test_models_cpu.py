"""CPU (torch reference ops) tests of the dense-tower models: each learns on synthetic data,
and a 2-rank gloo run of the same global batch matches the 1-rank run (BSP) -- SURVEY.md §4
items 3/5 (multi-worker semantics, end-to-end convergence)."""
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
