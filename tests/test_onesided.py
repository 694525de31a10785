"""Really asynchronous SSP / ASP (minips_amd/ps/onesided.py): rank 1 is an injected straggler.
SSP(s): rank 0 runs exactly s clocks ahead of the slowest rank and never s+1, and every value it
reads contains at least the updates of clocks < c - s of every rank (ssp_model.cpp:58-85);
ASP: rank 0 never waits (asp_model.cpp:18-26). No collective on the data path: Get / Add go
straight to the owners' rows (CPU: shared-memory shards; GPU: IPC-mapped HBM, two processes on
one card). Final values are exact (no lost update)."""
import time

import pytest
import torch

from test_ps_gloo import run_world

STEPS = 12


def _run(rank, world, consistency, s, dev):
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.onesided import OneSidedSparseTable

    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    comm = Comm(device=dev)
    t = OneSidedSparseTable(comm, num_rows=101, width=4, optimizer="add", consistency=consistency, staleness=s)
    shared = torch.tensor([5], device=dev)
    own = torch.tensor([60 + rank], device=dev)
    seen = []
    for c in range(STEPS):
        if rank == 1:
            time.sleep(0.03)  # straggler
        v = float(t.get_rows(shared)[0, 0])
        seen.append((c, t.staleness_seen[-1], v))
        t.add_keys(torch.cat([shared, own]), torch.ones(2, 4, device=dev))
        t.clock()
    t.drain()
    waited = t.waited_s
    comm.barrier()
    final = t.get_rows(torch.tensor([5, 60, 61], device=dev))[:, 0].tolist()
    comm.barrier()
    t.close()
    return seen, waited, final


def _ssp1(rank, world, dev=torch.device("cpu")):
    return _run(rank, world, "ssp", 1, dev)


def _ssp2(rank, world, dev=torch.device("cpu")):
    return _run(rank, world, "ssp", 2, dev)


def _asp(rank, world, dev=torch.device("cpu")):
    return _run(rank, world, "asp", 0, dev)


def _check(out, consistency, s, world=2):
    seen0, waited0, final0 = out[0]
    for rank, (_, _, fin) in out.items():
        assert fin == [world * STEPS, STEPS, STEPS], (rank, fin)  # every atomic add landed
    ahead = [st for _, st, _ in seen0]
    if consistency == "ssp":
        assert max(ahead) == s, ahead  # exactly s clocks ahead of the straggler, never s + 1
        assert waited0 > 0
        for c, _, v in seen0:  # SSP read guarantee: own clocks + every rank's clocks < c - s
            assert v >= c + (world - 1) * max(0, c - s), (c, v)
    else:
        assert waited0 == 0.0
        assert max(ahead) >= 4, ahead  # ran far ahead of the straggler


@pytest.mark.parametrize("fn,consistency,s", [(_ssp1, "ssp", 1), (_ssp2, "ssp", 2), (_asp, "asp", 0)],
                         ids=["ssp1", "ssp2", "asp"])
def test_onesided_staleness_cpu(fn, consistency, s):
    _check(run_world(fn, world=2), consistency, s)


def _g_ssp1(rank, world):
    return _run(rank, world, "ssp", 1, torch.device("cuda", 0))


def _g_asp(rank, world):
    return _run(rank, world, "asp", 0, torch.device("cuda", 0))


@pytest.mark.gpu
@pytest.mark.parametrize("fn,consistency,s", [(_g_ssp1, "ssp", 1), (_g_asp, "asp", 0)], ids=["ssp1", "asp"])
def test_onesided_staleness_gpu_ipc(dev, fn, consistency, s):
    """Two processes share cuda:0; each maps the other's shard through hipIpcOpenMemHandle and
    gathers / atomically adds rows with the gfx950 kernels (csrc/kernels/onesided.hip)."""
    _check(run_world(fn, world=2), consistency, s)


def _dlrm_run(rank, world, dev=torch.device("cpu"), steps=10):
    from minips_amd.models.dlrm import DLRM, DLRMConfig
    from minips_amd.ps.comm import Comm

    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    comm = Comm(device=dev)
    cfg = DLRMConfig(num_rows=5003, consistency="asp", transport="onesided", lr_sparse=0.05)
    m = DLRM(cfg, comm)
    dg = torch.Generator().manual_seed(4 + rank)
    losses = []
    for _ in range(steps):
        dense = torch.randn(64, cfg.n_dense, generator=dg)
        keys = torch.randint(0, cfg.num_rows, (64, cfg.F), generator=dg)
        y = (dense[:, 0] + 0.3 * (keys[:, 0] % 2).float() > 0).float()
        loss = m.train_step(dense.to(dev), keys.to(dev), y.to(dev))
        losses.append(float(loss) / 64)
    m.drain()
    comm.barrier()
    out = (losses, m.emb.clock_n, m.dense.step)
    m.emb.close()
    m.dense.close()
    return out


def test_dlrm_onesided_asp_cpu():
    """DLRM config 5 on the one-sided path: ASP async SGD, no collective per step."""
    out = run_world(_dlrm_run, world=2)
    for rank, (losses, ck, st) in out.items():
        assert ck == 10 and st == 10
        assert all(l == l for l in losses) and losses[-1] < losses[0], (rank, losses)


def _g_dlrm(rank, world):
    return _dlrm_run(rank, world, torch.device("cuda", 0))


@pytest.mark.gpu
def test_dlrm_onesided_asp_gpu_ipc(dev):
    out = run_world(_g_dlrm, world=2)
    for rank, (losses, ck, st) in out.items():
        assert ck == 10 and all(l == l for l in losses) and losses[-1] < losses[0], (rank, losses)
