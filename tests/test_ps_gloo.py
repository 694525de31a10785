"""Multi-process (gloo, CPU) tests of the GPU parameter-server data plane: the same code that
runs over RCCL on MI355X runs here over gloo with world_size 2."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _util import free_ports


def _worker(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, "ERROR " + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def run_world(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_ports(1)[0]
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, v = q.get(timeout=240)
            out[r] = v
            if isinstance(v, str) and v.startswith("ERROR"):
                break  # peers may be blocked in a collective with the failed rank
    finally:
        for p in procs:
            p.join(timeout=60 if len(out) == world else 1)
            if p.is_alive():
                p.kill()
    errs = [v for v in out.values() if isinstance(v, str) and v.startswith("ERROR")]
    # a failing rank closes its connections: show the root cause, not a peer's echo of it
    errs.sort(key=lambda e: "Connection closed" in e or "Connection reset" in e)
    assert not errs, errs[0]
    return out


# ------------------------------------------------------------------------------ sparse table
def _sparse_fn(rank, world):
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.tables import SparseTable

    comm = Comm(device=torch.device("cpu"))
    t = SparseTable(comm, num_rows=100, width=4, optimizer="add", pull_dtype=torch.float32, init_std=0.0)
    keys = torch.tensor([[3, 50], [97, 3], [rank, 60 + rank]])  # duplicates + cross-shard keys
    rows, plan = t.get(keys)
    before = rows[plan.inv].clone()
    g = torch.zeros(plan.U, 4)
    torch.ops.aten.index_add_(g, 0, plan.inv, torch.ones(keys.numel(), 4))
    t.add(plan, g)
    mid = t.get_rows(keys)  # BSP: the Add is invisible until Clock
    t.clock()
    after = t.get_rows(keys)
    return before.tolist(), mid.tolist(), after.tolist()


def test_sparse_table_push_pull_bsp():
    out = run_world(_sparse_fn)
    for rank, (before, mid, after) in out.items():
        assert all(v == 0.0 for row in before for v in row)
        assert mid == before
        keys = [3, 50, 97, 3, rank, 60 + rank]
        # key 3 is pushed twice by each of the 2 ranks; 50, 97 once each by both
        expect = {3: 4.0, 50: 2.0, 97: 2.0, 0: 1.0, 1: 1.0, 60: 1.0, 61: 1.0}
        for k, row in zip(keys, after):
            assert row == [expect[k]] * 4, (rank, k, row)


# ------------------------------------------------------------------------------ dense table
def _dense_fn(rank, world):
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.tables import DenseTable

    comm = Comm(device=torch.device("cpu"))
    t = DenseTable(comm, n_params=1000, optimizer="add", pull_dtype=torch.float32)
    t.load_full(torch.arange(1000, dtype=torch.float32))
    p0 = t.get()[:1000].clone()
    t.add(torch.full((1000,), float(rank + 1)))
    t.clock()
    p1 = t.get()[:1000].clone()
    sgd = DenseTable(comm, n_params=10, optimizer="sgd", lr=0.5, pull_dtype=torch.float32)
    sgd.load_full(torch.ones(10))
    sgd.add(torch.ones(10))
    sgd.clock()
    return p0.tolist(), p1.tolist(), sgd.get()[:10].tolist(), t.shard, t.base


def test_dense_table_rs_ag():
    out = run_world(_dense_fn)
    for rank, (p0, p1, s, shard, base) in out.items():
        assert p0 == [float(i) for i in range(1000)]
        assert p1 == [float(i) + 3.0 for i in range(1000)]  # 1 + 2 summed over ranks
        assert s == [0.0] * 10  # 1 - 0.5 * (1 + 1)
        assert base == rank * shard


# ------------------------------------------------------------------------------ Wide&Deep
CARDS = [50, 7, 300, 20, 5, 60, 90, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28]


def _wd_run(rank, world, steps=6, per_rank=64):
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig
    from minips_amd.ps.comm import Comm

    comm = Comm(device=torch.device("cpu"))
    cfg = WideDeepConfig(cards=CARDS)
    m = WideDeep(cfg, comm)
    # identical initial embedding rows regardless of the sharding
    g = torch.Generator().manual_seed(5)
    full = torch.randn(m.num_rows, cfg.row_width, generator=g) * 0.01
    full[:, cfg.emb_dim:] = 0
    m.emb.shard.copy_(full[m.emb.base: m.emb.base + m.emb.rows_local])
    data = CriteoSynth(per_rank * 2, cards=CARDS, device="cpu", seed=11)
    losses = []
    for _ in range(steps):
        dense, keys, y = data.next()
        lo, hi = (rank * per_rank, (rank + 1) * per_rank) if world > 1 else (0, 2 * per_rank)
        loss = m.train_step(dense[lo:hi], keys[lo:hi], y[lo:hi])
        t = loss.clone()
        comm.all_reduce_(t)
        losses.append(float(t) / (2 * per_rank))
    return losses, m.dense.full_master()[:2000].tolist()


def _wd_fn(rank, world):
    return _wd_run(rank, world)


def test_widedeep_two_ranks_match_one():
    two = run_world(_wd_fn)
    one_losses, one_master = _wd_run(0, 1)
    l0, m0 = two[0]
    l1, _ = two[1]
    assert l0 == l1  # the all-reduced loss is identical on both ranks
    for a, b in zip(l0, one_losses):
        assert abs(a - b) < 2e-3, (l0, one_losses)
    diff = max(abs(a - b) for a, b in zip(m0, one_master))
    assert diff < 2e-3


def _sparse_bf16_push_fn(rank, world):
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.tables import SparseTable

    comm = Comm(device=torch.device("cpu"))
    t = SparseTable(comm, num_rows=100, width=4, optimizer="add", pull_dtype=torch.float32, init_std=0.0,
                    push_dtype=torch.bfloat16)
    keys = torch.tensor([3, 50, 97, 3, rank])
    t.add_keys(keys, torch.full((5, 4), 0.5 * (rank + 1)))
    t.clock()
    return t.get_rows(keys).tolist()


def test_sparse_push_in_bf16():
    """The multi-GPU push sends gradient rows as bf16 (owner accumulates fp32)."""
    out = run_world(_sparse_bf16_push_fn)
    for rank, rows in out.items():
        expect = {3: 3.0, 50: 1.5, 97: 1.5, 0: 0.5, 1: 1.0}
        for k, row in zip([3, 50, 97, 3, rank], rows):
            assert row == [expect[k]] * 4, (rank, k, row)


# ------------------------------------------------------------------------------ fp64 dense table
def _fp64_bsp_fn(rank, world, steps=4, n=1000):
    """The reference's double tables (BSP): after clock t every rank pulls exactly the fp64 sum
    of t supersteps of every rank's deltas -- bit-for-bit, no fp32 rounding anywhere."""
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.tables import DenseTable

    comm = Comm(device=torch.device("cpu"))
    t = DenseTable(comm, n, optimizer="add", value_dtype=torch.float64)
    base = torch.arange(n, dtype=torch.float64)
    expect = torch.zeros(n, dtype=torch.float64)
    ok = True
    for s in range(steps):
        got = t.get()[:n].clone()
        ok = ok and bool(torch.equal(got, expect))
        t.add(0.1 * (rank + 1) * base + 1e-9 * s)
        t.clock()
        tot = torch.zeros(n, dtype=torch.float64)
        for r in range(world):
            tot = tot + (0.1 * (r + 1) * base + 1e-9 * s)
        expect = expect + tot
    t.drain()
    final = t.get()[:n]
    return ok, bool(torch.equal(final, expect)), str(final.dtype), float((final.float().double() - expect).abs().max())


def test_dense_fp64_bsp_exact_two_ranks():
    out = run_world(_fp64_bsp_fn)
    for r in (0, 1):
        ok, final_ok, dtype, f32_err = out[r]
        assert ok and final_ok and dtype == "torch.float64", out[r]
        assert f32_err > 0  # the values are not fp32-representable: fp64 was really kept


def test_dense_fp64_rejects_optimizers():
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.tables import DenseTable

    with pytest.raises(ValueError):
        DenseTable(Comm(device=torch.device("cpu")), 10, optimizer="adam", value_dtype=torch.float64)
