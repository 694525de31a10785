"""4- and 8-rank (gloo, CPU) correctness of every GPU-PS table and model against one rank
(reference: driver/engine_test.cpp:94-124, MultipleTasks with 3 engines). Integer / fp64 pushes
must be EXACT; Adam / Adagrad within float rounding; model losses within tolerance.

Edge cases covered: num_rows % world != 0, ranks owning none of the requested keys, a rank
that requests no keys at all, 8-way all-to-all-v split bookkeeping.
"""
import pytest
import torch

from test_ps_gloo import run_world

WORLDS = [4, 8]


# ------------------------------------------------------------------------------ sparse tables
def _rank_keys(rank):
    """Keys per rank: duplicates, cross-shard keys, keys near the table end; rank 3 asks none."""
    if rank == 3:
        return torch.empty(0, dtype=torch.int64)
    return torch.tensor([1, 1, 1002, 500 + rank, 7 * rank, 999, 3 * rank + 1, 1], dtype=torch.int64)


def _expected_rows(world, num_rows=1003):
    exp = torch.zeros(num_rows)
    for r in range(world):
        for k in _rank_keys(r).tolist():
            exp[k] += float(r + 1)
    return exp


def _sparse_exact_fn(route, low_keys):
    def fn(rank, world):
        from minips_amd.ps.comm import Comm
        from minips_amd.ps.tables import SparseTable

        torch.set_num_threads(1)
        comm = Comm(device=torch.device("cpu"))
        t = SparseTable(comm, num_rows=1003, width=3, optimizer="add", pull_dtype=torch.float32, init_std=0.0,
                        route=route)
        keys = _rank_keys(rank)
        if low_keys:  # every requested key lives on rank 0's range: ranks 1.. serve nothing
            keys = keys % 100
        seen = []
        for step in range(3):
            seen.append(t.get_rows(keys)[:, 0].tolist())  # every rank Gets (empty too)
            t.add_keys(keys, torch.full((keys.numel(), 3), float(rank + 1)))
            t.clock()
        all_keys = torch.arange(1003)
        final = t.get_rows(all_keys)
        return seen, final.tolist()

    return fn


def _sx_range(rank, world):
    return _sparse_exact_fn("range", False)(rank, world)


def _sx_mix(rank, world):
    return _sparse_exact_fn("mix", False)(rank, world)


def _sx_low(rank, world):
    return _sparse_exact_fn("range", True)(rank, world)


@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("fn,low", [(_sx_range, False), (_sx_mix, False), (_sx_low, True)],
                         ids=["range", "mix", "owners_idle"])
def test_sparse_table_exact(world, fn, low):
    out = run_world(fn, world=world)
    exp = torch.zeros(1003)
    for r in range(world):
        ks = _rank_keys(r) % 100 if low else _rank_keys(r)
        for k in ks.tolist():
            exp[k] += float(r + 1)
    for rank, (seen, final) in out.items():
        ks = (_rank_keys(rank) % 100 if low else _rank_keys(rank)).tolist()
        for step, vals in enumerate(seen):  # BSP: step i sees exactly i supersteps
            assert vals == [float(exp[k]) * step for k in ks], (rank, step)
        got = torch.tensor(final)
        assert torch.equal(got, exp[:, None].expand(-1, 3) * 3), rank


def _hash_exact(rank, world):
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.tables import HashSparseTable

    torch.set_num_threads(1)
    comm = Comm(device=torch.device("cpu"))
    t = HashSparseTable(comm, width=2, capacity=16)
    keys = torch.tensor([5, 5, 1 << 40, 123456789 + rank, 17 * rank, (1 << 62) + 3], dtype=torch.int64)
    for _ in range(2):
        t.add_keys(keys, torch.full((keys.numel(), 2), float(rank + 1)))
        t.clock()
    probe = torch.tensor([5, 1 << 40, (1 << 62) + 3] + [123456789 + r for r in range(world)], dtype=torch.int64)
    return t.get_rows(probe)[:, 0].tolist()


@pytest.mark.parametrize("world", WORLDS)
def test_hash_table_exact(world):
    out = run_world(_hash_exact, world=world)
    s = sum(r + 1 for r in range(world))
    expect = [2 * 2.0 * s, 2.0 * s, 2.0 * s] + [2.0 * (r + 1) for r in range(world)]
    for rank, got in out.items():
        # keys 17*rank collide with 0 for rank 0 only; not probed
        assert got == expect, (rank, got, expect)


# ------------------------------------------------------------------------------ dense tables
def _grad(rank, step, n):
    """Multiples of 1/64: fp32/fp64 sums are exact in any order, so the optimizers see bitwise
    the same gradient sum however the reduce-scatter groups the ranks."""
    return torch.round(torch.sin(torch.arange(n, dtype=torch.float64) * (rank + 1) + step) * 64) / 64


def _dense_fn(rank, world, n=1001, steps=3):
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.tables import DenseTable

    torch.set_num_threads(1)
    comm = Comm(device=torch.device("cpu"))
    exact = DenseTable(comm, n, optimizer="add", value_dtype=torch.float64)
    adam = DenseTable(comm, n, optimizer="adam", lr=1e-2, pull_dtype=torch.float32)
    adagrad = DenseTable(comm, n, optimizer="adagrad", lr=1e-1, pull_dtype=torch.float32)
    init = torch.linspace(-1, 1, n)
    adam.load_full(init)
    adagrad.load_full(init)
    for s in range(steps):
        g = _grad(rank, s, n)
        exact.add(g)
        adam.add(g.float())
        adagrad.add(g.float())
        for t in (exact, adam, adagrad):
            t.clock()
    return [t.full_master().tolist() for t in (exact, adam, adagrad)]


def _dense_ref(world, n=1001, steps=3):
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.tables import DenseTable

    comm = Comm(device=torch.device("cpu"))
    exact = DenseTable(comm, n, optimizer="add", value_dtype=torch.float64)
    adam = DenseTable(comm, n, optimizer="adam", lr=1e-2, pull_dtype=torch.float32)
    adagrad = DenseTable(comm, n, optimizer="adagrad", lr=1e-1, pull_dtype=torch.float32)
    init = torch.linspace(-1, 1, n)
    adam.load_full(init)
    adagrad.load_full(init)
    for s in range(steps):
        g = sum(_grad(r, s, n) for r in range(world))
        exact.add(g)
        adam.add(g.float())
        adagrad.add(g.float())
        for t in (exact, adam, adagrad):
            t.clock()
    return [t.full_master() for t in (exact, adam, adagrad)]


@pytest.mark.parametrize("world", WORLDS)
def test_dense_tables_match_one_rank(world):
    out = run_world(_dense_fn, world=world)
    ref_exact, ref_adam, ref_adagrad = _dense_ref(world)
    for rank, (ex, ad, ag) in out.items():
        assert torch.equal(torch.tensor(ex, dtype=torch.float64), ref_exact), rank
        assert torch.allclose(torch.tensor(ad), ref_adam, rtol=0, atol=1e-6), rank
        assert torch.allclose(torch.tensor(ag), ref_adagrad, rtol=0, atol=1e-6), rank


# ------------------------------------------------------------------------------ models
CARDS = [50, 7, 300, 20, 5, 60, 90, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28]
PER_RANK = 16


def _wd_run(rank, world, steps=4):
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig
    from minips_amd.ps.comm import Comm

    torch.set_num_threads(1)
    comm = Comm(device=torch.device("cpu"))
    cfg = WideDeepConfig(cards=CARDS)
    m = WideDeep(cfg, comm)
    g = torch.Generator().manual_seed(5)
    full = torch.randn(m.num_rows, cfg.row_width, generator=g) * 0.01
    full[:, cfg.emb_dim:] = 0
    m.emb.shard.copy_(full[m.emb.base: m.emb.base + m.emb.rows_local])
    total = PER_RANK * 8
    data = CriteoSynth(total, cards=CARDS, device="cpu", seed=11)
    per = total // world
    losses = []
    for _ in range(steps):
        dense, keys, y = data.next()
        sl = slice(rank * per, (rank + 1) * per)
        t = m.train_step(dense[sl], keys[sl], y[sl]).clone()
        comm.all_reduce_(t)
        losses.append(float(t) / total)
    return losses


def _dlrm_run(rank, world, steps=4):
    from minips_amd.models.dlrm import DLRM, DLRMConfig
    from minips_amd.ps.comm import Comm

    torch.set_num_threads(1)
    comm = Comm(device=torch.device("cpu"))
    cfg = DLRMConfig(num_rows=5003, transport="collective")  # ASP over collectives: exact across world sizes
    m = DLRM(cfg, comm)
    g = torch.Generator().manual_seed(9)
    full = torch.randn(cfg.num_rows, cfg.D, generator=g) * 0.05
    m.emb.shard.copy_(full[m.emb.base: m.emb.base + m.emb.rows_local])
    dg = torch.Generator().manual_seed(4)
    total = PER_RANK * 8
    per = total // world
    losses = []
    for _ in range(steps):
        dense = torch.randn(total, cfg.n_dense, generator=dg)
        keys = torch.randint(0, cfg.num_rows, (total, cfg.F), generator=dg)
        y = (dense[:, 0] + 0.3 * (keys[:, 0] % 2).float() > 0).float()
        sl = slice(rank * per, (rank + 1) * per)
        t = m.train_step(dense[sl], keys[sl], y[sl]).clone()
        m.drain()
        comm.all_reduce_(t)
        losses.append(float(t) / total)
    return losses


def _gpt2_run(rank, world, steps=3):
    from minips_amd.models.gpt2 import GPT2, GPT2Config
    from minips_amd.ps.comm import Comm

    torch.set_num_threads(1)
    comm = Comm(device=torch.device("cpu"))
    m = GPT2(GPT2Config(vocab=300, n_ctx=32, d=128, n_layer=2, n_head=2, lr=1e-3), comm)
    g = torch.Generator().manual_seed(2)
    tokens = torch.randint(0, 300, (8, 32), generator=g)
    targets = torch.roll(tokens, -1, 1)
    per = 8 // world
    losses = []
    for _ in range(steps):
        t = m.train_step(tokens[rank * per:(rank + 1) * per], targets[rank * per:(rank + 1) * per]).clone()
        comm.all_reduce_(t)
        losses.append(float(t) / tokens.numel())
    return losses


def _mlp_run(rank, world, steps=4):
    from minips_amd.data.synthetic import MnistSynth
    from minips_amd.models.mlp import MLP, MLPConfig
    from minips_amd.ps.comm import Comm

    torch.set_num_threads(1)
    comm = Comm(device=torch.device("cpu"))
    m = MLP(MLPConfig(), comm)
    total = PER_RANK * 8
    data = MnistSynth(total, device="cpu", seed=3)
    per = total // world
    losses = []
    for _ in range(steps):
        x, y = data.next()
        loss, _ = m.train_step(x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per])
        t = loss.clone()
        comm.all_reduce_(t)
        losses.append(float(t) / total)
    return losses


@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("run", [_wd_run, _dlrm_run, _gpt2_run, _mlp_run], ids=["widedeep", "dlrm", "gpt2", "mlp"])
def test_model_losses_match_one_rank(world, run):
    many = run_world(run, world=world)
    one = run(0, 1)
    for r in range(1, world):
        assert many[r] == many[0]  # the all-reduced loss is identical on every rank
    for a, b in zip(many[0], one):
        assert abs(a - b) <= 3e-3 * max(1.0, abs(b)), (many[0], one)


# ------------------------------------------------------------------------------ bucketed dense clocks
def _gpt2_bucket_run(rank, world, bucketed=True, steps=3):
    import json
    import os
    import tempfile

    from minips_amd.models.gpt2 import GPT2, GPT2Config
    from minips_amd.ps.comm import Comm
    from minips_amd.utils.metrics import MetricsLogger

    torch.set_num_threads(1)
    comm = Comm(device=torch.device("cpu"))
    m = GPT2(GPT2Config(vocab=300, n_ctx=32, d=128, n_layer=3, n_head=2, lr=1e-3, bucketed=bucketed), comm)
    g = torch.Generator().manual_seed(2)
    tokens = torch.randint(0, 300, (8, 32), generator=g)
    targets = torch.roll(tokens, -1, 1)
    per = 8 // world
    path = os.path.join(tempfile.mkdtemp(), f"m{rank}.jsonl")
    log = MetricsLogger(rank, path)
    for it in range(steps):
        m.train_step(tokens[rank * per:(rank + 1) * per], targets[rank * per:(rank + 1) * per])
        log.step(it, per * 32, 1.0, comm.stats)
    recs = [json.loads(l) for l in open(path)]
    n_buckets = len(m.table.buckets) if m.table.buckets else 0
    full = m.table.full_master()
    # the key bias has an analytically zero gradient (softmax is shift-invariant along a query row):
    # Adam normalises its reduction-order noise into +-lr steps, so it is left out of the comparison
    for blk in m.blocks:
        m.layout.view(full, blk["qkv"].name)[128:256, 128] = 0.0
    return full.tolist(), recs[-1].get("bucket_bytes"), n_buckets


def _gpt2_b(rank, world):
    return _gpt2_bucket_run(rank, world, True)


def _gpt2_nb(rank, world):
    return _gpt2_bucket_run(rank, world, False)


def test_gpt2_bucketed_clock_equals_unbucketed():
    """4 ranks: per-layer buckets (RS + Adam + AG issued during the backward) give the same
    parameters as one whole-table clock; the metrics JSONL carries per-bucket bytes."""
    b = run_world(_gpt2_b, world=4)
    nb = run_world(_gpt2_nb, world=4)
    for r in range(4):
        pb, bytes_b, nbk = b[r]
        pn, bytes_n, _ = nb[r]
        assert nbk == 4 and bytes_n is None  # embedding bucket + one per layer
        # the bucketed reduce-scatter sums in another order; after the key-bias noise above feeds back
        # through bf16 rounding, parameters agree to a small fraction of one Adam step (lr 1e-3) -- a
        # missed or stale bucket would move a whole layer by ~lr
        assert torch.allclose(torch.tensor(pb), torch.tensor(pn), rtol=0, atol=2e-4)
        assert len(bytes_b) == 4 and all(v > 0 for v in bytes_b.values()), bytes_b


def _sparse_f64(rank, world):
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.tables import SparseTable

    torch.set_num_threads(1)
    comm = Comm(device=torch.device("cpu"))
    t = SparseTable(comm, num_rows=1003, width=2, optimizer="add", init_std=0.0, value_dtype=torch.float64)
    keys = _rank_keys(rank)
    for step in range(3):
        t.add_keys(keys, torch.full((keys.numel(), 2), 0.1 * (rank + 1) + 1e-12 * step, dtype=torch.float64))
        t.clock()
    got = t.get_rows(torch.arange(1003))
    return str(got.dtype), got.tolist()


@pytest.mark.parametrize("world", WORLDS)
def test_sparse_table_fp64_exact(world):
    """The reference's double tables: sums exact in fp64 (not fp32-representable deltas)."""
    out = run_world(_sparse_f64, world=world)
    exp = torch.zeros(1003, dtype=torch.float64)
    for step in range(3):
        for r in range(world):
            for k in _rank_keys(r).tolist():
                exp[k] += 0.1 * (r + 1) + 1e-12 * step
    for rank, (dt, got) in out.items():
        assert dt == "torch.float64"
        g = torch.tensor(got, dtype=torch.float64)
        assert torch.allclose(g[:, 0], exp, rtol=1e-15, atol=1e-15), rank
        assert not torch.equal(g[:, 0].float().double(), g[:, 0])  # really fp64 values
