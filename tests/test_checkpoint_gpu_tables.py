"""Checkpoint / resume of the GPU-PS tables: round trip in all three
consistency models, resume equivalence (train k, save, train j == restore, train j), elastic
re-sharding (save at world 2, restore at world 1), and the reference text formats."""
import os

import pytest
import torch

from test_ps_gloo import run_world

CARDS = [50, 7, 300, 20, 5, 60, 90, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28]


def _wd(comm, consistency="bsp", staleness=0):
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig

    m = WideDeep(WideDeepConfig(cards=CARDS, consistency=consistency, staleness=staleness,
                                 transport="collective"), comm)
    g = torch.Generator().manual_seed(5)
    full = torch.randn(m.num_rows, m.cfg.row_width, generator=g) * 0.01
    full[:, m.cfg.emb_dim:] = 0
    m.emb.shard.copy_(full[m.emb.base: m.emb.base + m.emb.rows_local])
    return m


def _batches(n, per_rank, world, rank, seed=11):
    from minips_amd.data.synthetic import CriteoSynth

    data = CriteoSynth(per_rank * world, cards=CARDS, device="cpu", seed=seed)
    out = []
    for _ in range(n):
        d, k, y = data.next()
        lo, hi = rank * per_rank, (rank + 1) * per_rank
        out.append((d[lo:hi], k[lo:hi], y[lo:hi]))
    return out


def _tables(m):
    return {0: m.emb, 1: m.dense}


def _resume_fn(rank, world, prefix, consistency):
    from minips_amd.ps.checkpoint import Checkpointer
    from minips_amd.ps.comm import Comm

    comm = Comm(device=torch.device("cpu"))
    bs = _batches(6, 32, world, rank)
    m = _wd(comm, consistency, 1 if consistency == "ssp" else 0)
    for b in bs[:3]:
        m.train_step(*b)
    m.drain()
    ck = Checkpointer(comm, prefix)
    ck.save(_tables(m), iteration=3, blocking=True)
    ref = [float(m.train_step(*b)) for b in bs[3:]]
    m.drain()
    ref_master = m.dense.full_master().clone()
    # fresh model, restore, continue
    m2 = _wd(comm, consistency, 1 if consistency == "ssp" else 0)
    m2.emb.shard.zero_()
    it = Checkpointer(comm, prefix).load(_tables(m2))
    got = [float(m2.train_step(*b)) for b in bs[3:]]
    m2.drain()
    return it, ref, got, float((m2.dense.full_master() - ref_master).abs().max())


@pytest.mark.parametrize("consistency", ["bsp", "ssp", "asp"])
def test_checkpoint_resume_equivalence(tmp_path, consistency):
    prefix = str(tmp_path / "ck") + os.sep
    out = run_world(_ResumeFn(prefix, consistency), world=2)
    for r in (0, 1):
        it, ref, got, dmax = out[r]
        assert it == 3
        assert ref == got, (consistency, ref, got)
        assert dmax == 0.0
    # reference-format side files
    d = prefix + "iter_3/"
    assert open(prefix + "latest").read() == "3"
    prog = open(d + "server_progress_0_t1").read().split()
    assert prog[0] == "min_clock:3" and "100:3" in prog and "1100:3" in prog
    assert open(d + "worker_config_1").read().split() == ["1:3"]


class _ResumeFn:
    def __init__(self, prefix, consistency):
        self.prefix, self.consistency = prefix, consistency

    def __call__(self, rank, world):
        return _resume_fn(rank, world, self.prefix, self.consistency)


class _SaveFn:
    def __init__(self, prefix):
        self.prefix = prefix

    def __call__(self, rank, world):
        from minips_amd.ps.checkpoint import Checkpointer
        from minips_amd.ps.comm import Comm

        comm = Comm(device=torch.device("cpu"))
        m = _wd(comm)
        for b in _batches(2, 32, world, rank):
            m.train_step(*b)
        Checkpointer(comm, self.prefix).save(_tables(m), iteration=2, blocking=True)
        import torch.distributed as dist

        rows = [None] * world
        dist.all_gather_object(rows, m.emb.shard.tolist())
        # plain lists: a tensor sent through the result queue needs its sender alive
        return m.dense.full_master().tolist(), [r for part in rows for r in part]


def test_checkpoint_reshard_world2_to_world1(tmp_path):
    from minips_amd.ps.checkpoint import Checkpointer, load_text_params, parse_progress
    from minips_amd.ps.comm import Comm

    prefix = str(tmp_path / "ck") + os.sep
    out = run_world(_SaveFn(prefix), world=2)
    master2, emb2 = out[0]
    comm = Comm(device=torch.device("cpu"))
    m = _wd(comm)
    m.emb.shard.zero_()
    it = Checkpointer(comm, prefix).load(_tables(m))
    assert it == 2
    assert m.dense.full_master().tolist() == master2
    assert m.emb.shard.tolist() == emb2
    # the reference text format of the dense shard parses back to the same values
    from minips_amd._native import runtime

    d = prefix + "iter_2/"
    meta_rows = runtime().read_shard(d + "server_params_0_t1.bin")[0]["rows"]
    txt = load_text_params(d + "server_params_0_t1", meta_rows)
    assert torch.allclose(txt.float(), torch.tensor(master2[:meta_rows]), rtol=1e-6, atol=1e-9)
    assert parse_progress(d + "server_progress_1_t0")["min_clock"] == 2


@pytest.mark.gpu
def test_checkpoint_resume_on_gpu(dev, tmp_path):
    """Async D2H (side stream, pinned staging) + native writer on the real device."""
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.ps.checkpoint import Checkpointer
    from minips_amd.ps.comm import Comm

    comm = Comm(device=dev)
    prefix = str(tmp_path / "ck") + os.sep
    m = _wd(comm, "ssp", 1)
    data = CriteoSynth(256, cards=CARDS, device=dev, seed=3)
    for _ in range(3):
        m.train_step(*data.next())
    ck = Checkpointer(comm, prefix)
    ck.save(_tables(m), iteration=3)
    for _ in range(2):  # training continues while the checkpoint drains
        m.train_step(*data.next())
    ck.commit()
    m.drain()
    m2 = _wd(comm, "ssp", 1)
    assert Checkpointer(comm, prefix).load(_tables(m2)) == 3
    # restored state equals the state at iteration 3: replay the two steps and compare
    data2 = CriteoSynth(256, cards=CARDS, device=dev, seed=3)
    data2.skip(3)
    for _ in range(2):
        m2.train_step(*data2.next())
    m2.drain()
    # (float atomics in split-K GEMMs / scatter-adds: bitwise equality is not guaranteed on GPU)
    torch.testing.assert_close(m2.dense.master, m.dense.master, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(m2.emb.shard, m.emb.shard, rtol=1e-3, atol=1e-4)



def _fp64_table_roundtrip(device):
    from minips_amd.ps.checkpoint import Checkpointer
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.tables import DenseTable

    import tempfile

    n = 4099
    comm = Comm(device=torch.device(device))
    t = DenseTable(comm, n, optimizer="add", value_dtype=torch.float64)
    base = torch.arange(n, dtype=torch.float64)
    expect = torch.zeros(n, dtype=torch.float64)
    for s in range(5):
        assert torch.equal(t.get()[:n].cpu(), expect)
        d = 0.1 * base + 1e-9 * s
        t.add(d.to(device))
        t.clock()
        expect = expect + d
    t.drain()
    assert t.params.dtype == torch.float64 and torch.equal(t.full_master().cpu(), expect)
    with tempfile.TemporaryDirectory() as dname:
        Checkpointer(comm, os.path.join(dname, "ck")).save({"w": t}, iteration=5, blocking=True)
        t2 = DenseTable(comm, n, optimizer="add", value_dtype=torch.float64)
        assert Checkpointer(comm, os.path.join(dname, "ck")).load({"w": t2}) == 5
        assert torch.equal(t2.full_master().cpu(), expect)
        assert torch.equal(t2.get()[:n].cpu(), expect)


def test_dense_fp64_table_exact_cpu():
    """fp64 dense table (reference KVClientTable<double>): BSP adds are exact and a checkpoint
    round trip keeps every fp64 bit."""
    _fp64_table_roundtrip("cpu")


@pytest.mark.gpu
def test_dense_fp64_table_gpu_exact(dev):
    _fp64_table_roundtrip(dev)


@pytest.mark.gpu
@pytest.mark.parametrize("ring", [1 << 30, 1 << 16], ids=["pinned", "device_snapshot"])
def test_async_checkpoint_is_consistent_while_training(dev, tmp_path, ring):
    """A checkpoint saved without blocking while the next steps keep updating the shards holds
    exactly the state at the save (pinned: the compute stream waits for the D2H; above the ring
    size: a device-side snapshot streamed through the ring)."""
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig
    from minips_amd.ps.checkpoint import Checkpointer
    from minips_amd.ps.comm import Comm

    comm = Comm(device=dev)
    m = WideDeep(WideDeepConfig(cards=[1000, 50, 20000, 7, 300] + [20] * 21), comm)
    data = CriteoSynth(1024, cards=m.cfg.cards, device=dev, seed=1)
    for _ in range(2):
        m.train_step(*data.next())
    m.drain()
    ref_emb, ref_state, ref_dense = m.emb.shard.clone(), m.emb.state.clone(), m.dense.master.clone()
    ck = Checkpointer(comm, str(tmp_path / "ck_"), ring_bytes=ring)
    ck.save({0: m.emb, 1: m.dense}, iteration=2)  # async: returns before the files are written
    assert ck.last_mode == ("pinned" if ring > 1 << 20 else "device")
    for _ in range(4):  # these steps change every shard while the writer drains
        m.train_step(*data.next())
    ck.commit()
    assert not torch.equal(m.emb.shard, ref_emb)
    m2 = WideDeep(WideDeepConfig(cards=m.cfg.cards), comm)
    assert Checkpointer(comm, str(tmp_path / "ck_"), ring_bytes=ring).load({0: m2.emb, 1: m2.dense}) == 2
    assert torch.equal(m2.emb.shard, ref_emb) and torch.equal(m2.emb.state, ref_state)
    assert torch.equal(m2.dense.master, ref_dense)


@pytest.mark.gpu
def test_checkpoint_without_drain_waits_for_side_stream_adam(dev, tmp_path, monkeypatch):
    """One rank runs the dense Adam on the weight-gradient side stream and the main stream does not
    join it (WideDeep dense_side); a checkpoint saved right after a step, without model.drain(),
    must still hold the state after that Adam (DenseTable.hold -> drain): the Adam is held back
    10 ms by a spin kernel on the side stream, so a snapshot that did not wait would copy the
    pre-update master / m / v."""
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig
    from minips_amd.ps.checkpoint import Checkpointer
    from minips_amd.ps.comm import Comm
    from minips_amd.utils import streams

    comm = Comm(device=dev)
    cfg = WideDeepConfig(cards=[1000, 50, 20000, 7, 300] + [20] * 21)
    m = WideDeep(cfg, comm)
    data = CriteoSynth(1024, cards=cfg.cards, device=dev, seed=2)
    for _ in range(2):
        m.train_step(*data.next())
    idx = torch.device(dev).index or 0
    orig_clock = m.dense.clock

    def slow_clock():  # (on the side stream: the clock's Adam starts 10 ms late)
        streams.delay(streams.current_raw(idx), idx)
        orig_clock()

    monkeypatch.setattr(streams, "DELAY_US", 10000)
    monkeypatch.setattr(m.dense, "clock", slow_clock)
    m.train_step(*data.next())
    monkeypatch.setattr(streams, "DELAY_US", 0)
    assert m.__dict__.get("_side_pending") is not None  # the Adam was issued on the side stream
    Checkpointer(comm, str(tmp_path / "ck_")).save({0: m.emb, 1: m.dense}, iteration=3, blocking=True)
    m.drain()
    torch.cuda.synchronize()
    m2 = WideDeep(WideDeepConfig(cards=cfg.cards), comm)
    assert Checkpointer(comm, str(tmp_path / "ck_")).load({0: m2.emb, 1: m2.dense}) == 3
    assert torch.equal(m2.dense.master, m.dense.master)
    assert torch.equal(m2.dense.m, m.dense.m) and torch.equal(m2.dense.v, m.dense.v)
