"""End-to-end Wide&Deep PS step on the GPU vs the same model on the CPU reference path."""
import pytest
import torch

from minips_amd.data.synthetic import CriteoSynth
from minips_amd.models.widedeep import WideDeep, WideDeepConfig
from minips_amd.ps.comm import Comm

pytestmark = pytest.mark.gpu

CARDS = [100, 50, 3000, 7, 300, 20, 5, 60, 90, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26]


def _run(device, steps=12, consistency="bsp", staleness=0):
    torch.manual_seed(0)
    cfg = WideDeepConfig(cards=CARDS, consistency=consistency, staleness=staleness, transport="collective")
    m = WideDeep(cfg, Comm(device=torch.device(device)))
    m.emb.shard.copy_(_init_rows(m))
    data = CriteoSynth(512, cards=CARDS, device="cpu", seed=3)
    losses = []
    for _ in range(steps):
        dense, keys, y = data.next()
        losses.append(float(m.train_step(dense.to(device), keys.to(device), y.to(device)).item()) / 512)
    m.drain()
    return losses, m


def _init_rows(m):
    g = torch.Generator().manual_seed(9)
    r = torch.randn(m.emb.rows_local, m.cfg.row_width, generator=g) * 0.01
    r[:, m.cfg.emb_dim:] = 0
    return r.to(m.emb.shard.device)


def test_widedeep_gpu_matches_cpu(dev):
    l_cpu, m_cpu = _run("cpu")
    l_gpu, m_gpu = _run(dev)
    assert l_gpu[-1] < l_gpu[0]
    for a, b in zip(l_gpu, l_cpu):
        assert abs(a - b) < 2e-2 * max(1.0, abs(b)), (l_gpu, l_cpu)
    # Adam normalises every gradient to ~lr per step, so elements whose gradient is ~0 can
    # flip sign under different (but equally valid) bf16 / atomic summation orders: bound
    # those by lr*steps and require the bulk to agree tightly.
    diff = (m_gpu.dense.master.cpu() - m_cpu.dense.master).abs()
    assert float(diff.max()) <= 1e-3 * 12 * 1.5
    assert float((diff > 2e-3).float().mean()) < 1e-2


@pytest.mark.parametrize("s", [1, 2])
def test_collective_ssp_read_bound(dev, s):
    """SSP(s) on the collective path (clocks on the table's side stream, reads gated at clock
    c - s - 1): every read at clock c holds the pushes of clocks < c - s and never more than were
    issued, and reads DO run ahead of a slow apply (the side stream is slowed by a spin kernel
    before each clock) -- so the bound, not a synchronous apply, is what holds."""
    from minips_amd.ps.tables import SparseTable

    t = SparseTable(Comm(device=torch.device(dev)), 64, 4, optimizer="add", consistency="ssp", staleness=s,
                    pull_dtype=torch.float32, init_std=0.0)
    assert t.pipe.async_
    k = torch.tensor([7], device=dev)
    # a deterministic delay on the side stream (a ~9 TFLOP GEMM, several ms on any MI355X clock),
    # not a cycle-count spin, whose duration depends on the clock source
    a = torch.randn(8192, 8192, device=dev).to(torch.bfloat16)
    seen = []
    for c in range(16):
        v = float(t.get_rows(k)[0, 0])  # a Get at clock c
        seen.append((c, v))
        t.add_keys(k, torch.ones(1, 4, device=dev))
        with torch.cuda.stream(t.pipe.stream):
            for _ in range(8):
                torch.matmul(a, a)  # the clock's apply lands late
        t.clock()
    t.drain()
    for c, v in seen:
        assert max(0, c - s) <= v <= c, (s, seen)
    assert any(v < c for c, v in seen), seen  # the reads really were stale
    assert float(t.get_rows(k)[0, 0]) == 16


def test_widedeep_ssp_staleness_histogram(dev):
    """W&D SSP s=1 end to end: the metrics log's observed-staleness histogram never exceeds s."""
    from minips_amd.utils.metrics import get_logger

    log = get_logger()
    log.staleness_hist.clear()
    losses, _ = _run(dev, steps=10, consistency="ssp", staleness=1)
    assert all(l == l for l in losses) and losses[-1] < losses[0] + 0.05
    assert log.staleness_hist and max(log.staleness_hist) <= 1, log.staleness_hist


def test_widedeep_lookahead_depth_matches(dev):
    """Key plans issued 1 or 2 batches ahead on the planning stream (bench.py's data-loader
    depth) give the same training as planning each batch in its own step: planning reads no
    table state, so the lookahead changes no semantics."""
    data = CriteoSynth(512, cards=CARDS, device="cpu", seed=4)
    batches = [tuple(t.to(dev) for t in data.next()) for _ in range(8)]
    res = {}
    for depth in (0, 1, 2):
        torch.manual_seed(0)
        m = WideDeep(WideDeepConfig(cards=CARDS), Comm(device=torch.device(dev)))
        m.emb.shard.copy_(_init_rows(m))
        for k in range(1, depth):  # batches 1..depth-1 planned before the first step
            m.prefetch(batches[k][1])
        losses = []
        for i, (dense, keys, y) in enumerate(batches):
            nk = batches[i + depth][1] if depth and i + depth < len(batches) else None
            losses.append(float(m.train_step(dense, keys, y, next_keys=nk).item()) / 512)
        m.drain()
        res[depth] = losses
    # (the deterministic reductions of round 5: the round-3 bound again)
    for depth in (1, 2):
        for a, b in zip(res[depth], res[0]):
            assert abs(a - b) < 1e-4, (depth, res)


def test_widedeep_bsp_one_rank_bit_identical(dev):
    """Two same-seed Wide&Deep BSP runs at one rank, through the bench's look-ahead feeder and
    streams, end bit-identical (loss, dense master, embedding shard and Adagrad state): every
    reduction of the step has one fixed summation order (segment sums, bias column sums, the head's
    fold, the split-K planes folded by Adam) -- the reference BSP applies a superstep's Adds in one
    fixed order too (server/consistency/bsp_model.cpp:14-32)."""
    from minips_amd.models.feeder import LookaheadFeeder

    out = []
    for _ in range(2):
        comm = Comm(device=torch.device(dev))
        m = WideDeep(WideDeepConfig(cards=CARDS), comm)
        feeder = LookaheadFeeder(m, CriteoSynth(4096, cards=CARDS, device=dev, seed=11), comm)
        losses = [feeder.step().clone() for _ in range(6)]
        m.drain()
        torch.cuda.synchronize()
        out.append((torch.stack(losses).cpu(), m.dense.full_master().cpu(), m.emb.shard.cpu().clone(),
                    m.emb.state.cpu().clone()))
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)


def test_widedeep_fused_assemble_matches_gather(dev, monkeypatch):
    """One rank: the input assembled straight from the shard (SparseTable.get_source) trains
    exactly like the gathered Get + wd_assemble."""
    import minips_amd.ps.tables as tables

    res = {}
    for fused in (False, True):
        monkeypatch.setattr(tables, "_FUSED_ASSEMBLE", fused)
        losses, m = _run(dev, steps=6)
        res[fused] = (losses, m.emb.shard.cpu())
    (l0, s0), (l1, s1) = res[False], res[True]
    for a, b in zip(l0, l1):
        assert abs(a - b) <= 1e-4 * max(1.0, abs(a)), (l0, l1)
    assert float((s0 - s1).abs().max()) < 1e-3


def test_widedeep_wgrad_slabs_folded_by_adam(dev, monkeypatch):
    """One rank: the split-K weight gradients left in their slab planes and folded by the dense
    table's Adam kernel (DenseTable.slab_sink) train like the reduce-kernel path."""
    import minips_amd.ps.tables as tables

    res = {}
    for defer in (False, True):
        monkeypatch.setattr(tables, "_WGRAD_DEFER", defer)
        losses, m = _run(dev, steps=4)
        if defer:
            assert m.dense.slab_sink() is not None and not m.dense._sink._pending
        res[defer] = (losses, m.dense.master.cpu())
    (l0, p0), (l1, p1) = res[False], res[True]
    for a, b in zip(l0, l1):
        assert abs(a - b) <= 1e-3 * max(1.0, abs(a)), (l0, l1)
    diff = (p0 - p1).abs()
    assert float((diff > 2e-4).float().mean()) < 1e-2


@pytest.mark.parametrize("defer", [True, False])
def test_widedeep_launch_list_replay_bit_identical(dev, monkeypatch, defer):
    """The dense forward and backward chain replayed from the native launch list (layers.Replayer)
    train bit-identically to the op-by-op issue, with the split-K planes folded by Adam (defer) and
    with the list's own persistent reduce planes (no slab sink: the several-rank path)."""
    import minips_amd.models.widedeep as wd
    import minips_amd.ps.tables as tables
    from minips_amd.models.feeder import LookaheadFeeder

    monkeypatch.setattr(tables, "_WGRAD_DEFER", defer)
    out = {}
    for replay in (False, True):
        monkeypatch.setattr(wd, "_REPLAY", replay)
        comm = Comm(device=torch.device(dev))
        m = WideDeep(WideDeepConfig(cards=CARDS), comm)
        feeder = LookaheadFeeder(m, CriteoSynth(4096, cards=CARDS, device=dev, seed=11), comm)
        losses = [feeder.step().clone() for _ in range(6)]
        m.drain()
        torch.cuda.synchronize()
        if replay:
            assert len(m._replay._lists) >= 2  # the forward and the backward chain were recorded
        out[replay] = (torch.stack(losses).cpu(), m.dense.full_master().cpu(), m.emb.shard.cpu().clone())
    for a, b in zip(out[False], out[True]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("where", ["main", "fork", "use", "use+fork+main"])
def test_widedeep_one_rank_invariant_under_stream_delays(dev, monkeypatch, where):
    """Cross-stream ordering check of the one-rank BSP step: 300-us spins injected where streams
    hand off (MINIPS_STREAM_DEBUG delay modes: the forked side stream late, the compute stream late
    after each fork, the planning / clock streams late) leave the loss trajectory, the dense master
    and the embedding shard bit-identical. A consumer that misses its wait on a producer stream then
    reads data of the wrong step deterministically (the "main" spin exposed the side-stream Adam
    rewriting W1 under the embedding dgrad, profiles/r5/race_dgrad_adam.txt)."""
    from minips_amd.models.feeder import LookaheadFeeder
    from minips_amd.utils import streams

    def run():
        comm = Comm(device=torch.device(dev))
        m = WideDeep(WideDeepConfig(cards=CARDS), comm)
        feeder = LookaheadFeeder(m, CriteoSynth(4096, cards=CARDS, device=dev, seed=11), comm)
        losses = [feeder.step().clone() for _ in range(6)]
        m.drain()
        torch.cuda.synchronize()
        return torch.stack(losses).cpu(), m.dense.full_master().cpu(), m.emb.shard.cpu().clone()

    ref = run()
    monkeypatch.setattr(streams, "DELAY_US", 300)
    monkeypatch.setattr(streams, "DELAY_WHERE", set(where.split("+")))
    got = run()
    for a, b in zip(ref, got):
        assert torch.equal(a, b), where
