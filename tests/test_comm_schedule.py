"""The data plane's ordering contract (minips_amd/ps/comm.py): every rank issues the same
sequence of collectives on its single communicator, so RCCL's in-order execution cannot
cross two ranks' collectives, whatever the per-rank data (splits) and the HW-queue count.

The Wide&Deep step runs exactly as in bench.py (LookaheadFeeder, lookahead depth 2, lookahead
planning, sparse + dense clocks) on 4 and 8 gloo ranks under BSP and SSP; each rank records
(op, dtype, row width / fixed size) per collective and the records must be identical.
(Reference contract: the single FIFO sender, comm/mailbox.cpp:231-308, comm/sender.cpp:7-30.)
"""
import os

import pytest
import torch

from test_ps_gloo import run_world

CARDS = [50, 7, 300, 20, 5, 60, 90, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28]


def _schedule_fn(consistency, staleness):
    def fn(rank, world):
        from minips_amd.data.synthetic import CriteoSynth
        from minips_amd.models.feeder import LookaheadFeeder
        from minips_amd.models.widedeep import WideDeep, WideDeepConfig
        from minips_amd.ps.comm import Comm

        torch.set_num_threads(1)
        comm = Comm(device=torch.device("cpu"))
        model = WideDeep(WideDeepConfig(cards=CARDS, consistency=consistency, staleness=staleness,
                                       transport="collective"), comm)
        # different data per rank: different all-to-all splits, same op sequence
        data = CriteoSynth(32 + 8 * rank, cards=CARDS, device="cpu", seed=100 + rank)
        comm.trace = []
        feeder = LookaheadFeeder(model, data, comm, depth=2)
        for _ in range(4):
            feeder.step()
        model.drain()
        comm.barrier()
        return comm.trace

    return fn


def _bsp(rank, world):
    return _schedule_fn("bsp", 0)(rank, world)


def _ssp(rank, world):
    return _schedule_fn("ssp", 1)(rank, world)


@pytest.mark.parametrize("world", [4, 8])
@pytest.mark.parametrize("fn", [_bsp, _ssp], ids=["bsp", "ssp1"])
def test_collective_sequence_identical_across_ranks(world, fn):
    out = run_world(fn, world=world)
    ref = out[0]
    kinds = {op for op, _, _ in ref}
    assert {"a2a_counts", "reduce_scatter", "all_gather"} <= kinds, kinds
    assert kinds & {"a2av", "a2av_p2p"}, kinds
    for r in range(1, world):
        assert out[r] == ref, (r, next(i for i, (a, b) in enumerate(zip(out[r], ref)) if a != b)
                               if len(out[r]) == len(ref) else (len(out[r]), len(ref)))
    # look-ahead planning never sits in front of a step's own exchanges in the FIFO: within a
    # step (up to its dense all-gather) every key-routing collective (int64) precedes the row
    # exchanges, i.e. the planning of step n+1 / n+2 was issued at the end of step n
    seg = []
    for op, dt, size in ref:
        seg.append(dt)
        if op == "all_gather":
            first = next(i for i, d in enumerate(seg) if d != "int64")
            assert "int64" not in seg[first:], seg
            seg = []


def test_no_extra_communicators():
    """One communicator per rank: tables never create process groups of their own."""
    import torch.distributed as dist

    calls = []
    orig = dist.new_group

    def spy(*a, **k):  # pragma: no cover - only called on a regression
        calls.append(a)
        return orig(*a, **k)

    dist.new_group = spy
    try:
        from minips_amd.models.widedeep import WideDeep, WideDeepConfig
        from minips_amd.ps.comm import Comm

        WideDeep(WideDeepConfig(cards=CARDS, consistency="ssp", staleness=1, transport="collective"),
                 Comm(device=torch.device("cpu")))
    finally:
        dist.new_group = orig
    assert calls == []


def test_bench_four_ranks_cpu():
    """bench.py under torchrun at 4 ranks (gloo, CPU, small tables): the driver's multi-rank
    control flow -- feeder, barriers, max-over-ranks timing, one JSON line, honest labels."""
    import json
    import subprocess
    import sys

    from _util import ROOT, free_ports

    env = dict(os.environ, OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(free_ports(1)[0]), "bench.py", "--gpus", "4", "--steps", "3",
           "--warmup", "1", "--batch", "64", "--test-cards", ",".join(map(str, CARDS))]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 4 and out["config"]["world_size"] == 4 and out["config"]["backend"] == "gloo"
    assert out["config"]["global_batch"] == 256 and "over gloo" in out["config"]["parallelism"]
    assert out["config"]["model"].startswith("PLUMBING TEST")


def _emulated_trace(world, consistency, staleness):
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.feeder import LookaheadFeeder
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig
    from minips_amd.ps.comm import LoopbackComm

    torch.set_num_threads(1)
    comm = LoopbackComm(world, 0, device=torch.device("cpu"))
    model = WideDeep(WideDeepConfig(cards=CARDS, consistency=consistency, staleness=staleness,
                                       transport="collective"), comm)
    data = CriteoSynth(32, cards=CARDS, device="cpu", seed=100)
    comm.trace = []
    feeder = LookaheadFeeder(model, data, comm, depth=2)
    losses = [float(feeder.step()) for _ in range(4)]
    model.drain()
    comm.barrier()
    return comm.trace, losses, model


@pytest.mark.parametrize("fn,cons", [(_bsp, ("bsp", 0)), (_ssp, ("ssp", 1))], ids=["bsp", "ssp1"])
def test_emulated_rank_issues_the_real_rank_program(fn, cons):
    """bench.py --emulate-world: one process running rank 0 of a 4-rank job over LoopbackComm
    issues exactly the collective sequence (op, dtype, row width) of a real 4-rank gloo job, so
    its profile is the per-rank program of the N-rank step; the owner applies land in its own
    row range and the loss stays finite."""
    real = run_world(fn, world=4)[0]
    emu, losses, model = _emulated_trace(4, *cons)
    assert emu == real
    assert all(l == l and abs(l) < 1e6 for l in losses)
    assert model.emb.rows_local == model.emb.bounds_list[1] and model.dense.shard * 4 == model.dense.n_pad


def test_loopback_wire_model_matches_survey_formulas():
    """LoopbackComm's modelled link times (SURVEY §5.8, 7 xGMI links of 153 GB/s at 8 ranks): an
    all-to-all puts every peer segment on its own link, a ring RS/AG is per-link bound, a direct
    one uses all 7 links; plus the per-collective latency."""
    import pytest

    from minips_amd.ps.comm import LoopbackComm

    S = 8 << 20
    ring = LoopbackComm(8, wire="ring", link_gbps=153, latency_us=8, device=torch.device("cpu"))
    direct = LoopbackComm(8, wire="direct", link_gbps=153, latency_us=8, device=torch.device("cpu"))
    none = LoopbackComm(8, device=torch.device("cpu"))
    bw = 153e3  # bytes per us
    assert ring.wire_time_us("rs", S) == pytest.approx(7 / 8 * S / bw + 8)
    assert direct.wire_time_us("ag", S) == pytest.approx(S / (8 * bw) + 8)
    assert ring.wire_time_us("a2a", S) == pytest.approx(S / (8 * bw) + 8)
    assert direct.wire_time_us("a2a", S) == ring.wire_time_us("a2a", S)
    assert none.wire_time_us("rs", S) == 0.0
    with pytest.raises(ValueError):
        LoopbackComm(8, wire="mesh", device=torch.device("cpu"))
