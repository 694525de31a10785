"""The data plane's RCCL calls on real hardware. RCCL refuses two ranks on one device, so a
one-GPU box can only run a one-rank communicator; with ``Comm(force_collectives=True)`` every
Comm collective still goes through ProcessGroupNCCL (= RCCL) with exactly the dtypes, layouts
and split lists the tables use at N > 1 (bf16 row all-to-all-v with uneven splits, int64 count
exchange, fp32/fp64 reduce-scatter, in-place bf16/fp64 all-gather, MAX all-reduce of the bench's
timer, the barrier), so a layout or dtype RCCL rejects fails here instead of in the driver's
8-GPU scaling run."""
import datetime

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture()
def nccl_comm():
    from _util import free_ports
    from minips_amd.ps.comm import Comm

    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_ports(1)[0]}", rank=0, world_size=1,
                            device_id=dev, timeout=datetime.timedelta(seconds=60))
    try:
        assert dist.get_backend() == "nccl"
        yield Comm(device=dev, force_collectives=True)
    finally:
        dist.destroy_process_group()


def test_rccl_table_collectives(nccl_comm):
    comm = nccl_comm
    dev = comm.device
    assert comm._rc() is not None  # the native data plane (csrc/comm/rccl_comm.h) carries every call
    # sparse Get / Add: rows of width 33 (32 emb + 1 wide) in bf16, and fp32 gradient rows
    for dt in (torch.bfloat16, torch.float32):
        inp = torch.randn(1000, 33, device=dev).to(dt)
        out = torch.empty(1200, 33, dtype=dt, device=dev)
        comm.all_to_all_v(out, inp, [937], [937])
        torch.testing.assert_close(out[:937], inp[:937], rtol=0, atol=0)
        out.zero_()
        comm.all_to_all_v(out, inp, [937], [937], p2p=True)  # the SSP/ASP send/recv form
        torch.testing.assert_close(out[:937], inp[:937], rtol=0, atol=0)
    keys = torch.randint(0, 1 << 40, (500,), device=dev)
    kout = torch.empty(500, dtype=torch.int64, device=dev)
    comm.all_to_all_v(kout, keys, [500], [500])
    assert torch.equal(kout, keys)
    counts = torch.tensor([123], dtype=torch.int64, device=dev)
    recv = torch.empty_like(counts)
    comm.all_to_all_counts(recv, counts)
    assert recv.item() == 123
    assert comm.exchange_counts(counts) == ([123], [123])
    # dense Clock: reduce-scatter of the fp32 / fp64 gradient, in-place all-gather of the params
    for dt in (torch.float32, torch.float64):
        g = torch.randn(4096, dtype=dt, device=dev)
        shard = torch.empty(4096, dtype=dt, device=dev)
        comm.reduce_scatter(shard, g)
        torch.testing.assert_close(shard, g, rtol=0, atol=0)
    for dt in (torch.bfloat16, torch.float64):
        full = torch.randn(4096, device=dev).to(dt)
        ref = full.clone()
        comm.all_gather(full, full[:4096])  # the shard aliases its slot of the full buffer
        torch.testing.assert_close(full, ref, rtol=0, atol=0)
    t = torch.tensor([1.5], dtype=torch.float64, device=dev)
    comm.all_reduce_(t, op=dist.ReduceOp.MAX)
    assert t.item() == 1.5
    comm.barrier()
    assert comm.stats.calls > 0


def test_rccl_collectives_from_side_streams(nccl_comm):
    """Collectives issued from the planning stream and a clock stream (as the tables do) complete
    in issue order on the one communicator."""
    comm = nccl_comm
    dev = comm.device
    ps, cs = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    a = torch.arange(64 * 33, dtype=torch.float32, device=dev).view(64, 33).to(torch.bfloat16)
    b = torch.empty_like(a)
    g = torch.randn(1 << 16, device=dev)
    shard = torch.empty_like(g)
    for _ in range(5):
        with torch.cuda.stream(ps):
            ps.wait_stream(torch.cuda.current_stream(dev))
            comm.all_to_all_v(b, a, [64], [64])
        with torch.cuda.stream(cs):
            cs.wait_stream(torch.cuda.current_stream(dev))
            comm.reduce_scatter(shard, g)
    torch.cuda.synchronize(dev)
    assert torch.equal(b, a) and torch.equal(shard, g)


def test_rccl_destroy_reinit_restore(tmp_path, monkeypatch):
    """The in-place rollback path of minips_amd.train (rollback(): destroy the broken group ->
    re-init -> Comm.refresh -> reset_after_rollback -> restore the committed checkpoint -> go on)
    on real RCCL state: a world-1 NCCL group with every table collective forced through it and
    the tables' clock side streams active. Training after the restore repeats the losses of the
    run that continued from the checkpoint without the rollback."""
    from _util import free_ports
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig
    from minips_amd.ps.checkpoint import Checkpointer
    from minips_amd.ps.comm import Comm

    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)

    def init():
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_ports(1)[0]}", rank=0, world_size=1,
                                device_id=dev, timeout=datetime.timedelta(seconds=60))

    cards = [1000, 50, 2000, 7, 300, 20, 5, 60, 90, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26]
    init()
    try:
        comm = Comm(device=dev, force_collectives=True)
        model = WideDeep(WideDeepConfig(cards=cards), comm)
        assert model.emb.pipe.async_ and model.dense.pipe.async_
        tables = {0: model.emb, 1: model.dense}
        ck = Checkpointer(comm, prefix=str(tmp_path) + "/")
        data = CriteoSynth(512, cards=cards, device=dev, seed=3)
        batches = [data.next() for _ in range(7)]
        for i in range(3):
            model.train_step(*batches[i])
        ck.save(tables, iteration=3)
        ck.commit()
        ref = [float(model.train_step(*batches[i]).item()) for i in range(3, 7)]
        calls_before = comm.stats.calls
        assert calls_before > 0  # the clocks really went through RCCL
        model.drain()
        torch.cuda.synchronize(dev)
        dist.destroy_process_group()
        init()
        comm.refresh()
        assert comm.backend == "nccl" and comm.world == 1
        for t in tables.values():
            t.reset_after_rollback()
        if hasattr(model, "_pending_plans"):
            model._pending_plans = []
        assert ck.load(tables) == 3
        again = [float(model.train_step(*batches[i]).item()) for i in range(3, 7)]
        model.drain()
        torch.cuda.synchronize(dev)
        assert comm.stats.calls > calls_before
        for a, b in zip(again, ref):
            assert abs(a - b) <= 2e-3 * abs(b) + 1e-3, (again, ref)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_native_rccl_matches_c10d(nccl_comm, monkeypatch):
    """The native RCCL data plane and torch's ProcessGroupNCCL give identical results for every
    collective the tables issue (uneven bf16 row all-to-all-v, int64 keys, fp32 / fp64
    reduce-scatter, bf16 all-gather, MAX all-reduce)."""
    from minips_amd.ps import comm as cm

    dev = nccl_comm.device
    g = torch.Generator(device=dev).manual_seed(7)
    rows = torch.randn(777, 36, device=dev, generator=g).to(torch.bfloat16)
    keys = torch.randint(0, 1 << 40, (777,), device=dev, generator=g)
    grad = torch.randn(1 << 15, device=dev, generator=g)
    gd = grad.double()
    par = torch.randn(1 << 14, device=dev, generator=g).to(torch.bfloat16)
    outs = {}
    for native in (True, False):
        monkeypatch.setattr(cm, "_NATIVE_RCCL", native)
        c = cm.Comm(device=dev, force_collectives=True)
        assert (c._rc() is not None) == native
        r = torch.zeros(800, 36, dtype=torch.bfloat16, device=dev)
        c.all_to_all_v(r, rows, [777], [777])
        k = torch.zeros(800, dtype=torch.int64, device=dev)
        c.all_to_all_v(k, keys, [777], [777], p2p=True)
        rs, rsd = torch.empty_like(grad), torch.empty_like(gd)
        c.reduce_scatter(rs, grad)
        c.reduce_scatter(rsd, gd)
        ag = torch.empty_like(par)
        c.all_gather(ag, par)
        m = torch.tensor([2.5, -1.0], device=dev)
        c.all_reduce_(m, op=dist.ReduceOp.MAX)
        torch.cuda.synchronize(dev)
        outs[native] = [r, k, rs, rsd, ag, m]
    for a, b in zip(outs[True], outs[False]):
        assert torch.equal(a, b)


def test_native_rccl_watchdog_aborts_a_stuck_collective(nccl_comm):
    """A stream that stops completing (a collective waiting for a dead peer, here: 1.5 s of device
    spins queued behind one) is detected by the native communicator's watchdog within its
    timeout: the communicator is aborted and the next call raises the torch.distributed error the
    training driver's recovery handles (train._is_comm_failure) -- no hang."""
    import time

    from minips_amd._native import kernels
    from minips_amd.ps.comm import _rccl_call, _rccl_lib
    from minips_amd.train import _is_comm_failure

    dev = nccl_comm.device
    k = kernels()
    lib = _rccl_lib()
    rc = k.Rccl(lib, k.rccl_unique_id(lib), 1, 0, dev.index or 0, timeout_s=0.4, teardown=False)
    s = torch.cuda.Stream(device=dev)
    x = torch.ones(1024, device=dev)
    y = torch.empty_like(x)
    buf = torch.zeros(2, dtype=torch.int64, device=dev)
    with torch.cuda.stream(s):
        rc.all_gather(y, x)  # the stream is now watched
        for _ in range(150):  # 150 x 10 ms of spins: the stream makes no progress for ~1.5 s
            k.clock_probe(buf, 1_000_000, s.cuda_stream)
    t0 = time.monotonic()
    while not rc.aborted and time.monotonic() - t0 < 5.0:
        time.sleep(0.02)
    assert rc.aborted, "the watchdog did not abort the stuck communicator"
    assert "did not complete" in rc.async_error()
    with pytest.raises(dist.DistBackendError) as ei:
        with torch.cuda.stream(s):
            _rccl_call(rc.all_gather, y, x)
    assert _is_comm_failure(ei.value)
    torch.cuda.synchronize(dev)  # the spins drain; nothing is left running


def test_native_rccl_keeps_issue_order_across_streams(nccl_comm):
    """The data plane's deadlock-freedom argument (ps/comm.py, ordering contract 1) needs one
    communicator's collectives to run in issue order even when they are enqueued on different
    HIP streams: collective B on stream 2 must not finish before collective A, issued first on
    stream 1 behind a ~2 ms kernel. RCCL alone lets B overtake A (this test failed, B done at
    0.28 ms); RcclComm chains each collective after the previous one's completion event."""
    from minips_amd._native import kernels

    comm = nccl_comm
    dev = comm.device
    rc = comm._rc()
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    a, b = torch.ones(1 << 18, device=dev), torch.ones(1 << 18, device=dev)
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    e_spin, e_b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record(s1)
    s2.wait_event(t0)
    kernels().wire_spin(200000, 1, s1.cuda_stream)  # ~2 ms
    e_spin.record(s1)
    with torch.cuda.stream(s1):
        rc.all_reduce(a, 0)
    with torch.cuda.stream(s2):
        rc.all_reduce(b, 0)
    e_b.record(s2)
    torch.cuda.synchronize()
    assert t0.elapsed_time(e_b) >= t0.elapsed_time(e_spin), "RCCL ran a later collective ahead of an earlier one"
