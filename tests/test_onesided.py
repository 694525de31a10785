"""Asynchronous SSP / ASP with an owner-side optimizer apply (minips_amd/ps/onesided.py,
csrc/runtime/async_server.h, csrc/kernels/onesided.hip).

* straggler: rank 1 sleeps every clock. SSP(s): rank 0 runs exactly s clocks ahead of what every
  owner applied and never s + 1, and every value it reads holds the pushes of every rank's clocks
  < c - s (ssp_model.cpp:58-85); ASP: rank 0 never waits (asp_model.cpp:18-26). Final values are
  exact (no lost update).
* replay: the owners apply row-wise Adagrad (sparse) and Adam (dense) with their own state; an
  fp32 CPU replay of each owner's logged apply order reproduces its shard and state.
* models: Wide&Deep and DLRM on the one-sided transport with their real optimizers.
CPU: /dev/shm shards and inboxes, the same C++ server loop with the PyTorch reference apply.
GPU: two processes share cuda:0 and map each other's buffers through hipIpcOpenMemHandle.
"""
import time

import pytest
import torch

from test_ps_gloo import run_world

STEPS = 12


def _run(rank, world, consistency, s, dev):
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.onesided import AsyncSparseTable

    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    comm = Comm(device=dev)
    t = AsyncSparseTable(comm, num_rows=101, width=4, optimizer="add", consistency=consistency, staleness=s,
                         pull_dtype=torch.float32, init_std=0.0, route="range", max_keys=64)
    shared = torch.tensor([5], device=dev)
    own = torch.tensor([60 + rank], device=dev)
    seen = []
    for c in range(STEPS):
        if rank == 1:
            time.sleep(0.03)  # straggler
        v = float(t.get_rows(shared)[0, 0])
        seen.append((c, c - t.ps.board.min_applied(t.t), v))
        t.add_keys(torch.cat([shared, own]), torch.ones(2, 4, device=dev))
        t.clock()
    t.drain()
    comm.barrier()  # every rank drained: every push is applied everywhere
    final = t.get_rows(torch.tensor([5, 60, 61], device=dev))[:, 0].tolist()
    stats = t.staleness_stats()
    comm.barrier()
    t.close()
    return seen, stats, final


def _ssp1(rank, world, dev=torch.device("cpu")):
    return _run(rank, world, "ssp", 1, dev)


def _ssp2(rank, world, dev=torch.device("cpu")):
    return _run(rank, world, "ssp", 2, dev)


def _asp(rank, world, dev=torch.device("cpu")):
    return _run(rank, world, "asp", 0, dev)


def _check(out, consistency, s, world=2):
    seen0, stats0, _ = out[0]
    for rank, (_, _, fin) in out.items():
        assert fin == [world * STEPS, STEPS, STEPS], (rank, fin)  # every push applied exactly once
    if consistency == "ssp":
        # the staleness each read observed: exactly s clocks at the straggler, never s + 1
        assert stats0["max"] == s, stats0
        assert stats0["waited_s"] > 0 and stats0["gate_waits"] > 0, stats0
        for c, st, v in seen0:  # SSP read guarantee: every rank's clocks < c - s are in the row
            assert st <= s, (c, st)
            assert v >= world * max(0, c - s), (c, v)
    else:
        assert stats0["waited_s"] == 0.0 and stats0["gate_waits"] == 0, stats0
        assert stats0["max"] >= 4, stats0  # ran far ahead of the straggler


@pytest.mark.parametrize("fn,consistency,s", [(_ssp1, "ssp", 1), (_ssp2, "ssp", 2), (_asp, "asp", 0)],
                         ids=["ssp1", "ssp2", "asp"])
def test_async_staleness_cpu(fn, consistency, s):
    _check(run_world(fn, world=2), consistency, s)


def _g_ssp1(rank, world):
    return _run(rank, world, "ssp", 1, torch.device("cuda", 0))


def _g_asp(rank, world):
    return _run(rank, world, "asp", 0, torch.device("cuda", 0))


@pytest.mark.gpu
@pytest.mark.parametrize("fn,consistency,s", [(_g_ssp1, "ssp", 1), (_g_asp, "asp", 0)], ids=["ssp1", "asp"])
def test_async_staleness_gpu_ipc(dev, fn, consistency, s):
    """Two processes share cuda:0; each maps the other's shard and inbox through
    hipIpcOpenMemHandle, pushes with ps_push_rows and reads with ps_gather_rows, and its server
    thread applies the other's pushes (csrc/kernels/onesided.hip)."""
    _check(run_world(fn, world=2), consistency, s)


# ------------------------------------------------------------------------------ replay of the owner apply
ROWS, W, NP = 97, 8, 1000


def _push_of(r, c):
    """The (keys, grad rows) of requester r's clock c, and its dense gradient (deterministic)."""
    g = torch.Generator().manual_seed(1000 * r + c)
    keys = torch.randperm(ROWS, generator=g)[:20]  # unique keys, both owners, overlapping ranks
    rows = torch.randn(20, W, generator=g)
    dense = torch.randn(NP, generator=g) * 0.1
    return keys, rows, dense


def _replay_run(rank, world, dev=torch.device("cpu"), consistency="asp"):
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.onesided import AsyncDenseTable, AsyncSparseTable

    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    comm = Comm(device=dev)
    # (SSP: staleness 3 -- the straggler's sleeps then interleave the applies with the pushes)
    sp = AsyncSparseTable(comm, num_rows=ROWS, width=W, optimizer="rowwise_adagrad", lr=0.1, consistency=consistency,
                          pull_dtype=torch.float32, init_std=0.0, route="range", max_keys=64, split=6, staleness=3)
    dn = AsyncDenseTable(comm, NP, optimizer="adam", lr=0.01, consistency=consistency, pull_dtype=torch.float32,
                         staleness=3)
    assert sp.coalesced == dn.coalesced == (consistency == "ssp" and world > 1)
    sp.ps.server.set_log(True)
    comm.barrier()  # every owner logs before any peer pushes (else its first applies go unlogged)
    for c in range(STEPS):
        if rank == 1 and c % 3 == 0:
            time.sleep(0.01)  # vary the interleaving
        keys, rows, dense = _push_of(rank, c)
        sp.add_keys(keys.to(dev), rows.to(dev))
        sp.clock()
        dn.add(dense.to(dev))
        dn.clock()
    sp.drain()
    dn.drain()
    comm.barrier()
    # numpy (pickled by value): torch tensors would travel as shared-memory handles that die with
    # this process before the parent unpickles them
    out = dict(log=sp.ps.apply_log(), shard=sp.shard.cpu().numpy().copy(), state=sp.state.cpu().numpy().copy(),
               state2=sp.state2.cpu().numpy().copy(), base=sp.base, master=dn.master.cpu().numpy().copy(),
               m=dn.m.cpu().numpy().copy(), v=dn.v.cpu().numpy().copy(), dbase=dn.base, dshard=dn.shard)
    comm.barrier()
    return out


def _replay_check(out, world=2, coalesced=False):
    """ASP: replay every push in this owner's apply order. SSP (clock-coalesced): per clock, the
    requesters' rows summed per key in requester order and ONE row-wise Adagrad / Adam step at lr."""
    from minips_amd import ops

    for o, res in out.items():
        res = {k: torch.from_numpy(v) if hasattr(v, "dtype") and not isinstance(v, int) else v for k, v in res.items()}
        log = res["log"]
        assert len(log) == 2 * world * STEPS, len(log)  # every clock of every requester, both tables
        lo, hi = res["base"], res["base"] + res["shard"].shape[0]
        shard = torch.zeros(hi - lo, W)
        state = torch.zeros(hi - lo)
        state2 = torch.zeros(hi - lo)
        S, db = res["dshard"], res["dbase"]
        w = torch.zeros(S)
        m = torch.zeros(S)
        v = torch.zeros(S)
        step = 0
        if coalesced:
            for t, r, c in log:  # whole clocks, requesters in order
                assert r == [x for x in log if x[0] == t and x[2] == c].index((t, r, c)), log
            for c in range(STEPS):
                agg, dsum = {}, torch.zeros(NP)
                for r in range(world):
                    keys, rows, dense = _push_of(r, c)
                    for k, row in zip(keys.tolist(), rows):
                        if lo <= k < hi:
                            agg[k] = agg[k] + row if k in agg else row.clone()
                    dsum += dense
                ks = sorted(agg)
                ops.sparse_rowwise_adagrad(shard, state, torch.tensor(ks, dtype=torch.int64), lo,
                                           torch.stack([agg[k] for k in ks]), 0.1, 1e-8, state2=state2, split=6)
                g = torch.zeros(S)
                n = max(0, min(S, NP - db))
                g[:n] = dsum[db: db + n]
                ops.adam_apply(w, m, v, g, 0.01, 0.9, 0.999, 1e-8, 0.0, c + 1, 1.0, None)
            log = []
        for t, r, c in log:  # this owner's apply order
            keys, rows, dense = _push_of(r, c)
            if t == 0:
                mine = (keys >= lo) & (keys < hi)
                ops.sparse_rowwise_adagrad(shard, state, keys[mine], lo, rows[mine], 0.1, 1e-8, state2=state2,
                                           split=6)
            else:
                step += 1
                g = torch.zeros(S)
                n = max(0, min(S, NP - db))
                g[:n] = dense[db: db + n]
                ops.adam_apply(w, m, v, g, 0.01 / world, 0.9, 0.999, 1e-8, 0.0, step, 1.0, None)  # (push_lr)
        torch.testing.assert_close(res["shard"], shard, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(res["state"], state, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(res["state2"], state2, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(res["master"], w, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(res["m"], m, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(res["v"], v, rtol=1e-5, atol=1e-8)


def test_owner_apply_replay_cpu():
    _replay_check(run_world(_replay_run, world=2))


def _replay_ssp(rank, world):
    return _replay_run(rank, world, consistency="ssp")


def _g_replay_ssp(rank, world):
    return _replay_run(rank, world, torch.device("cuda", 0), consistency="ssp")


def test_owner_apply_replay_ssp_coalesced_cpu():
    """SSP: the owner applies a clock once every requester sent it, one optimizer step over the
    summed pushes (the reference's linear Add, ssp_model.cpp:54-56)."""
    _replay_check(run_world(_replay_ssp, world=2), coalesced=True)


def _g_replay(rank, world):
    return _replay_run(rank, world, torch.device("cuda", 0))


@pytest.mark.gpu
def test_owner_apply_replay_gpu_ipc(dev):
    """The owners' HIP applies (row-wise Adagrad with a split state, Adam) match an fp32 CPU replay
    of the same apply order."""
    _replay_check(run_world(_g_replay, world=2))


@pytest.mark.gpu
def test_owner_apply_replay_ssp_coalesced_gpu_ipc(dev):
    """The clock-coalesced HIP applies (ps_clock_adagrad with a split state, summed dense push +
    one Adam step per clock) match the fp32 CPU replay, at 2 and 4 requesters."""
    _replay_check(run_world(_g_replay_ssp, world=2), coalesced=True)
    _replay_check(run_world(_g_replay_ssp, world=4), world=4, coalesced=True)


# ------------------------------------------------------------------------------ models
def _dlrm_run(rank, world, dev=torch.device("cpu"), steps=10):
    from minips_amd.models.dlrm import DLRM, DLRMConfig
    from minips_amd.ps.comm import Comm

    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    comm = Comm(device=dev)
    cfg = DLRMConfig(num_rows=5003, D=16, consistency="asp", transport="onesided", lr_sparse=0.05, max_batch=64)
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
    out = (losses, m.emb.clock_n, m.dense.step, m.emb.optimizer, m.dense.optimizer)
    comm.barrier()
    return out


def test_dlrm_onesided_asp_cpu():
    """DLRM config 5 on the one-sided path: ASP, row-wise Adagrad + Adam applied by the owners."""
    out = run_world(_dlrm_run, world=2)
    for rank, (losses, ck, st, so, do) in out.items():
        assert ck == 10 and st == 10 and (so, do) == ("rowwise_adagrad", "adam")
        assert all(l == l for l in losses) and losses[-1] < losses[0], (rank, losses)


def _g_dlrm(rank, world):
    return _dlrm_run(rank, world, torch.device("cuda", 0))


@pytest.mark.gpu
def test_dlrm_onesided_asp_gpu_ipc(dev):
    out = run_world(_g_dlrm, world=2)
    for rank, (losses, ck, st, so, do) in out.items():
        assert ck == 10 and all(l == l for l in losses) and losses[-1] < losses[0], (rank, losses)


def _wd_losses(dev, transport, consistency, s, steps=30, B=256):
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig
    from minips_amd.ps.comm import Comm

    cards = [50, 7, 300, 20, 5, 60, 90, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28]
    cfg = WideDeepConfig(cards=cards, consistency=consistency, staleness=s, transport=transport, max_batch=B)
    m = WideDeep(cfg, Comm(device=dev))
    data = CriteoSynth(B, cards=cards, device=dev, seed=3)
    out = []
    for _ in range(steps):
        out.append(float(m.train_step(*data.next())) / B)
    m.drain()
    return out, m


def test_widedeep_onesided_ssp_tracks_bsp_cpu():
    """W&D SSP s=1 on the one-sided path (owner-side row-wise Adagrad + Adam) follows the BSP
    loss curve of the collective path (one rank; the apply of clock c-1 may land after Get c)."""
    bsp, _ = _wd_losses(torch.device("cpu"), "collective", "bsp", 0)
    ssp, m = _wd_losses(torch.device("cpu"), "onesided", "ssp", 1)
    assert m.emb.staleness_stats()["max"] <= 1
    a, b = sum(bsp[-10:]) / 10, sum(ssp[-10:]) / 10
    assert ssp[-1] < ssp[0] and abs(a - b) < 0.05 * a, (bsp, ssp)


@pytest.mark.gpu
def test_widedeep_onesided_ssp_tracks_bsp_gpu(dev):
    bsp, _ = _wd_losses(dev, "collective", "bsp", 0, steps=60, B=2048)
    ssp, m = _wd_losses(dev, "onesided", "ssp", 1, steps=60, B=2048)
    st = m.emb.staleness_stats()
    assert st["max"] <= 1, st
    a, b = sum(bsp[-20:]) / 20, sum(ssp[-20:]) / 20
    assert ssp[-1] < ssp[0] and abs(a - b) < 0.05 * a, (bsp, ssp)


# ------------------------------------------------------------------------------ checkpoint / restore
def _ckpt_run(rank, world, prefix):
    from minips_amd.ps.checkpoint import Checkpointer
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.onesided import AsyncDenseTable, AsyncSparseTable

    dev = torch.device("cpu")
    comm = Comm(device=dev)
    sp = AsyncSparseTable(comm, num_rows=ROWS, width=W, optimizer="rowwise_adagrad", lr=0.1, consistency="ssp",
                          staleness=1, pull_dtype=torch.float32, init_std=0.01, max_keys=64)
    dn = AsyncDenseTable(comm, NP, optimizer="adam", lr=0.01, consistency="ssp", staleness=1,
                         pull_dtype=torch.float32)
    ck = Checkpointer(comm, prefix)
    for c in range(6):
        keys, rows, dense = _push_of(rank, c)
        sp.get(keys)
        sp.add_keys(keys, rows)
        sp.clock()
        dn.get()
        dn.add(dense)
        dn.clock()
    ck.save({0: sp, 1: dn}, iteration=6, blocking=True)
    snap = (sp.shard.clone(), sp.state.clone(), dn.master.clone(), dn.v.clone())
    comm.barrier()  # nobody pushes before every rank took its copy
    for c in range(6, 9):  # train on past the checkpoint
        keys, rows, dense = _push_of(rank, c)
        sp.add_keys(keys, rows)
        sp.clock()
        dn.add(dense)
        dn.clock()
    sp.drain()
    dn.drain()
    comm.barrier()
    it = ck.load({0: sp, 1: dn})
    same = [torch.equal(a, b) for a, b in zip(snap, (sp.shard, sp.state, dn.master, dn.v))]
    clocks = (sp.clock_n, dn.clock_n, sp.ps.board.min_applied(sp.t))
    comm.barrier()  # every rank compared before anyone pushes again
    # training continues after the restore
    keys, rows, dense = _push_of(rank, 50)
    sp.get(keys)
    sp.add_keys(keys, rows)
    sp.clock()
    sp.drain()
    comm.barrier()
    return it, same, clocks, sp.clock_n


def test_async_checkpoint_restore_cpu(tmp_path):
    prefix = str(tmp_path) + "/ck_"
    out = run_world(_ckpt_fn(prefix), world=2)
    for rank, (it, same, clocks, after) in out.items():
        assert it == 6 and all(same), (rank, same)
        assert clocks == (6, 6, 6) and after == 7, (rank, clocks, after)


class _ckpt_fn:
    def __init__(self, prefix):
        self.prefix = prefix

    def __call__(self, rank, world):
        return _ckpt_run(rank, world, self.prefix)
