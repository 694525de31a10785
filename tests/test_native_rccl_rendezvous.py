"""The native RCCL data plane's rendezvous (minips_amd/ps/comm.py _native_rccl) at world > 1 on
CPU ranks: the RCCL calls are replaced by a fake, the protocol over the real c10d store is the
production one -- rank 0 publishes ONE unique id, every rank builds its communicator from that
same id, the keys are gone afterwards (a re-formed group starts clean), a second Comm over the
group reuses the communicator, and refresh() drops it so the next collective makes a new one; a
communicator whose self-test fails on ONE rank is dropped on every rank (the group falls back to
c10d together). (The RCCL calls themselves run on the GPU box at world 1: tests/test_rccl_gpu.py.)"""
import torch

from test_ps_gloo import run_world


class _FakeRccl:
    def __init__(self, lib, uid, world, rank, device, timeout_s=60.0, teardown=False):
        self.uid, self.world, self.rank, self.aborted = uid, world, rank, False
        self.why = None

    def abort(self, why=""):
        self.aborted, self.why = True, why


class _FakeKernels:
    made = 0

    def rccl_unique_id(self, lib):
        import os

        return os.urandom(128)

    def Rccl(self, *a, **kw):
        _FakeKernels.made += 1
        return _FakeRccl(*a, **kw)


def _rendezvous(rank, world):
    import torch.distributed as dist

    from minips_amd import _native
    from minips_amd.ps import comm as cm

    fake = _FakeKernels()
    _native.kernels = lambda: fake  # the fake RCCL behind the production rendezvous
    cm._rccl_selftest = lambda rc, comm: True  # (the data-plane self-test needs a GPU)
    c = cm.Comm()
    c.backend, c.device = "nccl", torch.device("cuda", 0)  # (as on a GPU rank; nothing touches a GPU)
    rc = c._rc()
    c2 = cm.Comm()
    c2.backend, c2.device = "nccl", torch.device("cuda", 0)
    same = c2._rc() is rc  # one communicator per group, shared by every Comm
    uids = [None] * world
    dist.all_gather_object(uids, rc.uid)
    dist.barrier()
    store = dist.distributed_c10d._get_default_store()
    tag = "minips_rccl/" + ",".join(str(r) for r in range(world))
    left = store.check([tag + "/id"]) if rank == 0 else False
    c.refresh()  # a re-formed group: the old communicator is aborted and forgotten
    c.backend, c.device = "nccl", torch.device("cuda", 0)
    dist.barrier()
    rc2 = c._rc()
    dist.barrier()
    return dict(rank=rc.rank, world=rc.world, all_same=len(set(uids)) == 1, same=same, left=left,
                aborted=rc.aborted, why=rc.why, new=rc2 is not rc, new_uid_differs=rc2.uid != rc.uid)


def test_native_rccl_rendezvous_four_ranks():
    out = run_world(_rendezvous, world=4)
    for r, o in out.items():
        assert o["rank"] == r and o["world"] == 4
        assert o["all_same"], o     # every rank joined with rank 0's unique id
        assert o["same"], o         # a second Comm over the group reuses the communicator
        assert not o["left"], o     # the id / ack keys were deleted after the rendezvous
        assert o["aborted"] and "re-formed" in o["why"], o
        assert o["new"] and o["new_uid_differs"], o


def _selftest_fails_on_one_rank(rank, world):
    import warnings

    from minips_amd import _native
    from minips_amd.ps import comm as cm

    fake = _FakeKernels()
    _native.kernels = lambda: fake
    cm._rccl_selftest = lambda rc, comm: comm.rank != 2  # a broken data plane on rank 2 only
    c = cm.Comm()
    c.backend, c.device = "nccl", torch.device("cuda", 0)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        rc = c._rc()
    made = [v for v in cm._RCCL_CACHE.values()]
    c2 = cm.Comm()
    c2.backend, c2.device = "nccl", torch.device("cuda", 0)
    return dict(rc=rc, again=c2._rc(), made=fake.made, warned=any("disabled" in str(x.message) for x in w),
                cached=[m[1] for m in made])


def test_native_rccl_selftest_failure_disables_it_on_every_rank():
    out = run_world(_selftest_fails_on_one_rank, world=4)
    for r, o in out.items():
        assert o["rc"] is None and o["again"] is None, o  # every rank on c10d, not only rank 2
        assert o["made"] == 1, o                          # no second attempt by a later Comm
        assert o["warned"] == (r == 0), o
