"""Collective helpers of the GPU data plane (RCCL over xGMI; gloo on CPU for tests).

The PS message patterns map onto collectives:
  C1/C2 sparse Get      -> all-to-all(counts) + all-to-all-v(keys) + all-to-all-v(rows)
  C3    sparse Add      -> all-to-all-v(grad rows) into the owner shards
  C1/C3 dense Get/Add   -> reduce-scatter(grads) / all-gather(params) of equal shards
  C6    Barrier         -> 1-element all-reduce on the group
With one rank every collective degenerates to a local copy (no RCCL launch at all).

On RCCL the collectives run on the rank's native data plane (csrc/comm/rccl_comm.h, the Rccl
binding): our own communicator over the RCCL torch loaded, each collective ONE enqueue from C++
onto the issuing stream (the all-to-all-v as grouped ncclSend / ncclRecv), a watchdog that aborts
the communicator when a collective stops completing; c10d (ProcessGroupNCCL) stays for the
rendezvous, the unique-id exchange (store) and anything outside the step (MINIPS_NATIVE_RCCL=0:
every collective through c10d).

Ordering contract (why the data plane cannot deadlock, whatever the HW-queue count)
-----------------------------------------------------------------------------------
The reference keeps one FIFO sender per process (comm/sender.cpp:7-30 feeding
comm/mailbox.cpp:231-308), so a worker's messages leave in program order. The GPU data plane
keeps the same contract with ONE communicator per rank:

1. Every collective of a rank goes through this Comm's single process group, whichever HIP
   stream issues it (compute, planning, a table's clock stream), and runs on the GPU in issue
   order: ProcessGroupNCCL enqueues on its one internal stream; the native plane makes each
   collective's stream wait for the previous collective's completion event (RcclComm::Call) --
   RCCL alone lets a collective enqueued on another stream overtake an earlier one
   (tests/test_rccl_gpu.py::test_native_rccl_keeps_issue_order_across_streams failed without the
   chain: the later one finished at 0.28 ms, the earlier one behind a 2 ms kernel). So the n-th
   collective of every rank is the same op (same kind, dtype and row width; all-to-all-v splits
   agree pairwise), executed after collectives < n.
2. Every rank issues the same program: the tables' issue points (plan, get, clock, advance)
   are identical on all ranks and never depend on timing or on a non-blocking query.
3. A host wait (an event of the count exchange) and a stream wait (wait_event) only target
   work issued EARLIER in that rank's program.
By induction over the issue order, collective n completes on every rank once collectives
< n have: nothing it waits for was issued after it, on any rank. Streams multiplexed onto
fewer hardware queues (GPU_MAX_HW_QUEUES, 4 by default) only delay, never reorder, packets
issued earlier, so the argument survives queue sharing. ``trace`` records the issue order;
tests/test_comm_schedule.py checks that 4- and 8-rank runs issue identical sequences.
"""
from __future__ import annotations

import contextlib
import datetime
import os
import threading
import time
import warnings
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from ..utils.metrics import _HOST_ON, _ROCTX_ON, range as _mrange


# The native RCCL data plane (csrc/comm/rccl_comm.h, ops_py Rccl): every collective of the step
# enqueued from C++ straight onto the issuing stream -- no c10d work object, no stream-sync events,
# no per-call Python beyond one binding call (c10d: 13-31 us of host time per collective,
# profiles/r5/host_issue.txt). NATIVE_RCCL off: the c10d ProcessGroupNCCL calls.
_NATIVE_RCCL = os.environ.get("MINIPS_NATIVE_RCCL", "1") != "0"
# process group -> (group, native communicator): one communicator per group, shared by every Comm
_RCCL_CACHE: dict = {}


def _rccl_lib() -> str:
    """The RCCL shared object torch loaded (dlopen'ed again by the native side: one RCCL per process)."""
    return os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")


def _native_rccl(comm: "Comm"):
    """The native communicator of ``comm``'s group: rank 0 of the group creates the unique id, the
    others read it from the c10d store and acknowledge, rank 0 then deletes the keys (a re-formed
    group later finds none of them), and every rank joins ncclCommInitRank. Collective: called at
    the same point of every rank's program (the first collective of the group)."""
    from .._native import kernels

    pg = comm.group if comm.group is not None else dist.group.WORLD
    hit = _RCCL_CACHE.get(id(pg))
    if hit is not None and hit[0] is pg and (hit[1] is None or not hit[1].aborted):
        return hit[1]  # (None: the self-test failed on some rank -- the group runs on c10d)
    k = kernels()
    lib = _rccl_lib()
    store = dist.distributed_c10d._get_default_store()
    tag = "minips_rccl/" + ",".join(str(r) for r in dist.get_process_group_ranks(pg))
    mode = os.environ.get("TORCH_NCCL_ASYNC_ERROR_HANDLING", "")
    with comm.waiting():
        if comm.rank == 0:
            store.set(tag + "/id", k.rccl_unique_id(lib))
        uid = store.get(tag + "/id")
        if comm.rank != 0:
            store.add(tag + "/ack", 1)
        else:
            t0 = time.monotonic()
            while int(store.add(tag + "/ack", 0)) < comm.world - 1:
                if time.monotonic() - t0 > float(os.environ.get("MINIPS_PG_TIMEOUT", "60")):
                    raise dist.DistBackendError(f"native RCCL rendezvous {tag}: peers missing")
                time.sleep(0.001)
            store.delete_key(tag + "/id")
            store.delete_key(tag + "/ack")
        # the watchdog's timeout and failure mode follow the process group's: TORCH_NCCL_ASYNC_ERROR_
        # HANDLING 1 / 3 end the process on a stuck collective, 2 (in-place rollback) raises instead
        rc, ok = None, 1
        try:
            rc = k.Rccl(lib, uid, comm.world, comm.rank, comm.device.index or 0,
                        timeout_s=float(os.environ.get("MINIPS_PG_TIMEOUT", "60")), teardown=mode in ("1", "3"))
            ok = int(_rccl_selftest(rc, comm))
        except RuntimeError as e:
            ok, why = 0, str(e)
        else:
            why = "wrong self-test result"
        # every rank takes the same path: if the communicator failed anywhere, the whole group falls
        # back to ProcessGroupNCCL (a rank on its own communicator while a peer waits in c10d hangs)
        if comm.world > 1:
            fdev = comm.device if dist.get_backend(pg) == "nccl" else torch.device("cpu")
            flag = torch.tensor([ok], dtype=torch.int32, device=fdev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=pg)
            ok = int(flag.item())
        if not ok:
            if rc is not None:
                rc.abort("native RCCL self-test failed on a rank")
            rc = None
            if comm.rank == 0:
                warnings.warn(f"native RCCL data plane disabled for {tag} ({why}); collectives run on c10d")
    _RCCL_CACHE[id(pg)] = (pg, rc)
    return rc


def _rccl_selftest(rc, comm: "Comm") -> bool:
    """One all-to-all-v (rank r sends r * P + p to peer p, two values to the next rank) and one
    all-reduce on the new communicator, checked on the host: a broken data plane is caught before
    a table's first exchange, while the group can still fall back together."""
    P, r, dev = comm.world, comm.rank, comm.device
    send = [2 if p == (r + 1) % P else 1 for p in range(P)]
    recv = [2 if p == (r - 1) % P else 1 for p in range(P)]
    vals = []
    for p in range(P):
        vals += [r * P + p] * send[p]
    inp = torch.tensor(vals, dtype=torch.int64, device=dev)
    out = torch.full((sum(recv),), -1, dtype=torch.int64, device=dev)
    want = []
    for p in range(P):
        want += [p * P + r] * recv[p]
    ones = torch.ones(4, dtype=torch.float32, device=dev)
    rc.all_to_all_v(out, inp, recv, send)
    rc.all_reduce(ones, 0)
    torch.cuda.current_stream(dev).synchronize()
    return out.tolist() == want and ones.tolist() == [float(P)] * 4


def _rccl_call(fn, *args):
    """A native RCCL enqueue; its failures surface as the torch.distributed error class the
    training driver's recovery recognises (train._is_comm_failure)."""
    try:
        return fn(*args)
    except RuntimeError as e:
        if str(e).startswith("rccl"):
            raise dist.DistBackendError(str(e)) from e
        raise


_REDOPS = {dist.ReduceOp.SUM: 0, dist.ReduceOp.MAX: 1, dist.ReduceOp.MIN: 2}


# handles of dedicated streams whose owner is gone, by (device index, priority): reused, never
# destroyed -- the caching allocator may still record events on a stream a freed tensor was
# record_stream()-ed to, so destroying one can crash a later free
_FREE_STREAMS: dict[tuple[int, int], list[int]] = {}


class _OwnedStream(torch.cuda.ExternalStream):
    """An ExternalStream over a stream this process created; back to the free list with its last
    reference (only LIVE users must not alias)."""

    def __del__(self):
        try:
            _FREE_STREAMS.setdefault((self.device.index or 0, self._minips_prio), []).append(int(self.cuda_stream))
        except Exception:  # interpreter shutdown
            pass


def dedicated_stream(device, priority: int = 0):
    """A HIP stream no other live stream aliases. torch.cuda.Stream() draws from a 32-per-priority
    round-robin pool, so a long-lived process that builds many tables (Engine.create_table, the
    test suite) would otherwise get the SAME HIP stream for two "independent" lanes -- e.g. a
    table's clock pipeline and the planning stream -- and serialise one behind the other. Falls
    back to the pool when the native extension is not built."""
    device = torch.device(device)
    idx = device.index or 0
    free = _FREE_STREAMS.get((idx, int(priority)))
    if free:
        h = free.pop()
    else:
        try:
            from .._native import kernels

            h = kernels().new_stream(idx, int(priority))
        except Exception:
            return torch.cuda.Stream(device=device, priority=priority)
    s = _OwnedStream(h, device=device)
    s._minips_prio = int(priority)
    return s


@dataclass
class CommStats:
    bytes_a2a: int = 0
    bytes_rs: int = 0
    bytes_ag: int = 0
    calls: int = 0
    bucket_bytes: dict = field(default_factory=dict)  # "t<table>b<k>" -> RS + AG bytes (bucketed clocks)

    def as_dict(self):
        return dict(bytes_a2a=self.bytes_a2a, bytes_rs=self.bytes_rs, bytes_ag=self.bytes_ag, calls=self.calls,
                    bucket_bytes=dict(self.bucket_bytes))


class Comm:
    """Rank/world/device bookkeeping plus the collectives used by the tables (one ordered
    communicator per rank: see the module docstring)."""

    emulated = False  # LoopbackComm: one rank of an N-rank job emulated on one device

    def __init__(self, group=None, device: torch.device | None = None, force_collectives: bool = False):
        """``force_collectives``: run every collective through the process group even at world 1
        (tests: the RCCL calls of the multi-rank data plane, with the tables' dtypes and layouts,
        executed on a one-GPU box)."""
        self.force = force_collectives
        self.initialized = dist.is_available() and dist.is_initialized()
        self.group = group
        self.rank = dist.get_rank(group) if self.initialized else 0
        self.world = dist.get_world_size(group) if self.initialized else 1
        self.backend = dist.get_backend(group) if self.initialized else "none"
        if device is None:
            device = torch.device("cuda",
                                  torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        self.device = device
        self.stats = CommStats()
        self._plan_stream = None
        # issue-order record of the collectives [(op, dtype, shape-invariant size)], enabled by
        # MINIPS_COMM_TRACE=1 or by assigning a list (tests)
        self.trace: list | None = [] if os.environ.get("MINIPS_COMM_TRACE") == "1" else None
        self._waiting = 0
        self._wlock = threading.Lock()
        # per-collective timing (bench.py's N > 1 diagnostics): a list of (kind, bytes, start, end)
        # -- HIP events on the issuing stream (GPU) or host clocks (gloo) -- when assigned
        self.timing: list | None = None

    def refresh(self):
        """Re-read rank / world / backend after the default process group was re-created (in-place
        rollback, minips_amd.train): every table keeps this same Comm object."""
        self.drop_native("the process group was re-formed")
        self._sb = 0  # the new group's store starts its barrier counters afresh
        self.initialized = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank(self.group) if self.initialized else 0
        self.world = dist.get_world_size(self.group) if self.initialized else 1
        self.backend = dist.get_backend(self.group) if self.initialized else "none"

    @contextlib.contextmanager
    def waiting(self):
        """Marks a host wait on peers (a blocking collective, a collective's result): the
        heartbeat reports state "comm", so the supervisor can tell a rank that waits for a stuck
        peer from the stuck rank itself."""
        with self._wlock:
            self._waiting += 1
        try:
            yield
        finally:
            with self._wlock:
                self._waiting -= 1

    def state(self) -> str:
        return "comm" if self._waiting > 0 else "run"

    def _rc(self):
        """The native RCCL communicator of this Comm's group (created at the first collective, shared
        by every Comm over the group), or None: not RCCL, staged gloo tests, NATIVE_RCCL off."""
        rc = self.__dict__.get("_rcc", False)
        if rc is False:
            rc = None
            if self.backend == "nccl" and _NATIVE_RCCL and self.device.type == "cuda" and self.initialized:
                rc = _native_rccl(self)
            self._rcc = rc
        return rc

    def drop_native(self, why: str = "dropped"):
        """Abort and forget the native communicator (rollback / rescale: its peers may be gone, and
        a re-formed group needs a new one)."""
        rc = self.__dict__.pop("_rcc", None)
        if rc:
            rc.abort(why)
            for k, v in list(_RCCL_CACHE.items()):
                if v[1] is rc:
                    del _RCCL_CACHE[k]

    def _bare(self, fn, *args, **kw):
        """A collective enqueued bare (_plain): no generator context managers, but still counted as
        a possible host wait -- an enqueue can block (the first collective of a communicator sets
        it up; a full proxy queue), and a rank blocked there on a stuck peer must report "comm"."""
        wl = self._wlock
        with wl:
            self._waiting += 1
        try:
            return fn(*args, **kw)
        finally:
            with wl:
                self._waiting -= 1

    def _plain(self) -> bool:
        """A collective can be enqueued bare: RCCL calls return at once (no host wait for the
        heartbeat's "comm" state to cover) and no timing / tracing wraps it -- the two generator
        context managers cost ~3-4 us per collective on the step's host path."""
        return self.backend == "nccl" and self.timing is None and not (_ROCTX_ON or _HOST_ON)

    @contextlib.contextmanager
    def _timed(self, kind: str, nbytes: int):
        """Around one collective when ``timing`` is on: its bytes and its time on the issuing
        stream (an RCCL call leaves the current stream waiting for it, so the end event fires
        when the collective completed)."""
        if _ROCTX_ON or _HOST_ON:
            with _mrange("comm." + kind):
                yield from self._timed_inner(kind, nbytes)
            return
        yield from self._timed_inner(kind, nbytes)

    def _timed_inner(self, kind: str, nbytes: int):
        if self.timing is None:
            yield
            return
        if self.device.type == "cuda":
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            yield
            b.record()
        else:
            a = time.perf_counter()
            yield
            b = time.perf_counter()
        self.timing.append((kind, int(nbytes), a, b))

    def timing_report(self, steps: int) -> dict:
        """Per collective kind: calls, bytes and ms per step, achieved GB/s (bytes / time spent in
        the collective) of the recorded window; clears the record."""
        rec, self.timing = self.timing or [], []
        if rec and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        out: dict = {}
        for kind, nb, a, b in rec:
            ms = a.elapsed_time(b) if self.device.type == "cuda" else (b - a) * 1e3
            e = out.setdefault(kind, {"calls": 0, "bytes": 0, "ms": 0.0})
            e["calls"] += 1
            e["bytes"] += nb
            e["ms"] += ms
        n = max(1, int(steps))
        return {k: dict(calls_per_step=round(e["calls"] / n, 3), mb_per_step=round(e["bytes"] / n / 2**20, 4),
                        ms_per_step=round(e["ms"] / n, 4),
                        gbps=round(e["bytes"] / (e["ms"] * 1e-3) / 1e9, 3) if e["ms"] > 0 else None)
                for k, e in sorted(out.items())}

    def _record(self, op: str, t: torch.Tensor | None = None, size=None):
        if self.trace is not None:
            self.trace.append((op, str(t.dtype).replace("torch.", "") if t is not None else "", size))

    def new_stream(self, priority: int = 0):
        """A HIP stream of this rank's device that no other stream aliases (see dedicated_stream)."""
        return dedicated_stream(self.device, priority)

    def plan_stream(self):
        """The HIP stream on which lookahead key planning runs (one per rank, shared by tables).
        (A CU-masked planning stream, which kept the latency-bound dedupe kernels off most CUs,
        measured no better in round 2 and is gone.) One rank: a low-priority HIP stream (priority 1,
        below the default 0 of the compute streams), so the dispatcher favours the step's own
        workgroups over the look-ahead planning's: W&D 0.358-0.359 vs 0.363-0.365 ms/step. Several
        ranks keep priority 0: the planning stream also carries the plan's count and key exchanges,
        which the next step's host waits on (8 emulated ranks 0.477-0.482 vs 0.440-0.444 at low
        priority; profiles/r5/ab_plan_priority.txt)."""
        if self._plan_stream is None and self.device.type == "cuda":
            self._plan_stream = dedicated_stream(self.device, 1 if self.world == 1 else 0)
        return self._plan_stream

    # -- helpers ------------------------------------------------------------------------
    def _staged(self, *ts) -> bool:
        """GPU tensors over a gloo group: the multi-rank GPU TEST harness (several ranks sharing
        one card, where RCCL refuses duplicate devices) stages them through host memory, so the
        streams / lanes / lookahead logic runs on the GPU at world > 1. Never a production path:
        init_distributed() picks RCCL whenever GPUs are present."""
        return self.backend == "gloo" and any(t.is_cuda for t in ts)

    @staticmethod
    def _host(t: torch.Tensor) -> torch.Tensor:
        # gloo moves raw 16-bit payloads as fp16 bit patterns (it has no bf16 / int16 path)
        t = t.detach().cpu()
        return t.view(torch.float16) if t.dtype == torch.bfloat16 else t

    @staticmethod
    def _back(dst: torch.Tensor, host: torch.Tensor):
        dst.copy_(host.view(dst.dtype) if dst.dtype == torch.bfloat16 else host)

    def all_to_all_v(self, out: torch.Tensor, inp: torch.Tensor, recv_splits: list[int], send_splits: list[int],
                     p2p: bool = False):
        """Rows of ``inp`` split by ``send_splits`` go to ranks 0..P-1; ``out`` gets recv_splits.

        p2p=True issues the exchange as grouped point-to-point send/recv pairs (one per peer
        with a non-empty message, the own segment copied locally) -- the SSP/ASP data path;
        otherwise one RCCL all-to-all-v."""
        if self.world > 1 and self._staged(out, inp):
            o = self._host(out[: sum(recv_splits)])
            self.all_to_all_v(o, self._host(inp[: sum(send_splits)]), recv_splits, send_splits, p2p)
            self._back(out[: sum(recv_splits)], o)
            return out
        self.stats.calls += 1
        if self.world > 1:
            self._record("a2av_p2p" if p2p else "a2av", inp, tuple(inp.shape[1:]))
        if self.world == 1 and not self.force:
            n = send_splits[0]
            if n:
                out[:n].copy_(inp[:n])
            return out
        nbytes = inp[: sum(send_splits)].numel() * inp.element_size()
        self.stats.bytes_a2a += nbytes
        rc = self._rc()
        if rc is not None:  # one grouped send / recv launch from C++ (both the a2a-v and the p2p form)
            o = out[: sum(recv_splits)]
            i = inp[: sum(send_splits)]
            if self._plain():
                self._bare(_rccl_call, rc.all_to_all_v, o, i, recv_splits, send_splits)
                return out
            with self.waiting(), self._timed("p2p_send_recv" if p2p else "all_to_all_v", nbytes):
                _rccl_call(rc.all_to_all_v, o, i, recv_splits, send_splits)
            return out
        if not p2p:
            o = out[: sum(recv_splits)]
            i = inp[: sum(send_splits)]
            if self._plain():
                self._bare(dist.all_to_all_single, o, i, recv_splits, send_splits, group=self.group)
                return out
            with self.waiting(), self._timed("all_to_all_v", nbytes):
                dist.all_to_all_single(o, i, recv_splits, send_splits, group=self.group)
            return out
        so = [0]
        for c in send_splits:
            so.append(so[-1] + c)
        ro = [0]
        for c in recv_splits:
            ro.append(ro[-1] + c)
        ops_ = []
        for peer in range(self.world):
            if peer == self.rank:
                if send_splits[peer]:
                    out[ro[peer]: ro[peer + 1]].copy_(inp[so[peer]: so[peer + 1]])
                continue
            if send_splits[peer]:
                ops_.append(dist.P2POp(dist.isend, inp[so[peer]: so[peer + 1]].contiguous(), peer, group=self.group))
            if recv_splits[peer]:
                ops_.append(dist.P2POp(dist.irecv, out[ro[peer]: ro[peer + 1]], peer, group=self.group))
        if ops_:
            with self.waiting(), self._timed("p2p_send_recv", nbytes):
                for r in dist.batch_isend_irecv(ops_):
                    r.wait()
        return out

    def all_to_all_counts(self, recv: torch.Tensor, counts: torch.Tensor):
        """Device-side all-to-all of per-destination counts (no host sync)."""
        if self.world == 1 and not self.force:
            recv.copy_(counts)
            return recv
        self._record("a2a_counts", counts, counts.numel())
        rc = None if self._staged(recv, counts) else self._rc()
        if rc is not None:
            self._bare(_rccl_call, rc.all_to_all, recv, counts)
        elif self._staged(recv, counts):
            r = torch.empty(recv.shape, dtype=recv.dtype)
            with self.waiting():
                dist.all_to_all_single(r, counts.cpu(), group=self.group)
            recv.copy_(r)
        elif self._plain():
            self._bare(dist.all_to_all_single, recv, counts, group=self.group)
        else:
            with self.waiting():
                dist.all_to_all_single(recv, counts, group=self.group)
        return recv

    def exchange_counts(self, counts: torch.Tensor) -> tuple[list[int], list[int]]:
        """all-to-all of per-destination counts; returns (send, recv) as host lists (1 sync)."""
        if self.world == 1 and not self.force:
            c = counts.tolist()
            return c, c
        recv = torch.empty_like(counts)
        self.all_to_all_counts(recv, counts)
        both = torch.stack([counts, recv]).cpu()
        return both[0].tolist(), both[1].tolist()

    def reduce_scatter(self, out_shard: torch.Tensor, inp: torch.Tensor):
        if self.world > 1 and self._staged(out_shard, inp):
            o = torch.empty(out_shard.shape, dtype=out_shard.dtype)
            self.reduce_scatter(o, inp.cpu())
            out_shard.copy_(o)
            return out_shard
        self.stats.calls += 1
        if self.world > 1:
            self._record("reduce_scatter", inp, inp.numel())
        if self.world == 1 and not self.force:
            out_shard.copy_(inp)
            return out_shard
        self.stats.bytes_rs += inp.numel() * inp.element_size()
        rc = self._rc()
        if self._plain():
            if rc is not None:
                self._bare(_rccl_call, rc.reduce_scatter, out_shard, inp)
            else:
                self._bare(dist.reduce_scatter_tensor, out_shard, inp, group=self.group)
            return out_shard
        with self.waiting(), self._timed("reduce_scatter", inp.numel() * inp.element_size()):
            if rc is not None:
                _rccl_call(rc.reduce_scatter, out_shard, inp)
            else:
                dist.reduce_scatter_tensor(out_shard, inp, group=self.group)
        return out_shard

    def all_gather(self, out_full: torch.Tensor, shard: torch.Tensor):
        if self.world > 1 and self._staged(out_full, shard):
            o = self._host(out_full)
            self.all_gather(o, self._host(shard).clone())
            self._back(out_full, o)
            return out_full
        self.stats.calls += 1
        if self.world > 1:
            self._record("all_gather", out_full, out_full.numel())
        if self.world == 1 and not self.force:
            if out_full.data_ptr() != shard.data_ptr():
                out_full.copy_(shard)
            return out_full
        self.stats.bytes_ag += out_full.numel() * out_full.element_size()
        if self.backend == "gloo" and shard.data_ptr() >= out_full.data_ptr() and \
                shard.data_ptr() < out_full.data_ptr() + out_full.numel() * out_full.element_size():
            shard = shard.clone()  # gloo does not support the in-place (aliased) form
        rc = self._rc()
        if self._plain():
            if rc is not None:
                self._bare(_rccl_call, rc.all_gather, out_full, shard)
            else:
                self._bare(dist.all_gather_into_tensor, out_full, shard, group=self.group)
            return out_full
        with self.waiting(), self._timed("all_gather", out_full.numel() * out_full.element_size()):
            if rc is not None:
                _rccl_call(rc.all_gather, out_full, shard)
            else:
                dist.all_gather_into_tensor(out_full, shard, group=self.group)
        return out_full

    def all_reduce_(self, t: torch.Tensor, op=None):
        if self.world == 1 and not self.force:
            return t
        self._record("all_reduce", t, t.numel())
        if self._staged(t):
            h = t.cpu()
            with self.waiting():
                dist.all_reduce(h, op=op or dist.ReduceOp.SUM, group=self.group)
            t.copy_(h)
            return t
        rc = self._rc()
        with self.waiting(), self._timed("all_reduce", t.numel() * t.element_size()):
            if rc is not None and (op or dist.ReduceOp.SUM) in _REDOPS:
                _rccl_call(rc.all_reduce, t, _REDOPS[op or dist.ReduceOp.SUM])
            else:
                dist.all_reduce(t, op=op or dist.ReduceOp.SUM, group=self.group)
        return t

    def store_barrier(self, tag: str, timeout_s: float | None = None):
        """Host barrier through the c10d store with its own long timeout (MINIPS_LONG_PHASE_TIMEOUT,
        default 3600 s), for the end of a phase whose length differs by rank -- a checkpoint restore
        (owner-range reads of up to ~85 GB per rank), a foreground checkpoint write. Without it the
        next collective would start its PG timeout (MINIPS_PG_TIMEOUT, 60 s) on the fast ranks and
        abort a healthy job; after it every rank is present and the collective completes at once.
        The heartbeat reports "comm" meanwhile (a rank waiting for slow peers is not stuck)."""
        if self.world == 1 and not self.force:
            return
        if not self.initialized:
            return
        store = dist.distributed_c10d._get_default_store()
        self._sb = getattr(self, "_sb", 0) + 1
        members = dist.get_process_group_ranks(self.group) if self.group is not None else range(self.world)
        key = f"minips_sb/{tag}/{self._sb}/" + ",".join(str(r) for r in members)
        store.add(key, 1)
        limit = timeout_s if timeout_s is not None else float(os.environ.get("MINIPS_LONG_PHASE_TIMEOUT", "3600"))
        t0 = time.monotonic()
        with self.waiting():
            while int(store.add(key, 0)) < self.world:
                if time.monotonic() - t0 > limit:
                    raise TimeoutError(f"store barrier {tag!r}: {int(store.add(key, 0))}/{self.world} ranks "
                                       f"after {limit:.0f} s")
                time.sleep(0.005)

    def barrier(self):
        if self.world == 1 and not self.force:
            return
        t = torch.zeros(1, device=self.device)
        self.all_reduce_(t)
        if t.is_cuda:
            with self.waiting():
                torch.cuda.synchronize(self.device)


class LoopbackComm(Comm):
    """Rank ``rank`` of a ``world``-rank job, emulated in ONE process on one device: every table is
    built and routed as that rank of the N-rank job (shard sizes, key ranges, buckets, ring
    buffers, lookahead depth) and takes every ``world > 1`` code path, but each collective is a
    loopback that moves the same bytes through this device's HBM instead of the fabric:

      all-to-all(counts)   recv = counts (every peer asks this owner for what it asks each peer)
      all-to-all-v         out = inp (requires recv_splits == send_splits, which the symmetric
                           counts give); the KEY exchange's segments are re-based into this
                           rank's own row range by the caller (SparseTable, ``emulated``), so the
                           owner-side dedupe and applies run on in-range rows of realistic count
      reduce-scatter       out = sum of the N equal slices of inp (reads N x shard, like the real
                           reduction of the peers' contributions)
      all-gather           every slot of out = this rank's shard (writes N x shard)
      barrier / all-reduce no-ops

    Wire time is excluded by default: ``bench.py --emulate-world N`` times the per-rank GPU and host
    program of an N-rank step on one GPU, so the step's kernels, host syncs and launch count can be
    profiled (rocprofv3) before an N-GPU node is available.

    ``wire`` (bench.py --emu-wire, MINIPS_EMU_WIRE) adds a modelled link time to each collective: a
    device spin on the collective's stream, on ``channels`` workgroups (the CUs an RCCL collective's
    channels hold), of latency + bytes / bandwidth per SURVEY §5.8 for 7 point-to-point xGMI links
    of ``link_gbps`` each:
      all-to-all(-v)          every peer segment on its own link: S_sent / ((P - 1) * link)
      RS / AG "ring"          one link per hop: (P - 1) / P * S / link
      RS / AG "direct"        all 7 links at once: (P - 1) / P * S / ((P - 1) * link)
    (S: the bytes this rank's collective moves; a fixed per-collective latency on top)."""

    emulated = True

    def __init__(self, world: int, rank: int = 0, device: torch.device | None = None, wire: str | None = None,
                 link_gbps: float | None = None, latency_us: float | None = None, channels: int | None = None):
        if world < 2 or not 0 <= rank < world:
            raise ValueError(f"LoopbackComm: rank {rank} of world {world}")
        super().__init__(device=device)
        self.world, self.rank = int(world), int(rank)
        self.backend = "loopback"
        self.initialized = False
        self.wire = (wire if wire is not None else os.environ.get("MINIPS_EMU_WIRE", "none")) or "none"
        if self.wire not in ("none", "ring", "direct"):
            raise ValueError(f"LoopbackComm wire model {self.wire!r}: none | ring | direct")
        self.link_gbps = float(link_gbps if link_gbps is not None else os.environ.get("MINIPS_EMU_LINK_GBPS", "153"))
        self.latency_us = float(latency_us if latency_us is not None else os.environ.get("MINIPS_EMU_LAT_US", "8"))
        self.channels = int(channels if channels is not None else os.environ.get("MINIPS_EMU_CHANNELS", "16"))
        self.wire_us = 0.0  # modelled link time issued so far (bench.py diag)

    def wire_time_us(self, kind: str, nbytes: int) -> float:
        """Modelled link time (us) of one collective moving ``nbytes`` on this rank: "a2a" (every peer
        segment on its own link) or "rs" / "ag" (ring: one link per hop; direct: all P - 1 links)."""
        if self.wire == "none":
            return 0.0
        P, bw = self.world, self.link_gbps * 1e3  # bytes per us
        if kind == "a2a" or self.wire == "direct":
            us = nbytes * (P - 1) / P / ((P - 1) * bw)
        else:
            us = (P - 1) / P * nbytes / bw
        return us + self.latency_us

    def _wire(self, kind: str, nbytes: int):
        """The modelled link time of one collective, spun on the current stream (GPU only)."""
        if self.wire == "none" or self.device.type != "cuda":
            return
        us = self.wire_time_us(kind, nbytes)
        self.wire_us += us
        from .._native import kernels

        kernels().wire_spin(max(1, min(1_000_000, int(us * 100))), self.channels, 0)

    def refresh(self):
        self._sb = 0

    def _rc(self):
        return None

    def _plain(self) -> bool:  # (the loopback copies stand in for RCCL's bare enqueue)
        return self.timing is None and not (_ROCTX_ON or _HOST_ON)

    def all_to_all_v(self, out, inp, recv_splits, send_splits, p2p: bool = False):
        if list(recv_splits) != list(send_splits):
            raise ValueError("LoopbackComm: an emulated exchange needs symmetric splits")
        self.stats.calls += 1
        self._record("a2av_p2p" if p2p else "a2av", inp, tuple(inp.shape[1:]))
        n = int(sum(send_splits))
        nbytes = n * inp[:1].numel() * inp.element_size()
        self.stats.bytes_a2a += nbytes
        self._wire("a2a", nbytes)
        if self._plain():
            if n and out.data_ptr() != inp.data_ptr():
                out[:n].copy_(inp[:n])
            return out
        with self._timed("p2p_send_recv" if p2p else "all_to_all_v", nbytes):
            if n and out.data_ptr() != inp.data_ptr():
                out[:n].copy_(inp[:n])
        return out

    def all_to_all_counts(self, recv, counts):
        self._record("a2a_counts", counts, counts.numel())
        self._wire("a2a", counts.numel() * counts.element_size())
        recv.copy_(counts)
        return recv

    def exchange_counts(self, counts):
        c = counts.tolist()
        return c, c

    def reduce_scatter(self, out_shard, inp):
        self.stats.calls += 1
        self._record("reduce_scatter", inp, inp.numel())
        self.stats.bytes_rs += inp.numel() * inp.element_size()
        self._wire("rs", inp.numel() * inp.element_size())
        with contextlib.nullcontext() if self._plain() else self._timed(
                "reduce_scatter", inp.numel() * inp.element_size()):
            if inp.is_cuda and inp.dtype == torch.float32 and out_shard.numel() % 4 == 0:
                from .._native import kernels

                kernels().emu_sum_slices(inp, out_shard, self.world)  # (slice order, one kernel)
            else:
                torch.sum(inp.view(self.world, -1), 0, out=out_shard.view(-1))
        return out_shard

    def all_gather(self, out_full, shard):
        self.stats.calls += 1
        self._record("all_gather", out_full, out_full.numel())
        self.stats.bytes_ag += out_full.numel() * out_full.element_size()
        self._wire("ag", out_full.numel() * out_full.element_size())
        with contextlib.nullcontext() if self._plain() else self._timed(
                "all_gather", out_full.numel() * out_full.element_size()):
            lo, hi = out_full.data_ptr(), out_full.data_ptr() + out_full.numel() * out_full.element_size()
            slots = list(out_full.view(self.world, -1))
            if lo <= shard.data_ptr() < hi:  # the in-place form: this rank's slot of out_full is the shard
                slots = [t for t in slots if t.data_ptr() != shard.data_ptr()]
            if out_full.is_cuda and len(slots) <= 16:
                from .._native import kernels

                kernels().multi_copy(slots, [shard.reshape(-1)] * len(slots))  # (one kernel)
            else:
                for t in slots:
                    t.copy_(shard.reshape(-1))
        return out_full

    def all_reduce_(self, t, op=None):
        self._record("all_reduce", t, t.numel())
        return t

    def store_barrier(self, tag: str, timeout_s: float | None = None):
        return

    def barrier(self):
        if self.trace is not None:  # (the real barrier is a 1-element fp32 all-reduce)
            self._record("all_reduce", torch.zeros(1), 1)


def init_distributed(backend: str | None = None) -> Comm:
    """Initialise torch.distributed from the torchrun env (RANK/WORLD_SIZE/MASTER_*).

    One process per GPU: the local rank selects the device; backend "nccl" is RCCL on ROCm.
    A collective that does not complete within MINIPS_PG_TIMEOUT seconds (default 60) aborts
    the communicator and ends the process with an error (RCCL async error handling), so a
    stuck peer turns into a non-zero exit the elastic supervisor restarts from, not a hang.
    """
    timeout = datetime.timedelta(seconds=float(os.environ.get("MINIPS_PG_TIMEOUT", "60")))
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            # MINIPS_DIST_BACKEND=gloo (+ MINIPS_SHARE_DEVICE=1): the multi-rank test harness on one
            # card (RCCL refuses two ranks on one device); production picks RCCL whenever GPUs exist
            backend = os.environ.get("MINIPS_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        local = int(os.environ.get("LOCAL_RANK", "0"))
        # test harness only: several ranks on one card (MINIPS_SHARE_DEVICE=1 -> all on device 0)
        if os.environ.get("MINIPS_SHARE_DEVICE") == "1":
            local = 0
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local), timeout=timeout)
        else:
            dist.init_process_group(backend, timeout=timeout)
            if torch.cuda.is_available():
                torch.cuda.set_device(local)
    elif torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    return Comm()
