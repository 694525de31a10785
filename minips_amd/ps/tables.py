"""GPU parameter-server tables: the KV Get/Add/Clock API over RCCL collectives.

Each rank (one process per MI355X) is both a worker and the server of one equal key range
of every table; shards live in that GPU's HBM.

DenseTable  (flat fp32 master, equal shards)     reference: VectorStorage + BSPModel
  get()    -> full parameter vector in the pull dtype (bf16 by default)
  add(g)   -> gradients accumulate into the local fp32 buffer (BSP: invisible until Clock)
  clock()  -> reduce-scatter(grad) -> fused optimizer on the owned shard -> all-gather
              (the all-gather IS the next pull, so Gets after a Clock see the new values;
              Gets before it see the start-of-superstep values: bsp_model.cpp:14-56)

SparseTable (row table, equal key ranges)        reference: MapStorage/VectorStorage rows
  get(keys)        -> hash dedupe + owner bucketing (HIP), all-to-all of counts and keys,
                      owner row gather (HIP), all-to-all of rows back
  add(plan, grads) -> buffered per-unique-key gradient rows
  clock()          -> all-to-all of gradient rows to the owners, owner-side dedupe +
                      segment sum (HIP) and row-wise Adagrad / SGD apply (HIP)

Consistency: "bsp" applies at every Clock. "ssp" with staleness s (and "asp") issues the
Clock's communication + apply on a dedicated HIP stream and only makes a later Get wait for
the update of clock c-s-1 (bounded-staleness pipelining: the next steps' compute overlaps
the collectives), which is exactly the SSP read guarantee (ssp_model.cpp:58-85).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch

from .. import ops
from .comm import Comm
from ..utils import streams
from ..utils.metrics import phase, traced


def even_bounds(num_rows: int, parts: int) -> list[int]:
    """Same split as the reference getRanges(): floor-sized ranges, the last takes the rest."""
    step = num_rows // parts
    b = [step * i for i in range(parts)] + [num_rows]
    return b


# multi-rank BSP clocks on the tables' side streams (OVERLAP False: inline on the compute stream --
# the overlap-vs-sync numerics test flips it before building its tables)
OVERLAP = True


def _overlap_default() -> bool:
    return OVERLAP


class _Pipeline:
    """Tracks in-flight Clock work issued on a side HIP stream.

    On the GPU every consistency model runs the Clock's communication + apply on the table's
    own stream (its collectives join the rank's single ordered communicator, ps/comm.py) and
    gates READS instead of the issue: a Get at clock c waits only for the update of clock
    c - s - 1. BSP is s = 0 (the Get waits for the previous Clock -- the reference rule that
    Gets after a Clock see the new values), but the Clock itself now overlaps with whatever the
    worker does before its next Get (the rest of the backward pass, the next batch's key
    planning and dense assembly). SSP(s) relaxes the gate to s clocks, ASP to a fixed
    pipelining depth. On CPU (gloo tests) the work runs inline.
    """

    def __init__(self, comm: Comm, consistency: str, staleness: int, overlap: bool | None = None,
                 kind: str = "", w1: bool = False):
        self.consistency = consistency
        # ASP on the collective path is pipelining, not a staleness model: its clocks are
        # collectives every rank joins, so the Get gate only bounds how many clocks may be in
        # flight (MINIPS_ASP_DEPTH, default 2). The unbounded ASP of the reference
        # (asp_model.cpp:23-26) is the one-sided transport (ps/onesided.py, asp_bound=None).
        asp_depth = int(os.environ.get("MINIPS_ASP_DEPTH", "2"))
        self.staleness = staleness if consistency == "ssp" else (0 if consistency == "bsp" else asp_depth)
        overlap = _overlap_default() if overlap is None else overlap
        if consistency == "bsp":
            # one rank has no communication to hide; ``w1`` (or a communicator that forces every
            # collective through its group at world 1, as an N-rank job would) still runs the
            # clock on a side stream there (the apply overlapping other compute)
            self.async_ = comm.device.type == "cuda" and overlap and (comm.world > 1 or w1
                                                                       or getattr(comm, "force", False))
        else:
            self.async_ = comm.device.type == "cuda" and self.staleness > 0
        self.stream = comm.new_stream() if self.async_ else None
        self.events: dict = {}
        self.clock = 0
        # fence-free ordering events from rings (no event object per clock, no system-scope
        # release: every consumer is on this device)
        if self.async_:
            self._evs = streams.EventRing(self.staleness + 8, fast=streams.fast_for("pipe"))
            self._forks = streams.EventRing(4, fast=streams.fast_for("pipe"))
        # ``retain`` (set by tables driven by a fencing LookaheadFeeder): the tensors a clock reads
        # on the side stream are kept referenced until the compute stream has waited for that
        # clock, plus one step (the feeder's fence then also orders the planning stream after
        # it), instead of record_stream -- which costs an allocator event per tensor per clock
        self.retain = False
        self._held: dict = {}
        self._grace: list = []

    def run(self, fn):
        """Run ``fn`` (the clock's communication+apply) for the current clock."""
        if not self.async_:
            fn()
        else:
            cur = streams.current(self.stream.device)
            fork = self._forks.next()
            fork.record(cur)
            self.stream.wait_event(fork)  # inputs produced on the compute stream
            with streams.use(self.stream):
                fn()
                ev = self._evs.next()
                ev.record(self.stream)
            self.events[self.clock] = ev
        self.clock += 1

    def wait_clock(self, c: int):
        """Make the compute stream wait until the Clock number ``c`` has been applied."""
        if not self.async_ or c < 0:
            return
        cur = streams.current(self.stream.device)
        done = [k for k in self.events if k <= c]
        if done:
            cur.wait_event(self.events[max(done)])  # the side stream is in-order
            for k in done:
                del self.events[k]
        if self._held or self._grace:
            self._grace = [v for k, v in self._held.items() if k <= c]  # (the previous grace list dies)
            for k in [k for k in self._held if k <= c]:
                del self._held[k]

    def wait_for_read(self):
        """Before a Get at clock c: updates of clocks <= c - s - 1 must be applied."""
        self.wait_clock(self.clock - self.staleness - 1)
        if self.async_ and self.events and self.consistency != "bsp":
            # observed staleness of this read: earlier clocks whose update is still in flight
            # (non-blocking event queries; the metrics JSONL reports the histogram per step)
            from ..utils.metrics import get_logger

            log = get_logger()
            log.observe_pending(len(self.events))
            log.observe_staleness(sum(1 for ev in self.events.values() if not ev.query()))

    def keep_alive(self, *tensors):
        """Tensors produced on the compute stream and consumed on the side stream (by the clock
        about to run)."""
        if self.async_:
            if self.retain:
                self._held.setdefault(self.clock, []).extend(tensors)
                return
            for t in tensors:
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(self.stream)

    def drain(self):
        if self.async_:
            cur = streams.current(self.stream.device)
            cur.wait_stream(self.stream)
            self.events.clear()
            self._grace = [v for v in self._held.values()]
            self._held.clear()

    def reset(self):
        """In-place rollback: forget in-flight clocks (issued on the broken communicator)."""
        self.events.clear()
        self._held.clear()
        self._grace = []


def merge_buckets(starts, n_params: int, min_elems: float) -> list:
    """Layer start offsets -> bucket start offsets: walking down from the last layer, a bucket is
    closed at a layer start once it holds >= ``min_elems`` elements (the first bucket takes what is
    left); offset 0 always starts one."""
    cuts, top = [], n_params
    for s in sorted({int(x) for x in starts} - {0}, reverse=True):
        if top - s >= min_elems:
            cuts.append(s)
            top = s
    return [0] + sorted(cuts)


# WGRAD_DEFER off: split-K weight gradients of one rank reduce into the gradient buffer (a
# reduce kernel per GEMM) instead of being folded by the Adam kernel
_WGRAD_DEFER = True


class _SlabSink:
    """Split-K weight-gradient slabs pending for a DenseTable's next Adam (DenseTable.slab_sink):
    persistent fp32 planes per gradient region (re-used every step: the next step's GEMM is issued
    after this step's Adam on the stream order of the step; with a ring of gradient buffers each
    buffer has its own planes, reused under the ring's own clock wait), folded by the Adam kernel
    that applies the region -- the whole-gradient Adam, or the Adam of the bucket holding it (at
    most 4 regions per Adam launch)."""

    def __init__(self, table):
        self.t = table
        self._bufs = {}
        self._pending = []  # (byte address of the region, slab, nsplit, elements)

    def _range_of(self, dw):
        """Byte range [a, b) of the Adam launch that will apply ``dw``: its bucket or the gradient."""
        g = self.t.grad
        if getattr(self.t, "buckets", None) is None:
            return g.data_ptr(), g.data_ptr() + g.numel() * g.element_size()
        off = (dw.data_ptr() - g.data_ptr()) // g.element_size()
        lo, hi = self.t.buckets[self.t.bucket_of(off)]
        if off + dw.numel() > hi:
            return None  # the region spans two buckets
        return g.data_ptr() + lo * g.element_size(), g.data_ptr() + hi * g.element_size()

    def accepts(self, dw) -> bool:
        g = self.t.grad
        if not (dw.device == g.device and dw.dtype == g.dtype
                and g.data_ptr() <= dw.data_ptr() < g.data_ptr() + g.numel() * g.element_size()
                and (dw.data_ptr() - g.data_ptr()) % 16 == 0):
            return False
        r = self._range_of(dw)
        return r is not None and sum(1 for a, _, _, _ in self._pending if r[0] <= a < r[1]) < 4

    def slab(self, dw, split_k: int):
        key = (dw.data_ptr(), dw.numel())
        buf = self._bufs.get(key)
        need = int(split_k) * dw.numel()
        if buf is None or buf.numel() < need:
            buf = self._bufs[key] = torch.empty(need, dtype=torch.float32, device=dw.device)
        return buf

    def add(self, dw, slab, nsplit: int):
        self._pending.append((dw.data_ptr(), slab, int(nsplit), dw.numel()))

    def take(self, g):
        """The pending slabs inside gradient range ``g`` (removed), offsets relative to ``g``."""
        gp, ge = g.data_ptr(), g.data_ptr() + g.numel() * g.element_size()
        out, keep = [], []
        for e in self._pending:
            a, slab, nsplit, numel = e
            if gp <= a and a + 4 * numel <= ge:
                out.append((slab, nsplit, numel, (a - gp) // 4))
            else:
                keep.append(e)
        self._pending = keep
        return out


class DenseTable:
    def __init__(self, comm: Comm, n_params: int, optimizer: str = "adam", lr: float = 1e-3,
                 pull_dtype=torch.bfloat16, consistency: str = "bsp", staleness: int = 0, table_id: int = 0,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, p2p: bool = False,
                 value_dtype=torch.float32, buckets=None, overlap_w1: bool = False, bucket_mb: float | None = None):
        """``value_dtype`` float64 gives the reference's ``double`` tables (KVClientTable<double>
        with VectorStorage::SubAdd, server/vector_storage.hpp:28-38): optimizer "add" only, pulled
        in fp64, so BSP sums are exact for exactly representable deltas.

        ``buckets`` (multi-rank): element offsets where the model's layers start. The clock then
        runs per bucket -- reduce-scatter of the bucket's gradient, the optimizer on the owned
        slice, all-gather of the bucket's parameters -- and a bucket is issued as soon as the
        model calls ``bucket_ready(k)`` during its backward, so the communication of the late
        layers overlaps the backward of the early ones (SURVEY §5.8 bucket sizing: per-layer
        buckets of 8-64 MB). Ownership is then bucket-major: rank r owns the r-th slice of every
        bucket (the shard buffers are those slices in bucket order); checkpoints keep the
        canonical contiguous layout (shard_state / finish_restore convert).

        ``bucket_mb`` (with ``buckets``): merge consecutive layers into buckets of at least this many
        MB of fp32 gradient, walking from the last layer (the first whose backward completes) -- few,
        large collectives for the per-link bandwidth of the xGMI mesh instead of one per small
        layer.

        ``overlap_w1``: at world 1 too, run the clock on the table's side stream and, with
        ``buckets``, apply each bucket as soon as the backward finished its layer (one rank has
        no communication to hide, but the per-bucket optimizer then overlaps the remaining
        backward instead of running after it)."""
        if value_dtype not in (torch.float32, torch.float64):
            raise ValueError(f"value_dtype {value_dtype}")
        if value_dtype == torch.float64:
            if optimizer != "add":
                raise ValueError("fp64 dense tables support the reference's plain add apply only")
            pull_dtype = torch.float64
        self.value_dtype = value_dtype
        self.comm = comm
        self.table_id = table_id
        self.n_params = n_params
        align = 64 * comm.world
        self.n_pad = int(math.ceil(n_params / align) * align)
        self.shard = self.n_pad // comm.world
        self.base = comm.rank * self.shard
        dev = comm.device
        self.optimizer = optimizer
        self.lr = lr
        self.betas, self.eps, self.weight_decay = betas, eps, weight_decay
        self.pull_dtype = pull_dtype
        self.master = torch.zeros(self.shard, dtype=value_dtype, device=dev)
        self.m = torch.zeros_like(self.master) if optimizer in ("adam", "adagrad") else None
        self.v = torch.zeros_like(self.master) if optimizer == "adam" else None
        self.params = torch.zeros(self.n_pad, dtype=pull_dtype, device=dev)
        self.grad = torch.zeros(self.n_pad, dtype=value_dtype, device=dev)
        self.grad_shard = torch.zeros(self.shard, dtype=value_dtype, device=dev)
        self.step = 0
        # the Adam step also lives on the device (advanced inside the clock) so that a clock
        # captured in a HIP graph replays with the right bias correction
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self.pipe = _Pipeline(comm, consistency, staleness, kind="dense", w1=overlap_w1)
        self._pending = False
        # async clocks: a ring of staleness+2 gradient buffers, so the side stream reduces clock
        # t's gradients while the compute stream already writes clock t+1's.
        self._ring = [self.grad] + [torch.zeros_like(self.grad) for _ in range(self.pipe.staleness + 1)] \
            if self.pipe.async_ else [self.grad]
        self.buckets = None
        if buckets is not None and bucket_mb:
            buckets = merge_buckets(buckets, n_params, bucket_mb * 2**20 / self.master.element_size())
        if buckets is not None and (comm.world > 1 or self.pipe.async_):
            self._init_buckets(buckets)

    # -- bucketed clocks ----------------------------------------------------------------------
    def _init_buckets(self, starts):
        W = self.comm.world
        unit = 64 * W
        # a bucket starts at the first aligned offset at or after a layer start: it then holds the
        # tail of its layer plus at most `unit` elements of the NEXT layer, whose backward finished
        # earlier -- so a bucket is complete when its own layer's backward is
        edges = sorted({0, self.n_pad} | {min(self.n_pad, -(-int(x) // unit) * unit) for x in starts})
        self.buckets = [(a, b) for a, b in zip(edges[:-1], edges[1:]) if b > a]
        self._boff, off = [], 0
        for lo, hi in self.buckets:
            self._boff.append((off, (hi - lo) // W))
            off += (hi - lo) // W
        assert off == self.shard
        self._issued: set = set()
        self._bstat = [(f"t{self.table_id}b{k}", (hi - lo) * (self.grad.element_size() + self.params.element_size()))
                       for k, (lo, hi) in enumerate(self.buckets)]

    def bucket_of(self, offset: int) -> int:
        """Index of the bucket holding element ``offset``."""
        for k, (lo, hi) in enumerate(self.buckets):
            if lo <= offset < hi:
                return k
        raise IndexError(offset)

    def bucket_for_layer(self, start: int) -> int | None:
        """The bucket a layer starting at element ``start`` completes (None: not bucketed)."""
        if self.buckets is None:
            return None
        unit = 64 * self.comm.world
        return self.bucket_of(min(self.n_pad - 1, -(-int(start) // unit) * unit))

    def _own_piece(self, k: int):
        lo, _ = self.buckets[k]
        off, sz = self._boff[k]
        g0 = lo + self.comm.rank * sz
        return off, sz, g0

    def _step_dev_for_clock(self, first: bool = True):
        """The Adam step's device twin ``step_dev`` advances only inside a HIP-graph capture (a
        replayed step must read a fresh step on the device; GraphedStep sets it
        from the host step before capturing). Eager clocks pass the host step: no extra kernel
        on the clock's stream. Returns the step_dev argument for adam_apply."""
        if not (self.master.is_cuda and torch.cuda.is_current_stream_capturing()):
            return None
        if first:
            self.step_dev.add_(1)
        return self.step_dev

    def sync_step_dev(self):
        """Before a HIP-graph capture: the device step twin = the host step."""
        self.step_dev.fill_(int(self.step))

    def _bucket_views(self, k: int, grad: torch.Tensor):
        """The views one bucket's clock works on (persistent buffers: built once per bucket and
        gradient buffer of the ring -- ~10 slicing ops per bucket per clock off the host path)."""
        key = (k, grad.data_ptr())
        cache = self.__dict__.setdefault("_bview", {})
        v = cache.get(key)
        if v is None:
            lo, hi = self.buckets[k]
            off, sz, g0 = self._own_piece(k)
            sl = slice(off, off + sz)
            v = cache[key] = (grad[lo:hi], self.grad_shard[sl], self.master[sl],
                              self.m[sl] if self.m is not None else None, self.v[sl] if self.v is not None else None,
                              self.params[g0: g0 + sz], self.params[lo:hi])
        return v

    @traced("dense.bucket_work")
    def _bucket_work(self, k: int, grad: torch.Tensor, step: int):
        comm = self.comm
        sd = self._step_dev_for_clock(first=not self._issued)
        self._issued.add(k)
        g_b, gs_own, w, m, v, p_own, p_b = self._bucket_views(k, grad)
        local = comm.world == 1 and not comm.force  # one rank owns the whole bucket: no copy
        packed = False
        if local:
            gs = g_b
        else:
            sink = getattr(self, "_sink", None)
            if sink is not None and comm.world > 1:  # the bucket's split-K planes folded into its RS input
                send = self.__dict__.get("_rs_send")
                if send is None:
                    send = self._rs_send = torch.empty_like(self.grad)
                lo, hi = self.buckets[k]
                ops.slab_pack(g_b, send[lo:hi], sink.take(g_b))
                comm.reduce_scatter(gs_own, send[lo:hi])
                packed = True
            else:
                comm.reduce_scatter(gs_own, g_b)
            gs = gs_own
        out = p_own if self.pull_dtype == torch.bfloat16 else None
        zeroed = False
        if self.optimizer == "adam":
            sink = getattr(self, "_sink", None)  # (one rank: the bucket's split-K wgrad planes)
            slabs = sink.take(gs) if sink is not None and local else ()
            ops.adam_apply(w, m, v, gs, self.lr, self.betas[0], self.betas[1], self.eps, self.weight_decay, step, 1.0,
                           out, step_dev=sd, zero_g=local, slabs=slabs)
            zeroed = local or packed  # the kernel (or the pack) cleared the gradient
        elif self.optimizer == "adagrad":
            ops.adagrad_apply(w, m, gs, self.lr, self.eps, 1.0, out)
        elif self.optimizer == "sgd":
            ops.sgd_apply(w, gs, self.lr, 1.0, out)
        elif self.optimizer == "add":
            w.add_(gs)
            if out is not None:
                ops.cast_f32_bf16(w, out)
        else:
            raise ValueError(self.optimizer)
        if out is None:
            p_own.copy_(w)
        comm.all_gather(p_b, p_own)
        if not (zeroed or packed):
            g_b.zero_()
        key, nb = self._bstat[k]
        bb = comm.stats.bucket_bytes
        bb[key] = bb.get(key, 0) + nb

    @traced("dense.bucket_ready")
    def bucket_ready(self, k: int, events=()):
        """The gradients of bucket ``k`` are complete (every writer is on the current stream or
        behind ``events``): issue its reduce-scatter + apply + all-gather now (on the clock
        stream when clocks are asynchronous, so it overlaps the rest of the backward)."""
        if self.buckets is None or k in self._issued:
            return
        self._pending = True  # the gradients were written in place into self.grad
        grad, step = self.grad, self.step + 1
        if self.pipe.async_:
            st = self.pipe.stream
            fork = self.pipe._forks.next()
            fork.record(streams.current(st.device))
            st.wait_event(fork)
            for ev in events:
                if ev is not None:
                    st.wait_event(ev)
            # (the gradient ring's buffers are persistent: nothing to keep alive)
            with streams.use(st):
                self._bucket_work(k, grad, step)
        else:
            # synchronous clocks: the bucket's collectives run on the current stream, which must
            # still wait for the gradients' producers on other streams (the weight-gradient side
            # stream) -- with the HIP default of 4 hardware queues the two streams happened to
            # share a queue, which hid the missing wait; with 8 they run concurrently
            if grad.is_cuda:
                cur = streams.current(grad.device)
                for ev in events:
                    if ev is not None:
                        cur.wait_event(ev)
            self._bucket_work(k, grad, step)

    def _full_from_pieces(self, t: torch.Tensor) -> torch.Tensor:
        """All-gather a bucket-major shard buffer into the full vector in canonical order."""
        W = self.comm.world
        gathered = torch.empty(W * self.shard, dtype=t.dtype, device=t.device)
        self.comm.all_gather(gathered, t)
        gathered = gathered.view(W, self.shard)
        full = torch.empty(self.n_pad, dtype=t.dtype, device=t.device)
        for (lo, _), (off, sz) in zip(self.buckets, self._boff):
            full[lo: lo + W * sz].view(W, sz).copy_(gathered[:, off: off + sz])
        return full

    def _pieces_from_full(self, full: torch.Tensor, dst: torch.Tensor):
        for k in range(len(self.buckets)):
            off, sz, g0 = self._own_piece(k)
            dst[off: off + sz].copy_(full[g0: g0 + sz])

    # -- init / views -----------------------------------------------------------------------
    def load_full(self, full: torch.Tensor):
        """Initialise from the full vector (identical on every rank)."""
        assert full.numel() == self.n_params
        flat = torch.zeros(self.n_pad, dtype=self.value_dtype, device=self.comm.device)
        flat[: self.n_params] = full.to(self.comm.device, self.value_dtype)
        if self.buckets is not None:
            self._pieces_from_full(flat, self.master)
        else:
            self.master.copy_(flat[self.base: self.base + self.shard])
        self.params.copy_(flat.to(self.pull_dtype))

    def full_master(self) -> torch.Tensor:
        """All-gather of the master values (checkpoint / tests)."""
        self.drain()
        if self.buckets is not None:
            return self._full_from_pieces(self.master)[: self.n_params]
        out = torch.empty(self.n_pad, dtype=self.value_dtype, device=self.comm.device)
        self.comm.all_gather(out, self.master)
        return out[: self.n_params]

    # -- KV API -----------------------------------------------------------------------------
    @traced("dense.get")
    def get(self) -> torch.Tensor:
        self.pipe.wait_for_read()
        return self.params

    @traced("dense.add")
    def add(self, grad: torch.Tensor | None = None):
        """Accumulate a gradient (or mark the in-place-written self.grad as pushed)."""
        if grad is not None:
            self.grad[: grad.numel()] += grad.reshape(-1).to(self.value_dtype)
        self._pending = True

    @traced("dense.clock")
    def clock(self):
        grad = self.grad
        step = self.step + 1
        self.step = step
        pending = self._pending
        self._pending = False

        comm = self.comm

        if self.buckets is not None:
            def work():  # the buckets the backward did not issue yet, in order
                if pending:
                    for k in range(len(self.buckets)):
                        if k not in self._issued:
                            self._bucket_work(k, grad, step)
                else:
                    self._step_dev_for_clock()
                self._issued = set()

            self.pipe.run(work)
            if self.pipe.async_:
                self.grad = self._ring[step % len(self._ring)]
                self.pipe.wait_clock(step - len(self._ring))
            return

        def work():
            sd = self._step_dev_for_clock()
            if pending:
                if comm.world == 1:  # the whole gradient is the owned shard
                    # Adam clears it in the same pass (one fewer full-size kernel per clock)
                    cleared = self._apply(grad, step, zero_g=grad.numel() == self.shard, step_dev=sd)
                else:
                    sink = getattr(self, "_sink", None)
                    if sink is not None:
                        # the split-K weight-gradient planes folded into the reduce-scatter input and
                        # the gradient cleared, in one pass (no split-K reduce kernels, no fill)
                        send = self.__dict__.get("_rs_send")
                        if send is None:
                            send = self._rs_send = torch.empty_like(grad)
                        ops.slab_pack(grad, send, sink.take(grad))
                        comm.reduce_scatter(self.grad_shard, send)
                        cleared = True
                    else:
                        comm.reduce_scatter(self.grad_shard, grad)
                        cleared = False
                    self._apply(self.grad_shard, step, step_dev=sd)
                comm.all_gather(self.params, self.params[self.base: self.base + self.shard])
            else:
                cleared = False
            if not cleared:
                grad.zero_()

        self.pipe.run(work)
        if self.pipe.async_:
            # next buffer of the ring: it was last used by clock step-len(ring); wait for it
            self.grad = self._ring[step % len(self._ring)]
            self.pipe.wait_clock(step - len(self._ring))

    def slab_sink(self):
        """A sink for split-K weight gradients whose K slices this table's next clock folds in
        (ops.linear_wgrad(defer=...): no reduce kernel, no pass of the sum through the gradient
        buffer): one rank's Adam, or several ranks' reduce-scatter pack of the clock or of each
        bucket (ops.slab_pack); None for other optimizers at one rank."""
        # several ranks: the planes are folded by the reduce-scatter's pack (clock / bucket)
        if (not _WGRAD_DEFER or self.comm.device.type != "cuda"
                or (self.comm.world == 1 and self.optimizer != "adam")
                or (self.comm.world > 1 and self.value_dtype != torch.float32)
                or (self.pipe.async_ and len(self._ring) < 2)):
            # (an asynchronous clock applies after the next step's GEMMs ran: those write the next
            # buffer of the gradient ring -- and its own planes -- which the ring's clock wait protects)
            return None
        sink = getattr(self, "_sink", None)
        if sink is None:
            sink = self._sink = _SlabSink(self)
        return sink

    def _apply(self, g: torch.Tensor, step: int, zero_g: bool = False, step_dev=None) -> bool:
        """Apply the optimizer to the owned shard; True if ``g`` was cleared on the way."""
        out = self.params[self.base: self.base + self.shard] if self.pull_dtype == torch.bfloat16 else None
        if self.optimizer == "adam":
            sink = getattr(self, "_sink", None)
            slabs = sink.take(g) if sink is not None else ()
            ops.adam_apply(self.master, self.m, self.v, g, self.lr, self.betas[0], self.betas[1], self.eps,
                           self.weight_decay, step, 1.0, out, step_dev=step_dev, zero_g=zero_g, slabs=slabs)
            if out is None:
                self.params[self.base: self.base + self.shard].copy_(self.master)
            return zero_g
        elif self.optimizer == "adagrad":
            ops.adagrad_apply(self.master, self.m, g, self.lr, self.eps, 1.0, out)
        elif self.optimizer == "sgd":
            ops.sgd_apply(self.master, g, self.lr, 1.0, out)
        elif self.optimizer == "add":  # the reference server apply: w += delta
            self.master.add_(g)
            if out is not None:
                ops.cast_f32_bf16(self.master, out)
        else:
            raise ValueError(self.optimizer)
        if out is None:
            self.params[self.base: self.base + self.shard].copy_(self.master)
        return False

    def hold(self, event):
        """A clock of this table was issued on another stream (WideDeep runs one rank's dense Adam
        on its weight-gradient side stream and does not join it): ``event`` marks its end, and the
        next drain() -- every checkpoint's shard_state() -- makes the current stream wait for it, so
        a snapshot never copies master / m / v from the middle of that Adam."""
        self._held = event

    def drain(self):
        self.pipe.drain()
        ev = self.__dict__.pop("_held", None)
        if ev is not None:
            streams.current(self.comm.device).wait_event(ev)

    def reset_after_rollback(self):
        self.pipe.reset()
        self._pending = False
        self.__dict__.pop("_held", None)
        for g in self._ring:
            g.zero_()

    # -- checkpoint hooks (minips_amd.ps.checkpoint) -------------------------------------------
    def shard_state(self):
        """(meta, {name: tensor}) of the owned shard: fp32 master + optimizer state, padding
        beyond n_params excluded."""
        self.drain()
        rows = max(0, min(self.shard, self.n_params - self.base))
        if self.buckets is not None:  # canonical contiguous layout: the same files as unbucketed
            arrays = {n: self._full_from_pieces(t)[self.base: self.base + rows]
                      for n, t in (("master", self.master), ("m", self.m), ("v", self.v)) if t is not None}
        else:
            arrays = {"master": self.master[:rows]}
            if self.m is not None:
                arrays["m"] = self.m[:rows]
            if self.v is not None:
                arrays["v"] = self.v[:rows]
        meta = dict(global_rows=self.n_params, base=self.base, rows=rows, cols=1, clock=self.step,
                    table_id=self.table_id, rank=self.comm.rank, world=self.comm.world, kind="dense")
        return meta, arrays

    def restore_range(self):
        """Global element range [lo, hi) this rank restores (checkpoint.Checkpointer.load)."""
        return self.base, max(self.base, min(self.base + self.shard, self.n_params))

    def restore_dst(self):
        """Device destinations of the checkpointed arrays, [rows, 1] in restore_range order."""
        tabs = (("master", self.master), ("m", self.m), ("v", self.v))
        if self.buckets is not None:  # land in the canonical layout, redistribute in finish_restore
            self._canon = {n: torch.zeros_like(t) for n, t in tabs if t is not None}
            return {n: t.view(-1, 1) for n, t in self._canon.items()}
        return {n: t.view(-1, 1) for n, t in tabs if t is not None}

    def finish_restore(self, clock: int):
        """After the rows landed: clocks, then re-pull (all-gather) the parameters."""
        self.step = int(clock)
        self.step_dev.fill_(int(clock))
        self.pipe.clock = int(clock)
        if self.buckets is not None:
            full = None
            for n, c in self._canon.items():
                g = torch.empty(self.n_pad, dtype=c.dtype, device=c.device)
                self.comm.all_gather(g, c)
                self._pieces_from_full(g, getattr(self, n))
                if n == "master":
                    full = g
            self._canon = None
            self.params.copy_(full.to(self.pull_dtype))
            return
        own = self.params[self.base: self.base + self.shard]
        if self.pull_dtype == torch.bfloat16:
            ops.cast_f32_bf16(self.master, own)
        else:
            own.copy_(self.master)
        self.comm.all_gather(self.params, own)


def column_spec(columns, device):
    """(bases, cards) of [B, F] batches with disjoint column key ranges -> the per-column sort
    planner's (base tensor, bit widths, device bit widths), or None when a column needs > 32 bits."""
    if columns is None:
        return None
    bases, cards = columns
    bits = [max(1, (int(c) - 1).bit_length()) for c in cards]
    if max(bits) > 32:
        return None
    return (torch.as_tensor(list(bases), dtype=torch.int64, device=device), bits,
            torch.tensor(bits, dtype=torch.int32, device=device))


_ROUTE_PRIMES = (402653189, 201326611, 100663319, 50331653, 25165843, 12582917, 6291469, 3145739, 1572869)


def _route_multiplier(num_rows: int) -> int:
    """A prime multiplier coprime to num_rows with key * A < 2^63 (0: no mixing possible)."""
    for p in _ROUTE_PRIMES:
        if num_rows % p and num_rows * p < (1 << 63) and p < num_rows:
            return p
    return 0


# the dedupe counts each unique key's lookups for the embedding-backward CSR (one pass less);
# CSR_FUSED off counts in emb_build_csr instead
_CSR_FUSED = True
# SORTED_EMB on: plans carry the CSR's inverse permutation (csr[2]: each lookup's row in
# member order) so the embedding dgrad writes its output pre-sorted and the backward streams it
# contiguously instead of gathering 64-byte pieces. Measured on one MI355X (W&D step, 3 x 400
# steps each, tools/gpu_round.sh ab): 0.4244 vs 0.4151 ms with the gather path -- the segment sums get
# faster (66 -> 36 us) but the dgrad's scattered 64-byte stores cost more -- so it is off.
SORTED_EMB = False


def _with_positions(csr):
    return (*csr, ops.emb_csr_positions(csr[0])) if SORTED_EMB else csr


@dataclass
class SparsePlan:
    """Routing of one batch's keys. Row counts are host ints on multi-rank runs (the all-to-all
    splits need them anyway); on one rank the unique count stays on the GPU (``U_dev``) and
    buffers are sized by the upper bound ``cap`` -- no host round trip per step."""
    keys_n: int
    inv: torch.Tensor          # [n] position of each requested key in the unique order
    uniq: torch.Tensor         # [n] unique keys grouped by owner (first U valid)
    cap: int                   # rows to allocate for per-unique-key buffers (>= U)
    send: list | None          # keys requested from each owner
    recv: list | None          # keys each requester asked from me
    recv_keys: torch.Tensor    # [M] keys I serve (grouped by requester)
    U_dev: torch.Tensor | None = None   # [1] device-side U (None: cap == U exactly)
    own_uniq: torch.Tensor | None = None
    own_inv: torch.Tensor | None = None
    own_U_dev: torch.Tensor | None = None
    own_slots: torch.Tensor | None = None  # [own cap * P] received row per (owned row, requester)
    csr: tuple | None = None   # (members, memrow) lookups grouped by unique row (emb backward)
    extra: dict = field(default_factory=dict)
    _U: int | None = None

    @property
    def U(self) -> int:
        """Exact unique-key count (host; syncs once when only the device count exists)."""
        if self._U is None:
            self._U = self.cap if self.U_dev is None else int(self.U_dev.item())
        return self._U


# Key planning of [B, F] batches with disjoint column key ranges (SparseTable ``columns``) on one
# rank: per-column radix sort without atomics (ops.plan_sorted) instead of the hash dedupe, whose
# Bitmap planning (ops.bitmap_plan) for range tables whose key space is small next to the batch
# (bitmap bytes <= _BITMAP_RATIO x keys): uniformly drawn ids dedupe without a hash table. Measured
# on one MI355X: sparse LR (16.6M rows, 4.2M keys: 0.5 B/key) 1.26 -> 0.83 ms/step; DLRM (10^8
# rows, 426K keys: 29 B/key) 0.69 -> 0.71 ms (the map scans and the separate CSR build cost more
# than the hash inserts there), so the default ratio keeps DLRM on the hash dedupe.
# BITMAP_PLAN off keeps the hash dedupe everywhere.
_BITMAP_PLAN = True
_BITMAP_RATIO = 16
# memory-side atomics slow the concurrently running step; SORT_PLAN off keeps the hash path
_SORT_PLAN = True

# one rank: W&D assembles its input straight from the fp32 shard (SparseTable.get_source +
# ops.wd_assemble_tab) instead of gathering the batch's unique rows first (FUSED_ASSEMBLE off)
_FUSED_ASSEMBLE = True


class _PendingPlan:
    """A plan whose dedupe + count exchange was issued on the planning stream (lookahead)."""
    __slots__ = ("keys", "F", "flat", "uniq", "inv", "counts", "U_dev", "host", "event", "csr", "cev", "exchanged")


class SparseTable:
    _local_apply = True  # this rank applies its pushes itself (the one-sided tables' owners apply)
    # hash tables need exact host counts (insert-on-miss must not see padding keys)
    _exact_counts = False

    def __init__(self, comm: Comm, num_rows: int, width: int, optimizer: str = "rowwise_adagrad",
                 lr: float = 0.01, eps: float = 1e-8, pull_dtype=torch.bfloat16, consistency: str = "bsp",
                 staleness: int = 0, split: int | None = None, table_id: int = 0, init_std: float = 0.01,
                 seed: int = 1234, p2p: bool | None = None, push_dtype=None, route: str = "mix",
                 value_dtype=torch.float32, columns=None):
        """``value_dtype`` float64: the reference's double tables (CreateTable<double>,
        lr_example.cpp:182; values read as double, kv_client_table.hpp:96-101) -- optimizer "add"
        (VectorStorage::SubAdd), rows pulled and pushed in fp64 (f64.hip kernels).

        ``columns`` = (bases, cards): a caller whose [B, F] key batches hold disjoint ranges per
        column (column f's keys in [bases[f], bases[f] + cards[f]), e.g. concatenated feature
        tables) lets one-rank planning use the atomic-free per-column sort (ops.plan_sorted).

        ``value_dtype`` bfloat16: rows stored in bf16 (half the HBM: the 10B x 64 DLRM table fits
        8 x 288 GB), gradients and optimizer state in fp32, applies rounded stochastically
        (bf16rows.hip); rows of 16 / 32 / 64 values."""
        if value_dtype not in (torch.float32, torch.float64, torch.bfloat16):
            raise ValueError(f"value_dtype {value_dtype}")
        if value_dtype == torch.float64:
            if optimizer != "add":
                raise ValueError("fp64 sparse tables support the reference's plain add apply only")
            pull_dtype = push_dtype = torch.float64
        if value_dtype == torch.bfloat16 and width not in (16, 32, 64):
            raise ValueError("bf16 sparse rows hold 16, 32 or 64 values")
        self.value_dtype = value_dtype
        # gradients / pushes of a bf16 table are fp32 (only the stored rows are bf16)
        self.grad_dtype = torch.float32 if value_dtype == torch.bfloat16 else value_dtype
        self._applies = 0  # apply counter: keys the stochastic rounding of bf16 rows
        self.seed = seed
        self.comm = comm
        self.columns = column_spec(columns, comm.device)
        # Key -> row placement. "range": row = key (the reference's contiguous range partition).
        # "mix" (default): row = key * A mod num_rows, a bijection (A prime, coprime to num_rows),
        # then the same equal ranges: contiguous key blocks (a big feature of a concatenated
        # table, or a hot id range) spread over every shard instead of overloading one owner --
        # on Criteo-shaped batches the busiest of 8 range owners serves 6x the rows of the
        # quietest. Rows, checkpoints and re-sharding live in the routed space (it depends on
        # num_rows only, so any world size agrees).
        self.route_mult = _route_multiplier(num_rows) if route == "mix" else 0
        # gradient rows cross xGMI in bf16 on multi-GPU runs (half the push bytes; the owner
        # accumulates in fp32), fp32 otherwise
        self.push_dtype = push_dtype or (torch.bfloat16 if comm.device.type == "cuda" and comm.world > 1
                                         else torch.float32)
        self.table_id = table_id
        self.num_rows = num_rows
        self.width = width
        self.optimizer, self.lr, self.eps = optimizer, lr, eps
        self.pull_dtype = pull_dtype
        self.split = split
        dev = comm.device
        b = even_bounds(num_rows, comm.world)
        self.bounds_list = b
        self.bounds = torch.tensor(b, dtype=torch.int64, device=dev)
        self.base = b[comm.rank]
        self.rows_local = b[comm.rank + 1] - b[comm.rank]
        # LoopbackComm re-bases the keys this rank asks of owner s to offset (key - bounds[s]) of its
        # own range (_finish_plan); the last owner's range is up to P - 1 rows longer than the
        # others', so an emulated shard carries that many spare rows (offsets stay collision-free)
        self._rows_alloc = self.rows_local + (num_rows % comm.world if comm.emulated else 0)
        g = torch.Generator(device=dev)
        g.manual_seed(seed + 7919 * comm.rank)
        self.shard = torch.empty(self._rows_alloc, width, dtype=value_dtype, device=dev)
        if init_std > 0:
            self.shard.normal_(0.0, init_std, generator=g)
        else:
            self.shard.zero_()
        self.state = torch.zeros(self._rows_alloc, dtype=torch.float32, device=dev) \
            if optimizer == "rowwise_adagrad" else None
        self.state2 = torch.zeros_like(self.state) if (self.state is not None and split is not None) else None
        self._init_comm(consistency, staleness, p2p)

    def _init_comm(self, consistency, staleness, p2p):
        comm = self.comm
        self.pipe = _Pipeline(comm, consistency, staleness, kind="sparse")
        # SSP/ASP move rows with point-to-point send/recv by default, BSP with all-to-all-v
        self.p2p = (consistency != "bsp") if p2p is None else p2p
        self._pending: list = []
        self._own_bounds = torch.tensor([0, (1 << 63) - 1], dtype=torch.int64, device=comm.device)

    # -- KV API -----------------------------------------------------------------------------
    def _route_keys(self, keys: torch.Tensor) -> torch.Tensor:
        """Keys as exchanged between ranks and stored: the global row of each key."""
        if self.route_mult:
            return (keys * self.route_mult) % self.num_rows
        return keys

    def _serve_index(self, plan: SparsePlan):
        """(row table, row index tensor, base) for the rows this rank serves in ``plan``."""
        return self.shard, plan.recv_keys, self.base

    def _owner_rows(self, keys: torch.Tensor, plan=None):
        """(row index tensor, base) of owned unique keys being updated."""
        return keys, self.base

    def _owner_keys(self, plan: SparsePlan):
        """The owned unique keys a push of ``plan`` updates (exact-count plans only)."""
        if self.comm.world == 1:
            return plan.uniq[: plan.cap]
        if plan.own_uniq is None:
            return None
        return plan.own_uniq[: plan.extra.get("own_U", len(plan.recv_keys))]

    @traced("sparse.start_plan")
    def _start_plan(self, keys: torch.Tensor, csr: bool = False, exchange: bool = True) -> _PendingPlan:
        """Dedupe + owner bucketing (+ the all-to-all of the per-owner counts unless
        ``exchange`` is False: _exchange_counts does it later), issued on the current stream;
        the counts land in pinned host memory behind an event. ``csr`` also groups the lookups
        by unique row for the embedding backward (it depends on the keys only)."""
        pp = _PendingPlan()
        pp.keys = keys
        pp.F = keys.shape[1] if keys.dim() == 2 else 1
        flat = keys.reshape(-1).to(torch.int64)
        rmult = getattr(self, "route_mult", 0)
        want_csr = csr and flat.is_cuda
        fused = want_csr and _CSR_FUSED
        n = flat.numel()
        zeroed = None
        cols = getattr(self, "columns", None)  # (HashSparseTable has no column ranges)
        if (cols is not None and _SORT_PLAN and flat.is_cuda and self.comm.world <= 16 and keys.dim() == 2
                and keys.shape[0] <= 16384 and keys.shape[1] == cols[0].numel()
                and max(cols[1]) + (self.comm.world - 1).bit_length() <= 32):  # (owner bits ride in the sort key)
            # disjoint column key ranges: atomic-free per-column sort (ops.plan_sorted), unique keys
            # regrouped by owner, and the embedding backward's lookup CSR on the way
            pp.flat = flat
            res = ops.plan_sorted(keys if keys.dtype == torch.int64 else keys.to(torch.int64), cols[0], cols[1], rmult,
                                  self.num_rows if rmult else 0, bits_dev=cols[2], bounds=self.bounds,
                                  positions=want_csr and SORTED_EMB)
            pp.uniq, pp.inv, pp.counts, pp.U_dev = res[:4]
            pp.csr = tuple(res[4:]) if want_csr else None  # (members, memrow[, positions][, rowstart])
            pp.host = pp.event = pp.cev = None
            pp.exchanged = self.comm.world == 1
            if exchange:
                self._exchange_counts(pp)
            return pp
        if (_BITMAP_PLAN and flat.is_cuda and cols is None and type(self)._route_keys is SparseTable._route_keys
                and self.num_rows <= (1 << 36) and self.num_rows // 8 <= _BITMAP_RATIO * max(n, 1)):
            # bounded key space: bitmap dedupe (sorted unique keys, grouped by owner by construction)
            pp.flat = flat
            pp.uniq, pp.inv, pp.counts, pp.U_dev = ops.bitmap_plan(flat, self.bounds, self.num_rows, rmult,
                                                                   oor=self._oor_counter())
            pp.csr = _with_positions(ops.emb_build_csr(pp.inv, pp.F, n)) if want_csr else None
            pp.host = pp.event = pp.cev = None
            pp.exchanged = self.comm.world == 1
            if exchange:
                self._exchange_counts(pp)
            return pp
        if rmult:  # range tables: the routing is fused into the dedupe kernel
            pp.flat = flat
            res = ops.unique_bucketize_n(flat, self.bounds, pp.F, rmult, self.num_rows,
                                         extra_zero_ints=2 * n if want_csr else 0, csr_counts=fused)
        else:
            pp.flat = self._route_keys(flat)
            res = ops.unique_bucketize_n(pp.flat, self.bounds, pp.F, extra_zero_ints=2 * n if want_csr else 0,
                                         csr_counts=fused)
        if want_csr:  # the CSR's counters were cleared by the dedupe's single memset, and the
            res, zeroed = res  # dedupe already counted each unique key's lookups into them
        pp.uniq, pp.inv, pp.counts, pp.U_dev = res
        pp.csr = _with_positions(ops.emb_build_csr(pp.inv, pp.F, n, zeroed=zeroed, counts_ready=fused)) \
            if want_csr else None
        pp.host = pp.event = pp.cev = None
        pp.exchanged = self.comm.world == 1
        if exchange:
            self._exchange_counts(pp)
        return pp

    @traced("sparse.exchange_counts")
    def _exchange_counts(self, pp: _PendingPlan):
        """All-to-all of the plan's per-owner counts on the current stream; the counts land in
        pinned host memory behind ``pp.cev`` (the host reads them to size the key exchange)."""
        if pp.exchanged:
            return
        pp.exchanged = True
        if not pp.counts.is_cuda:
            recv = torch.empty_like(pp.counts)
            self.comm.all_to_all_counts(recv, pp.counts)
            pp.host = torch.stack([pp.counts, recv])
            return
        # [send counts | received counts] in one device buffer -> one copy into a pinned slot of a
        # ring (no pinned allocation, no event object per plan); the event carries the system-scope
        # release the host read needs
        ring = self.__dict__.get("_count_ring")
        P = pp.counts.numel()
        if ring is None or ring[0][0][0].shape[1] != P:
            n = 8  # > look-ahead depth + 2 plans in flight
            ring = self._count_ring = ([(torch.empty(2, P, dtype=torch.int64, device=pp.counts.device),
                                         torch.empty(2, P, dtype=torch.int64, pin_memory=True),
                                         torch.cuda.Event()) for _ in range(n)], [0])
        slots, i = ring
        both, host, ev = slots[i[0]]
        i[0] = (i[0] + 1) % len(slots)
        both[0].copy_(pp.counts)
        self.comm.all_to_all_counts(both[1], pp.counts)
        host.copy_(both, non_blocking=True)
        ev.record()
        pp.host, pp.cev = host, ev

    @traced("sparse.plan_async")
    def plan_async(self, keys: torch.Tensor, csr: bool = False, keys_on_plan_stream: bool = False,
                   fenced: bool = False):
        """Lookahead: start planning ``keys`` (a LATER batch) on the planning stream, so its
        dedupe, count exchange (and lookup CSR) overlap the current step; pass the result to
        get(plan=...). Planning reads no table state, so issuing it early changes no
        consistency semantics. ``keys_on_plan_stream``: the keys were produced on the planning
        stream itself (a data producer running there), so planning need not wait for the
        compute stream at all. On the CPU the same two halves run at the same issue points
        (inline), so a gloo run issues exactly the collective sequence of an RCCL run.

        ``fenced``: the caller orders the planning stream after each step's compute-stream work
        (LookaheadFeeder's end-of-step fence), so the plan's buffers -- allocated on the planning
        stream and read on the compute stream -- need no per-tensor ``record_stream``: each
        record_stream costs an allocator event on the compute stream when the tensor is freed,
        and those events cost the W&D step ~30 us (tools/step_probe.py ablation). Only valid while the
        plan is consumed inside the fenced step (one rank, synchronous clocks)."""
        if self._exact_counts:
            return self.plan(keys, csr)
        if self.comm.device.type != "cuda":
            return self._start_plan(keys, csr, exchange=False)
        ps = self.comm.plan_stream()
        cur = streams.current(self.comm.device)
        if not keys_on_plan_stream:
            ps.wait_stream(cur)  # the keys are produced on the compute stream
        with streams.use(ps):
            pp = self._start_plan(keys, csr, exchange=False)
            ring = self.__dict__.get("_plan_evs")
            if ring is None:  # (plans are consumed within a few steps of their issue)
                ring = self._plan_evs = streams.EventRing(16, fast=streams.fast_for("plan"))
            pp.event = ring.next()
            pp.event.record(ps)
        if fenced:
            # the feeder fences the planning stream after every step and the clocks retain what
            # their side streams read (_Pipeline.retain): no per-tensor stream bookkeeping
            self.pipe.retain = True
            return pp
        keys.record_stream(ps)
        for t in (pp.flat, pp.uniq, pp.inv, pp.counts, pp.U_dev, *(pp.csr or ())):
            if t is not None:  # produced on the planning stream, consumed on the compute stream
                t.record_stream(cur)
        return pp

    @traced("sparse.finish_plan")
    def _finish_plan(self, pp: _PendingPlan) -> SparsePlan:
        dev = self.comm.device
        comm = self.comm
        n = pp.flat.numel()
        if pp.event is not None:
            streams.current(dev).wait_event(pp.event)
        if not pp.exchanged:  # nobody issued the count exchange yet: do it here
            self._exchange_counts(pp)
        if self.comm.world == 1:
            if self._exact_counts or dev.type != "cuda":
                U = int(pp.U_dev.item())
                return SparsePlan(n, pp.inv, pp.uniq, U, [U], [U], pp.uniq[:U], csr=pp.csr, _U=U)
            return SparsePlan(n, pp.inv, pp.uniq, n, None, None, pp.uniq, U_dev=pp.U_dev, csr=pp.csr)
        if pp.cev is not None and not pp.cev.query():
            # the only possible host wait of a step: the all-to-all splits (with look-ahead depth 2
            # they were exchanged a step earlier, so normally they are in already: no wait)
            with self.comm.waiting(), phase("sparse.count_wait"):
                pp.cev.synchronize()
        send, recv = pp.host[0].tolist(), pp.host[1].tolist()
        U, M = int(sum(send)), int(sum(recv))
        recv_keys = torch.empty(M, dtype=torch.int64, device=dev)
        comm.all_to_all_v(recv_keys, pp.uniq, recv, send, p2p=self.p2p)
        if comm.emulated and M and type(self)._route_keys is SparseTable._route_keys:
            # LoopbackComm: the keys came back as this rank's own requests to every owner; re-base
            # them into its own row range, as the peers' requests to this owner would be: offset
            # key - bounds[s] within owner s's range (s = min(key // step, P - 1)), so distinct keys
            # of one requester segment stay distinct (the direct owner apply has one writer per
            # (row, requester) entry) -- the shard has the last range's spare rows (_rows_alloc)
            step = self.bounds_list[1]
            if recv_keys.is_cuda:
                from .._native import kernels

                kernels().emu_rebase(recv_keys, step, comm.world, self.base)
            else:
                q = torch.div(recv_keys, step, rounding_mode="floor").clamp_(max=comm.world - 1)
                recv_keys.sub_(q.mul_(step)).add_(self.base)
        p = SparsePlan(n, pp.inv, pp.uniq, U, send, recv, recv_keys, csr=pp.csr, _U=U)
        if M > 0 and self._owner_direct_ok():
            p.extra["direct"] = True  # the push applies by direct addressing: no owner-side plan
        elif M > 0:
            # owner-side dedupe of the keys requested by all ranks (the push sums their rows): they
            # lie in this rank's own row range, a bounded space -> the bitmap planner when its map
            # is small per key (W&D at 8 ranks: 4.2M local rows for ~10^5-10^6 requested keys)
            if (_BITMAP_PLAN and recv_keys.is_cuda and type(self)._route_keys is SparseTable._route_keys
                    and 0 < self._rows_alloc // 8 <= _BITMAP_RATIO * M):
                if getattr(self, "_own_local_bounds", None) is None:
                    self._own_local_bounds = torch.tensor([0, self._rows_alloc], dtype=torch.int64, device=dev)
                ou, oi, _, oU = ops.bitmap_plan(recv_keys - self.base, self._own_local_bounds, self._rows_alloc,
                                                oor=self._oor_counter())
                ou = ou + self.base
            else:
                ou, oi, _, oU = ops.unique_bucketize_n(recv_keys, self._own_bounds)
            p.own_uniq, p.own_inv, p.own_U_dev = ou, oi, oU
            if self._exact_counts:
                p.extra["own_U"] = int(oU.item())
            if self._owner_fused_ok():
                # per owned row, the received row of every requester (each requester pushes a key
                # at most once): the clock's apply sums them in requester order in one kernel
                p.own_slots = ops.owner_slots(oi, recv, M)
        return p

    # the direct-addressed owner apply keeps an int2 {stamp, row} per (owned row, requester)
    _direct_max_bytes = 2 << 30

    def _owner_direct_ok(self) -> bool:
        """The fused owner apply (below) by direct addressing (ops.owner_push_adagrad): no bitmap
        dedupe, no slot scatter at planning time, when the rows x requesters table fits the budget
        (W&D at 8 ranks: 4.2M rows x 8 x 8 B = 270 MB; a 10^9-row shard keeps the planned path)."""
        return self._owner_fused_ok() and self.rows_local * self.comm.world * 8 <= self._direct_max_bytes

    def _owner_fused_ok(self) -> bool:
        """Several ranks, row-wise Adagrad on an fp32 range shard: the owner applies its pushes
        with ops.owner_rows_adagrad (segment sums + apply fused, deterministic) instead of
        scatter-add into a zeroed buffer + a separate apply."""
        return (self.comm.world > 1 and self.comm.world <= 16 and self._local_apply
                and self.optimizer == "rowwise_adagrad" and self.value_dtype == torch.float32
                and type(self)._owner_rows is SparseTable._owner_rows and 16 < self.width <= 64
                and self.width % 4 == 0)

    def plan(self, keys: torch.Tensor, csr: bool = False) -> SparsePlan:
        return self._finish_plan(self._start_plan(keys, csr))

    def _oor_counter(self) -> torch.Tensor:
        """Device count of keys the bitmap planner found outside [0, num_rows) (they would alias
        row 0); read at the next host sync point (drain), never per step."""
        c = getattr(self, "_oor", None)
        if c is None:
            c = self._oor = torch.zeros(1, dtype=torch.int64, device=self.comm.device)
        return c

    def _check_keys(self):
        c = getattr(self, "_oor", None)
        if c is not None:
            n = int(c.item())
            if n:
                c.zero_()
                raise ValueError(f"table {self.table_id}: {n} keys outside [0, {self.num_rows}) were planned "
                                 f"(their Gets read and their Adds wrote row 0)")

    @traced("sparse.advance_plan")
    def advance_plan(self, pending, finish: bool = True):
        """Later halves of lookahead planning, called once the current step is issued (so these
        collectives follow the step's own row exchanges and clocks in the rank's single ordered
        communicator, ps/comm.py): issue the count exchange of a pending plan if it is not done
        yet; with ``finish``, then wait (host) for the counts and issue the all-to-all of its
        keys and the owner-side dedupe on the planning stream, so that only the row gather and
        the row exchange remain on the critical path of the step that uses the plan."""
        if not isinstance(pending, _PendingPlan) or self.comm.world == 1:
            return pending
        if self.comm.device.type != "cuda":
            self._exchange_counts(pending)
            return self._finish_plan(pending) if finish else pending
        ps = self.comm.plan_stream()
        cur = streams.current(self.comm.device)
        if not pending.exchanged:
            with streams.use(ps):
                self._exchange_counts(pending)
        if not finish:
            return pending
        with streams.use(ps):
            plan = self._finish_plan(pending)
            ring = self.__dict__.get("_ready_evs")
            if ring is None:
                ring = self._ready_evs = streams.EventRing(16, fast=streams.fast_for("plan"))
            ev = ring.next()
            ev.record(ps)
        if not self.pipe.retain:  # (retain: the plan's tensors live until its clock was waited for)
            for t in (plan.recv_keys, plan.own_uniq, plan.own_inv, plan.own_U_dev, plan.own_slots):
                if t is not None:
                    t.record_stream(cur)
        plan.extra["ready"] = ev
        return plan

    @traced("sparse.get")
    def get(self, keys: torch.Tensor, plan=None):
        """Pull rows of ``keys``. Returns (rows [cap, width] in unique order, plan); the row of
        keys[i] is rows[plan.inv[i]]. ``plan`` may be a plan_async() handle for these keys."""
        if plan is None:
            plan = self.plan(keys)
        elif isinstance(plan, _PendingPlan):
            plan = self._finish_plan(plan)
        ready = plan.extra.pop("ready", None)
        if ready is not None:  # keys exchanged on the planning stream (advance_plan)
            streams.current(self.comm.device).wait_event(ready)
        self.pipe.wait_for_read()  # BSP: the previous Clock's apply; SSP: clock c-s-1
        dev = self.comm.device
        served = torch.empty(len(plan.recv_keys), self.width, dtype=self.pull_dtype, device=dev)
        table, index, base = self._serve_index(plan)
        ops.gather_rows(table, index, base, served, n_dev=plan.U_dev if self.comm.world == 1 else None)
        if self.comm.world == 1:  # the served rows ARE the requested rows: no exchange, no copy
            return served, plan
        rows = torch.empty(plan.cap, self.width, dtype=self.pull_dtype, device=dev)
        self.comm.all_to_all_v(rows, served, plan.send, plan.recv, p2p=self.p2p)
        return rows, plan

    @traced("sparse.get_source")
    def get_source(self, keys: torch.Tensor, plan=None):
        """The Get without its row gather, for a consumer that reads the rows in place (one rank,
        fp32 range shard, bf16 pull): returns (plan, table, index, base) -- the row of unique u
        is table[index[u] - base] -- after the same ordering as get() (plan ready, BSP/SSP read
        gate). None when the rows must be gathered (several ranks, hash / bf16 / fp64 tables)."""
        if not (self.comm.world == 1 and self.comm.device.type == "cuda" and type(self)._serve_index is
                SparseTable._serve_index and self.shard.dtype == torch.float32
                and self.pull_dtype == torch.bfloat16 and _FUSED_ASSEMBLE
                and getattr(self, "pipe", None) is not None):  # (the asynchronous one-sided table: no pipe)
            return None
        if plan is None:
            plan = self.plan(keys)
        elif isinstance(plan, _PendingPlan):
            plan = self._finish_plan(plan)
        ready = plan.extra.pop("ready", None)
        if ready is not None:
            streams.current(self.comm.device).wait_event(ready)
        self.pipe.wait_for_read()
        table, index, base = self._serve_index(plan)
        return plan, table, index, base

    def get_rows(self, keys: torch.Tensor) -> torch.Tensor:
        """Reference-style Get: the values of every requested key, in request order."""
        rows, plan = self.get(keys)
        return rows[plan.inv]

    @traced("sparse.add")
    def add(self, plan: SparsePlan, grad_rows: torch.Tensor):
        """Push gradient rows (aligned with the plan's unique order; rows >= U are ignored)."""
        assert grad_rows.shape[0] >= plan.cap and grad_rows.dtype in (getattr(self, "grad_dtype", torch.float32),
                                                                      self.push_dtype)
        self._pending.append((plan, grad_rows))

    @traced("sparse.add_lookup_grads")
    def add_lookup_grads(self, plan: SparsePlan, dX: torch.Tensor, dwide, F: int, D: int, x_off: int = 0,
                         sorted_rows: bool = False):
        """Push the gradient of every lookup of ``plan``'s batch: dX[b, x_off + f*D : +D] for
        lookup (b, f) (+ dwide[b] into column D of the row). The table reduces them per unique
        row -- the Add of the reference's worker, which sends one summed row per key -- with the
        deterministic segment sum (ops.wd_emb_backward), straight into the push dtype (bf16 rows
        at several GPU ranks: no cast pass), then pushes them by add()."""
        dev = self.comm.device
        gdt = self.push_dtype if self.comm.world > 1 else getattr(self, "grad_dtype", torch.float32)
        grad_rows = (torch.empty if dev.type == "cuda" else torch.zeros)(max(plan.cap, 1), self.width, dtype=gdt,
                                                                         device=dev)
        ops.wd_emb_backward(dX, dwide, plan.inv, F, D, grad_rows, x_off=x_off, csr=plan.csr, sorted_rows=sorted_rows)
        self.add(plan, grad_rows)

    def add_keys(self, keys: torch.Tensor, vals: torch.Tensor):
        """Reference-style Add(keys, vals) (duplicates are summed)."""
        plan = self.plan(keys)
        vdt = getattr(self, "grad_dtype", torch.float32)
        g = torch.zeros(max(plan.cap, 1), self.width, dtype=vdt, device=self.comm.device)
        ops.scatter_add_rows(vals.reshape(keys.numel(), self.width).to(vdt).contiguous(), plan.inv, g)
        self.add(plan, g)

    @traced("sparse.clock")
    def clock(self):
        pending, self._pending = self._pending, []
        for plan, g in pending:
            self.pipe.keep_alive(g, plan.uniq, plan.recv_keys, plan.own_uniq, plan.own_inv, plan.U_dev,
                                 plan.own_U_dev, plan.own_slots)

        def work():
            for plan, grad_rows in pending:
                self._push(plan, grad_rows)

        self.pipe.run(work)

    @traced("sparse.push")
    def _push(self, plan: SparsePlan, grad_rows):
        dev = self.comm.device
        if self.comm.world == 1:
            keys, g, n_dev, n = plan.uniq, grad_rows, plan.U_dev, plan.cap
        else:
            M = len(plan.recv_keys)
            recv = torch.empty(M, self.width, dtype=self.push_dtype, device=dev)
            send = grad_rows[: plan.U]
            if send.dtype != self.push_dtype:
                send = send.to(self.push_dtype)
            self.comm.all_to_all_v(recv, send, plan.recv, plan.send, p2p=self.p2p)
            if M == 0:
                return
            if plan.extra.get("direct"):  # stamp + sum + row-wise Adagrad, no owner-side plan
                rs = self.__dict__.get("_rs")
                if rs is None and dev.type == "cuda":
                    rs = self._rs = torch.full((self._rows_alloc * self.comm.world * 2,), -1, dtype=torch.int32,
                                               device=dev)
                self._stamp = self.__dict__.get("_stamp", -1) + 1
                ops.owner_push_adagrad(self.shard, self.state, plan.recv_keys, self.base, recv, plan.recv, rs,
                                       self._stamp, self.lr, self.eps, state2=self.state2, split=self.split)
                return
            if plan.own_slots is not None:  # segment sums + row-wise Adagrad in one pass
                ops.owner_rows_adagrad(self.shard, self.state, plan.own_uniq, M, self.base, recv, plan.own_slots,
                                       len(plan.recv), self.lr, self.eps, state2=self.state2, split=self.split,
                                       n_dev=plan.own_U_dev)
                return
            n = plan.extra.get("own_U", M)
            g = torch.zeros(n, self.width, dtype=getattr(self, "grad_dtype", torch.float32), device=dev)
            ops.scatter_add_rows(recv, plan.own_inv, g)
            keys, n_dev = plan.own_uniq, (None if "own_U" in plan.extra else plan.own_U_dev)
        keys, base = self._owner_rows(keys[:n], plan)
        self._apply_rows(keys, base, g[:n], n_dev)

    def _apply_rows(self, keys, base, g, n_dev=None):
        if getattr(self, "value_dtype", None) == torch.bfloat16:
            self._applies += 1
            if self.optimizer not in ("rowwise_adagrad", "sgd", "add"):
                raise ValueError(self.optimizer)
            opt = "rowwise_adagrad" if self.optimizer == "rowwise_adagrad" else "add"
            scale = -self.lr if self.optimizer == "sgd" else 1.0
            ops.sparse_apply_bf16(opt, self.shard, self.state, keys, base, g.contiguous(), self.lr, self.eps, scale,
                                  state2=self.state2, split=self.split, step=self._applies, seed=self.seed, n_dev=n_dev)
            return
        if self.optimizer == "rowwise_adagrad":
            ops.sparse_rowwise_adagrad(self.shard, self.state, keys, base, g, self.lr, self.eps,
                                       state2=self.state2, split=self.split, n_dev=n_dev)
        elif self.optimizer == "sgd":
            ops.sparse_sgd(self.shard, keys, base, g.contiguous(), -self.lr, n_dev=n_dev)
        elif self.optimizer == "add":
            ops.sparse_sgd(self.shard, keys, base, g.contiguous(), 1.0, n_dev=n_dev)
        else:
            raise ValueError(self.optimizer)

    def drain(self):
        self.pipe.drain()
        self._check_keys()

    def reset_after_rollback(self):
        self.pipe.reset()
        self._pending = []

    # -- checkpoint hooks (minips_amd.ps.checkpoint) -------------------------------------------
    def shard_state(self):
        self.drain()
        arrays = {"params": self.shard}
        if self.state is not None:
            arrays["state"] = self.state
        if self.state2 is not None:
            arrays["state2"] = self.state2
        meta = dict(global_rows=self.num_rows, base=self.base, rows=self.rows_local, cols=self.width,
                    clock=self.pipe.clock, table_id=self.table_id, rank=self.comm.rank, world=self.comm.world,
                    kind="sparse")
        if self.value_dtype == torch.bfloat16:
            meta["applies"] = int(self._applies)  # the stochastic-rounding stream resumes where it was
        return meta, arrays

    def restore_meta(self, meta: dict):
        """Checkpoint meta of this rank's shard (ps/checkpoint.py, before the rows land): bf16 rows
        continue their stochastic-rounding stream instead of replaying steps 0, 1, ...."""
        if "applies" in meta:
            self._applies = int(meta["applies"])

    def restore_range(self):
        return self.base, self.base + self.rows_local

    def restore_dst(self):
        out = {"params": self.shard}
        if self.state is not None:
            out["state"] = self.state.view(-1, 1)
        if self.state2 is not None:
            out["state2"] = self.state2.view(-1, 1)
        return out

    def finish_restore(self, clock: int):
        self.pipe.clock = int(clock)


# ------------------------------------------------------------------------------------------------
MASK63 = (1 << 63) - 1
_M1, _M2 = 0x5BD1E9955BD1E995 & MASK63 | 1, 0x1B873593C2B2AE35 & MASK63 | 1


def mix63(k: torch.Tensor) -> torch.Tensor:
    """Bijection of [0, 2^63): xor-shifts and odd multiplies mod 2^63 (int64 arithmetic wraps mod
    2^64; the mask keeps 63 bits). Spreads arbitrary user keys evenly over the rank ranges."""
    x = k & MASK63
    x = x ^ (x >> 31)
    x = (x * _M1) & MASK63
    x = x ^ (x >> 29)
    x = (x * _M2) & MASK63
    x = x ^ (x >> 32)
    return x


class HashSparseTable(SparseTable):
    """Unbounded key space (reference MapStorage, server/map_storage.hpp): keys in [0, 2^63) are
    mixed by a bijection and range-partitioned over the ranks; each rank stores its keys in a GPU
    open-addressing hash table (csrc/kernels/hashtable.hip) whose rows are created on first
    touch -- zero (MapStorage's default-insert) or a deterministic per-key uniform init -- and
    grows (rehash, doubling) past 70% load. The Get/Add/Clock protocol is SparseTable's.

    No host sync on the hot path: the lookups take the dedupe's device-side unique count (the
    kernel resolves only that prefix), the growth check runs against a host-side upper bound of
    the size (inserts so far <= keys submitted) and reads the device counters only when that
    bound crosses the load limit, and the key-range check (keys < 2^63) and the table-full flag
    are read at those same sync points (or drain / size())."""

    _exact_counts = False

    def __init__(self, comm: Comm, width: int, capacity: int = 1 << 16, optimizer: str = "add", lr: float = 0.01,
                 eps: float = 1e-8, pull_dtype=torch.float32, consistency: str = "bsp", staleness: int = 0,
                 table_id: int = 0, init_std: float = 0.0, seed: int = 1234, p2p: bool | None = None,
                 push_dtype=None):
        self.comm = comm
        self.table_id = table_id
        self.push_dtype = push_dtype or torch.float32  # MapStorage values are exact sums: keep fp32
        self.num_rows = MASK63
        self.width = width
        self.optimizer, self.lr, self.eps = optimizer, lr, eps
        self.pull_dtype = pull_dtype
        self.split = None
        dev = comm.device
        b = even_bounds(MASK63, comm.world)
        self.bounds_list = b
        self.bounds = torch.tensor(b, dtype=torch.int64, device=dev)
        self.base = b[comm.rank]
        self.rows_local = 0
        self.init_scale = float(init_std) * math.sqrt(3.0)
        self.seed = int(seed)
        cap = 1 << max(4, int(capacity - 1).bit_length())
        self._alloc(cap)
        self.counters = torch.zeros(2, dtype=torch.int32, device=dev)
        self._size_ub = 0  # host-side upper bound of the occupied slots
        self._neg = None   # device flag: a negative (>= 2^63 unsigned) key was seen
        self._init_comm(consistency, staleness, p2p)

    def _alloc(self, cap: int):
        dev = self.comm.device
        self.capacity = cap
        self.tab_keys = torch.full((cap,), -1, dtype=torch.int64, device=dev)
        self.shard = torch.zeros(cap, self.width, dtype=torch.float32, device=dev)
        self.state = torch.zeros(cap, dtype=torch.float32, device=dev) if self.optimizer == "rowwise_adagrad" \
            else None
        self.state2 = None

    def _route_keys(self, keys):
        if keys.is_cuda:  # checked at the next sync point (no host round trip per batch)
            neg = (keys < 0).any()
            self._neg = neg if self._neg is None else (self._neg | neg)
        elif bool((keys < 0).any()):
            raise ValueError("HashSparseTable keys must be in [0, 2^63)")
        return mix63(keys)

    def _sync_counters(self) -> int:
        """One host read of the device counters (+ the deferred checks); returns the size."""
        size, full = (int(v) for v in self.counters.tolist())
        if self._neg is not None:
            neg, self._neg = bool(self._neg), None
            if neg:
                raise ValueError("HashSparseTable keys must be in [0, 2^63)")
        if full:
            raise RuntimeError("hash table full")
        self._size_ub = size
        return size

    def size(self) -> int:
        return self._sync_counters()

    def _slots(self, keys: torch.Tensor, grow: bool = True, n_dev=None) -> torch.Tensor:
        """Lookup-or-insert of keys[:n_dev] (n_dev: device count, None = all). ``grow=False``:
        the keys are known to be present (no insert, no growth check) -- safe inside side-stream
        clock work."""
        need = keys.numel()
        if need == 0:
            return torch.empty(0, dtype=torch.int64, device=keys.device)
        if grow:
            if self._size_ub + need > 0.7 * self.capacity and self._sync_counters() + need > 0.7 * self.capacity:
                self._grow(max(self.capacity * 2, 1 << int(math.ceil(math.log2((self._size_ub + need) / 0.5)))))
            self._size_ub += need
        slots = torch.empty(need, dtype=torch.int64, device=keys.device)
        ops.hash_slots(self.tab_keys, keys, slots, self.shard, self.init_scale, self.seed, self.counters, n_dev=n_dev)
        return slots

    def _grow(self, new_cap: int):
        # The rehash copies the rows on the current stream: every clock issued so far (SSP/ASP
        # applies on the pipe stream write into the current rows) must land first, and the old
        # buffers stay reserved for the streams that used them (lost updates / reuse).
        self.pipe.drain()
        old = (self.tab_keys, self.shard, self.state)
        self._alloc(new_cap)
        cnt = torch.zeros(2, dtype=torch.int32, device=self.comm.device)
        ops.hash_rehash(old[0], old[1], old[2], self.tab_keys, self.shard, self.state, cnt)
        self.counters[0] = cnt[0]
        self.counters[1] = 0
        if self.pipe.stream is not None:
            for t in old:
                if t is not None:
                    t.record_stream(self.pipe.stream)

    def _own_n_dev(self, plan):
        """Device count of the valid owned unique keys of ``plan`` (None: all are valid)."""
        if plan is None:
            return None
        if self.comm.world == 1:
            return plan.U_dev
        return None if "own_U" in plan.extra else plan.own_U_dev

    def _serve_index(self, plan):
        # insert-on-miss: unseen keys get their initial row (one rank: the unique prefix only)
        slots = self._slots(plan.recv_keys, n_dev=plan.U_dev if self.comm.world == 1 else None)
        plan.extra["served_slots"] = slots
        plan.extra["served_cap"] = self.capacity
        return self.shard, slots, 0

    @traced("hash.add")
    def add(self, plan: SparsePlan, grad_rows: torch.Tensor):
        """Resolve (insert-on-miss) the owner slots NOW, on the issuing stream: the clock's apply
        may run on the pipe stream, where a table growth must never happen."""
        keys = self._owner_keys(plan)
        if keys is not None and "own_slots" not in plan.extra:
            served = plan.extra.get("served_slots")
            if served is not None and self.comm.world == 1 and plan.extra.get("served_cap") == self.capacity:
                plan.extra["own_slots"] = served  # one rank: the pushed keys ARE the served keys
            else:
                # keys served by this plan's Get are present already: a lookup, no growth check
                plan.extra["own_slots"] = self._slots(keys, grow=served is None, n_dev=self._own_n_dev(plan))
            plan.extra["own_cap"] = self.capacity
        super().add(plan, grad_rows)

    def _owner_rows(self, keys, plan=None):
        slots = plan.extra.get("own_slots") if plan is not None else None
        if slots is None or self.capacity != plan.extra.get("own_cap"):
            # the table grew after add() (a rehash moves rows): the keys are present, so a
            # lookup-only probe re-resolves them without any growth on this stream
            slots = self._slots(keys, grow=False, n_dev=self._own_n_dev(plan))
        return slots, 0

    def drain(self):
        super().drain()
        if self.counters.is_cuda:
            self._sync_counters()  # surface a deferred key-range / table-full error

    # -- checkpoint hooks: (key, row, state) triples of the occupied slots, sorted by key ------
    def shard_state(self):
        """Sorted by (mixed) key, so a restore at any world size finds its key range by binary
        search in the file instead of reading every rank's whole table."""
        self.drain()
        occ = (self.tab_keys >= 0).nonzero().squeeze(1)
        keys, order = torch.sort(self.tab_keys[occ])
        slots = occ[order]
        arrays = {"keys": keys.view(-1, 1), "params": self.shard[slots]}
        if self.state is not None:
            arrays["state"] = self.state[slots].view(-1, 1)
        meta = dict(global_rows=MASK63, base=0, rows=int(keys.numel()), cols=self.width, clock=self.pipe.clock,
                    table_id=self.table_id, rank=self.comm.rank, world=self.comm.world, kind="hash")
        return meta, arrays

    def restore_range(self):
        return self.bounds_list[self.comm.rank], self.bounds_list[self.comm.rank + 1]

    def restore_insert(self, chunk: dict):
        """Insert checkpointed (key, params, state) rows of this rank's key range."""
        keys = chunk["keys"].reshape(-1)
        slots = self._slots(keys)
        self.shard[slots] = chunk["params"].to(self.shard.dtype)
        if self.state is not None and "state" in chunk:
            self.state[slots] = chunk["state"].reshape(-1).to(self.state.dtype)

    def finish_restore(self, clock: int):
        self.pipe.clock = int(clock)
