"""Look-ahead batch feeder shared by bench.py, the training driver and the schedule tests.

A batch is generated ``depth`` steps ahead, like a prefetching data loader, and ON the planning
stream, so its generation and key routing (dedupe + count all-to-all, SparseTable.plan_async)
run beside the current step; planning reads no table state, so issuing it early changes no
consistency semantics. The compute stream waits for a batch's event before using it.

On the CPU (gloo tests) the same calls run inline at the same issue points, so a CPU run
issues exactly the collective sequence of a GPU run (ps/comm.py, ordering contract).
"""
from __future__ import annotations

import collections

import torch

from ..utils import streams
from ..utils.metrics import traced


def default_depth(world: int) -> int:
    # several ranks: 3 -- the one host wait of a step (a plan's all-to-all split sizes) lands on
    # counts issued two steps earlier: 8 emulated ranks 0.467 vs 0.494-0.502 ms/step at depth 2
    # (depth 4: 0.467-0.470; profiles/r5/ab_lookahead.txt); one rank: the planning starts mid-step
    # (plan_wait below), so its batch is planned two steps ahead (3: 0.358 either way).
    # LookaheadFeeder(depth=...) / bench.py --lookahead override it.
    return 3 if world > 1 else 2


class LookaheadFeeder:
    """``fence`` (default on): after each step the planning stream waits for
    the compute stream (one event per step). Everything the planning stream hands to a step --
    the batch and its key plan -- is then safe to recycle from the planning stream once the step
    is issued, so neither needs ``record_stream`` (an allocator event per tensor on the compute
    stream when it is freed: ~30 us per W&D step for the ~10 tensors). The planning work of later
    batches is issued after the fence anyway, so no overlap is lost."""

    def __init__(self, model, data, comm, depth: int | None = None, fence: bool | None = None):
        self.model, self.data, self.comm = model, data, comm
        self.cuda = comm.device.type == "cuda"
        self.plan_stream = comm.plan_stream() if self.cuda else None
        self.main = torch.cuda.current_stream(comm.device) if self.cuda else None
        self.depth = depth or default_depth(comm.world)
        if fence is None:
            fence = True
        self.fence = bool(fence and self.cuda)
        if self.fence:
            model._fenced = True
        # the look-ahead planning (batch generation, key sort, CSR) waits for the point of the step
        # where the model issues it (WideDeep: after the dgrad chain), so its ~120 us of kernels run
        # beside the memory-bound embedding backward instead of squeezing the forward GEMMs (a
        # 256x256-tile GEMM that loses the 26 CUs of the per-column sort runs a second round of
        # tiles): one rank 0.351-0.352 vs 0.368 ms/step at depth 2; 8 emulated ranks at depth 3
        # 0.428-0.433 vs 0.463-0.506 (profiles/r5/ab_plan_wait.txt; at depth 2 the next plan's count
        # exchange waited instead: 0.575-0.586 vs 0.500-0.505)
        self.plan_wait = self.fence
        # batch-ready and fence events: reused from rings (a wait binds to the record before it;
        # each event's wait is issued within depth + 1 steps of its record)
        if self.cuda:
            from ..utils.streams import EventRing

            self._evring = EventRing(2 * self.depth + 4, fast=streams.fast_for("plan"))
            self._fence_ring = EventRing(8, fast=streams.fast_for("plan"))
        self.queue = collections.deque(self._produce() for _ in range(self.depth))
        for (_, k, _), _ev in list(self.queue)[1:]:
            model.prefetch(k, keys_on_plan_stream=self.cuda)

    @traced("feeder.produce")
    def _produce(self):
        if not self.cuda:
            return self.data.next(), None
        with streams.use(self.plan_stream):
            b = self.data.next()
            ev = self._evring.next()
            ev.record(self.plan_stream)
        if not self.fence:
            for t in b:
                t.record_stream(self.main)
        return b, ev

    @traced("feeder.step")
    def step(self):
        (dense, keys, labels), ev = self.queue.popleft()
        # the batch was generated on the planning stream before its key plan: a step whose plan
        # was prefetched waits on the plan's event before it touches the batch (SparseTable.get),
        # so the batch event is only needed when the step plans the keys itself
        planned = self.fence and any(k is keys for k, _ in getattr(self.model, "_pending_plans", ()))
        if ev is not None and not planned:
            self.main.wait_event(ev)

        def next_keys():  # called by train_step where it issues the look-ahead planning
            if self.plan_wait:  # the planning work starts on the GPU at this point of the step
                ev = self._fence_ring.next()
                ev.record(self.main)
                self.plan_stream.wait_event(ev)
            self.queue.append(self._produce())
            return self.queue[-1][0][1]

        loss = self.model.train_step(dense, keys, labels, next_keys=next_keys, next_on_plan_stream=self.cuda)
        if self.fence:  # the planning stream's later work (and buffer reuse) follows this step
            ev = self._fence_ring.next()
            ev.record(self.main)
            self.plan_stream.wait_event(ev)
        return loss


class LookaheadPlans:
    """Mixin of the recommendation models (WideDeep, DLRM): key plans issued ahead of the step
    that uses them (``self.emb`` is the SparseTable). A plan goes through three issue points,
    each placed so that the rank's single ordered communicator (ps/comm.py) never holds a
    look-ahead collective in front of the current step's own exchanges:

      prefetch (step n-d, planning stream)   dedupe + owner bucketing, no collective
      end of step n-d                        all-to-all of the per-owner counts
      end of step n-d+1 (d >= 2)             host reads the counts (issued a step earlier: no
                                             wait on the current step), all-to-all of the keys
                                             + owner-side dedupe
      step n                                 row gather + row exchange only

    With depth 1 the last two halves run at the start of step n (SparseTable._finish_plan)."""

    def prefetch(self, keys, keys_on_plan_stream: bool = False):
        """Start routing a future batch's keys on the planning stream; train_step picks the
        plan up when that batch comes (a batch may be several steps ahead: data-loader depth).
        A model driven by a fencing LookaheadFeeder (``_fenced``) skips the per-tensor stream
        bookkeeping of the plan (SparseTable.plan_async ``fenced``)."""
        pend = self.__dict__.setdefault("_pending_plans", [])
        pend.append([keys, self.emb.plan_async(keys, csr=True, keys_on_plan_stream=keys_on_plan_stream,
                                               fenced=self.__dict__.get("_fenced", False))])

    def _take_plan(self, keys):
        pend = self.__dict__.setdefault("_pending_plans", [])
        for i, (k, pp) in enumerate(pend):
            if k is keys:
                del pend[: i + 1]  # older entries were never consumed: drop them
                return pp
        return self.emb.plan(keys, csr=True)

    def _advance_next_plan(self):
        """The step is issued: run the prefetched plans' collectives now, after this step's own
        row exchanges and clocks (SparseTable.advance_plan): the older plans exchange their keys,
        the newest one (planned by this very step) only its counts."""
        pend = self.__dict__.get("_pending_plans") or []
        # (finishing only the next step's plan -- its counts then two steps old -- measured slower:
        # its key exchange then lands right before its consumer, 0.555-0.595 vs 0.439-0.511 ms at 8
        # emulated ranks, profiles/r5/ab_lookahead.txt)
        for e in pend[:-1]:
            e[1] = self.emb.advance_plan(e[1], finish=True)
        if pend:
            pend[-1][1] = self.emb.advance_plan(pend[-1][1], finish=False)
