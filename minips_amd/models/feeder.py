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
import os

import torch

from ..utils import streams
from ..utils.metrics import traced


def default_depth(world: int) -> int:
    # one rank: depth 1 (measured neutral, 1/2/3 within 0.522-0.530 ms/step); several ranks: 2,
    # so the one host wait of a step (a plan's all-to-all split sizes) lands on counts issued a
    # whole step earlier
    return max(1, int(os.environ.get("MINIPS_LOOKAHEAD", "2" if world > 1 else "1")))


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
        # batch-ready and fence events: reused from rings (a wait binds to the record before it;
        # each event's wait is issued within depth + 1 steps of its record)
        if self.cuda:
            from ..utils.streams import EventRing

            self._evring = EventRing(2 * self.depth + 4, fast=streams.fast_for("plan"))
            self._fence_ring = EventRing(4, fast=streams.fast_for("plan"))
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
        for e in pend[:-1]:
            e[1] = self.emb.advance_plan(e[1], finish=True)
        if pend:
            pend[-1][1] = self.emb.advance_plan(pend[-1][1], finish=False)


def _batch_plan_tensors(batch, pp) -> list:
    """The device tensors one step hands to the next: the look-ahead batch and its pending key
    plan (deduplicated by storage: the flat key view aliases the batch keys)."""
    out, seen = [], set()
    for t in (*batch, pp.flat, pp.uniq, pp.inv, pp.counts, pp.U_dev, *(pp.csr or ())):
        if t is None or t.data_ptr() in seen:
            continue
        seen.add(t.data_ptr())
        out.append(t)
    return out


class GraphedFeeder:
    """One rank's whole training step -- next batch generation and key planning on the planning
    stream, sparse Get, forward, backward (weight gradients on the side stream), Add, Clock --
    captured into ONE HIP graph and replayed (torch.cuda.CUDAGraph = hipGraph on ROCm). This
    removes the host issue cost (~0.37 ms of Python + launches per step) from the critical path.

    Why a one-rank step is capturable: every size is static (buffers sized by the batch, unique
    counts kept on the device and consumed by n_dev-bounded kernels), the Adam step and the data
    generator's counter advance on the device, and nothing syncs with the host. The step consumes
    the batch + plan produced by the previous step: the captured step copies the batch + plan it
    produced into those static input slots at its end (after every reader joined), so the graph
    replays in a closed loop. Host-side clocks (checkpoint metadata) advance per replay."""

    def __init__(self, feeder: LookaheadFeeder, tables=()):
        f = feeder
        if not (f.cuda and f.comm.world == 1 and f.depth == 1):
            raise ValueError("GraphedFeeder: one rank on a GPU with look-ahead depth 1")
        for t in tables:
            if getattr(t, "pipe", None) is not None and t.pipe.async_:
                raise ValueError("GraphedFeeder needs synchronous clocks")
        self.f, self.tables = f, list(tables)
        torch.cuda.synchronize(f.comm.device)
        # an eager step may leave its side-stream tail for the next step to wait on (WideDeep's
        # _side_pending); it is complete now, and a capture must not wait on events from outside it
        f.model.__dict__.pop("_side_pending", None)
        batch, _ev = f.queue[0]
        pend = f.model._pending_plans
        if len(pend) != 1 or pend[0][0] is not batch[1]:
            raise ValueError("GraphedFeeder: expected exactly the next batch's pending plan")
        pp = pend[0][1]
        pp.event = None  # already complete; a capture must not wait on an event recorded outside it
        f.queue[0] = (batch, None)
        static = _batch_plan_tensors(batch, pp)
        saved = [(getattr(t, "step", None), t.pipe.clock) for t in self.tables]
        # device twins of the host counters (Adam step, data draw): eager steps leave them alone,
        # the captured step advances them on the device
        for t in self.tables:
            if hasattr(t, "sync_step_dev"):
                t.sync_step_dev()
        if hasattr(f.data, "graph_prepare"):
            f.data.graph_prepare()
        saved_draws = getattr(f.data, "_host_step", None)
        self.graph = torch.cuda.CUDAGraph()
        main, ps = f.main, f.plan_stream
        with torch.cuda.graph(self.graph, stream=main):
            ps.wait_stream(main)  # fork: the planning stream's work joins the capture
            self.loss = f.step()
            main.wait_stream(ps)  # join before the static slots are overwritten
            (nb, _), = f.queue
            npp = pend[-1][1]
            produced = _batch_plan_tensors(nb, npp)
            if [(t.shape, t.dtype) for t in produced] != [(t.shape, t.dtype) for t in static]:
                raise RuntimeError("GraphedFeeder: the step's batch/plan layout is not static")
            # one launch for every slot (11 separate copy nodes cost ~110 us of dispatch gaps)
            pairs = [(d, s) for d, s in zip(static, produced) if d.numel()]
            if pairs and all(d.is_contiguous() and s.is_contiguous() for d, s in pairs):
                from .._native import kernels

                kernels().multi_copy([d for d, _ in pairs], [s for _, s in pairs])
            else:
                for dst, src in pairs:
                    dst.copy_(src)
        # the capture ran nothing: restore the host view (static batch + plan are the next input)
        f.queue.clear()
        f.queue.append((batch, None))
        pend[:] = [[batch[1], pp]]
        for t, (st, ck) in zip(self.tables, saved):
            if st is not None:
                t.step = st
            t.pipe.clock = ck
        if saved_draws is not None:
            f.data._host_step = saved_draws

    def step(self):
        self.graph.replay()
        for t in self.tables:  # the host-side counters an eager step advances
            if hasattr(t, "step"):
                t.step += 1
            t.pipe.clock += 1
        if hasattr(self.f.data, "graph_replayed"):
            self.f.data.graph_replayed(1)
        return self.loss
