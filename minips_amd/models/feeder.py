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


def default_depth(world: int) -> int:
    # one rank: depth 1 (measured neutral, 1/2/3 within 0.522-0.530 ms/step); several ranks: 2,
    # so the one host wait of a step (a plan's all-to-all split sizes) lands on counts issued a
    # whole step earlier
    return max(1, int(os.environ.get("MINIPS_LOOKAHEAD", "2" if world > 1 else "1")))


class LookaheadFeeder:
    def __init__(self, model, data, comm, depth: int | None = None):
        self.model, self.data, self.comm = model, data, comm
        self.cuda = comm.device.type == "cuda"
        self.plan_stream = comm.plan_stream() if self.cuda else None
        self.main = torch.cuda.current_stream(comm.device) if self.cuda else None
        self.depth = depth or default_depth(comm.world)
        self.queue = collections.deque(self._produce() for _ in range(self.depth))
        for (_, k, _), _ev in list(self.queue)[1:]:
            model.prefetch(k, keys_on_plan_stream=self.cuda)

    def _produce(self):
        if not self.cuda:
            return self.data.next(), None
        with torch.cuda.stream(self.plan_stream):
            b = self.data.next()
            ev = torch.cuda.Event()
            ev.record(self.plan_stream)
        for t in b:
            t.record_stream(self.main)
        return b, ev

    def step(self):
        (dense, keys, labels), ev = self.queue.popleft()
        if ev is not None:
            self.main.wait_event(ev)

        def next_keys():  # called by train_step where it issues the look-ahead planning
            self.queue.append(self._produce())
            return self.queue[-1][0][1]

        return self.model.train_step(dense, keys, labels, next_keys=next_keys, next_on_plan_stream=self.cuda)
