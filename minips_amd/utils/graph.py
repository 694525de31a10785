"""HIP-graph capture of a static-shape training step (launch-bound models, e.g. the 3-layer MLP).

A step of a small model issues ~20 kernels of a few microseconds each, so the host (Python +
launch) is the bottleneck, not the GPU. ``GraphedStep`` captures one step into a HIP graph (via
``torch.cuda.CUDAGraph``, HIP graphs on ROCm) and replays it: one launch per step. Requirements,
met by the dense models on one rank: static shapes, inputs copied into fixed buffers, no host
syncs inside, and optimizer state that advances on the device (DenseTable keeps a device twin of
the Adam step, ``step_dev``, which a captured clock advances; it is set from the host step here).
Host-side bookkeeping that Python would have done per step (``DenseTable.step``,
the clock counter) is advanced by ``replay`` so checkpoints stay consistent.
"""
from __future__ import annotations

import torch


class GraphedStep:
    def __init__(self, fn, example_inputs, tables=(), warmup: int = 3):
        """fn(*inputs) -> outputs (tensors). The ``warmup`` steps are real training steps on
        ``example_inputs``; the captured step only runs on replay."""
        self.fn = fn
        self.tables = list(tables)
        self.static = [t.clone() for t in example_inputs]
        dev = self.static[0].device
        cur = torch.cuda.current_stream(dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(cur)
        with torch.cuda.stream(side):  # warm-up on a side stream (allocator pools settle)
            for _ in range(warmup):
                fn(*self.static)
        cur.wait_stream(side)
        for t in self.tables:
            if getattr(t, "pipe", None) is not None and t.pipe.async_:
                raise ValueError("GraphedStep needs synchronous clocks (a ring of gradient buffers "
                                 "would be frozen into the graph)")
        # capture records the step without running it: the host counters the Python step
        # advanced during capture are rolled back, so only the ``warmup`` steps count
        saved = [(t.step, t.pipe.clock) for t in self.tables]
        for t in self.tables:  # the captured clock advances the Adam step on the device
            if hasattr(t, "sync_step_dev"):
                t.sync_step_dev()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = fn(*self.static)
        for t, (st, ck) in zip(self.tables, saved):
            t.step, t.pipe.clock = st, ck

    def __call__(self, *inputs):
        for dst, src in zip(self.static, inputs):
            dst.copy_(src, non_blocking=True)
        self.graph.replay()
        for t in self.tables:  # the host-side counters a Python step would have advanced
            t.step = getattr(t, "step", 0) + 1
            t.pipe.clock += 1
        return self.out
