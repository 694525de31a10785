"""File-backed data for the PS ranks and host->device prefetch.

LibsvmData       a rank's shard of libsvm files (path, directory or comma list), loaded by the
                 native block-assigner + mmap line reader (csrc/runtime/io.cc, one block queue per
                 rank, N loader threads) into CSR tensors; ``batches()`` walks it in consecutive
                 mini-batches from a random start point, wrapping (lib/batch_data_sampler.cpp:42-71)
PrefetchToDevice double-buffered host->device copies: a producer thread fills pinned host
                 buffers from any batch iterator while the GPU trains on the previous batch; the
                 copies run on a side HIP stream and the compute stream waits on their event.
"""
from __future__ import annotations

import queue
import threading

import torch

from .._native import runtime


class LibsvmData:
    def __init__(self, path: str, rank: int = 0, world: int = 1, threads: int = 4, one_based: bool = True):
        rowptr, cols, vals, labels = runtime().load_libsvm(path, rank, world, threads, one_based)
        self.rowptr = torch.from_numpy(rowptr)
        self.cols = torch.from_numpy(cols)
        self.vals = torch.from_numpy(vals).float()
        self.labels = torch.from_numpy(labels).float()
        self.n = self.labels.numel()

    def __len__(self):
        return self.n

    def batch(self, start: int, size: int):
        """CSR batch of rows start .. start+size (wrapping)."""
        idx = (torch.arange(size) + start) % max(self.n, 1)
        lens = self.rowptr[idx + 1] - self.rowptr[idx]
        rp = torch.zeros(size + 1, dtype=torch.int64)
        rp[1:] = torch.cumsum(lens, 0)
        gather = torch.cat([torch.arange(int(self.rowptr[i]), int(self.rowptr[i + 1])) for i in idx.tolist()]) \
            if size else torch.empty(0, dtype=torch.int64)
        return rp, self.cols[gather], self.vals[gather], self.labels[idx]

    def batches(self, size: int, seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        pos = int(torch.randint(0, max(self.n, 1), (1,), generator=g))
        while True:
            yield self.batch(pos, size)
            pos = (pos + size) % max(self.n, 1)


class PrefetchToDevice:
    def __init__(self, iterator, device, depth: int = 2):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self.q: queue.Queue = queue.Queue(maxsize=max(1, depth))
        self._it = iterator
        self._stop = False
        self._th = threading.Thread(target=self._produce, name="minips-prefetch", daemon=True)
        self._th.start()

    def _produce(self):
        try:
            for item in self._it:
                if self._stop:
                    return
                tensors = [t.pin_memory() if self.cuda else t for t in item]
                if self.cuda:
                    with torch.cuda.stream(self.stream):
                        dev = [t.to(self.device, non_blocking=True) for t in tensors]
                        ev = torch.cuda.Event()
                        ev.record(self.stream)
                else:
                    dev, ev = tensors, None
                self.q.put((dev, ev))
        except BaseException as e:  # surfaced on the consumer side
            self.q.put((e, None))
        self.q.put((None, None))

    def __iter__(self):
        return self

    def __next__(self):
        dev, ev = self.q.get()
        if dev is None:
            raise StopIteration
        if isinstance(dev, BaseException):
            raise dev
        if ev is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            for t in dev:
                t.record_stream(cur)
        return dev

    def close(self):
        self._stop = True
