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
    def __init__(self, path: str, rank: int = 0, world: int = 1, threads: int = 4, one_based: bool = True,
                 assigner: str = "", host: str = ""):
        # path: local / webhdfs:// / hdfs:// (csrc/runtime/fs.h); assigner "host:port": blocks come
        # from the locality-aware BlockAssignerServer instead of the static rank partition
        rowptr, cols, vals, labels = runtime().load_libsvm(path, rank, world, threads, one_based, assigner=assigner,
                                                           host=host)
        self.rowptr = torch.from_numpy(rowptr)
        self.cols = torch.from_numpy(cols)
        self.vals = torch.from_numpy(vals).float()
        self.labels = torch.from_numpy(labels).float()
        self.n = self.labels.numel()

    def __len__(self):
        return self.n

    def to(self, device) -> "LibsvmData":
        """Keep the whole shard resident in device memory (288 GB of HBM holds webspam/kdd12-sized
        shards many times over): batches are then cut on the GPU with no host work per step."""
        self._rp_host = self.rowptr.cpu()
        self.rowptr, self.cols, self.vals, self.labels = (t.to(device) for t in
                                                          (self.rowptr, self.cols, self.vals, self.labels))
        return self

    def _span(self, a: int, b: int):
        """Rows [a, b) (no wrap) as a contiguous CSR slice: no per-row work; the bounds come from a
        host copy of rowptr, so cutting a batch of HBM-resident data needs no device sync."""
        if not hasattr(self, "_rp_host"):
            self._rp_host = self.rowptr.cpu()
        lo, hi = int(self._rp_host[a]), int(self._rp_host[b])
        return self.rowptr[a: b + 1] - lo, lo, hi

    def batch(self, start: int, size: int):
        """CSR batch of rows start .. start+size (wrapping): consecutive samples from a start point as
        the reference sampler takes them (lib/batch_data_sampler.cpp:50-71), cut as at most two
        contiguous CSR slices (vectorised; runs where the data lives, host or HBM)."""
        n = max(self.n, 1)
        start %= n
        parts, rows_left, pos = [], size, start
        while rows_left > 0:
            take = min(rows_left, n - pos)
            parts.append((pos, pos + take))
            rows_left -= take
            pos = 0
        rps, cols, vals, labels, off = [], [], [], [], 0
        for a, b in parts:
            rp, lo, hi = self._span(a, b)
            rps.append((rp[1:] if rps else rp) + off)
            off = off + (hi - lo)
            cols.append(self.cols[lo:hi])
            vals.append(self.vals[lo:hi])
            labels.append(self.labels[a:b])
        if not parts:
            z = self.rowptr[:1] * 0
            return z, self.cols[:0], self.vals[:0], self.labels[:0]
        return torch.cat(rps), torch.cat(cols), torch.cat(vals), torch.cat(labels)

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
