"""Checkpoint / resume of the GPU parameter-server tables.

Every checkpoint goes to ``<prefix>iter_<k>/`` and becomes the restore point only when it is
committed: after every rank finished writing, a barrier, then rank 0 atomically rewrites
``<prefix>latest`` (= k) and drops older iteration directories. A failure while a checkpoint is
still being written therefore restores the previous complete one, never a mix of iterations.
Files inside an iteration directory, one set per rank ``my_id``, keep the reference names and
text formats:

  server_params_<id>_t<table>.bin  binary sidecar: header + fp32 shard + optimizer state
                                   (native writer, csrc/runtime/shard_io.cc)
  server_params_<id>_t<table>      reference text format "<local_idx>:<val> " of the non-zero
                                   parameters (vector_storage.hpp:54-73), small tables only
  server_progress_<id>_t<table>    "min_clock:<c> <tid>:<c> ..." (progress_tracker.hpp:68-85),
                                   exact clocks (no RoundHundred), tids in SimpleIdMapper layout
  worker_config_<id>               "<worker_id>:<iteration> " (svm_dumper.hpp:51-66)

Saving is asynchronous: the shards are copied device -> pinned host on a side HIP stream, and a
background thread writes the files (the C++ writer releases the GIL), so training continues
while the checkpoint drains. ``wait()`` joins it. Loading reads every rank's sidecar of a table
and copies the overlap of each piece's global row range with the local shard, so a checkpoint
taken at one world size restores at another (elastic restart). The reference defects are fixed:
text restore parses its own format, BSP/ASP tables checkpoint (no hang), one file per table.
"""
from __future__ import annotations

import glob
import os
import threading
import time

import torch

from .._native import runtime
from ..utils.metrics import get_logger

_DT = {torch.float32: "float32", torch.bfloat16: "bfloat16", torch.float64: "float64", torch.int64: "int64",
       torch.int32: "int32"}
_TD = {v: k for k, v in _DT.items()}
WORKER_TID_OFFSET = 100  # SimpleIdMapper: workers of node n are n*1000 + [100, 1000)


def _prefix_path(prefix: str, name: str) -> str:
    return prefix + name


class Checkpointer:
    def __init__(self, comm, prefix: str, my_id: int | None = None, text_limit: int = 1 << 22):
        self.comm = comm
        self.prefix = prefix
        self.my_id = comm.rank if my_id is None else my_id
        self.text_limit = text_limit  # write the reference text file when a shard has <= this many values
        self._writer = runtime().ShardWriter()
        self._stream = torch.cuda.Stream(device=comm.device) if comm.device.type == "cuda" else None
        self._host: dict = {}
        self._thread: threading.Thread | None = None
        self._error: BaseException | None = None
        self._pending_iter: int | None = None
        self.last_seconds = 0.0
        self.keep = 2

    # ------------------------------------------------------------------------------ save
    def _staging(self, key, t: torch.Tensor) -> torch.Tensor:
        h = self._host.get(key)
        if h is None or h.shape != t.shape or h.dtype != t.dtype:
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=t.is_cuda)
            self._host[key] = h
        return h

    def iter_dir(self, iteration: int) -> str:
        return f"{self.prefix}iter_{int(iteration)}/"

    def save(self, tables: dict, iteration: int, blocking: bool = False):
        """Checkpoint every table ({table_id: table}) at ``iteration`` (collective: all ranks).
        The write drains in the background; ``commit()`` (collective) publishes it."""
        self.commit()
        t0 = time.perf_counter()
        out = self.iter_dir(iteration)
        for t in tables.values():
            t.drain()
        # every rank's clock of every table -> the progress files carry the whole tracker view
        clocks = torch.tensor([int(t.shard_state()[0]["clock"]) for t in tables.values()], dtype=torch.float64,
                              device=self.comm.device)
        allc = torch.empty(self.comm.world * clocks.numel(), dtype=torch.float64, device=self.comm.device)
        self.comm.all_gather(allc, clocks)
        allc = allc.view(self.comm.world, -1).cpu()
        jobs = []
        cur = torch.cuda.current_stream(self.comm.device) if self._stream is not None else None
        if self._stream is not None:
            self._stream.wait_stream(cur)
        for k, (tid, table) in enumerate(sorted(tables.items())):
            meta, arrays = table.shard_state()
            host = {}
            for name, dev in arrays.items():
                h = self._staging((tid, name), dev)
                if self._stream is not None:
                    with torch.cuda.stream(self._stream):
                        h.copy_(dev, non_blocking=True)
                        dev.record_stream(self._stream)
                else:
                    h.copy_(dev)
                host[name] = h
            jobs.append((tid, meta, host, allc[:, k].tolist()))
        ev = None
        if self._stream is not None:
            ev = torch.cuda.Event()
            ev.record(self._stream)

        def work():
            try:
                if ev is not None:
                    ev.synchronize()
                for tid, meta, host, clk in jobs:
                    base = f"server_params_{self.my_id}_t{tid}"
                    arrays = [(n, h.data_ptr(), _DT[h.dtype], h.shape[0] if h.dim() else 1,
                               h.shape[1] if h.dim() > 1 else 1) for n, h in host.items()]
                    n_vals = sum(h.numel() for h in host.values()) // max(1, len(host))
                    text = _prefix_path(out, base) if n_vals <= self.text_limit and meta["kind"] != "hash" else ""
                    self._writer.submit(_prefix_path(out, base + ".bin"), meta, arrays, text)
                    self._write_progress(out, tid, clk)
                self._write_worker_config(out, iteration)
                self._writer.wait_all()
                err = self._writer.take_error()
                if err:
                    raise RuntimeError(err)
                self.last_seconds = time.perf_counter() - t0
                get_logger().event("checkpoint", iteration=iteration, seconds=round(self.last_seconds, 4),
                                   tables=len(jobs), prefix=self.prefix)
            except BaseException as e:  # surfaced by wait()
                self._error = e

        self._thread = threading.Thread(target=work, name="minips-ckpt", daemon=True)
        self._thread.start()
        self._pending_iter = int(iteration)
        if blocking:
            self.commit()

    def try_commit(self) -> bool:
        """Publish the in-flight checkpoint if every rank's background writer has finished
        (collective: one tiny MIN all-reduce while a checkpoint is pending, nothing otherwise);
        training never blocks on the disk. Returns whether it was published."""
        if self._pending_iter is None:
            return False
        done = torch.tensor([0.0 if (self._thread is not None and self._thread.is_alive()) else 1.0],
                            device=self.comm.device)
        self.comm.all_reduce_(done, op=__import__("torch.distributed", fromlist=["ReduceOp"]).ReduceOp.MIN)
        if float(done.item()) < 1.0:
            return False
        self.commit()
        return True

    def commit(self):
        """Finish the in-flight checkpoint on every rank and publish it (collective)."""
        if self._pending_iter is None:
            return
        self.wait()
        self.comm.barrier()
        it, self._pending_iter = self._pending_iter, None
        if self.comm.rank == 0:
            tmp = self.prefix + "latest.tmp"
            with open(tmp, "w") as f:
                f.write(str(it))
            os.replace(tmp, self.prefix + "latest")
            # the prefix is a path prefix (reference style, e.g. "/ckpt/lr_"), not necessarily a
            # directory: list its directory and match "<basename>iter_<n>"
            pdir, stem = os.path.split(self.prefix)
            tag = stem + "iter_"
            done = sorted(int(d[len(tag):]) for d in os.listdir(pdir or ".")
                          if d.startswith(tag) and d[len(tag):].isdigit())
            for old in done[:-self.keep]:
                if old != it:
                    import shutil

                    shutil.rmtree(self.iter_dir(old), ignore_errors=True)
        self.comm.barrier()

    def wait(self):
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._error is not None:
            e, self._error = self._error, None
            raise e

    def _write_progress(self, out: str, tid: int, clocks: list):
        path = _prefix_path(out, f"server_progress_{self.my_id}_t{tid}")
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        parts = [f"min_clock:{int(min(clocks))}"]
        parts += [f"{r * 1000 + WORKER_TID_OFFSET}:{int(c)}" for r, c in enumerate(clocks)]
        with open(path, "w") as f:
            f.write(" ".join(parts) + " ")

    def _write_worker_config(self, out: str, iteration: int):
        path = _prefix_path(out, f"worker_config_{self.my_id}")
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        runtime().dump_config_data(path, {int(self.comm.rank): int(iteration)})

    # ------------------------------------------------------------------------------ load
    def latest(self) -> int | None:
        try:
            return int(open(self.prefix + "latest").read().strip())
        except (OSError, ValueError):
            return None

    def exists(self) -> bool:
        return self.latest() is not None

    def load(self, tables: dict, iteration: int | None = None) -> int:
        """Restore every table from the sidecars of all ranks of the latest committed checkpoint
        (or ``iteration``); returns the saved iteration."""
        it = self.latest() if iteration is None else int(iteration)
        if it is None:
            raise FileNotFoundError(f"no committed checkpoint under {self.prefix!r} (missing 'latest')")
        src = self.iter_dir(it)
        for tid, table in sorted(tables.items()):
            files = sorted(glob.glob(glob.escape(src) + f"server_params_*_t{tid}.bin"))
            if not files:
                raise FileNotFoundError(f"no checkpoint shards for table {tid} under {src!r}")
            pieces, clock = [], None
            my_meta = table.shard_state()[0]
            for path in files:
                meta, arrays = runtime().read_shard(path)
                if meta["global_rows"] != my_meta["global_rows"] or meta["cols"] != my_meta["cols"]:
                    raise ValueError(f"{path}: table shape {meta['global_rows']}x{meta['cols']} does not match "
                                     f"{my_meta['global_rows']}x{my_meta['cols']}")
                lo, hi = meta["base"], meta["base"] + meta["rows"]
                if meta["kind"] != "hash" and (hi <= my_meta["base"] or lo >= my_meta["base"] + my_meta["rows"]):
                    if meta["rank"] == self.my_id:
                        clock = meta["clock"]
                    continue
                tens = {}
                for name, dt, rows, cols, buf in arrays:
                    t = torch.frombuffer(buf, dtype=_TD[dt]) if len(buf) else torch.empty(0, dtype=_TD[dt])
                    tens[name] = t.view(int(rows), int(cols)).to(self.comm.device)
                pieces.append((meta, tens))
                if meta["rank"] == self.my_id or clock is None:
                    clock = meta["clock"]
            table.load_shard_pieces(pieces, clock or 0)
        cfg_path = _prefix_path(src, f"worker_config_{self.my_id}")
        if os.path.exists(cfg_path):
            cfg = runtime().load_config_data(cfg_path)
            it = int(cfg.get(int(self.comm.rank), it))
        get_logger().event("restore", iteration=it, prefix=self.prefix, tables=len(tables))
        return it


def load_text_params(path: str, n: int) -> torch.Tensor:
    """Reader of the reference text format (correct, unlike vector_storage.hpp:75-90)."""
    return torch.from_numpy(runtime().read_text_params(path, n))


def parse_progress(path: str) -> dict:
    out = {}
    for tok in open(path).read().split():
        k, v = tok.split(":")
        out[k if k == "min_clock" else int(k)] = int(v)
    return out

