"""Checkpoint / resume of the GPU parameter-server tables.

Every checkpoint goes to ``<prefix>iter_<k>/`` and becomes the restore point only when it is
committed: after every rank finished writing, a barrier, then rank 0 atomically rewrites
``<prefix>latest`` (= k) and drops older iteration directories. A failure while a checkpoint is
still being written therefore restores the previous complete one, never a mix of iterations.
Files inside an iteration directory, one set per rank ``my_id``, keep the reference names and
text formats:

  server_params_<id>_t<table>.bin  binary sidecar (format v2, csrc/runtime/shard_io.h): header
                                   with per-array file offsets + fp32 shard + optimizer state
  server_params_<id>_t<table>      reference text format "<local_idx>:<val> " of the non-zero
                                   parameters (vector_storage.hpp:54-73), shards up to text_limit
                                   values (text_limit < 0: every shard; streamed from the same
                                   ring chunks as the binary file, so any size)
After a commit, ``<prefix>server_params_<id>`` / ``server_progress_<id>`` / ``worker_config_<id>``
(the reference's flat names; table k > 0 as ``..._t<k>``) link into the committed iteration.
  server_progress_<id>_t<table>    "min_clock:<c> <tid>:<c> ..." (progress_tracker.hpp:68-85),
                                   exact clocks (no RoundHundred), tids in SimpleIdMapper layout
  worker_config_<id>               "<worker_id>:<iteration> " (svm_dumper.hpp:51-66)

Consistent snapshot, bounded host memory (sized for a 10B-row table: ~85 GB of shard per rank)
---------------------------------------------------------------------------------------------
The reference dumps from the server thread, so no Add races the dump (ssp_model.cpp:112-125).
Here the shard must not change between the start and the end of its device -> host copy:
  * shard <= ``ring_bytes`` (default 1 GiB): D2H into pinned staging on the checkpoint stream;
    the compute stream waits for that copy (only), then the files are written in the background.
  * larger, and HBM has room for a copy: a device-side snapshot (D2D clone, ~3 TB/s); the
    compute stream waits for the clone only; the background writer streams the snapshot through
    a pinned ring of ``ring_bytes`` (two slots, D2H of chunk i+1 overlapping pwrite of chunk i).
  * larger, no HBM headroom: the same ring streaming from the live shard, in the foreground
    (training waits, like the reference's synchronous dump).
Host staging never exceeds ``ring_bytes`` (``peak_staging_bytes`` records it).

Restore reads the header of every file of a table (a few hundred bytes) and preads exactly the
rows of the global range this rank owns (hash tables: keys are stored sorted, the owned key
range is found by binary search), so an N -> M reshard reads every payload byte once in total.
The reference defects are fixed: text restore parses its own format, BSP/ASP tables checkpoint
(no hang), one file per table.
"""
from __future__ import annotations

import glob
import json
import os
import threading
import time

import numpy as np
import torch

from .._native import runtime
from ..utils.metrics import get_logger
from .fault import slow_io_delay, slow_pause_delay

_DT = {torch.float32: "float32", torch.bfloat16: "bfloat16", torch.float64: "float64", torch.int64: "int64",
       torch.int32: "int32"}
_TD = {v: k for k, v in _DT.items()}
WORKER_TID_OFFSET = 100  # SimpleIdMapper: workers of node n are n*1000 + [100, 1000)
_RING_DEFAULT = int(os.environ.get("MINIPS_CKPT_RING_MB", "1024")) << 20


_FIXED_META = ("global_rows", "base", "rows", "cols", "clock", "table_id", "rank", "world", "kind")

def _prefix_path(prefix: str, name: str) -> str:
    return prefix + name


def _as2d(t: torch.Tensor) -> torch.Tensor:
    if t.dim() == 0:
        return t.reshape(1, 1)
    if t.dim() == 1:
        return t.reshape(-1, 1)
    return t.reshape(t.shape[0], -1) if t.numel() else t.reshape(t.shape[0], max(1, int(np.prod(t.shape[1:]))))


class Checkpointer:
    def __init__(self, comm, prefix: str, my_id: int | None = None, text_limit: int = 1 << 22,
                 ring_bytes: int | None = None):
        self.comm = comm
        self.prefix = prefix
        self.my_id = comm.rank if my_id is None else my_id
        self.text_limit = text_limit  # write the reference text file when a shard has <= this many values
        self.ring_bytes = int(ring_bytes or _RING_DEFAULT)
        self.cuda = comm.device.type == "cuda"
        self._stream = torch.cuda.Stream(device=comm.device) if self.cuda else None
        self._host: dict = {}
        self._ring: list = []
        self._staging_now = 0
        self.peak_staging_bytes = 0
        self.last_mode = None
        self._thread: threading.Thread | None = None
        self._error: BaseException | None = None
        self._pending_iter: int | None = None
        self.last_seconds = 0.0
        self.keep = 2

    # ------------------------------------------------------------------------------ staging
    def _alloc_host(self, nbytes: int) -> torch.Tensor:
        t = torch.empty(nbytes, dtype=torch.uint8, pin_memory=self.cuda)
        self._staging_now += nbytes
        self.peak_staging_bytes = max(self.peak_staging_bytes, self._staging_now)
        return t

    def _release_staging(self):
        self._host.clear()
        self._ring = []
        self._staging_now = 0

    def _ring_slots(self, max_row_bytes: int):
        """Two pinned slots of ring_bytes / 2 each (at least one row of the widest array)."""
        slot = max(self.ring_bytes // 2, max_row_bytes)
        if not self._ring or self._ring[0].numel() < slot:
            self._ring = []
            self._ring = [self._alloc_host(slot) for _ in range(2)]
        return self._ring

    # ------------------------------------------------------------------------------ save
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
        # asynchronous tables: every rank drained its pushes (the all-gather above ordered that), so
        # every push so far is applied; the owners' server threads now stop until the snapshot is
        # taken (the reference SSPModel::Dump runs inside its server thread, ssp_model.cpp:112-125)
        paused = [t for t in tables.values() if hasattr(t, "snapshot_begin")]
        if paused:
            slow_pause_delay(self.comm.rank)  # fault injection (tests): a rank late to pause
        for t in paused:
            t.snapshot_begin()
        if paused:
            # every owner is paused before ANY rank resumes training: otherwise a fast rank could
            # push clock c + 1 into a slow owner that has not paused yet, its snapshot would hold
            # rows of c + 1 under meta clock c, and a restore would apply that push twice
            self.comm.store_barrier(f"ckpt_pause_{int(iteration)}")
        jobs = []
        for k, (tid, table) in enumerate(sorted(tables.items())):
            meta, arrays = table.shard_state()
            jobs.append((tid, meta, {n: _as2d(a) for n, a in arrays.items()}, allc[:, k].tolist()))
        total = sum(a.numel() * a.element_size() for _, _, arrs, _ in jobs for a in arrs.values())
        self._release_staging()
        mode = self._snapshot_mode(total)
        self.last_mode = mode
        cur = torch.cuda.current_stream(self.comm.device) if self.cuda else None
        if mode == "pinned":
            # whole shards fit the staging budget: one D2H per array on the checkpoint stream; the
            # compute stream waits for these copies before it can touch the shards again
            if self.cuda:
                self._stream.wait_stream(cur)
            staged = []
            for tid, meta, arrs, clk in jobs:
                host = {}
                for name, a in arrs.items():
                    h = self._alloc_host(a.numel() * a.element_size()).view(a.dtype).view(a.shape)
                    if self.cuda:
                        with torch.cuda.stream(self._stream):
                            h.copy_(a, non_blocking=True)
                    else:
                        h.copy_(a)
                    host[name] = h
                staged.append((tid, meta, host, clk))
            ev = None
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record(self._stream)
                cur.wait_event(ev)  # no Add/apply may run before the D2H copies finished
            jobs = staged
        elif mode == "device":
            self._stream.wait_stream(cur)
            snap = []
            with torch.cuda.stream(self._stream):
                for tid, meta, arrs, clk in jobs:
                    snap.append((tid, meta, {n: a.clone() for n, a in arrs.items()}, clk))
                ev = torch.cuda.Event()
                ev.record(self._stream)
            cur.wait_event(ev)  # the clone is the consistent image; training continues after it
            jobs = snap
        else:
            ev = None
            if self.cuda:
                self._stream.wait_stream(cur)

        if paused and mode != "stream":  # resume once the snapshot copies are complete
            if ev is not None:
                ev.synchronize()
            for t in paused:
                t.snapshot_end()
            paused = []

        def work():
            try:
                slow_io_delay(self.comm.rank)  # fault injection (tests): a slow checkpoint disk
                if ev is not None:
                    ev.synchronize()
                for tid, meta, arrs, clk in jobs:
                    self._write_table(out, tid, meta, arrs, host_ready=(mode == "pinned"))
                    self._write_progress(out, tid, clk)
                self._write_worker_config(out, iteration)
                self.last_seconds = time.perf_counter() - t0
                get_logger().event("checkpoint", iteration=iteration, seconds=round(self.last_seconds, 4),
                                   tables=len(jobs), prefix=self.prefix, mode=mode, bytes=int(total),
                                   peak_staging=int(self.peak_staging_bytes))
            except BaseException as e:  # surfaced by wait()
                self._error = e

        self._pending_iter = int(iteration)
        if mode == "stream":  # no room for a snapshot: write from the live shards, training waits
            try:
                work()
            finally:
                for t in paused:
                    t.snapshot_end()
            self._thread = None
            if self._error is not None:
                e, self._error = self._error, None
                raise e
        else:
            self._thread = threading.Thread(target=work, name="minips-ckpt", daemon=True)
            self._thread.start()
        if blocking:
            self.commit()

    def _snapshot_mode(self, total: int) -> str:
        if total <= self.ring_bytes:
            return "pinned"
        if self.cuda:
            free, _ = torch.cuda.mem_get_info(self.comm.device)
            if free > total + (2 << 30):
                return "device"
        return "stream"

    def _write_table(self, out: str, tid: int, meta: dict, arrs: dict, host_ready: bool):
        base = f"server_params_{self.my_id}_t{tid}"
        desc = [(n, _DT[a.dtype], a.shape[0], a.shape[1]) for n, a in arrs.items()]
        w = runtime().ShardFileWriter(_prefix_path(out, base + ".bin"), meta, desc)
        first = next(iter(arrs.values()), None)
        n_vals = first.numel() if first is not None else 0
        # the reference text file of the parameters, fed from the same chunks as the binary file
        # (no extra host copy, any shard size); text_limit < 0 writes it for every shard
        want_text = first is not None and meta["kind"] != "hash" and (self.text_limit < 0 or
                                                                       n_vals <= self.text_limit)
        text = runtime().TextParamsWriter(_prefix_path(out, base)) if want_text else None
        for k, (name, a) in enumerate(arrs.items()):
            tw = text if k == 0 else None
            if host_ready or not a.is_cuda:
                self._write_host_array(w, k, a, tw)
            else:
                self._stream_array(w, k, a, tw)
        w.close()
        if text is not None:
            text.close()
        extra = {k: v for k, v in meta.items() if k not in _FIXED_META}
        if extra:  # table state beyond the binary header (e.g. the bf16 rows' rounding stream)
            with open(_prefix_path(out, base + ".json"), "w") as f:
                json.dump(extra, f)

    def _write_host_array(self, w, k: int, a: torch.Tensor, text=None):
        """Host-resident array: written in ring-sized pieces (a CPU table streams through the ring
        so it never needs a second whole-shard host copy)."""
        if a.shape[0] == 0:
            return
        a = a.contiguous()
        rb = a.shape[1] * a.element_size()
        step = max(1, (self.ring_bytes // 2) // rb)
        for r0 in range(0, a.shape[0], step):
            n = min(step, a.shape[0] - r0)
            w.write_rows(k, r0, a[r0:].data_ptr(), n)
            if text is not None:
                text.append(a[r0:].data_ptr(), _DT[a.dtype], n, a.shape[1])

    def _stream_array(self, w, k: int, a: torch.Tensor, text=None):
        """Device array -> file through the two-slot pinned ring: the D2H of chunk i+1 runs on
        the checkpoint stream while chunk i is written."""
        rows = a.shape[0]
        if rows == 0:
            return
        rb = a.shape[1] * a.element_size()
        slots = self._ring_slots(rb)
        step = max(1, slots[0].numel() // rb)
        prev = None

        def put(p_r0, p_n, p_dst):
            w.write_rows(k, p_r0, p_dst.data_ptr(), p_n)
            if text is not None:
                text.append(p_dst.data_ptr(), _DT[a.dtype], p_n, a.shape[1])

        for i, r0 in enumerate(range(0, rows, step)):
            n = min(step, rows - r0)
            dst = slots[i % 2][: n * rb].view(a.dtype).view(n, a.shape[1])
            with torch.cuda.stream(self._stream):
                dst.copy_(a[r0: r0 + n], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._stream)
            if prev is not None:
                p_ev, p_r0, p_n, p_dst = prev
                p_ev.synchronize()
                put(p_r0, p_n, p_dst)
            prev = (ev, r0, n, dst)
        p_ev, p_r0, p_n, p_dst = prev
        p_ev.synchronize()
        put(p_r0, p_n, p_dst)

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
        self.comm.store_barrier("ckpt_commit")  # write times differ by rank: no PG timeout here
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
        self._link_reference_names(it)

    def _link_reference_names(self, it: int):
        """The reference's flat names (<prefix>server_params_<my_id>, server_progress_<my_id>,
        worker_config_<my_id>; vector_storage.hpp:54-73, progress_tracker.hpp:68-85,
        svm_dumper.hpp:51-66) as symlinks into the committed iteration: table 0 keeps the plain
        name, table k > 0 gets "_t<k>". Swapped atomically (symlink + rename), local prefixes only."""
        src = self.iter_dir(it)
        pdir = os.path.dirname(self.prefix) or "."
        names = [(f"worker_config_{self.my_id}", f"worker_config_{self.my_id}")]
        for f in sorted(glob.glob(glob.escape(src) + f"server_p*_{self.my_id}_t*")):
            name = os.path.basename(f)
            if name.endswith(".bin"):
                continue
            stem, tid = name.rsplit("_t", 1)
            names.append((name, stem if tid == "0" else name))
        for have, ref in names:
            target = os.path.join(src, have)
            if not os.path.exists(target):
                continue
            link = self.prefix + ref
            tmp = link + f".lnk{os.getpid()}"
            try:
                os.symlink(os.path.relpath(target, pdir), tmp)
                os.replace(tmp, link)
            except OSError:
                try:
                    os.unlink(tmp)
                except OSError:
                    pass

    def abandon(self):
        """In-place rollback: finish the local writer, drop the uncommitted checkpoint (its commit
        would be a collective on the broken group)."""
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        self._error = None
        self._pending_iter = None
        self._release_staging()

    def wait(self):
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        self._release_staging()
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
        """Restore every table from the latest committed checkpoint (or ``iteration``), reading
        only the rows this rank owns; returns the saved iteration."""
        it = self.latest() if iteration is None else int(iteration)
        if it is None:
            raise FileNotFoundError(f"no committed checkpoint under {self.prefix!r} (missing 'latest')")
        src = self.iter_dir(it)
        self._release_staging()
        for tid, table in sorted(tables.items()):
            files = sorted(glob.glob(glob.escape(src) + f"server_params_*_t{tid}.bin"))
            if not files:
                raise FileNotFoundError(f"no checkpoint shards for table {tid} under {src!r}")
            my_meta = table.shard_state()[0]
            heads = [runtime().read_shard_header(p) for p in files]
            clock = None
            for path, (meta, _) in zip(files, heads):
                if meta["global_rows"] != my_meta["global_rows"] or meta["cols"] != my_meta["cols"]:
                    raise ValueError(f"{path}: table shape {meta['global_rows']}x{meta['cols']} does not match "
                                     f"{my_meta['global_rows']}x{my_meta['cols']}")
                if meta["rank"] == self.my_id or clock is None:
                    clock = meta["clock"]
            lo, hi = table.restore_range()
            if my_meta["kind"] == "hash":
                for path, (meta, arrays) in zip(files, heads):
                    self._load_hash_file(table, path, meta, arrays, lo, hi)
            else:
                dst = table.restore_dst()
                for path, (meta, arrays) in zip(files, heads):
                    a, b = max(lo, meta["base"]), min(hi, meta["base"] + meta["rows"])
                    if a >= b:
                        continue  # nothing of this file is ours: not a byte read
                    for name, dt, rows, cols, off in arrays:
                        d = dst.get(name)
                        if d is not None:
                            self._read_rows_into(path, off, _TD[dt], int(cols), a - meta["base"], b - a,
                                                 d[a - lo: b - lo])
            if hasattr(table, "restore_meta"):
                extras = []
                for path in files:
                    jp = path[: -len(".bin")] + ".json"
                    if os.path.exists(jp):
                        with open(jp) as f:
                            extras.append((f"server_params_{self.my_id}_t{tid}.bin" in path, json.load(f)))
                if extras:  # this rank's own entry, else (a rescaled restore) the first one
                    table.restore_meta(next((e for mine, e in extras if mine), extras[0][1]))
            table.finish_restore(clock or 0)
        self._release_staging()
        slow_io_delay(self.comm.rank)  # fault injection (tests): a rank whose restore reads are slow
        # restore times differ by rank (owner-range reads): meet on a long-timeout host barrier
        # before the next collective can start its PG timeout
        self.comm.store_barrier("restore")
        cfg_path = _prefix_path(src, f"worker_config_{self.my_id}")
        if os.path.exists(cfg_path):
            cfg = runtime().load_config_data(cfg_path)
            it = int(cfg.get(int(self.comm.rank), it))
        get_logger().event("restore", iteration=it, prefix=self.prefix, tables=len(tables),
                           bytes_read=int(runtime().shard_bytes_read()))
        return it

    def _read_rows_into(self, path, off, dtype, cols, r0, n, dst: torch.Tensor):
        """pread rows [r0, r0+n) into dst ([n, cols] view on the table's device) through the ring."""
        esz = torch.empty(0, dtype=dtype).element_size()
        rb = cols * esz
        slots = self._ring_slots(rb)
        step = max(1, slots[0].numel() // rb)
        for i, s in enumerate(range(0, n, step)):
            m = min(step, n - s)
            host = slots[i % 2][: m * rb]
            runtime().read_rows(path, int(off), rb, int(r0 + s), m, host.data_ptr())
            src = host.view(dtype).view(m, cols)
            d = dst[s: s + m]
            d.copy_(src.reshape(d.shape).to(d.dtype))  # synchronous: the slot is reused next round

    def _load_hash_file(self, table, path, meta, arrays, lo, hi):
        """Hash shards store their (mixed) keys sorted: binary-search the owned key range [lo, hi)
        and stream only those rows."""
        desc = {name: (dt, int(rows), int(cols), int(off)) for name, dt, rows, cols, off in arrays}
        kdt, nrows, _, koff = desc["keys"]
        probe = np.empty(1, dtype=np.int64)

        def lower_bound(key):
            a, b = 0, nrows
            while a < b:
                mid = (a + b) // 2
                runtime().read_rows(path, koff, 8, mid, 1, probe.ctypes.data)
                if int(probe[0]) < key:
                    a = mid + 1
                else:
                    b = mid
            return a

        i0, i1 = lower_bound(lo), lower_bound(hi)
        if i0 >= i1:
            return
        width = max(desc[n][2] for n in desc) * 8
        step = max(1, (self.ring_bytes // 4) // width)
        for s in range(i0, i1, step):
            m = min(step, i1 - s)
            chunk = {}
            for name, (dt, _, cols, off) in desc.items():
                t = torch.empty(m, cols, dtype=_TD[dt], device=self.comm.device)
                self._read_rows_into(path, off, _TD[dt], cols, s, m, t)
                chunk[name] = t
            table.restore_insert(chunk)


def load_text_params(path: str, n: int) -> torch.Tensor:
    """Reader of the reference text format (correct, unlike vector_storage.hpp:75-90)."""
    return torch.from_numpy(runtime().read_text_params(path, n))


def parse_progress(path: str) -> dict:
    out = {}
    for tok in open(path).read().split():
        k, v = tok.split(":")
        out[k if k == "min_clock" else int(k)] = int(v)
    return out
