"""Asynchronous SSP / ASP parameter server for GPU ranks: one-sided rows over xGMI and an
owner-side optimizer apply.

A collective rendezvous at every clock (all-to-all, reduce-scatter) makes every rank wait for the
slowest one, whatever the staleness setting. The reference's servers apply each Add as it arrives
(SSPModel::Add, server/consistency/ssp_model.cpp:54-56; ASPModel::Add, asp_model.cpp:18-21) with
the table's own update rule, answer a Get immediately (ASP, asp_model.cpp:23-26) or once the
slowest worker is within ``staleness`` clocks (SSP, ssp_model.cpp:58-85), and never make a worker
wait for a peer's pushes. These tables do the same with no collective on the data path:

* every rank hipMallocs its shard and an inbox and exports both (hipIpcGetMemHandle); every rank
  maps every peer's buffers (hipIpcOpenMemHandle, peer access over xGMI);
* Get  = ``ps_gather_rows``: the requested rows straight from the owners' HBM (16-byte loads);
* Add + Clock = ``ps_push_rows``: the requester writes its deduplicated (key, gradient row)
  batch, grouped by owner, into slot ``clock % depth`` of its ring in each owner's inbox (the
  per-owner row counts go into the slot headers on the device: no host round trip), then a
  native thread publishes ``sent`` on the PSBoard once those writes completed;
* the owner's AsyncServer thread (csrc/runtime/async_server.h) -- the ServerThread of
  server/server_thread.cpp -- sleeps on the board, applies every arrived slot with the table's
  optimizer and the OWNER's state (row-wise Adagrad, Adam, Adagrad, SGD or the reference's plain
  add; csrc/kernels/onesided.hip HipApplier) on its own high-priority stream, and publishes
  ``applied``;
* SSP tables with a stateful optimizer (row-wise Adagrad, Adam, Adagrad) on several ranks are served
  clock-coalesced (AsyncServer::SetCoalesce): the owner applies clock c once every requester
  sent it, as ONE optimizer step over the P pushes summed per key in requester order -- the BSP
  update of that clock. The reference's SSP server applies each Add on arrival as ``+=``
  (ssp_model.cpp:54-56), which is linear in the pushes; one scale-invariant Adagrad / Adam step
  per push is not (a key pushed by all 4 ranks moved up to ~2.8x a BSP step: the round-5 4-rank
  loss spike, profiles/r5/ssp_probe.txt). ASP keeps the per-arrival apply (asp_model.cpp:18-21);
* SSP gate (a Get at own clock c): every owner has applied every requester's clocks < c - s,
  i.e. min applied >= c - s (csrc/runtime/ps_board.h); ASP never waits (``asp_bound`` optionally
  bounds it the same way); a requester reuses an inbox slot only after every owner applied it;
* consistency of one-sided reads: each owner's applies of a batch run under its write lock and
  every Get / dense pull under the read locks of the owners (GPU: lock words in the owners'
  fine-grained HBM, csrc/kernels/onesided.hip; CPU: the board's lock lines), so a read never sees
  half of an owner's batch -- the reference's server thread serialises Add and Get the same way
  (server/server_thread.cpp:23-61). Dense pulls are lazy: an owner's shard is re-pulled only when
  the cached copy is older than the staleness bound allows;
* storage: range rows in fp32 or bf16 (stochastic rounding, the 10B-row DLRM table), or Map
  storage (AsyncHashTable: the owner's open-addressing table, insert on apply, a Get of an absent
  key reads 0 -- server/map_storage.hpp:13-26).

The same code runs on CPU ranks (gloo tests): shards and inboxes are /dev/shm files mapped by
every rank, the server thread is the same C++ loop calling back into the PyTorch reference
optimizers. Reference semantics kept: BSP stays on the collective tables (ps/tables.py).
"""
from __future__ import annotations

import collections
import contextlib
import os
import time
import uuid

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from .comm import Comm
from ..utils import streams
from ..utils.metrics import traced
from .tables import SparsePlan, SparseTable, _PendingPlan, column_spec, even_bounds, _route_multiplier

_MAX_TABLES = 16
_SLOT_HEADER = 64
# memory kind of the buffers peers read while their owner writes (shards, pull copies): 0
# coarse-grained + the explicit release (ps_write_unlock: every XCD's L2 written back) / acquire
# (the gathers' L2 invalidate) of onesided.hip, 1 fine-grained. Inboxes are always uncached, the
# lock lines always fine-grained.
_SHARD_MEM = 0
# inbox memory kind (default 2 uncached: the owner's apply reads what peers wrote, never an L2
# copy of the slot from `depth` clocks ago); PS_INBOX_MEM off is an A/B timing knob only
_INBOX_MEM = 2
_PUSH_STREAM = os.environ.get("MINIPS_PS_PUSH_STREAM", "0") == "1"
# clock-coalesced SSP applies need a (stamp, index) entry per owned row and requester: 8 * P bytes
# per row (W&D at 8 ranks: 34 MB per rank); above this many bytes a table falls back to applying
# push by push (the 10B-row DLRM table would need 80 GB per rank at 8 ranks -- it runs ASP)
_COALESCE_MAX_BYTES = 32 << 30
# PS_LOCKS off: no owner locks (A/B timing only: reads may see half of a batch)
_LOCKS = True


def _align(n: int, a: int) -> int:
    return (n + a - 1) // a * a


_OPT_CODES = {"add": 0, "sgd": 1, "rowwise_adagrad": 2, "adagrad": 3, "adam": 4}


class AsyncPS:
    """The asynchronous PS context of one rank (one per Comm): the shared progress board, the
    owner's server thread and the requester's clock publisher. Tables register in creation
    order, which is the same on every rank."""

    @classmethod
    def of(cls, comm: Comm) -> "AsyncPS":
        ps = getattr(comm, "_async_ps", None)
        if ps is None or ps.closed:
            ps = cls(comm)
            comm._async_ps = ps
        return ps

    def __init__(self, comm: Comm):
        from .._native import runtime

        self.comm = comm
        self.world, self.rank = comm.world, comm.rank
        self.cuda = comm.device.type == "cuda"
        name = f"minips_ps_{uuid.uuid4().hex[:16]}" if comm.rank == 0 else None
        if comm.world > 1:
            box = [name]
            dist.broadcast_object_list(box, src=0, group=comm.group)
            name = box[0]
        self.name = name
        self.board = runtime().PSBoard(name, self.world, self.rank, _MAX_TABLES)
        if self.cuda:
            from .._native import kernels

            k = kernels()
            # one rank: every owner is this device -- agent-scope ordering suffices, no system fences
            k.ps_set_fences(comm.world > 1)
            self.server = k.AsyncServer(name, self.world, self.rank, _MAX_TABLES, comm.device.index or 0)
            self._anchor = torch.zeros(1, device=comm.device)
            # the rank's error word (a device spin that timed out sets a bit) and the control lines
            # (one lock word per table) every rank maps from every owner
            self.err = k.HostWord()
            self.server.set_error_word(self.err.device_ptr)
            dev_i = comm.device.index or 0
            buf, handle = k.ipc_alloc(k.PS_CTRL_BYTES, dev_i, 1)
            handles = [None] * comm.world
            if comm.world > 1:
                dist.all_gather_object(handles, handle, group=comm.group)
            self.ctrl = [buf if r == comm.rank else k.ipc_open(handles[r], k.PS_CTRL_BYTES, dev_i)
                         for r in range(comm.world)]
            self._line = k.PS_CTRL_LINE
            self.held = torch.zeros(k.PS_HELD_SLOTS, dtype=torch.int32, device=comm.device)
            self._held_n = 0
            self._locks: dict = {}
        else:
            self.server = runtime().AsyncServer(name, self.world, self.rank, _MAX_TABLES, self._apply_cpu)
        self.server.start()
        self.tables: dict[int, object] = {}
        # a straggler that never publishes again is a failure (the supervisor restarts the set),
        # not an infinite hang of every other rank
        self.timeout = float(os.environ.get("MINIPS_SSP_GATE_TIMEOUT", "600"))
        self.closed = False
        self._paused = 0
        if comm.world > 1:
            comm.barrier()  # every rank attached the board
        if comm.rank == 0:
            self.board.unlink()  # mapped everywhere: the name is no longer needed (no /dev/shm leak)

    def register(self, table) -> int:
        t = len(self.tables)
        if t >= _MAX_TABLES:
            raise RuntimeError(f"at most {_MAX_TABLES} asynchronous tables per rank")
        self.tables[t] = table
        return t

    def _apply_cpu(self, t: int, r: int, c: int):
        if r < 0:  # a clock-coalesced table: every requester's slot of clock c in one apply
            self.tables[t]._apply_clock_cpu(c)
        else:
            self.tables[t]._apply_slot_cpu(r, c)

    def check(self):
        err = self.server.error()
        if err:
            raise RuntimeError(f"async PS server of rank {self.rank}: {err}")
        if self.cuda:
            perr = self.server.publish_error()
            if perr:
                raise RuntimeError(f"async PS clock publisher of rank {self.rank}: {perr}")
            bits = self.err.value
            if bits:
                raise RuntimeError(f"async PS of rank {self.rank}: device error bits {bits:#x} (1: a read lock "
                                   "timed out, 2: a write lock timed out, 4: a Map-storage table is full)")
        if self.board.aborted:
            raise RuntimeError(f"async PS: the job was aborted (code {self.board.aborted}: a peer failed or the "
                               "supervisor restarts the rank set)")

    def abort(self, code: int = 1):
        """Make every rank's waits on this board give up at once (a peer is gone)."""
        self.board.set_abort(int(code))

    # -- the owners' reader / writer locks ----------------------------------------------------
    def own_lock(self, t: int) -> int:
        """Device address of this owner's lock word of table t (0 on CPU ranks: board locks)."""
        return self.ctrl[self.rank].data_ptr() + t * self._line if self.cuda and _LOCKS else 0

    def _lock_tensor(self, t: int) -> torch.Tensor:
        lt = self._locks.get(t)
        if lt is None:
            lt = self._locks[t] = torch.tensor([c.data_ptr() + t * self._line for c in self.ctrl], dtype=torch.int64,
                                               device=self.comm.device)
        return lt

    @contextlib.contextmanager
    def read_locked(self, t: int):
        """Every owner's read lock of table t around the enclosed reads (GPU: taken and released by
        kernels on the current stream, around the read kernels issued inside)."""
        if self.cuda and not _LOCKS:
            yield
        elif self.cuda:
            from .._native import kernels

            k = kernels()
            slot = self.held.data_ptr() + 4 * (self._held_n % self.held.numel())
            self._held_n += 1
            locks = self._lock_tensor(t)
            k.ps_read_lock(locks, slot, self.err.device_ptr)
            try:
                yield
            finally:
                k.ps_read_unlock(locks, slot)
        else:
            if not self.board.read_lock(t, self.timeout if self.timeout > 0 else 0.0):
                self.check()
                raise TimeoutError(f"async PS: read lock of table {t} timed out")
            try:
                yield
            finally:
                self.board.read_unlock(t)

    @traced("ps.wait")
    def wait(self, fn, *args, what: str = "") -> float:
        """Run a board wait in slices, surfacing a server error instead of waiting it out."""
        t0 = time.perf_counter()
        while True:
            w = fn(*args, 0.25)
            if w >= 0:
                return time.perf_counter() - t0
            self.check()
            if 0 < self.timeout < time.perf_counter() - t0:
                raise TimeoutError(f"async PS: {what} still waiting after {self.timeout:.0f} s (board "
                                   f"sent {[self.board.snapshot_sent(t) for t in self.tables]})")

    def publish(self, t: int, clock: int):
        """sent[t] = clock once the work issued so far (this clock's pushes) has completed."""
        if self.cuda:
            self.server.publish_after(t, clock, self._anchor)
        else:
            self.board.publish_sent(t, clock)

    def pause(self):
        """Stop applying (checkpoint snapshot / restore); nested with resume()."""
        if self._paused == 0:
            self.server.pause()
            self.check()
        self._paused += 1

    def resume(self):
        self._paused = max(0, self._paused - 1)
        if self._paused == 0:
            self.server.resume()

    def apply_log(self) -> list:
        """(table, requester, clock) triples in this owner's apply order (server.set_log(True)
        before the applies)."""
        flat = self.server.take_log()
        return [tuple(flat[i: i + 3]) for i in range(0, len(flat), 3)]

    def close(self):
        if not self.closed:
            self.server.stop()
            self.closed = True


class _AsyncTable:
    """Shared parts of the asynchronous tables: shared buffers, clocks, gate, flow control."""

    def _init_async(self, comm: Comm, consistency: str, staleness: int, depth, asp_bound):
        if consistency not in ("ssp", "asp"):
            raise ValueError("asynchronous tables serve SSP / ASP (BSP uses the collective tables)")
        self.comm = comm
        self.consistency = consistency
        self.staleness = int(staleness) if consistency == "ssp" else 0
        # ASP is unbounded (asp_model.cpp:23-26) unless asp_bound (or MINIPS_ASP_BOUND, the
        # training driver's --asp_bound) sets the same gate as SSP
        if asp_bound is None and os.environ.get("MINIPS_ASP_BOUND", "") not in ("", "none"):
            asp_bound = int(os.environ["MINIPS_ASP_BOUND"])
        self.asp_bound = None if asp_bound is None or consistency != "asp" else int(asp_bound)
        self.cuda = comm.device.type == "cuda"
        self.ps = AsyncPS.of(comm)
        self.t = self.ps.register(self)
        bound = self.staleness if consistency == "ssp" else (self.asp_bound or 0)
        self.depth = int(depth) if depth else max(4, bound + 3)
        self.clock_n = 0
        self.waited_s = 0.0
        self.gate_waits = 0
        self.staleness_hist: collections.Counter = collections.Counter()
        self._cpu_files: list = []

    # -- shared buffers ---------------------------------------------------------------------
    def _share(self, nbytes: list, tag: str, kind: int = 1) -> list:
        """One buffer per rank (rank r's of nbytes[r] bytes, zero-filled), every one mapped here:
        uint8 tensors [P]. GPU: IPC handles of ipc_alloc memory -- ``kind`` 0 coarse-grained, 1
        fine-grained, 2 uncached (inboxes: written by peers); CPU: /dev/shm files."""
        comm, me = self.comm, self.comm.rank
        if self.cuda:
            from .._native import kernels

            buf, handle = kernels().ipc_alloc(max(256, int(nbytes[me])), comm.device.index or 0, int(kind))
            handles = [None] * comm.world
            if comm.world > 1:
                dist.all_gather_object(handles, handle, group=comm.group)
            return [buf if r == me else kernels().ipc_open(handles[r], max(256, int(nbytes[r])), comm.device.index or 0)
                    for r in range(comm.world)]
        paths = [f"/dev/shm/{self.ps.name}_t{self.t}_{tag}_{r}" for r in range(comm.world)]
        mine = np.memmap(paths[me], dtype=np.uint8, mode="w+", shape=(max(256, int(nbytes[me])),))
        mine.flush()
        self._cpu_files.append(paths[me])
        if comm.world > 1:
            dist.barrier(group=comm.group)  # every rank's file exists
        return [torch.from_numpy(np.memmap(p, dtype=np.uint8, mode="r+", shape=(max(256, int(nbytes[r])),)))
                for r, p in enumerate(paths)]

    def _finish_init(self):
        if self.comm.world > 1:
            self.comm.barrier()  # every rank mapped every buffer and registered the table
        for p in self._cpu_files:  # mapped everywhere: unlink now (nothing left behind in /dev/shm)
            try:
                os.unlink(p)
            except FileNotFoundError:
                pass
        self._cpu_files = []

    # -- clocks -----------------------------------------------------------------------------
    def _gate(self, c: int | None = None):
        """SSP: a Get at own clock c waits until every owner applied every worker's clocks
        < c - s (ssp_model.cpp:58-85); ASP: no wait unless asp_bound is set. ``c``: the reading
        worker's own progress when several workers share this rank (minips_amd.engine)."""
        c = self.clock_n if c is None else int(c)
        bound = self.staleness if self.consistency == "ssp" else self.asp_bound
        board, t = self.ps.board, self.t
        if bound is not None and c - bound > 0 and board.min_applied(t) < c - bound:
            self.waited_s += self.ps.wait(board.wait_min_applied, t, c - bound, what=f"SSP gate of table {t}")
            self.gate_waits += 1
        # observed staleness of this read: own clocks not yet in every shard
        self.staleness_hist[c - min(c, board.min_applied(t))] += 1

    def _reserve_slot(self) -> int:
        """Inbox slot of the current clock, free once every owner applied clock c - depth."""
        c = self.clock_n
        need = c - self.depth + 1
        board, t, me = self.ps.board, self.t, self.comm.rank
        if need > 0 and board.min_applied_from(t, me) < need:
            self.ps.wait(board.wait_applied_from, t, me, need, what=f"inbox slot of table {t}")
        return c % self.depth

    def _advance(self):
        self.clock_n += 1
        self.ps.publish(self.t, self.clock_n)

    def drain(self):
        """Until every owner applied this rank's clocks so far."""
        if hasattr(self, "_check_keys"):
            self._check_keys()
        board, t, me = self.ps.board, self.t, self.comm.rank
        if self.clock_n == 0:
            return
        self.ps.wait(board.wait_sent_at_least, t, me, self.clock_n, what="clock publisher")
        self.ps.wait(board.wait_applied_from, t, me, self.clock_n, what=f"drain of table {self.t}")

    def quiesce_owner(self):
        """Until this rank's server applied everything sent to it so far (tests, snapshots)."""
        board, t, me = self.ps.board, self.t, self.comm.rank
        sent = board.snapshot_sent(t)
        t0 = time.perf_counter()
        while any(board.applied(t, me, r) < sent[r] for r in range(self.comm.world)):
            self.ps.check()
            if 0 < self.ps.timeout < time.perf_counter() - t0:
                raise TimeoutError("async PS: owner quiesce timed out")
            time.sleep(0.0005)

    def staleness_stats(self) -> dict:
        h = dict(sorted(self.staleness_hist.items()))
        return dict(hist=h, max=max(h) if h else 0, gate_waits=self.gate_waits, waited_s=round(self.waited_s, 6))

    # -- checkpoint / restore ---------------------------------------------------------------
    def snapshot_begin(self):
        """Checkpointer.save, after every rank drained: no apply runs until snapshot_end()."""
        self.ps.pause()

    def snapshot_end(self):
        self.ps.resume()

    def _restore_clock(self, clock: int):
        """After the rows landed (server paused since restore_dst): every rank restarts at
        ``clock`` -- its sent counter and its owner row of the board -- then all resume."""
        board, t = self.ps.board, self.t
        # host barriers with the long timeout (restore times differ by rank): (a) every rank is
        # done reading this table's counters (a peer may still be draining its old clocks) before
        # any rank resets them, (b) nobody pushes before every rank reset its sent counter and row
        self.comm.store_barrier(f"async_restore_a_t{t}")
        self.clock_n = int(clock)
        board.publish_sent(t, self.clock_n)
        board.publish_applied_row(t, self.clock_n)
        self.staleness_hist.clear()
        self.comm.store_barrier(f"async_restore_b_t{t}")
        self.ps.resume()

    def reset_after_rollback(self):
        raise RuntimeError("asynchronous tables restart the whole rank set (no in-place rollback)")

    def close(self):
        self.drain()


class AsyncSparseTable(_AsyncTable, SparseTable):
    _local_apply = False  # pushes go to the owners' inboxes: no in-place apply in the backward
    """Row table (equal key ranges, optional routing) with SSP / ASP over the one-sided path.
    Same planning API as SparseTable (plan / plan_async / advance_plan / get / add /
    add_lookup_grads / add_keys / clock), so the models switch transports by construction.

    ``max_keys``: keys per clock a rank may push (an inbox slot holds that many rows; the models
    pass B * F)."""

    _exact_counts = False

    def __init__(self, comm: Comm, num_rows: int, width: int, optimizer: str = "rowwise_adagrad", lr: float = 0.01,
                 eps: float = 1e-8, pull_dtype=torch.bfloat16, consistency: str = "ssp", staleness: int = 0,
                 split: int | None = None, table_id: int = 0, init_std: float = 0.01, seed: int = 1234,
                 route: str = "mix", columns=None, max_keys: int = 1 << 16, depth: int | None = None,
                 asp_bound: int | None = None, value_dtype=torch.float32):
        if optimizer not in ("add", "sgd", "rowwise_adagrad"):
            raise ValueError(f"sparse optimizer {optimizer!r}: add | sgd | rowwise_adagrad")
        if value_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"one-sided rows are fp32 or bf16, not {value_dtype}")
        if value_dtype == torch.bfloat16 and width not in (16, 32, 64):
            raise ValueError("bf16 rows hold 16, 32 or 64 values")
        self._init_async(comm, consistency, staleness, depth, asp_bound)
        # bf16 rows: half the HBM (config 5's 10B x 64 table: 1.28 TB of rows over 8 x 288 GB); the
        # owner's optimizer math and state stay fp32, the row goes back to bf16 by stochastic rounding
        self.value_dtype = value_dtype
        self.push_dtype = self.grad_dtype = torch.float32
        self._applies = 0  # apply counter (CPU path): keys the stochastic rounding of bf16 rows
        self.seed = int(seed)
        self.columns = column_spec(columns, comm.device)
        self.route_mult = _route_multiplier(num_rows) if route == "mix" else 0
        self.table_id = table_id
        self.num_rows, self.width = num_rows, width
        self.optimizer, self.lr, self.eps = optimizer, lr, eps
        self.pull_dtype = pull_dtype
        self.split = split
        self.p2p = False
        self._pending: list = []
        self._own_bounds = torch.tensor([0, (1 << 63) - 1], dtype=torch.int64, device=comm.device)
        P, me, dev = comm.world, comm.rank, comm.device
        b = even_bounds(num_rows, P)
        self.bounds_list = b
        self.bounds = torch.tensor(b, dtype=torch.int64, device=dev)
        self.base = b[me]
        self.rows_local = b[me + 1] - b[me]
        rows_of = [b[r + 1] - b[r] for r in range(P)]
        self.cap = _align(max(2, int(max_keys)), 2)
        self.slot_bytes = _align(_SLOT_HEADER + self.cap * (8 + 4 * width), 256)
        esz = 2 if value_dtype == torch.bfloat16 else 4
        shards = self._share([esz * width * n for n in rows_of], "shard", kind=_SHARD_MEM)
        self._shards = shards
        self._views = [s[: esz * width * n].view(value_dtype).view(n, width) for s, n in zip(shards, rows_of)]
        self.shard = self._views[me]
        if init_std > 0:
            g = torch.Generator(device=dev)
            g.manual_seed(seed + 7919 * me)
            if value_dtype == torch.float32:
                self.shard.normal_(0.0, init_std, generator=g)
            else:  # drawn in fp32 (chunks: the 10B-row shards), rounded to bf16
                step = 1 << 24
                for r0 in range(0, self.rows_local, step):
                    tmp = torch.empty(min(step, self.rows_local - r0), width, dtype=torch.float32, device=dev)
                    self.shard[r0: r0 + tmp.shape[0]].copy_(tmp.normal_(0.0, init_std, generator=g))
        self.state = torch.zeros(self.rows_local, dtype=torch.float32, device=dev) \
            if optimizer == "rowwise_adagrad" else None
        self.state2 = torch.zeros_like(self.state) if (self.state is not None and split is not None) else None
        # SSP + row-wise Adagrad: one Adagrad step per row per clock over every requester's push
        # (module docstring); the owner's direct-addressed (stamp, index) table of that apply
        # (the clock kernel moves rows in float4 pieces: W % 4 == 0, W <= 64)
        # (one rank: a clock holds one push -- the per-push apply is the same update, one kernel)
        self.coalesced = (consistency == "ssp" and P > 1 and optimizer == "rowwise_adagrad" and width % 4 == 0
                          and width <= 64 and 8 * P * self.rows_local <= _COALESCE_MAX_BYTES)
        self._rs = torch.zeros(2 * P * self.rows_local, dtype=torch.int32, device=dev) \
            if self.coalesced and self.cuda else None
        self._inbox = self._share([P * self.depth * self.slot_bytes] * P, "inbox", kind=_INBOX_MEM)
        self._register_server()
        self._finish_init()

    def _register_server(self, hash_cap: int = 0, hkeys: int = 0):
        comm, me, dev = self.comm, self.comm.rank, self.comm.device
        if self.cuda:
            self.bases = torch.tensor([s.data_ptr() for s in self._shards], dtype=torch.int64, device=dev)
            self.inbox_ptrs = torch.tensor([s.data_ptr() for s in self._inbox], dtype=torch.int64, device=dev)
            D1 = self.split if self.split is not None else self.width
            self.ps.server.add_sparse(self.t, _OPT_CODES[self.optimizer], self.shard.data_ptr(), self.width,
                                      self.width, self.state.data_ptr() if self.state is not None else 0,
                                      self.state2.data_ptr() if self.state2 is not None else 0, D1, self.base,
                                      float(self.lr), float(self.eps), self.cap, self._inbox[me].data_ptr(),
                                      self.slot_bytes, self.depth, int(self.value_dtype == torch.bfloat16),
                                      self.seed & 0xFFFFFFFF, int(hash_cap), int(hkeys), self.ps.own_lock(self.t),
                                      rs=self._rs.data_ptr() if getattr(self, "_rs", None) is not None else 0,
                                      coalesce=bool(getattr(self, "coalesced", False)))
            torch.cuda.synchronize(dev)  # shard init + state zeroing done before any peer reads
        else:
            self.ps.server.set_coalesce(self.t, bool(getattr(self, "coalesced", False)))
            self.ps.server.enable(self.t)

    # -- planning: SparseTable's dedupe + owner grouping, no count exchange ----------------------
    def _finish_plan(self, pp: _PendingPlan) -> SparsePlan:
        if pp.event is not None:
            streams.current(self.comm.device).wait_event(pp.event)
        n = pp.flat.numel()
        if n > self.cap:
            raise ValueError(f"a batch of {n} keys exceeds the inbox slot ({self.cap} rows): raise max_keys")
        counts = pp.counts[: self.comm.world]
        if not self.cuda:
            U = int(pp.U_dev.reshape(-1)[0])
            p = SparsePlan(n, pp.inv, pp.uniq, U, None, None, pp.uniq[:U], csr=pp.csr, _U=U)
        else:
            p = SparsePlan(n, pp.inv, pp.uniq, n, None, None, pp.uniq, U_dev=pp.U_dev, csr=pp.csr)
        p.extra["counts"] = counts
        return p

    def plan(self, keys: torch.Tensor, csr: bool = False) -> SparsePlan:
        return self._finish_plan(self._start_plan(keys, csr, exchange=False))

    def plan_async(self, keys: torch.Tensor, csr: bool = False, keys_on_plan_stream: bool = False,
                   fenced: bool = False):
        if not self.cuda:
            return self._start_plan(keys, csr, exchange=False)
        ps = self.comm.plan_stream()
        cur = streams.current(self.comm.device)
        if not keys_on_plan_stream:
            ps.wait_stream(cur)
        with streams.use(ps):
            pp = self._start_plan(keys, csr, exchange=False)
            ring = self.__dict__.get("_plan_evs")
            if ring is None:
                # (same-device ordering: fence-free unless MINIPS_STREAM_DEBUG sysfence=plan)
                ring = self._plan_evs = streams.EventRing(16, fast=streams.fast_for("plan"))
            pp.event = ring.next()
            pp.event.record(ps)
        if not fenced:
            keys.record_stream(ps)
            for t in (pp.flat, pp.uniq, pp.inv, pp.counts, pp.U_dev, *(pp.csr or ())):
                if t is not None:  # (csr: positions may be None)
                    t.record_stream(cur)
        return pp

    def advance_plan(self, pending, finish: bool = True):
        return pending  # nothing to exchange

    def _fused_lookup_ok(self, *a) -> bool:
        return False

    # -- KV API -----------------------------------------------------------------------------
    @traced("async_sparse.get")
    def get(self, keys: torch.Tensor, plan=None, clock: int | None = None):
        """Rows of the unique keys ([cap, width], unique order) and the plan; rows[plan.inv[i]]
        is the row of keys[i]. No collective: rows come straight from the owners' HBM."""
        if plan is None:
            plan = self.plan(keys)
        elif isinstance(plan, _PendingPlan):
            plan = self._finish_plan(plan)
        self._gate(clock)
        out = torch.empty(max(plan.cap, 1), self.width, dtype=self.pull_dtype, device=self.comm.device)
        with self.ps.read_locked(self.t):
            self._gather(plan, out)
        return out, plan

    def _gather(self, plan, out):
        if self.cuda:
            from .._native import kernels

            if self.value_dtype == torch.bfloat16:
                kernels().ps_gather_rows_bf16tab(self.bases, self.bounds, plan.uniq, plan.U_dev, self.width, out)
            else:
                kernels().ps_gather_rows(self.bases, self.bounds, plan.uniq, plan.U_dev, self.width, out)
        else:
            u = plan.uniq[: plan.U]
            for o in range(self.comm.world):
                lo, hi = self.bounds_list[o], self.bounds_list[o + 1]
                m = (u >= lo) & (u < hi)
                if bool(m.any()):
                    out[: plan.U][m] = self._views[o][u[m] - lo].to(out.dtype)

    @traced("async_sparse.clock")
    def clock(self):
        """Push this clock's gradient rows into the owners' inboxes, then publish the clock."""
        pending, self._pending = self._pending, []
        if len(pending) > 1:
            pending = [self._merge(pending)]
        slot = self._reserve_slot()
        off = (self.comm.rank * self.depth + slot) * self.slot_bytes
        if self.cuda:
            from .._native import kernels

            # the push (and the publish event behind it) on a stream of its own, after the compute
            # stream's work so far; nothing later on the compute stream depends on it (reads are
            # gated by the board), so the step's remaining backward runs beside the copy into the
            # inboxes: W&D SSP 0.396-0.403 vs 0.402-0.404, DLRM-10B 0.681-0.683 vs 0.692-0.694 ms
            # (profiles/r4/ab_push_stream.txt). Opt-in (MINIPS_PS_PUSH_STREAM=1). The hand-off events
            # are same-device stream orderings and fence-free (streams.fast_for): the 4-rank SSP loss
            # spike once blamed on them showed with every event system-fenced and with the push
            # stream off too -- it was the per-push optimizer step, fixed by the clock-coalesced SSP
            # apply (profiles/r5/ssp_probe.txt)
            pst = self._push_stream() if _PUSH_STREAM else None
            if pst is not None:
                ev = self._push_evs.next()
                ev.record(streams.current(self.comm.device))
                pst.wait_event(ev)
            with streams.use(pst):
                if pending:
                    plan, g = pending[0]
                    g = g.contiguous()
                    kernels().ps_push_rows(plan.uniq, plan.extra["counts"], plan.U_dev, plan.cap, g,
                                           self.inbox_ptrs, off, self.cap)
                    if pst is not None:  # produced on the compute stream, read on the push stream
                        for t in (g, plan.uniq, plan.extra["counts"], plan.U_dev):
                            if isinstance(t, torch.Tensor) and t.is_cuda:
                                t.record_stream(pst)
                else:
                    kernels().ps_set_headers(self.inbox_ptrs, off, 0)
                self._advance()
            return
        self._push_cpu(pending[0] if pending else None, off)
        self._advance()

    def _push_stream(self):
        st = self.__dict__.get("_pst")
        if st is None:
            st = self._pst = self.comm.new_stream()
            # fence-free by default (streams.fast_for("push"); MINIPS_STREAM_DEBUG sysfence=push
            # fences them): the push reads the gradient rows on the same device, which the stream
            # order alone makes visible; its IPC stores into peers' inboxes are released by the
            # publish event's system-scope completion (onesided.hip header)
            self._push_evs = streams.EventRing(8, fast=streams.fast_for("push"))
        return st

    def _merge(self, pending):
        """Several Adds in one clock: one deduplicated batch (duplicates summed)."""
        keys, rows = [], []
        for plan, g in pending:
            U = plan.U
            keys.append(plan.uniq[:U])
            rows.append(g[:U])
        allk, allg = torch.cat(keys), torch.cat(rows)
        uniq, inv, counts, U_dev = ops.unique_bucketize_n(allk, self.bounds)
        g = torch.zeros(max(allk.numel(), 1), self.width, dtype=torch.float32, device=self.comm.device)
        ops.scatter_add_rows(allg.contiguous(), inv, g)
        U = int(U_dev.reshape(-1)[0])
        p = SparsePlan(allk.numel(), inv, uniq, allk.numel() if self.cuda else U, None, None, uniq,
                       U_dev=U_dev if self.cuda else None, _U=U)
        p.extra["counts"] = counts[: self.comm.world]
        return p, g

    # -- CPU data path (gloo tests) ----------------------------------------------------------
    def _push_cpu(self, item, off: int):
        W, cap = self.width, self.cap
        if item is None:
            for o in range(self.comm.world):
                self._inbox[o][off: off + 8].view(torch.int64)[0] = 0
            return
        plan, g = item
        counts = [int(c) for c in plan.extra["counts"].tolist()]
        s = 0
        for o, n in enumerate(counts):
            buf = self._inbox[o]
            keys = buf[off + _SLOT_HEADER: off + _SLOT_HEADER + 8 * cap].view(torch.int64)
            rows = buf[off + _SLOT_HEADER + 8 * cap: off + _SLOT_HEADER + 8 * cap + 4 * W * cap].view(torch.float32)
            keys[:n] = plan.uniq[s: s + n]
            rows.view(cap, W)[:n] = g[s: s + n].to(torch.float32)
            buf[off: off + 8].view(torch.int64)[0] = n  # the header last (the board publish orders it)
            s += n

    def _apply_slot_cpu(self, r: int, c: int):
        W, cap = self.width, self.cap
        off = (r * self.depth + c % self.depth) * self.slot_bytes
        buf = self._inbox[self.comm.rank]
        n = int(buf[off: off + 8].view(torch.int64)[0])
        if n == 0:
            return
        keys = buf[off + _SLOT_HEADER: off + _SLOT_HEADER + 8 * n].view(torch.int64).clone()
        g = buf[off + _SLOT_HEADER + 8 * cap: off + _SLOT_HEADER + 8 * cap + 4 * W * n].view(torch.float32)
        g = g.view(n, W).clone()
        self._apply_rows(keys, g)

    def _apply_clock_cpu(self, c: int):
        """Clock-coalesced apply (CPU twin of ps_clock_adagrad): every requester's rows of clock
        c summed per key in requester order, one optimizer step per row."""
        W, cap = self.width, self.cap
        buf = self._inbox[self.comm.rank]
        keys, rows = [], []
        for r in range(self.comm.world):
            off = (r * self.depth + c % self.depth) * self.slot_bytes
            n = int(buf[off: off + 8].view(torch.int64)[0])
            if n:
                keys.append(buf[off + _SLOT_HEADER: off + _SLOT_HEADER + 8 * n].view(torch.int64).clone())
                g = buf[off + _SLOT_HEADER + 8 * cap: off + _SLOT_HEADER + 8 * cap + 4 * W * n].view(torch.float32)
                rows.append(g.view(n, W).clone())
        if not keys:
            return
        allk = torch.cat(keys)
        uniq, inv = torch.unique(allk, return_inverse=True)
        g = torch.zeros(uniq.numel(), W, dtype=torch.float32)
        g.index_add_(0, inv, torch.cat(rows))  # sequential on the CPU: requester order per key
        self._apply_rows(uniq, g)

    def _apply_rows(self, keys, g):
        if self.value_dtype == torch.bfloat16:
            opt = "rowwise_adagrad" if self.optimizer == "rowwise_adagrad" else "add"
            scale = 1.0 if self.optimizer == "add" else -self.lr
            ops.sparse_apply_bf16(opt, self.shard, self.state, keys, self.base, g, self.lr, self.eps, scale,
                                  state2=self.state2, split=self.split, step=self._applies, seed=self.seed)
            self._applies += 1
            return
        if self.optimizer == "rowwise_adagrad":
            ops.sparse_rowwise_adagrad(self.shard, self.state, keys, self.base, g, self.lr, self.eps,
                                       state2=self.state2, split=self.split)
        else:
            ops.sparse_sgd(self.shard, keys, self.base, g, 1.0 if self.optimizer == "add" else -self.lr)

    # -- checkpoint hooks (minips_amd.ps.checkpoint) -------------------------------------------
    def shard_state(self):
        self.drain()
        arrays = {"params": self.shard}
        if self.state is not None:
            arrays["state"] = self.state
        if self.state2 is not None:
            arrays["state2"] = self.state2
        meta = dict(global_rows=self.num_rows, base=self.base, rows=self.rows_local, cols=self.width,
                    clock=self.clock_n, table_id=self.table_id, rank=self.comm.rank, world=self.comm.world,
                    kind="sparse", applies=self._apply_count())
        return meta, arrays

    def _apply_count(self) -> int:
        return int(self.ps.server.step(self.t)) if self.cuda else int(self._applies)

    def restore_meta(self, meta: dict):
        """Checkpoint meta of this rank's shard (before finish_restore): the bf16 rounding stream."""
        n = int(meta.get("applies", 0))
        if self.cuda:
            self.ps.server.set_step(self.t, n)
        else:
            self._applies = n

    def restore_range(self):
        return self.base, self.base + self.rows_local

    def restore_dst(self):
        self.ps.pause()  # the rows land with no apply running (resumed in finish_restore)
        out = {"params": self.shard}
        if self.state is not None:
            out["state"] = self.state.view(-1, 1)
        if self.state2 is not None:
            out["state2"] = self.state2.view(-1, 1)
        return out

    def finish_restore(self, clock: int):
        if self.cuda:
            torch.cuda.synchronize(self.comm.device)
        self._restore_clock(clock)


class AsyncHashTable(AsyncSparseTable):
    """Map storage on the one-sided path (reference MapStorage, server/map_storage.hpp:13-26):
    keys in [0, 2^63) are mixed by the same bijection as the collective HashSparseTable and
    range-partitioned over the owners; each owner keeps an open-addressing table of fixed
    ``capacity`` (power of two) in its fine-grained HBM -- keys [cap] int64 (-1 empty) and rows
    [cap, W] fp32 (+ row-wise Adagrad state). The owner's server thread inserts a key on its first
    Add (row 0 + update); a Get probes the owners' tables one-sidedly and reads 0 for an absent
    key (MapStorage::SubGet's default-insert, without the insert: a read never writes the
    owner's table). Capacity is fixed (no rehash under one-sided readers): a full table is a
    device error bit, raised at the next check."""

    def __init__(self, comm: Comm, width: int, capacity: int = 1 << 16, optimizer: str = "add", lr: float = 0.01,
                 eps: float = 1e-8, pull_dtype=torch.float32, consistency: str = "ssp", staleness: int = 0,
                 table_id: int = 0, max_keys: int = 1 << 16, depth: int | None = None, asp_bound: int | None = None,
                 **_unused):
        from .tables import MASK63

        if optimizer not in ("add", "sgd", "rowwise_adagrad"):
            raise ValueError(f"sparse optimizer {optimizer!r}: add | sgd | rowwise_adagrad")
        self._init_async(comm, consistency, staleness, depth, asp_bound)
        self.value_dtype = self.push_dtype = self.grad_dtype = torch.float32
        self._applies, self.seed = 0, 0
        self.columns = None
        self.route_mult = 0
        self.table_id = table_id
        self.num_rows, self.width = MASK63, width
        self.optimizer, self.lr, self.eps = optimizer, lr, eps
        self.pull_dtype = pull_dtype
        self.split = None
        self.p2p = False
        self._pending: list = []
        self._own_bounds = torch.tensor([0, (1 << 63) - 1], dtype=torch.int64, device=comm.device)
        P, me, dev = comm.world, comm.rank, comm.device
        b = even_bounds(MASK63, P)
        self.bounds_list = b
        self.bounds = torch.tensor(b, dtype=torch.int64, device=dev)
        self.base = 0  # rows are addressed by slot
        self.capacity = cap = 1 << max(4, int(capacity - 1).bit_length())
        self.rows_local = cap
        self.cap = _align(max(2, int(max_keys)), 2)
        self.slot_bytes = _align(_SLOT_HEADER + self.cap * (8 + 4 * width), 256)
        self._hk = self._share([8 * cap] * P, "hkeys", kind=_SHARD_MEM)
        self._hkeys = [h[: 8 * cap].view(torch.int64) for h in self._hk]
        self._hkeys[me].fill_(-1)
        shards = self._share([4 * width * cap] * P, "shard", kind=_SHARD_MEM)
        self._shards = shards
        self._views = [s[: 4 * width * cap].view(torch.float32).view(cap, width) for s in shards]
        self.shard = self._views[me]
        self.state = torch.zeros(cap, dtype=torch.float32, device=dev) if optimizer == "rowwise_adagrad" else None
        self.state2 = None
        self.coalesced, self._rs = False, None  # (Map storage applies push by push)
        self._inbox = self._share([P * self.depth * self.slot_bytes] * P, "inbox", kind=_INBOX_MEM)
        self._neg = None
        if self.cuda:
            self._hkey_ptrs = torch.tensor([h.data_ptr() for h in self._hk], dtype=torch.int64, device=dev)
            self._hval_ptrs = torch.tensor([s.data_ptr() for s in shards], dtype=torch.int64, device=dev)
        self._register_server(hash_cap=cap, hkeys=self._hkeys[me].data_ptr())
        self._finish_init()

    def _route_keys(self, keys: torch.Tensor) -> torch.Tensor:
        from .tables import mix63

        if keys.is_cuda:  # checked at drain (no host round trip per batch)
            neg = (keys < 0).any()
            self._neg = neg if self._neg is None else (self._neg | neg)
        elif bool((keys < 0).any()):
            raise ValueError("Map-storage keys must be in [0, 2^63)")
        return mix63(keys)

    def _check_keys(self):
        if self._neg is not None:
            neg, self._neg = bool(self._neg), None
            if neg:
                raise ValueError("Map-storage keys must be in [0, 2^63)")

    def _gather(self, plan, out):
        if self.cuda:
            from .._native import kernels

            kernels().ps_hash_gather(self._hkey_ptrs, self._hval_ptrs, self.bounds, self.capacity, plan.uniq,
                                     plan.U_dev, self.width, out)
            return
        u = plan.uniq[: plan.U].tolist()
        rows = torch.zeros(len(u), self.width, dtype=torch.float32)
        for i, k in enumerate(u):
            o = next(r for r in range(self.comm.world) if self.bounds_list[r] <= k < self.bounds_list[r + 1])
            s = self._find_cpu(self._hkeys[o], k)
            if s >= 0:
                rows[i] = self._views[o][s]
        out[: plan.U] = rows.to(out.dtype)

    def _find_cpu(self, hk: torch.Tensor, k: int) -> int:
        cap = self.capacity
        s = ops._mix64_int(k) & (cap - 1)
        for _ in range(cap):
            cur = int(hk[s])
            if cur == k:
                return s
            if cur == -1:
                return -1
            s = (s + 1) & (cap - 1)
        return -1

    def _apply_rows(self, keys, g):
        slots = torch.empty(keys.numel(), dtype=torch.int64)
        counters = torch.zeros(2, dtype=torch.int32)
        ops.hash_slots(self._hkeys[self.comm.rank], keys, slots, self.shard, 0.0, 0, counters)
        if int(counters[1]):
            raise RuntimeError(f"one-sided Map-storage table full (capacity {self.capacity})")
        if self.optimizer == "rowwise_adagrad":
            ops.sparse_rowwise_adagrad(self.shard, self.state, slots, 0, g, self.lr, self.eps)
        else:
            ops.sparse_sgd(self.shard, slots, 0, g, 1.0 if self.optimizer == "add" else -self.lr)

    def size(self) -> int:
        """Occupied slots of this owner's table."""
        self.drain()
        return int((self._hkeys[self.comm.rank] >= 0).sum())

    # -- checkpoint hooks: (key, row, state) of the occupied slots, sorted by key (the collective
    # HashSparseTable's format, so either transport restores the other's files)
    def shard_state(self):
        self.drain()
        hk = self._hkeys[self.comm.rank]
        occ = (hk >= 0).nonzero().squeeze(1)
        keys, order = torch.sort(hk[occ])
        slots = occ[order]
        arrays = {"keys": keys.view(-1, 1), "params": self.shard[slots]}
        if self.state is not None:
            arrays["state"] = self.state[slots].view(-1, 1)
        from .tables import MASK63

        meta = dict(global_rows=MASK63, base=0, rows=int(keys.numel()), cols=self.width, clock=self.clock_n,
                    table_id=self.table_id, rank=self.comm.rank, world=self.comm.world, kind="hash")
        return meta, arrays

    def restore_range(self):
        self.ps.pause()  # resumed in finish_restore
        self._hkeys[self.comm.rank].fill_(-1)
        self.shard.zero_()
        if self.state is not None:
            self.state.zero_()
        return self.bounds_list[self.comm.rank], self.bounds_list[self.comm.rank + 1]

    def restore_insert(self, chunk: dict):
        keys = chunk["keys"].reshape(-1).to(self.comm.device)
        slots = torch.empty(keys.numel(), dtype=torch.int64, device=self.comm.device)
        counters = torch.zeros(2, dtype=torch.int32, device=self.comm.device)
        ops.hash_slots(self._hkeys[self.comm.rank], keys, slots, self.shard, 0.0, 0, counters)
        # a full table returns slot -1 for the keys it could not place: writing through them would
        # overwrite the last slot's row (restores onto fewer owners put more keys on each)
        full = int(counters[1].item())
        if full:
            occupied = int((self._hkeys[self.comm.rank] >= 0).sum().item())
            raise RuntimeError(f"one-sided Map-storage table {self.table_id} full while restoring: {full} of "
                               f"{keys.numel()} keys found no slot (capacity {self.capacity}, {occupied} occupied); "
                               f"create the table with capacity >= {2 * (occupied + full)}")
        self.shard[slots] = chunk["params"].to(self.shard.dtype)
        if self.state is not None and "state" in chunk:
            self.state[slots] = chunk["state"].reshape(-1).to(self.state.dtype)


class AsyncDenseTable(_AsyncTable):
    """A flat dense parameter vector (equal shards, like ps.tables.DenseTable) on the one-sided
    path: Get pulls every owner's shard whose version changed since the last pull (bf16 copies
    the owner's apply writes), Add + Clock pushes each owner's slice of the gradient into its
    inbox, and the owner applies Adam / Adagrad / SGD / add with its own m / v state.
    SSP (Adam / Adagrad): clock-coalesced -- the owner sums the P pushes of a clock (requester
    order) and takes ONE optimizer step at lr, one Adam step count per clock: BSP's update.
    ASP: one optimizer step per push, as an asynchronous PS server does (each Add applied on
    arrival); every rank pushes the whole gradient every clock, so one clock is P pushes and the
    scale-invariant optimizers (a step moves ~lr whatever the gradient's size) take lr / P per
    push (``push_lr``) -- with lr per push a 4-rank run moved the weights 4x as far and spiked
    (tools/ssp_probe.py, profiles/r5/ssp_probe.txt). SGD / add are linear: the P pushes sum to the
    BSP step at lr either way.
    Same API as DenseTable (grad written in place by the models, get / add / clock / load_full /
    full_master)."""

    buckets = None

    def __init__(self, comm: Comm, n_params: int, optimizer: str = "adam", lr: float = 1e-3,
                 consistency: str = "ssp", staleness: int = 0, pull_dtype=torch.bfloat16, table_id: int = 0,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, depth: int | None = None,
                 asp_bound: int | None = None):
        if optimizer not in ("add", "sgd", "adagrad", "adam"):
            raise ValueError(f"dense optimizer {optimizer!r}: add | sgd | adagrad | adam")
        self._init_async(comm, consistency, staleness, depth, asp_bound)
        P, me, dev = comm.world, comm.rank, comm.device
        self.table_id, self.n_params = table_id, n_params
        self.optimizer, self.lr = optimizer, lr
        self.coalesced = consistency == "ssp" and P > 1 and optimizer in ("adam", "adagrad")
        self.push_lr = lr / P if optimizer in ("adam", "adagrad") and not self.coalesced else lr
        self.betas, self.eps, self.weight_decay = betas, eps, weight_decay
        self.pull_dtype = pull_dtype
        self.value_dtype = torch.float32
        self.n_pad = _align(n_params, 64 * P)
        self.shard = self.n_pad // P
        self.base = me * self.shard
        self.slot_bytes = _align(_SLOT_HEADER + 4 * self.shard, 256)
        masters = self._share([4 * self.shard] * P, "master", kind=_SHARD_MEM)
        self._masters = [m[: 4 * self.shard].view(torch.float32) for m in masters]
        self.master = self._masters[me]
        # what peers pull: the bf16 copy the apply writes (half the xGMI bytes), or the fp32 master
        self._pull_bf16 = self.cuda and pull_dtype == torch.bfloat16
        if self._pull_bf16:
            pulls = self._share([2 * self.shard] * P, "pull", kind=_SHARD_MEM)
            self._pulls = [p[: 2 * self.shard].view(torch.bfloat16) for p in pulls]
        else:
            self._pulls = self._masters
        self.m = torch.zeros(self.shard, dtype=torch.float32, device=dev) if optimizer in ("adam", "adagrad") \
            else None
        self.v = torch.zeros_like(self.m) if optimizer == "adam" else None
        self._inbox = self._share([P * self.depth * self.slot_bytes] * P, "inbox", kind=_INBOX_MEM)
        self.params = torch.zeros(self.n_pad, dtype=pull_dtype, device=dev)
        self.grad = torch.zeros(self.n_pad, dtype=torch.float32, device=dev)
        self._seen = [-1] * P          # owner version of the cached copy (sum of its applied clocks)
        self._seen_applied = [-1] * P  # min over requesters of the owner's applied clocks at that pull
        self.pulls = 0                 # owner shards pulled so far (lazy-pull accounting)
        self._pending = False
        self.step = 0
        self.cpu_step = 0
        if self.cuda:
            self._inbox_ptrs = torch.tensor([b.data_ptr() for b in self._inbox], dtype=torch.int64, device=dev)
            self._pull_ptrs = torch.tensor([b.data_ptr() for b in self._pulls], dtype=torch.int64, device=dev)
            self._slot_views = [b for b in self._inbox]
            # the coalesced apply's summed gradient and its active-push count
            self._sum = torch.zeros(self.shard, dtype=torch.float32, device=dev) if self.coalesced else None
            self._sum_active = torch.zeros(1, dtype=torch.int64, device=dev) if self.coalesced else None
            self.ps.server.add_dense(self.t, _OPT_CODES[optimizer], self.master.data_ptr(),
                                     self.m.data_ptr() if self.m is not None else 0,
                                     self.v.data_ptr() if self.v is not None else 0,
                                     self._pulls[me].data_ptr() if self._pull_bf16 else 0, self.shard,
                                     float(self.push_lr),
                                     float(betas[0]), float(betas[1]), float(eps), float(weight_decay), 0,
                                     self._inbox[me].data_ptr(), self.slot_bytes, self.depth, self.ps.own_lock(self.t),
                                     sum=self._sum.data_ptr() if self.coalesced else 0,
                                     sum_active=self._sum_active.data_ptr() if self.coalesced else 0,
                                     coalesce=self.coalesced)
        else:
            self.ps.server.set_coalesce(self.t, self.coalesced)
            self.ps.server.enable(self.t)
        self._finish_init()

    # the clock (push + headers + host publish of this stream's event) may be issued from any
    # stream of the device: WideDeep issues it on its weight-gradient side stream
    side_clock_ok = True

    @property
    def clock_count(self):
        return self.clock_n

    def load_full(self, full: torch.Tensor):
        """Initialise from the full vector (identical on every rank)."""
        flat = torch.zeros(self.n_pad, dtype=torch.float32, device=self.comm.device)
        flat[: self.n_params] = full.to(self.comm.device, torch.float32)
        self.master.copy_(flat[self.base: self.base + self.shard])
        if self._pull_bf16:
            self._pulls[self.comm.rank].copy_(self.master.to(torch.bfloat16))
        self.params.copy_(flat.to(self.pull_dtype))
        board = self.ps.board
        self._seen = [board.owner_version(self.t, o) for o in range(self.comm.world)]
        self._seen_applied = [min(board.applied(self.t, o, r) for r in range(self.comm.world))
                              for o in range(self.comm.world)]
        if self.cuda:
            torch.cuda.synchronize(self.comm.device)
        if self.comm.world > 1:
            self.comm.barrier()

    def full_master(self) -> torch.Tensor:
        self.drain()
        return torch.cat([m.to(self.comm.device) for m in self._masters])[: self.n_params].clone()

    @traced("async_dense.get")
    def get(self, clock: int | None = None) -> torch.Tensor:
        """Pull the owners' shards the read needs (SSP-gated). Lazy: with a staleness bound s, an
        owner's cached copy that already holds every requester's clocks < c - s is served as is
        (it is as fresh as SSP requires), so a shard is re-pulled about every s clocks instead of
        every clock; unbounded ASP re-pulls whatever changed. The pull runs under the owners' read
        locks: every shard is copied between two of its owner's apply batches."""
        self._gate(clock)
        board, t, P = self.ps.board, self.t, self.comm.world
        c = self.clock_n if clock is None else int(clock)
        bound = self.staleness if self.consistency == "ssp" else self.asp_bound
        need, ver, app = [], {}, {}
        for o in range(P):
            v = board.owner_version(t, o)
            if v == self._seen[o]:
                continue
            if bound is not None and self._seen_applied[o] >= c - bound:
                continue
            need.append(o)
            # read BEFORE the copy: what the locked copy holds is at least this new
            ver[o] = v
            app[o] = min(board.applied(t, o, r) for r in range(P))
        if need:
            with self.ps.read_locked(t):
                if self.cuda:
                    from .._native import kernels

                    kernels().ps_pull(self._pull_ptrs, need, self.shard * self.params.element_size(), self.params)
                else:
                    for o in need:
                        self.params[o * self.shard: (o + 1) * self.shard].copy_(self._pulls[o])
            for o in need:
                self._seen[o], self._seen_applied[o] = ver[o], app[o]
            self.pulls += len(need)
        return self.params

    @traced("async_dense.add")
    def add(self, grad: torch.Tensor | None = None):
        if grad is not None:
            self.grad[: grad.numel()] += grad.reshape(-1).to(torch.float32)
        self._pending = True

    def slab_sink(self):
        """Split-K weight gradients left in fp32 planes that this table's push sums on the way into
        the inboxes (ops.linear_wgrad(defer=...): no reduce kernels, no pass through self.grad);
        None off the GPU push path . The planes are rewritten by the
        next clock's GEMMs, which the stream order puts after this clock's push."""
        from .tables import _WGRAD_DEFER, _SlabSink

        if not (_WGRAD_DEFER and self.cuda and self.shard % 4 == 0):
            return None
        sink = self.__dict__.get("_sink")
        if sink is None:
            sink = self._sink = _SlabSink(self)
        return sink

    @traced("async_dense.clock")
    def clock(self):
        slot = self._reserve_slot()
        off = (self.comm.rank * self.depth + slot) * self.slot_bytes
        S = self.shard
        sink = self.__dict__.get("_sink")
        slabs = sink.take(self.grad) if sink is not None else []
        if slabs and not (self._pending and self.cuda and S % 4 == 0):
            raise RuntimeError("async dense table: deferred weight-gradient planes need the GPU push path")
        if self._pending:
            if self.cuda and S % 4 == 0:  # one pass: every owner's slice into its slot, grad cleared
                from .._native import kernels

                kernels().ps_push_dense(self.grad, self._inbox_ptrs, off + _SLOT_HEADER, S, slabs)
            else:
                for o in range(self.comm.world):
                    dst = self._inbox[o][off + _SLOT_HEADER: off + _SLOT_HEADER + 4 * S].view(torch.float32)
                    dst.copy_(self.grad[o * S: (o + 1) * S])
                self.grad.zero_()
        if self.cuda:
            from .._native import kernels

            kernels().ps_set_headers(self._inbox_ptrs, off, 1 if self._pending else 0)
        else:
            for o in range(self.comm.world):
                self._inbox[o][off: off + 8].view(torch.int64)[0] = 1 if self._pending else 0
        self._pending = False
        self.step += 1
        self._advance()

    def _apply_slot_cpu(self, r: int, c: int):
        off = (r * self.depth + c % self.depth) * self.slot_bytes
        buf = self._inbox[self.comm.rank]
        if self.optimizer == "adam":
            self.cpu_step += 1  # one optimizer step per push, an empty one included (as the GPU applier)
        if int(buf[off: off + 8].view(torch.int64)[0]) == 0:
            return
        g = buf[off + _SLOT_HEADER: off + _SLOT_HEADER + 4 * self.shard].view(torch.float32).clone()
        if self.optimizer == "adam":
            ops.adam_apply(self.master, self.m, self.v, g, self.push_lr, self.betas[0], self.betas[1], self.eps,
                           self.weight_decay, self.cpu_step, 1.0, None)
        elif self.optimizer == "adagrad":
            ops.adagrad_apply(self.master, self.m, g, self.push_lr, self.eps, 1.0, None)
        elif self.optimizer == "sgd":
            ops.sgd_apply(self.master, g, self.lr, 1.0, None)
        else:
            self.master.add_(g)

    def _apply_clock_cpu(self, c: int):
        """Clock-coalesced apply (CPU twin of ps_clock_sum_dense + the optimizer): the active pushes
        of clock c summed in requester order, one optimizer step at lr."""
        buf = self._inbox[self.comm.rank]
        if self.optimizer == "adam":
            self.cpu_step += 1  # one optimizer step per clock (BSP's count)
        g, active = torch.zeros(self.shard, dtype=torch.float32), 0
        for r in range(self.comm.world):
            off = (r * self.depth + c % self.depth) * self.slot_bytes
            if int(buf[off: off + 8].view(torch.int64)[0]) != 0:
                g += buf[off + _SLOT_HEADER: off + _SLOT_HEADER + 4 * self.shard].view(torch.float32)
                active += 1
        if not active:
            return
        if self.optimizer == "adam":
            ops.adam_apply(self.master, self.m, self.v, g, self.lr, self.betas[0], self.betas[1], self.eps,
                           self.weight_decay, self.cpu_step, 1.0, None)
        else:
            ops.adagrad_apply(self.master, self.m, g, self.lr, self.eps, 1.0, None)

    # -- checkpoint hooks ------------------------------------------------------------------------
    def shard_state(self):
        self.drain()
        rows = max(0, min(self.shard, self.n_params - self.base))
        arrays = {"master": self.master[:rows]}
        if self.m is not None:
            arrays["m"] = self.m[:rows]
        if self.v is not None:
            arrays["v"] = self.v[:rows]
        meta = dict(global_rows=self.n_params, base=self.base, rows=rows, cols=1, clock=self.clock_n,
                    table_id=self.table_id, rank=self.comm.rank, world=self.comm.world, kind="dense")
        return meta, arrays

    def restore_range(self):
        return self.base, max(self.base, min(self.base + self.shard, self.n_params))

    def restore_dst(self):
        self.ps.pause()
        tabs = (("master", self.master), ("m", self.m), ("v", self.v))
        return {n: t.view(-1, 1) for n, t in tabs if t is not None}

    def finish_restore(self, clock: int):
        if self._pull_bf16:
            self._pulls[self.comm.rank].copy_(self.master.to(torch.bfloat16))
        # one optimizer step per clock (coalesced) or per push of every requester
        steps = int(clock) * (1 if self.coalesced else self.comm.world)
        if self.cuda:
            self.ps.server.set_step(self.t, steps)
            torch.cuda.synchronize(self.comm.device)
        self.cpu_step = steps
        self.step = int(clock)
        self._seen = [-1] * self.comm.world  # re-pull everything
        self._seen_applied = [-1] * self.comm.world
        self._restore_clock(clock)
        self.get()
