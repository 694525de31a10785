"""Really asynchronous SSP / ASP for GPU ranks: one-sided row access over xGMI.

A collective rendezvous at every clock (all-to-all, reduce-scatter) makes every rank wait for the
slowest one, whatever the staleness setting. The reference's ASPModel replies and applies
immediately (server/consistency/asp_model.cpp:18-26) and SSPModel lets a worker run up to
``staleness`` clocks ahead of the slowest worker (ssp_model.cpp:58-85, progress_tracker.cpp:46-72).
This table gets the same semantics with NO collective on the data path:

* every rank hipMallocs its shard (equal key ranges, fp32 rows) and exports it with
  hipIpcGetMemHandle; every rank maps every peer shard (hipIpcOpenMemHandle, peer access over
  xGMI), so any GPU addresses the whole table through a device table of base pointers
  (csrc/kernels/onesided.hip);
* Get = direct gather of the requested rows from their owners' HBM; Add + Clock = atomic
  scatter-add into the owners' rows (``add``: w += delta, the reference SubAdd; ``sgd``:
  w -= lr * g, the ASP async SGD of the DLRM config) -- the owner does nothing;
* progress: a clock vector in host shared memory (/dev/shm, one slot per rank; the native
  csrc/runtime/clock_board.h, futex wake-ups). A rank
  publishes clock c+1 only after its clock-c adds completed on the GPU (a publisher thread
  waits on the event recorded after them), so a reader that sees clock c+1 sees those adds.
* SSP gate (a Get at own clock c): wait until min over ranks >= c - staleness -- the
  reference's "buffer the Get while progress > min_clock + staleness". ASP never waits.

The same code runs on CPU ranks (gloo tests) with the shards in /dev/shm files (np.memmap) and
a per-owner file lock around the scatter-add in place of the GPU atomics.
"""
from __future__ import annotations

import fcntl
import os
import queue
import threading
import time
import uuid
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from .comm import Comm
from .tables import even_bounds


class ClockBoard:
    """Per-rank clocks in a /dev/shm segment shared by the ranks of one node: the native board
    (csrc/runtime/clock_board.h -- one cache line per rank, release stores, a futex the SSP gate
    sleeps on instead of polling from Python)."""

    def __init__(self, comm: Comm, name: str | None = None):
        from .._native import runtime

        self.comm = comm
        self.world, self.rank = comm.world, comm.rank
        if name is None:
            name = f"minips_clock_{uuid.uuid4().hex}" if comm.rank == 0 else None
            if comm.world > 1:
                box = [name]
                dist.broadcast_object_list(box, src=0, group=comm.group)
                name = box[0]
        self.path = os.path.join("/dev/shm", name)
        self.owner = comm.rank == 0
        self._b = runtime().ClockBoard(name, max(1, self.world), self.rank, self.owner)

    def publish(self, clock: int):
        self._b.publish(int(clock))

    def get(self, rank: int) -> int:
        return self._b.get(rank)

    def min_clock(self) -> int:
        return self._b.min_clock()

    def wait_min(self, target: int, timeout_s: float = 0.0) -> float:
        """Block (GIL released, futex sleep) until min clock >= target; returns seconds waited."""
        return self._b.wait_min_at_least(int(target), float(timeout_s))

    def snapshot(self) -> list:
        return list(self._b.snapshot())

    def close(self):
        if self.owner:
            self._b.unlink()


@dataclass
class OneSidedPlan:
    """Routing of one batch: the unique keys (no per-owner grouping needed: the kernels find
    each key's owner)."""
    keys_n: int
    inv: torch.Tensor        # [n] position of each requested key in the unique order
    uniq: torch.Tensor       # [n] unique keys (first U valid)
    cap: int
    U_dev: torch.Tensor | None = None
    csr: tuple | None = None
    extra: dict = field(default_factory=dict)
    _U: int | None = None

    @property
    def U(self) -> int:
        if self._U is None:
            self._U = self.cap if self.U_dev is None else int(self.U_dev.item())
        return self._U


class OneSidedSparseTable:
    def __init__(self, comm: Comm, num_rows: int, width: int, optimizer: str = "sgd", lr: float = 0.01,
                 consistency: str = "asp", staleness: int = 0, pull_dtype=torch.float32, init_std: float = 0.0,
                 seed: int = 1234, table_id: int = 0):
        if optimizer not in ("add", "sgd"):
            raise ValueError("one-sided tables apply by atomic adds: optimizer 'add' or 'sgd'")
        if consistency not in ("ssp", "asp"):
            raise ValueError("one-sided tables serve SSP / ASP (BSP uses the collective SparseTable)")
        self.comm, self.table_id = comm, table_id
        self.num_rows, self.width = num_rows, width
        self.optimizer, self.lr = optimizer, lr
        self.consistency = consistency
        self.staleness = staleness if consistency == "ssp" else 0
        self.pull_dtype = pull_dtype
        dev = comm.device
        self.cuda = dev.type == "cuda"
        b = even_bounds(num_rows, comm.world)
        self.bounds_list = b
        self.bounds = torch.tensor(b, dtype=torch.int64, device=dev)
        self.base = b[comm.rank]
        self.rows_local = b[comm.rank + 1] - b[comm.rank]
        self._own_bounds = torch.tensor([0, (1 << 63) - 1], dtype=torch.int64, device=dev)
        rows_of = [b[r + 1] - b[r] for r in range(comm.world)]
        nbytes = [max(4 * width * n, 256) for n in rows_of]
        if self.cuda:
            from .._native import kernels

            buf, handle = kernels().ipc_alloc(nbytes[comm.rank], dev.index)
            handles = [None] * comm.world
            if comm.world > 1:
                dist.all_gather_object(handles, handle, group=comm.group)
            else:
                handles = [handle]
            self._mapped = [buf if r == comm.rank else kernels().ipc_open(handles[r], nbytes[r], dev.index)
                            for r in range(comm.world)]
            self.bases = torch.tensor([m.data_ptr() for m in self._mapped], dtype=torch.int64, device=dev)
            self.shard = buf[: 4 * width * self.rows_local].view(torch.float32).view(self.rows_local, width)
            self._locks = None
        else:
            name = f"minips_tab_{uuid.uuid4().hex}" if comm.rank == 0 else None
            if comm.world > 1:
                box = [name]
                dist.broadcast_object_list(box, src=0, group=comm.group)
                name = box[0]
            self._paths = [os.path.join("/dev/shm", f"{name}_{r}") for r in range(comm.world)]
            mine = np.memmap(self._paths[comm.rank], dtype=np.float32, mode="w+", shape=(max(1,
                                                                                             self.rows_local), width))
            mine[:] = 0
            mine.flush()
            if comm.world > 1:
                dist.barrier(group=comm.group)  # every shard file exists
            self._views = [torch.from_numpy(np.memmap(p, dtype=np.float32, mode="r+",
                                                      shape=(max(1, rows_of[r]), width)))
                           for r, p in enumerate(self._paths)]
            self.shard = self._views[comm.rank][: self.rows_local]
            self._locks = [open(p, "rb") for p in self._paths]
        if init_std > 0:
            g = torch.Generator(device=dev)
            g.manual_seed(seed + 7919 * comm.rank)
            self.shard.normal_(0.0, init_std, generator=g)
        self.board = ClockBoard(comm)
        # a straggler that never publishes again is a failure (the supervisor restarts the set),
        # not an infinite hang of every other rank
        self.gate_timeout_s = float(os.environ.get("MINIPS_SSP_GATE_TIMEOUT", "600"))
        self.clock_n = 0
        self._pending: list = []
        self.waited_s = 0.0
        self.staleness_seen: list = []
        if self.cuda:
            self._pub_q: queue.Queue = queue.Queue()
            self._pub = threading.Thread(target=self._publisher, name="minips-clock-pub", daemon=True)
            self._pub.start()
        if comm.world > 1:
            comm.barrier()  # every rank mapped every shard and initialised its own rows

    # ------------------------------------------------------------------------------ progress
    def _publisher(self):
        while True:
            item = self._pub_q.get()
            if item is None:
                return
            ev, c = item
            ev.synchronize()  # this clock's atomic adds have completed in the owners' HBM
            self.board.publish(c)

    def _gate(self):
        """SSP: a Get at own clock c waits while c > min_clock + staleness (ssp_model.cpp:58-85)."""
        c = self.clock_n
        if self.consistency == "ssp":
            self.waited_s += self.board.wait_min(c - self.staleness, self.gate_timeout_s)
        self.staleness_seen.append(c - self.board.min_clock())

    # ------------------------------------------------------------------------------ KV API
    def _plan(self, keys: torch.Tensor) -> OneSidedPlan:
        flat = keys.reshape(-1).to(torch.int64)
        uniq, inv, _, U_dev = ops.unique_bucketize_n(flat, self._own_bounds)
        if self.cuda:
            return OneSidedPlan(flat.numel(), inv, uniq, flat.numel(), U_dev=U_dev)
        U = int(U_dev.reshape(-1)[0])
        return OneSidedPlan(flat.numel(), inv, uniq, U, _U=U)

    def get(self, keys: torch.Tensor, plan=None):
        """Rows of the unique keys ([cap, width], unique order) and the plan (rows[plan.inv[i]]
        is the row of keys[i]). No collective: rows come straight from the owners' HBM."""
        plan = plan or self._plan(keys)
        self._gate()
        out = torch.empty(max(plan.cap, 1), self.width, dtype=self.pull_dtype, device=self.comm.device)
        if self.cuda:
            from .._native import kernels

            kernels().remote_gather(self.bases, self.bounds, plan.uniq, plan.U_dev, self.width, out)
        else:
            u = plan.uniq[: plan.U]
            for r in range(self.comm.world):
                lo, hi = self.bounds_list[r], self.bounds_list[r + 1]
                m = (u >= lo) & (u < hi)
                if bool(m.any()):
                    out[: plan.U][m] = self._views[r][u[m] - lo].to(out.dtype)
        return out, plan

    def get_rows(self, keys: torch.Tensor) -> torch.Tensor:
        rows, plan = self.get(keys)
        return rows[plan.inv]

    # SparseTable-compatible planning API (models call plan / plan_async / advance_plan): a plan
    # is a local dedupe only, there is no count exchange to overlap
    def plan(self, keys: torch.Tensor, csr: bool = False) -> OneSidedPlan:
        return self._plan(keys)

    def plan_async(self, keys: torch.Tensor, csr: bool = False, keys_on_plan_stream: bool = False):
        return self._plan(keys)

    def advance_plan(self, pending, finish: bool = True):
        return pending

    def add(self, plan: OneSidedPlan, grad_rows: torch.Tensor):
        assert grad_rows.shape[0] >= plan.cap and grad_rows.dtype == torch.float32
        self._pending.append((plan, grad_rows))

    def add_lookup_grads(self, plan: OneSidedPlan, dX: torch.Tensor, dwide, F: int, D: int, x_off: int = 0):
        """Per-lookup gradients (SparseTable.add_lookup_grads): segment-summed per unique row here,
        then atomically added into the owners' rows at the clock."""
        dev = self.comm.device
        g = (torch.empty if dev.type == "cuda" else torch.zeros)(max(plan.cap, 1), self.width, dtype=torch.float32,
                                                                 device=dev)
        ops.wd_emb_backward(dX, dwide, plan.inv, F, D, g, x_off=x_off, U_dev=getattr(plan, "U_dev", None),
                            csr=getattr(plan, "csr", None))
        self.add(plan, g)

    def add_keys(self, keys: torch.Tensor, vals: torch.Tensor):
        plan = self._plan(keys)
        g = torch.zeros(max(plan.cap, 1), self.width, dtype=torch.float32, device=self.comm.device)
        ops.scatter_add_rows(vals.reshape(keys.numel(), self.width).to(torch.float32).contiguous(), plan.inv, g)
        self.add(plan, g)

    def clock(self):
        """Apply the buffered adds into the owners' rows (atomics), then publish clock+1."""
        scale = 1.0 if self.optimizer == "add" else -self.lr
        pending, self._pending = self._pending, []
        for plan, g in pending:
            if self.cuda:
                from .._native import kernels

                kernels().remote_scatter_add(self.bases, self.bounds, plan.uniq, g.contiguous(), scale, plan.U_dev)
            else:
                u = plan.uniq[: plan.U]
                for r in range(self.comm.world):
                    lo, hi = self.bounds_list[r], self.bounds_list[r + 1]
                    m = (u >= lo) & (u < hi)
                    if bool(m.any()):
                        fcntl.flock(self._locks[r], fcntl.LOCK_EX)
                        try:
                            self._views[r].index_add_(0, u[m] - lo, scale * g[: plan.U][m])
                        finally:
                            fcntl.flock(self._locks[r], fcntl.LOCK_UN)
        self.clock_n += 1
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.comm.device))
            self._pub_q.put((ev, self.clock_n))
        else:
            self.board.publish(self.clock_n)

    def drain(self):
        """Wait until this rank's clocks are applied and published."""
        if self.cuda:
            torch.cuda.current_stream(self.comm.device).synchronize()
            while not self._pub_q.empty() or self.board.get(self.comm.rank) < self.clock_n:
                time.sleep(0.0005)

    def close(self):
        self.drain()
        if self.cuda:
            self._pub_q.put(None)
            self._pub.join(timeout=5)
        self.board.close()
        if not self.cuda:
            for f in self._locks:
                f.close()
            if self.comm.rank == 0:
                for p in self._paths:
                    try:
                        os.unlink(p)
                    except FileNotFoundError:
                        pass

    # -- checkpoint hooks (minips_amd.ps.checkpoint) -------------------------------------------
    def shard_state(self):
        self.drain()
        meta = dict(global_rows=self.num_rows, base=self.base, rows=self.rows_local, cols=self.width,
                    clock=self.clock_n, table_id=self.table_id, rank=self.comm.rank, world=self.comm.world,
                    kind="sparse")
        return meta, {"params": self.shard}

    def restore_range(self):
        return self.base, self.base + self.rows_local

    def restore_dst(self):
        return {"params": self.shard}

    def finish_restore(self, clock: int):
        self.clock_n = int(clock)
        self.board.publish(self.clock_n)

    def reset_after_rollback(self):
        self._pending = []


class OneSidedDenseTable:
    """A flat dense parameter vector on the one-sided path (ASP / SSP async SGD): the vector is
    cut into rows of ``row`` values, row-partitioned over the ranks like a sparse table; Get
    gathers every row from its owner's HBM (the pull), Add + Clock atomically adds -lr * grad
    into the owners' rows. Same API as ps.tables.DenseTable (grad buffer written in place by
    the models, get / add / clock / load_full / full_master)."""

    def __init__(self, comm: Comm, n_params: int, lr: float = 1e-3, consistency: str = "asp", staleness: int = 0,
                 pull_dtype=torch.bfloat16, table_id: int = 0, row: int = 64, optimizer: str = "sgd"):
        self.comm, self.n_params, self.table_id = comm, n_params, table_id
        self.row = row
        self.rows = -(-n_params // row)
        self.n_pad = self.rows * row
        self.lr = lr
        self.pull_dtype = pull_dtype
        self.optimizer = optimizer
        self.t = OneSidedSparseTable(comm, self.rows, row, optimizer=optimizer, lr=lr, consistency=consistency,
                                     staleness=staleness, pull_dtype=torch.float32, table_id=table_id)
        dev = comm.device
        self._keys = torch.arange(self.rows, dtype=torch.int64, device=dev)
        self._plan = OneSidedPlan(self.rows, self._keys, self._keys, self.rows, _U=self.rows)
        self.params = torch.zeros(self.n_pad, dtype=pull_dtype, device=dev)
        self.grad = torch.zeros(self.n_pad, dtype=torch.float32, device=dev)
        self._full = torch.empty(self.rows, row, dtype=torch.float32, device=dev)
        self._pending = False
        self.step = 0

    @property
    def clock_n(self):
        return self.t.clock_n

    def load_full(self, full: torch.Tensor):
        flat = torch.zeros(self.n_pad, dtype=torch.float32, device=self.comm.device)
        flat[: self.n_params] = full.to(self.comm.device, torch.float32)
        lo, hi = self.t.base, self.t.base + self.t.rows_local
        self.t.shard.copy_(flat.view(self.rows, self.row)[lo:hi])
        self.params.copy_(flat.to(self.pull_dtype))
        if self.comm.world > 1:
            self.comm.barrier()

    def full_master(self) -> torch.Tensor:
        self.drain()
        rows, _ = self.t.get(self._keys, plan=self._plan)
        return rows.reshape(-1)[: self.n_params]

    def get(self) -> torch.Tensor:
        rows, _ = self.t.get(self._keys, plan=self._plan)
        self.params.copy_(rows.reshape(-1).to(self.pull_dtype))
        return self.params

    def add(self, grad: torch.Tensor | None = None):
        if grad is not None:
            self.grad[: grad.numel()] += grad.reshape(-1).to(torch.float32)
        self._pending = True

    def clock(self):
        if self._pending:
            self.t.add(self._plan, self.grad.view(self.rows, self.row).clone())
            self.grad.zero_()
        self._pending = False
        self.t.clock()
        self.step += 1

    def drain(self):
        self.t.drain()

    def close(self):
        self.t.close()

    def shard_state(self):
        meta, arrays = self.t.shard_state()
        meta.update(global_rows=self.rows, kind="sparse")
        return meta, arrays

    def restore_range(self):
        return self.t.restore_range()

    def restore_dst(self):
        return self.t.restore_dst()

    def finish_restore(self, clock: int):
        self.t.finish_restore(clock)
        self.step = int(clock)
        self.get()

    def reset_after_rollback(self):
        self.t.reset_after_rollback()
        self._pending = False
        self.grad.zero_()
