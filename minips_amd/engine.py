"""The Engine API on GPU ranks: tables by ``create_table``, tasks by ``run``, several workers per
rank with their own clocks -- the reference's driver/engine.hpp for one process per MI355X.

Reference parity
  Engine::CreateTable<Val>(ranges, ModelType, StorageType, staleness)   driver/engine.hpp:289-357
  Engine::Run(MLTask): one user thread per local worker with an Info    driver/engine.cpp:246-297
  MLTask {lambda, worker alloc, tables}                                 driver/ml_task.hpp:12-66
  Info {thread_id, worker_id, CreateKVClientTable}                      driver/info.hpp:17-43
  KVClientTable::{Get, Add, Clock, CheckPoint}                          worker/kv_client_table.hpp:45-71
  ProgressTracker over the worker tids (unique-min rule)                server/util/progress_tracker.cpp
  worker thread ids node*1000 + [100, 1000)                             driver/simple_id_mapper.cpp:49-62

How the workers of one rank meet the GPU tables (one table shard per rank, not per thread):
  * every worker's Clock advances ITS tid in the native ProgressTracker (minips_amd._runtime) of
    the table; the rank's table clock advances when the tracker's min clock does -- the reference's
    server-side rule (a clock is complete when the slowest worker clocked);
  * transport "onesided" (SSP / ASP, ps/onesided.py): workers run free. A worker's Get is gated
    on ITS OWN progress p: every owner applied every worker's clocks < p - s -- the per-worker
    SSP guarantee of ssp_model.cpp:58-85, with the slowest worker of every rank included (a
    rank publishes the min over its workers). Adds of all local workers join the rank's push of
    the clock in which they happened;
  * transport "collective" (BSP, or SSP/ASP over RCCL): every table operation is
    a collective, so the local workers go in lockstep: their Gets of a clock are served by ONE
    combined Get (BSP: every worker of the superstep reads the same values, exactly the
    reference's), their Adds are summed into the one push of the clock. Workers must then issue
    the same sequence of Get / Add / Clock (the reference apps do).
"""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass, field
from typing import Callable

import torch

from .ps.comm import Comm, init_distributed

WORKER_TID_BASE = 100  # SimpleIdMapper: worker threads take node*1000 + [100, 1000)


def create_table(comm: Comm, kind: str = "sparse", *, num_rows: int = 0, width: int = 1, n_params: int = 0,
                 model: str = "bsp", staleness: int = 0, storage: str = "vector", transport: str = "collective",
                 optimizer: str = "add", lr: float = 0.01, value_dtype=torch.float32, pull_dtype=None,
                 table_id: int = 0, **kw):
    """One PS table on this rank (collective over the ranks of ``comm``: every rank creates the same
    tables in the same order). ``kind`` "sparse" (rows of ``width`` values, keys in [0, num_rows);
    storage "map": unbounded 63-bit keys in a GPU hash table) or "dense" (one vector of
    ``n_params``); ``model`` bsp | ssp | asp; ``transport`` collective (RCCL) | onesided (the
    asynchronous PS, SSP / ASP only; range rows in fp32 or bf16, or Map storage)."""
    from .ps.tables import DenseTable, HashSparseTable, SparseTable

    model = model.lower()
    storage = storage.lower()
    if transport == "onesided":
        from .ps.onesided import AsyncDenseTable, AsyncHashTable, AsyncSparseTable

        if kind == "dense":
            if value_dtype != torch.float32:
                raise ValueError("one-sided dense tables keep an fp32 master")
            return AsyncDenseTable(comm, n_params, optimizer=optimizer, lr=lr, consistency=model, staleness=staleness,
                                   pull_dtype=pull_dtype or torch.bfloat16, table_id=table_id, **kw)
        if storage == "map":
            if value_dtype != torch.float32:
                raise ValueError("one-sided Map storage keeps fp32 rows (MapStorage sums exactly)")
            return AsyncHashTable(comm, width, optimizer=optimizer, lr=lr, consistency=model, staleness=staleness,
                                  pull_dtype=pull_dtype or torch.float32, table_id=table_id, **kw)
        return AsyncSparseTable(comm, num_rows, width, optimizer=optimizer, lr=lr, consistency=model,
                                staleness=staleness, pull_dtype=pull_dtype or torch.float32, table_id=table_id,
                                value_dtype=value_dtype, **kw)
    if kind == "dense":
        return DenseTable(comm, n_params, optimizer=optimizer, lr=lr, consistency=model, staleness=staleness,
                          pull_dtype=pull_dtype or (torch.float64 if value_dtype == torch.float64 else torch.bfloat16),
                          table_id=table_id, value_dtype=value_dtype, **kw)
    if storage == "map":
        return HashSparseTable(comm, width, optimizer=optimizer, lr=lr, consistency=model, staleness=staleness,
                               pull_dtype=pull_dtype or torch.float32, table_id=table_id, **kw)
    return SparseTable(comm, num_rows, width, optimizer=optimizer, lr=lr, consistency=model, staleness=staleness,
                       pull_dtype=pull_dtype or (torch.float64 if value_dtype == torch.float64 else torch.float32),
                       table_id=table_id, value_dtype=value_dtype, **kw)


@dataclass
class MLTask:
    """What Engine.run executes: ``fn(info)`` on every worker (driver/ml_task.hpp)."""
    fn: Callable | None = None
    workers_per_rank: int = 1
    alloc: dict = field(default_factory=dict)  # rank -> workers (overrides workers_per_rank)
    tables: list | None = None                  # table ids the workers use (None: every table)

    def set_lambda(self, fn):
        self.fn = fn

    def set_worker_alloc(self, alloc):
        """[(rank, n_workers)] like the reference's WorkerAlloc list (node id -> rank)."""
        self.alloc = {int(r): int(n) for r, n in alloc}

    def set_tables(self, tables):
        self.tables = list(tables)

    def workers_on(self, rank: int) -> int:
        return self.alloc.get(rank, self.workers_per_rank)


class _Group:
    """The workers of this rank on one table: their progress (native ProgressTracker), and either
    the lockstep combiner (collective transport) or per-worker gating (one-sided)."""

    def __init__(self, engine: "Engine", table_id: int, tids: list):
        from ._native import runtime

        self.engine, self.table_id = engine, table_id
        self.table = engine.tables[table_id]
        self.onesided = hasattr(self.table, "ps")
        self.tracker = runtime().ProgressTracker()
        self.tracker.init(tids)
        self.base_clock = getattr(self.table, "clock_n", 0) if self.onesided else 0
        self.W = len(tids)
        self.lock = threading.Lock()
        self.cv = threading.Condition(self.lock)
        # lockstep state
        self._gen = 0
        self._arrived: list = []
        self._results: dict = {}
        self._error: BaseException | None = None
        # adds of the current clock (both modes): (keys, vals)
        self._adds: list = []

    # -- progress ---------------------------------------------------------------------------
    def progress(self, tid: int) -> int:
        return self.tracker.get_progress(tid)

    def _rank_clock(self, tid: int) -> bool:
        """Advance tid; True when the rank's min clock moved (this worker completes the clock)."""
        return self.tracker.advance_and_get_changed_min_clock(tid) != -1

    # -- one-sided: workers run free ------------------------------------------------------------
    def _async_get(self, tid, keys):
        p = self.base_clock + self.progress(tid)
        if keys is None:
            return self.table.get(clock=p)
        rows, plan = self.table.get(keys, clock=p)
        return rows[plan.inv]

    def _async_clock(self, tid):
        with self.lock:
            done = self._rank_clock(tid)
            if not done:
                return
            adds, self._adds = self._adds, []
            self._push(adds)
            self.table.clock()

    def _push(self, adds):
        t = self.table
        if not adds:
            return
        if hasattr(t, "add_keys"):
            keys = torch.cat([k.reshape(-1) for k, _ in adds])
            vals = torch.cat([v.reshape(k.numel(), -1) for k, v in adds])
            t.add_keys(keys, vals)
        else:  # dense: sum of the workers' gradient vectors
            g = adds[0][1].reshape(-1).clone()
            for _, v in adds[1:]:
                g += v.reshape(-1)
            t.add(g)

    # -- collective: lockstep ----------------------------------------------------------------------
    def _lockstep(self, tid, op, payload):
        """Every local worker calls the same op; the last to arrive runs the combined op."""
        with self.cv:
            gen = self._gen
            self._arrived.append((tid, op, payload))
            if len(self._arrived) == self.W:
                arrived, self._arrived = self._arrived, []
                try:
                    self._results = self._run_combined(arrived)
                    self._error = None
                except BaseException as e:  # every worker of the generation sees it
                    self._results, self._error = {}, e
                self._gen += 1
                self.cv.notify_all()
            else:
                while self._gen == gen:
                    self.cv.wait()
            if self._error is not None:
                raise self._error
            return self._results.get(tid)

    def _run_combined(self, arrived):
        ops = {op for _, op, _ in arrived}
        if len(ops) != 1:
            raise RuntimeError(f"workers of one rank issued different table ops in lockstep: {sorted(ops)} "
                               "(collective tables need the same Get/Add/Clock sequence on every worker)")
        op = ops.pop()
        t = self.table
        if op == "get":
            if arrived[0][2] is None:  # dense
                v = t.get()
                return {tid: v for tid, _, _ in arrived}
            keys = [k.reshape(-1) for _, _, k in arrived]
            rows = t.get_rows(torch.cat(keys))
            out, o = {}, 0
            for (tid, _, _), k in zip(arrived, keys):
                out[tid] = rows[o: o + k.numel()]
                o += k.numel()
            return out
        if op == "add":
            self._adds.extend(p for _, _, p in arrived)
            return {}
        if op == "clock":
            for tid, _, _ in arrived:
                self._rank_clock(tid)
            adds, self._adds = self._adds, []
            self._push(adds)
            t.clock()
            return {}
        raise ValueError(op)

    # -- the KV API of one worker ------------------------------------------------------------------
    def get(self, tid, keys):
        if self.onesided:
            return self._async_get(tid, keys)
        return self._lockstep(tid, "get", keys)

    def add(self, tid, keys, vals):
        if self.onesided:
            with self.lock:
                self._adds.append((keys, vals))
            return
        self._lockstep(tid, "add", (keys, vals))

    def clock(self, tid):
        if self.onesided:
            self._async_clock(tid)
        else:
            self._lockstep(tid, "clock", None)


class KVClientTable:
    """One worker's view of a table (worker/kv_client_table.hpp): Get blocks and returns the values
    of ``keys`` in request order; Add and Clock are asynchronous."""

    def __init__(self, group: _Group, tid: int):
        self.group, self.tid = group, tid

    def get(self, keys: torch.Tensor | None = None) -> torch.Tensor:
        return self.group.get(self.tid, keys)

    def add(self, keys: torch.Tensor | None, vals: torch.Tensor):
        self.group.add(self.tid, keys, vals)

    def clock(self):
        self.group.clock(self.tid)

    def progress(self) -> int:
        return self.group.progress(self.tid)

    # reference spellings
    Get, Add, Clock = get, add, clock


@dataclass
class Info:
    """Per-worker context (driver/info.hpp): its thread id, its task-wide worker id, the rank and
    device, and the table views."""
    thread_id: int
    worker_id: int
    local_id: int
    rank: int
    device: torch.device
    num_workers: int
    _groups: dict = field(default_factory=dict, repr=False)

    def create_kv_client_table(self, table_id: int) -> KVClientTable:
        return KVClientTable(self._groups[table_id], self.thread_id)

    CreateKVClientTable = create_kv_client_table


class Engine:
    """One per rank: ``create_table`` (collective), ``barrier``, ``run(task)``, ``checkpoint`` /
    ``restore``, ``stop``."""

    def __init__(self, comm: Comm | None = None):
        self.comm = comm or init_distributed()
        self.rank, self.world = self.comm.rank, self.comm.world
        self.tables: dict[int, object] = {}
        self._ckpt = None

    # reference: Engine::CreateTable<Val>(ranges, ModelType, StorageType, staleness)
    def create_table(self, kind: str = "sparse", **kw) -> int:
        tid = len(self.tables)
        self.tables[tid] = create_table(self.comm, kind, table_id=tid, **kw)
        return tid

    CreateTable = create_table

    def table(self, tid: int):
        return self.tables[tid]

    def barrier(self):
        self.comm.barrier()

    Barrier = barrier

    def run(self, task: MLTask) -> list:
        """Run task.fn(info) on this rank's workers (threads); returns their results in local
        order. Task-wide worker ids are consecutive over the ranks (driver/worker_spec.cpp)."""
        if task.fn is None:
            raise ValueError("MLTask has no lambda")
        counts = [task.workers_on(r) for r in range(self.world)]
        W = counts[self.rank]
        first = sum(counts[: self.rank])
        tids = [self.rank * 1000 + WORKER_TID_BASE + w for w in range(W)]
        groups = {t: _Group(self, t, tids) for t in (list(self.tables) if task.tables is None else task.tables)}
        results: list = [None] * W
        errors: list = []

        def body(w):
            info = Info(tids[w], first + w, w, self.rank, self.comm.device, sum(counts), groups)
            try:
                if self.comm.device.type == "cuda":
                    torch.cuda.set_device(self.comm.device)
                results[w] = task.fn(info)
            except BaseException as e:  # noqa: BLE001 - re-raised on the calling thread
                errors.append(e)
                for g in groups.values():  # free lockstep peers waiting for this worker
                    with g.cv:
                        g._error = e
                        g._gen += 1
                        g.cv.notify_all()

        if W == 1:
            body(0)
        else:
            threads = [threading.Thread(target=body, args=(w,), name=f"minips-worker-{w}") for w in range(W)]
            for th in threads:
                th.start()
            for th in threads:
                th.join()
        if errors:
            raise errors[0]
        for t in groups.values():
            t.table.drain()
        return results

    Run = run

    def checkpoint(self, prefix: str, iteration: int):
        """Every table's shards at ``iteration`` (collective; the reference's KVClientTable::
        CheckPoint, answered by every server)."""
        from .ps.checkpoint import Checkpointer

        if self._ckpt is None or self._ckpt.prefix != prefix:
            self._ckpt = Checkpointer(self.comm, prefix)
        self._ckpt.save(self.tables, iteration, blocking=True)

    def restore(self, prefix: str) -> int:
        from .ps.checkpoint import Checkpointer

        return Checkpointer(self.comm, prefix).load(self.tables)

    def stop(self):
        """StopEverything: drain every table, meet, release the asynchronous server."""
        for t in self.tables.values():
            t.drain()
        self.comm.barrier()
        ps = getattr(self.comm, "_async_ps", None)
        if ps is not None:
            ps.close()

    StopEverything = stop


def main_env_engine() -> Engine:
    """An Engine from the torchrun environment (tests / apps)."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    return Engine(init_distributed())
