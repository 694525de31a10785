"""Observability of a PS rank.

MetricsLogger   structured JSONL per rank (``$MINIPS_METRICS_DIR/rank<r>.jsonl`` when set):
                step records (step time, samples/s, bytes pushed/pulled per collective and the
                achieved GB/s, staleness histogram, pending-buffer depth) and events (checkpoint,
                restore, fault-tolerance phases). Without the env var it only keeps counters.
range(name)     roctx range around Get / Add / Clock / collectives (and, natively, the owner's
traced(name)    apply batches: csrc/runtime/trace.h), so the phases show up in
                ``rocprofv3 --marker-trace`` timelines. Off unless MINIPS_ROCTX=1 (then
                librocprofiler-sdk-roctx is loaded): a disabled ``traced`` leaves the method
                untouched and a disabled ``range`` returns a shared null context.
                MINIPS_ROCTX=host instead accumulates each range's inclusive HOST time
                (perf_counter_ns) in HOST_TIMES -- the per-phase issue cost of a step
                (bench.py --host-phases prints it per step).
fault_tolerance_phase(n, detail)
                the reference's "[Fault Tolerance][PhaseN][ts] ..." line (base/utils.hpp:24-53).
"""
from __future__ import annotations

import collections
import contextlib
import ctypes
import json
import os
import sys
import threading
import time

_ROCTX = None
_ROCTX_TRIED = False
_ROCTX_ON = os.environ.get("MINIPS_ROCTX", "0") == "1"
_HOST_ON = os.environ.get("MINIPS_ROCTX", "0") == "host"
_NULL = contextlib.nullcontext()
# MINIPS_ROCTX=host: name -> [inclusive ns, calls]
HOST_TIMES: dict = collections.defaultdict(lambda: [0, 0])


class _HostRange:
    __slots__ = ("name", "t0")

    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        self.t0 = time.perf_counter_ns()
        return self

    def __exit__(self, *exc):
        e = HOST_TIMES[self.name]
        e[0] += time.perf_counter_ns() - self.t0
        e[1] += 1
        return False


def _roctx():
    global _ROCTX, _ROCTX_TRIED
    if not _ROCTX_TRIED:
        _ROCTX_TRIED = True
        if _ROCTX_ON:
            for name in ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
                         "libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
                try:
                    lib = ctypes.CDLL(name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    _ROCTX = lib
                    break
                except (OSError, AttributeError):
                    continue
    return _ROCTX


class _Range:
    __slots__ = ("lib", "name")

    def __init__(self, lib, name: str):
        self.lib, self.name = lib, name.encode()

    def __enter__(self):
        self.lib.roctxRangePushA(self.name)
        return self

    def __exit__(self, *exc):
        self.lib.roctxRangePop()
        return False


def phase(name: str):
    """A host-time phase (MINIPS_ROCTX=host), else the shared null context (one global check)."""
    return _HostRange(name) if _HOST_ON else _NULL


def host_times_reset():
    HOST_TIMES.clear()


def range(name: str):  # noqa: A001 - mirrors the roctx naming
    """roctx range context (a shared no-op context when roctx is off)."""
    if _HOST_ON:
        return _HostRange(name)
    lib = _roctx() if _ROCTX_ON else None
    return _NULL if lib is None else _Range(lib, name)


def traced(name: str):
    """Method decorator: the call runs inside roctx range ``name`` when MINIPS_ROCTX=1 at import;
    otherwise the method is returned unchanged (zero cost on the step's host path)."""

    def deco(fn):
        import functools

        if _HOST_ON:
            @functools.wraps(fn)
            def timed(*args, **kwargs):
                with _HostRange(name):
                    return fn(*args, **kwargs)

            return timed
        if not _ROCTX_ON:
            return fn

        @functools.wraps(fn)
        def wrapped(*args, **kwargs):
            lib = _roctx()
            if lib is None:
                return fn(*args, **kwargs)
            lib.roctxRangePushA(name.encode())
            try:
                return fn(*args, **kwargs)
            finally:
                lib.roctxRangePop()

        return wrapped

    return deco


class MetricsLogger:
    def __init__(self, rank: int = 0, path: str | None = None):
        self.rank = rank
        self.path = path
        self._f = None
        self._lock = threading.Lock()
        self.staleness_hist: collections.Counter = collections.Counter()
        self.pending_depth_max = 0
        self.steps = 0
        self._last = None

    def _write(self, rec: dict):
        if self.path is None:
            return
        with self._lock:
            if self._f is None:
                os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
                self._f = open(self.path, "a", buffering=1)
            self._f.write(json.dumps(rec) + "\n")

    def event(self, kind: str, **fields):
        self._write(dict(ts=time.time(), rank=self.rank, event=kind, **fields))

    def observe_staleness(self, s: int):
        self.staleness_hist[int(s)] += 1

    def observe_pending(self, depth: int):
        self.pending_depth_max = max(self.pending_depth_max, int(depth))

    def step(self, step: int, samples: int, seconds: float, comm_stats=None, **extra):
        """One training-step record; comm_stats is a CommStats (bytes since the last call)."""
        self.steps += 1
        rec = dict(ts=time.time(), rank=self.rank, step=step, step_ms=round(seconds * 1e3, 4),
                   samples_per_s=round(samples / seconds, 1) if seconds > 0 else None)
        if comm_stats is not None:
            d = comm_stats.as_dict()
            buckets = d.pop("bucket_bytes", {})
            prev = self._last or {k: 0 for k in d}
            delta = {k: d[k] - prev.get(k, 0) for k in d}
            prev_b = prev.get("bucket_bytes", {})
            self._last = dict(d, bucket_bytes=buckets)
            if buckets:  # per-bucket RS + AG bytes of bucketed dense clocks (this step)
                rec["bucket_bytes"] = {k: v - prev_b.get(k, 0) for k, v in buckets.items()}
            moved = delta["bytes_a2a"] + delta["bytes_rs"] + delta["bytes_ag"]
            rec.update(bytes_pushed=delta["bytes_a2a"] // 2 + delta["bytes_rs"],
                       bytes_pulled=delta["bytes_a2a"] - delta["bytes_a2a"] // 2 + delta["bytes_ag"],
                       collectives=delta["calls"],
                       xgmi_gbps=round(moved / seconds / 1e9, 3) if seconds > 0 else None)
        if self.staleness_hist:
            rec["staleness_hist"] = dict(self.staleness_hist)
        if self.pending_depth_max:
            rec["pending_depth_max"] = self.pending_depth_max
        rec.update(extra)
        self._write(rec)
        return rec

    def close(self):
        with self._lock:
            if self._f is not None:
                self._f.close()
                self._f = None


_LOGGER: MetricsLogger | None = None


def get_logger() -> MetricsLogger:
    global _LOGGER
    if _LOGGER is None:
        rank = int(os.environ.get("RANK", "0"))
        d = os.environ.get("MINIPS_METRICS_DIR")
        _LOGGER = MetricsLogger(rank, os.path.join(d, f"rank{rank}.jsonl") if d else None)
    return _LOGGER


_PHASES = {1: "Phase1", 2: "Phase2 detect failure", 3: "Phase3 restart", 4: "Phase4 recover",
           5: "Phase5 others recovered"}


def fault_tolerance_phase(phase: int, detail: str = "", stream=None):
    """Reference log line "[Fault Tolerance][Phase<n>][<unix ms>] <name>: <detail>" (base/utils.hpp:24-53),
    same text as the native runtime's CheckFaultTolerance."""
    ts = int(time.time() * 1000)
    line = f"[Fault Tolerance][Phase{phase}][{ts}] {_PHASES.get(phase, 'Phase?')}" + (f": {detail}" if detail else "")
    print(line, file=stream or sys.stderr, flush=True)
    get_logger().event("fault_tolerance", phase=phase, detail=detail, ts_ms=ts)
    return line
