"""Low-overhead HIP stream helpers for the per-step issue path.

``torch.cuda.current_stream(dev)`` and ``with torch.cuda.stream(s):`` resolve the device through
several Python layers (``_get_device_index`` -> ``_get_device_attr`` -> ``is_available`` ...) on
every call: ~19 such resolutions per W&D step cost ~25-40 us of its ~0.3 ms host issue
(tools/step_probe.py cprofile). These helpers go straight to the C entry points torch itself ends
in (``_cuda_getCurrentStream`` / ``_cuda_setStream`` / ``_cuda_getCurrentRawStream``), with the
same semantics for a stream of the process's own device (one device per rank here).
"""
from __future__ import annotations

import os

import torch

# MINIPS_STREAM_DEBUG (race diagnostics; tests/test_multirank_gpu.py, tools/gpu_round.sh race): comma-separated
#   delay=<us>         every work segment issued on another stream through use() or SideStream.fork()
#                      starts with an n-us device spin, so a consumer that misses its wait on a producer
#                      stream reads stale data deterministically instead of by timing luck -- and a
#                      missing edge no longer hides behind the latency of a system-fence event
#   where=use+fork     which segments get the spin: "use" (streams.use: planning, clock pipelines, the
#                      one-sided push stream), "fork" (SideStream.fork: the weight-gradient stream),
#                      "main" (at every SideStream.fork the stream forked FROM continues late: a side
#                      stream that writes what the compute stream still reads then runs first -- the
#                      hazard the other spins hide; tests/test_widedeep_gpu.py stream-delay test)
#   sysfence=<groups>  the ordering events of these groups ('+'-separated) carry a system-scope fence
#                      instead of none: side (SideStream fork / join / marks), pipe (table clock
#                      pipelines), plan (planning-stream hand-offs: feeder, plans), push (the one-sided
#                      push stream's hand-off), all
def _parse_debug(spec: str) -> dict:
    out = {}
    for item in filter(None, (x.strip() for x in spec.split(","))):
        k, _, v = item.partition("=")
        out[k] = v
    return out


_DEBUG = _parse_debug(os.environ.get("MINIPS_STREAM_DEBUG", ""))
DELAY_US = int(_DEBUG.get("delay", "0") or 0)
DELAY_WHERE = set(_DEBUG.get("where", "use+fork").split("+"))
SYSFENCE = set(filter(None, _DEBUG.get("sysfence", "").split("+")))


def fast_for(group: str) -> bool:
    """Fence-free (same-device ordering only) events for ``group`` unless the debug mode asks for
    system-scope fences there."""
    return group not in SYSFENCE and "all" not in SYSFENCE


_delay_bufs: dict = {}


def delay(raw_stream: int, dev_index: int):
    """Spin DELAY_US microseconds on ``raw_stream`` (a one-wave kernel on the 100 MHz clock)."""
    if DELAY_US <= 0:
        return
    buf = _delay_bufs.get(dev_index)
    if buf is None:
        buf = _delay_bufs[dev_index] = torch.zeros(2, dtype=torch.int64, device=torch.device("cuda", dev_index))
    from .._native import kernels

    kernels().clock_probe(buf, min(1_000_000, DELAY_US * 100), raw_stream)


_get = torch._C._cuda_getCurrentStream if hasattr(torch._C, "_cuda_getCurrentStream") else None
_set = torch._C._cuda_setStream if hasattr(torch._C, "_cuda_setStream") else None
_raw = torch._C._cuda_getCurrentRawStream if hasattr(torch._C, "_cuda_getCurrentRawStream") else None


def _index(dev) -> int:
    if isinstance(dev, int):
        return dev
    if isinstance(dev, torch.device) and dev.index is not None:
        return dev.index
    if isinstance(dev, torch.cuda.Stream):
        return dev.device_index
    return torch.cuda.current_device()


def current(dev=None) -> torch.cuda.Stream:
    """torch.cuda.current_stream(dev) without the device resolution layers."""
    d = _get(_index(dev))
    return torch.cuda.Stream(stream_id=d[0], device_index=d[1], device_type=d[2])


def current_raw(dev=None) -> int:
    """The current stream's hipStream_t handle (torch.cuda.current_stream(dev).cuda_stream)."""
    return _raw(_index(dev))


class use:
    """``with use(stream):`` == ``with torch.cuda.stream(stream):`` for a stream of the current
    device (restores the previous current stream of that device on exit); ``None``: no-op."""

    __slots__ = ("s", "prev")

    def __init__(self, s):
        self.s = s
        self.prev = None

    def __enter__(self):
        s = self.s
        if s is not None:
            self.prev = _get(s.device_index)
            _set(stream_id=s.stream_id, device_index=s.device_index, device_type=s.device_type)
            if DELAY_US > 0 and "use" in DELAY_WHERE:
                delay(_raw(s.device_index), s.device_index)
        return s

    def __exit__(self, *exc):
        p = self.prev
        if p is not None:
            _set(stream_id=p[0], device_index=p[1], device_type=p[2])
            self.prev = None
        return False


class FastEvent:
    """A same-device ordering event with torch.cuda.Event's record / wait / query / synchronize
    (duck-typed: torch's Stream.wait_event(ev) calls ev.wait(stream)), backed by ops_py FastEvent
    (hipEventDisableTiming | hipEventDisableSystemFence: its record does not write back the L2 for
    the host, which the default event does on every record -- a queue bubble of several us)."""

    __slots__ = ("ev",)

    def __init__(self):
        from .._native import kernels

        self.ev = kernels().FastEvent()

    def record(self, stream=None):
        self.ev.record(stream.cuda_stream if stream is not None else _raw(torch.cuda.current_device()))

    def wait(self, stream=None):
        self.ev.wait(stream.cuda_stream if stream is not None else _raw(torch.cuda.current_device()))

    def query(self) -> bool:
        return self.ev.query()

    def synchronize(self):
        self.ev.synchronize()


class EventRing:
    """A fixed ring of reusable events (torch.cuda.Event, or FastEvent when ``fast``):
    a stream wait binds to the record issued before it, so re-recording an event after its waits
    were issued is safe -- no event object created and destroyed per use."""

    __slots__ = ("evs", "i")

    def __init__(self, n: int = 8, fast: bool = False):
        self.evs = [FastEvent() if fast else torch.cuda.Event() for _ in range(n)]
        self.i = 0

    def next(self):
        ev = self.evs[self.i]
        self.i = (self.i + 1) % len(self.evs)
        return ev
