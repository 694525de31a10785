"""Host-sync audit of a training loop: counts every point where the host waits for the GPU.

    with SyncAudit() as a:
        for _ in range(n):
            a.step_begin(); step(); a.step_end()
    print(a.report())

Two sources are counted, each attributed to the calling ``file:line``:
  * torch's own synchronizing ops (``.item()``, ``.tolist()``, ``.cpu()`` of a device tensor,
    ``nonzero`` ...) through ``torch.cuda.set_sync_debug_mode("warn")``;
  * explicit waits -- ``torch.cuda.synchronize``, ``Event.synchronize``, ``Stream.synchronize``
    -- by wrapping them for the duration of the audit.
Sites inside ``ps/comm.py`` are the gloo staging copies of the multi-rank test harness (several
ranks sharing one card over gloo: every collective round-trips through host memory by
construction); they are reported separately, because the RCCL path has no such copies.

The report also carries the host issue time per step (``step_begin`` -> ``step_end`` wall time,
no GPU wait at the end), next to the wall time per step of the audited window -- issue << wall
means the GPU is the bottleneck (the host runs ahead), issue ~ wall means the host is.
"""
from __future__ import annotations

import collections
import os
import sys
import time
import warnings

import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_STAGING = os.path.join(_PKG, "ps", "comm.py")


def _site(depth: int = 2) -> str:
    f = sys._getframe(depth)
    # walk out of torch / this module to the first frame of the caller's code
    while f is not None and (f.f_code.co_filename.startswith(os.path.dirname(torch.__file__))
                             or f.f_code.co_filename == __file__):
        f = f.f_back
    if f is None:
        return "?"
    return f"{os.path.relpath(f.f_code.co_filename, os.path.dirname(_PKG))}:{f.f_lineno}"


class SyncAudit:
    def __init__(self):
        self.sites = collections.Counter()
        self.issue = []
        self._t_step = None
        self._t0 = None
        self._saved = []
        self._warn_ctx = None
        self._warn_log = None
        self._mode = None

    # -- instrumentation ----------------------------------------------------------------
    def _wrap(self, owner, name):
        orig = getattr(owner, name)
        audit = self

        def wrapped(*a, **k):
            audit.sites[_site()] += 1
            return orig(*a, **k)

        setattr(owner, name, wrapped)
        self._saved.append((owner, name, orig))

    def __enter__(self):
        if torch.cuda.is_available():
            self._mode = torch.cuda.get_sync_debug_mode()
            torch.cuda.set_sync_debug_mode("warn")
        self._warn_ctx = warnings.catch_warnings(record=True)
        self._warn_log = self._warn_ctx.__enter__()
        warnings.simplefilter("always")
        self._wrap(torch.cuda, "synchronize")
        self._wrap(torch.cuda.Event, "synchronize")
        self._wrap(torch.cuda.Stream, "synchronize")
        self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        for owner, name, orig in reversed(self._saved):
            setattr(owner, name, orig)
        self._saved.clear()
        if self._mode is not None:
            torch.cuda.set_sync_debug_mode(self._mode)
        for w in self._warn_log:
            if "synchroniz" in str(w.message):
                self.sites[f"{os.path.relpath(w.filename, os.path.dirname(_PKG))}:{w.lineno}"] += 1
        self._warn_ctx.__exit__(*exc)
        self._wall = time.perf_counter() - self._t0
        return False

    # -- per step -----------------------------------------------------------------------
    def step_begin(self):
        self._t_step = time.perf_counter()

    def step_end(self):
        self.issue.append(time.perf_counter() - self._t_step)

    # -- results ------------------------------------------------------------------------
    def report(self, wall_s: float | None = None) -> dict:
        n = max(1, len(self.issue))
        staging = {s: c for s, c in self.sites.items() if s.startswith("minips_amd/ps/comm.py")}
        other = {s: c for s, c in self.sites.items() if s not in staging}
        iss = sorted(self.issue) or [0.0]
        wall = self._wall if wall_s is None else wall_s
        return {
            "steps": len(self.issue),
            "host_issue_ms_median": round(iss[len(iss) // 2] * 1e3, 4),
            "host_issue_ms_min": round(iss[0] * 1e3, 4),
            "wall_ms_per_step": round(wall * 1e3 / n, 4),
            "syncs_per_step": round(sum(other.values()) / n, 3),
            "sync_sites": dict(sorted(other.items())),
            "staging_syncs_per_step": round(sum(staging.values()) / n, 3),
        }
