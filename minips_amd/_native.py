"""Loader for the in-tree native modules.

* ``_runtime``  -- the C++ parameter-server runtime (engine, consistency models, control
  plane, checkpoint I/O); CPU only, always required.
* ``_kernels``  -- the gfx950 HIP kernels (torch extension). Required whenever a GPU tensor
  reaches an op: on a GPU box a missing or stale build raises instead of silently falling
  back to eager PyTorch.
"""
from __future__ import annotations

import importlib
import os

_kernels = None
_kernels_err: Exception | None = None
_runtime = None
_runtime_err: Exception | None = None


def kernels():
    """Return the HIP kernel module or raise a loud error."""
    global _kernels, _kernels_err
    if _kernels is None and _kernels_err is None:
        try:
            import torch  # noqa: F401  (libtorch must be loaded first)

            _kernels = importlib.import_module("minips_amd._kernels")
        except Exception as e:  # pragma: no cover - depends on the build
            _kernels_err = e
    if _kernels is None:
        raise RuntimeError(
            "minips_amd._kernels (gfx950 HIP kernels) is not built or failed to load: "
            f"{_kernels_err!r}. Run `python tools/build.py` (or __graft_entry__.build())."
        )
    return _kernels


def runtime():
    """Return the C++ runtime module or raise."""
    global _runtime, _runtime_err
    if _runtime is None and _runtime_err is None:
        try:
            _runtime = importlib.import_module("minips_amd._runtime")
        except Exception as e:  # pragma: no cover
            _runtime_err = e
    if _runtime is None:
        raise RuntimeError(
            f"minips_amd._runtime (C++ PS runtime) is not built: {_runtime_err!r}. Run `python tools/build.py`."
        )
    return _runtime


def kernels_available() -> bool:
    try:
        kernels()
        return True
    except RuntimeError:
        return False


def native_dir() -> str:
    return os.path.dirname(os.path.abspath(__file__))
