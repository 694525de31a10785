#!/usr/bin/env python3
"""In-tree native build for minips_amd (no setuptools, no JIT cache).

Targets
  runtime   csrc/runtime/*.cc            -> build/obj/rt_*.o  (g++ -O2, C++17)
  rt_py     csrc/bindings/runtime_py.cc  -> minips_amd/_runtime*.so   (pybind11)
  tests     csrc/tests/runtime_test.cc   -> build/bin/runtime_test
  apps      csrc/apps/*.cc               -> build/bin/<app>
  kernels   csrc/kernels/*.hip           -> build/obj/k_*.o   (hipcc --offload-arch=gfx950)
  comm      csrc/comm/*.cc               -> build/obj/c_*.o   (native RCCL data plane, linked into ops_py)
  ops_py    csrc/bindings/ops_py.cpp     -> minips_amd/_kernels*.so   (hipcc, torch headers)
  san_thread / san_address   runtime + runtime_test + apps built with -fsanitize=thread|address
            (host code only) -> build/san_<kind>/bin/ (race detection on the runtime)

Rebuilds are mtime-driven: a target is rebuilt when any of its sources or any header in
its source directories is newer than the output.  `python tools/build.py [targets...]`.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "build")
OBJ = os.path.join(BUILD, "obj")
BIN = os.path.join(BUILD, "bin")
PKG = os.path.join(ROOT, "minips_amd")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
JOBS = max(1, min(int(os.environ.get("MAX_JOBS", "8")), 16))
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"

CXX = os.environ.get("CXX", "g++")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXXFLAGS = ["-O2", "-std=c++17", "-fPIC", "-pthread", "-Wall", "-Wno-unused-function", "-Wno-sign-compare"]
HIPFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {cmd[-1]}")


def _mtime(p: str) -> float:
    try:
        return os.path.getmtime(p)
    except OSError:
        return -1.0


def _stale(out: str, inputs: list[str]) -> bool:
    t = _mtime(out)
    return t < 0 or any(_mtime(i) > t for i in inputs)


def _headers(*dirs: str) -> list[str]:
    hs: list[str] = []
    for d in dirs:
        hs += glob.glob(os.path.join(ROOT, d, "*.h")) + glob.glob(os.path.join(ROOT, d, "*.cuh"))
        hs += glob.glob(os.path.join(ROOT, d, "*.hpp"))
    return hs


def _run_to(out: str, cmd: list[str]) -> None:
    """Link shared objects to a temporary name and rename: a copy of the tree taken meanwhile (a
    GPU run's snapshot) sees the old library or the new one, never a half-written file."""
    if not out.endswith(".so"):
        _run(cmd)
        return
    tmp = out + ".tmp"
    _run([tmp if c == out else c for c in cmd])
    os.replace(tmp, out)


def _compile_many(jobs: list[tuple[str, list[str], list[str]]]) -> None:
    """jobs: (out, inputs, cmd)."""
    todo = [j for j in jobs if _stale(j[0], j[1])]
    if not todo:
        return
    with cf.ThreadPoolExecutor(JOBS) as ex:
        futs = [ex.submit(_run_to, out, cmd) for out, _, cmd in todo]
        for f in futs:
            f.result()


def _torch_flags() -> tuple[list[str], list[str]]:
    import torch.utils.cpp_extension as ce  # noqa: WPS433

    inc = []
    new_api = "device_type" in ce.include_paths.__code__.co_varnames
    for p in ce.include_paths("cuda") if new_api else ce.include_paths(True):
        inc += ["-I", p]
    new_api = "device_type" in ce.library_paths.__code__.co_varnames
    libdir = ce.library_paths("cuda")[0] if new_api else ce.library_paths(True)[0]
    py_inc = sysconfig.get_paths()["include"]
    cflags = inc + ["-I", py_inc, "-DTORCH_EXTENSION_NAME=_kernels", "-DTORCH_API_INCLUDE_EXTENSION_H",
                    "-D_GLIBCXX_USE_CXX11_ABI=1", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1"]
    ldflags = ["-L", libdir, "-Wl,-rpath," + libdir, "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python",
               "-lc10_hip", "-ltorch_hip"]
    return cflags, ldflags


def runtime_objs() -> list[str]:
    os.makedirs(OBJ, exist_ok=True)
    hdrs = _headers("csrc/runtime")
    jobs, objs = [], []
    for src in sorted(glob.glob(os.path.join(ROOT, "csrc/runtime/*.cc"))):
        out = os.path.join(OBJ, "rt_" + os.path.basename(src)[:-3] + ".o")
        objs.append(out)
        jobs.append((out, [src] + hdrs, [CXX, *CXXFLAGS, "-c", src, "-o", out]))
    _compile_many(jobs)
    return objs


def build_runtime_py(objs: list[str]) -> str:
    import pybind11

    src = os.path.join(ROOT, "csrc/bindings/runtime_py.cc")
    out = os.path.join(PKG, "_runtime" + EXT)
    inc = ["-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"]]
    cmd = [CXX, *CXXFLAGS, "-shared", *inc, src, *objs, "-o", out]
    _compile_many([(out, [src] + objs + _headers("csrc/runtime"), cmd)])
    return out


def build_tests(objs: list[str]) -> str:
    os.makedirs(BIN, exist_ok=True)
    src = os.path.join(ROOT, "csrc/tests/runtime_test.cc")
    out = os.path.join(BIN, "runtime_test")
    hdrs = _headers("csrc/runtime", "csrc/tests")
    _compile_many([(out, [src] + objs + hdrs, [CXX, *CXXFLAGS, src, *objs, "-o", out])])
    return out


def build_apps(objs: list[str]) -> list[str]:
    os.makedirs(BIN, exist_ok=True)
    outs, jobs = [], []
    hdrs = _headers("csrc/runtime", "csrc/apps")
    for src in sorted(glob.glob(os.path.join(ROOT, "csrc/apps/*.cc"))):
        out = os.path.join(BIN, os.path.basename(src)[:-3])
        outs.append(out)
        jobs.append((out, [src] + objs + hdrs, [CXX, *CXXFLAGS, src, *objs, "-o", out]))
    _compile_many(jobs)
    return outs


# runtime pieces the kernel module links too: the async PS server thread and its board
# (csrc/runtime/async_server.h drives the HIP applier of csrc/kernels/onesided.hip)
KERNEL_RT = ("ps_board", "async_server")


def kernel_objs() -> list[str]:
    os.makedirs(OBJ, exist_ok=True)
    hdrs = _headers("csrc/kernels") + [os.path.join(ROOT, "csrc/runtime", h + ".h") for h in KERNEL_RT]
    jobs, objs = [], []
    for src in sorted(glob.glob(os.path.join(ROOT, "csrc/kernels/*.hip"))):
        out = os.path.join(OBJ, "k_" + os.path.basename(src)[:-4] + ".o")
        objs.append(out)
        jobs.append((out, [src] + hdrs, [HIPCC, *HIPFLAGS, "-c", src, "-o", out]))
    _compile_many(jobs)
    return objs


def comm_objs() -> list[str]:
    """csrc/comm/*.cc (the native RCCL data plane: host code over hip / rccl headers; RCCL itself is
    dlopen'ed at run time, the copy torch loaded)."""
    os.makedirs(OBJ, exist_ok=True)
    hdrs = _headers("csrc/comm")
    jobs, objs = [], []
    for src in sorted(glob.glob(os.path.join(ROOT, "csrc/comm/*.cc"))):
        out = os.path.join(OBJ, "c_" + os.path.basename(src)[:-3] + ".o")
        objs.append(out)
        jobs.append((out, [src] + hdrs, [HIPCC, "-O2", "-std=c++17", "-fPIC", "-Wall", "-I/opt/rocm/include", "-c", src,
                                         "-o", out]))
    _compile_many(jobs)
    return objs


def build_ops_py(kobjs: list[str], robjs: list[str] = ()) -> str:
    src = os.path.join(ROOT, "csrc/bindings/ops_py.cpp")
    out = os.path.join(PKG, "_kernels" + EXT)
    bobj = os.path.join(OBJ, "ops_py.o")
    cflags, ldflags = _torch_flags()
    kobjs = list(kobjs) + [o for o in robjs if os.path.basename(o)[3:-2] in KERNEL_RT]
    hdrs = _headers("csrc/kernels", "csrc/bindings", "csrc/comm") + [os.path.join(ROOT, "csrc/runtime", h + ".h")
                                                                     for h in KERNEL_RT]
    _compile_many([(bobj, [src] + hdrs, [HIPCC, "-O2", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
                                         *cflags, "-c", src, "-o", bobj])])
    _compile_many([(out, [bobj] + kobjs,
                    [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", bobj, *kobjs, "-o", out, *ldflags,
                     "-ldl"])])
    return out


def build_sanitized(kind: str) -> list[str]:
    """The CPU runtime, its unit/integration tests and the apps under a sanitizer."""
    d = os.path.join(BUILD, f"san_{kind}")
    obj, bin_ = os.path.join(d, "obj"), os.path.join(d, "bin")
    os.makedirs(obj, exist_ok=True)
    os.makedirs(bin_, exist_ok=True)
    flags = [f for f in CXXFLAGS if f != "-O2"] + ["-O1", "-g", f"-fsanitize={kind}", "-fno-omit-frame-pointer"]
    hdrs = _headers("csrc/runtime")
    jobs, objs = [], []
    for src in sorted(glob.glob(os.path.join(ROOT, "csrc/runtime/*.cc"))):
        out = os.path.join(obj, os.path.basename(src)[:-3] + ".o")
        objs.append(out)
        jobs.append((out, [src] + hdrs, [CXX, *flags, "-c", src, "-o", out]))
    _compile_many(jobs)
    outs, jobs = [], []
    srcs = [os.path.join(ROOT, "csrc/tests/runtime_test.cc")] + sorted(glob.glob(os.path.join(ROOT, "csrc/apps/*.cc")))
    for src in srcs:
        out = os.path.join(bin_, os.path.basename(src)[:-3])
        outs.append(out)
        jobs.append((out, [src] + objs + _headers("csrc/runtime", "csrc/tests", "csrc/apps"),
                     [CXX, *flags, src, *objs, "-o", out]))
    _compile_many(jobs)
    return outs


def main(argv: list[str]) -> int:
    targets = set(argv) or {"runtime", "rt_py", "tests", "apps", "kernels", "ops_py"}
    for kind in ("thread", "address"):
        if f"san_{kind}" in targets:
            for o in build_sanitized(kind):
                print("built", o)
            targets.discard(f"san_{kind}")
            if not targets:
                return 0
    objs = runtime_objs()
    if "rt_py" in targets:
        print("built", build_runtime_py(objs))
    if "tests" in targets:
        print("built", build_tests(objs))
    if "apps" in targets:
        for o in build_apps(objs):
            print("built", o)
    if targets & {"kernels", "ops_py"}:
        kobjs = kernel_objs() + comm_objs()
        print("built", build_ops_py(kobjs, objs))  # always relink: a stale .so would silently run old kernels
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
