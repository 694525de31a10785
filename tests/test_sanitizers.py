"""The native runtime's unit + integration tests under ThreadSanitizer and AddressSanitizer
(+ LeakSanitizer), host code only (the reference had no sanitizer builds and
several known races). Any sanitizer report fails the run (halt_on_error / exitcode)."""
import os
import subprocess

import pytest

from _util import ROOT, ensure_built


@pytest.mark.parametrize("kind,env", [
    ("thread", {"TSAN_OPTIONS": "halt_on_error=1 exitcode=66"}),
    ("address", {"ASAN_OPTIONS": "detect_leaks=1 halt_on_error=1"}),
])
def test_runtime_under_sanitizer(kind, env):
    ensure_built(f"san_{kind}")
    exe = os.path.join(ROOT, "build", f"san_{kind}", "bin", "runtime_test")
    r = subprocess.run([exe], cwd=ROOT, env=dict(os.environ, **env), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-6000:])
    assert "cases passed" in r.stdout + r.stderr


@pytest.mark.parametrize("model", ["BSP", "SSP", "ASP"])
def test_lr_app_two_nodes_under_tsan(tmp_path, model):
    """The LR app (2 processes x 2 worker threads, TCP mailbox, server threads) race-free under TSan."""
    from _util import write_hostfile
    from minips_amd import launch

    ensure_built("san_thread")
    hf = write_hostfile(str(tmp_path / "hosts"), 2)
    logs = str(tmp_path / "logs")
    old = {k: os.environ.get(k) for k in ("MINIPS_BIN_DIR", "TSAN_OPTIONS")}
    os.environ.update(MINIPS_BIN_DIR=os.path.join(ROOT, "build", "san_thread", "bin"),
                      TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    try:
        rcs = launch.launch_nodes("lr", hf, ["--num_workers_per_node=2", "--num_iters=60", "--batch_size=10",
                                             "--num_dims=2000", f"--kModelType={model}", "--kStaleness=1"],
                                  log_dir=logs, timeout=240)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    text = "".join(open(os.path.join(logs, f"node_{i}.log")).read() for i in range(2))
    assert rcs == [0, 0] and "ThreadSanitizer" not in text, (rcs, text[-4000:])
