"""Runs the native C++ unit tests (ports of every reference gtest, see csrc/tests)."""
import os
import subprocess

from _util import ROOT, ensure_built


def test_native_runtime_suite():
    ensure_built("runtime", "tests")
    r = subprocess.run([os.path.join(ROOT, "build/bin/runtime_test")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "cases passed" in r.stdout
