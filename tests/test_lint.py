"""The repository lint (tools/lint.py; the reference's CI runs cpplint + clang-format,
.travis.yml:36-49, scripts/lint.py:9-12) is clean."""
import subprocess
import sys

from _util import ROOT


def test_repository_lint_clean():
    r = subprocess.run([sys.executable, "tools/lint.py"], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-4000:]
