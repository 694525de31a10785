#!/usr/bin/env python3
"""Repository lint (the reference runs cpplint + clang-format in CI, scripts/lint.py:9-12; neither
tool is installed here, so the rules that matter are checked directly).

C++ / HIP (csrc/**): 120 columns, no tabs, no trailing whitespace, `#pragma once` in headers,
no `using namespace` in headers, no CUDA-compat / dual-platform shims (`__HIP_PLATFORM_*`,
`cuda_runtime.h`, hipify leftovers), no `__threadfence()` (the MI355X playbook: agent-scope
release/acquire fences, never the heavyweight device fence, in cross-workgroup protocols).
Python (minips_amd/, tools/, tests/, top-level): parses, 120 columns, no tabs / trailing
whitespace, no unused imports (names bound by an import and never referenced; `__init__`
re-exports and `# noqa` lines exempt).

    python tools/lint.py            # exit 1 and one line per finding
"""
from __future__ import annotations

import ast
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAX = 120
SHIMS = re.compile(r"__HIP_PLATFORM_|cuda_runtime\.h|hipify|__CUDA_ARCH__|cudaStream_t")


def _text_checks(path, lines, out):
    for i, l in enumerate(lines, 1):
        if len(l.rstrip("\n")) > MAX and "http" not in l:
            out.append(f"{path}:{i}: line longer than {MAX} columns")
        if "\t" in l:
            out.append(f"{path}:{i}: tab character")
        if l.rstrip("\n") != l.rstrip("\n").rstrip():
            out.append(f"{path}:{i}: trailing whitespace")


def lint_cpp(path, out):
    lines = open(path).readlines()
    _text_checks(path, lines, out)
    text = "".join(lines)
    if path.endswith(".h") and "#pragma once" not in text:
        out.append(f"{path}:1: header without #pragma once")
    if path.endswith(".h") and re.search(r"^using namespace ", text, re.M):
        out.append(f"{path}: `using namespace` in a header")
    for i, l in enumerate(lines, 1):
        code = l.split("//")[0]
        if SHIMS.search(code):
            out.append(f"{path}:{i}: CUDA-compat / dual-platform shim")
        if "__threadfence()" in code:
            out.append(f"{path}:{i}: __threadfence() (use agent-scope release/acquire fences)")


class _Names(ast.NodeVisitor):
    def __init__(self):
        self.used = set()

    def visit_Name(self, n):
        self.used.add(n.id)

    def visit_Attribute(self, n):
        root = n
        while isinstance(root, ast.Attribute):
            root = root.value
        if isinstance(root, ast.Name):
            self.used.add(root.id)
        self.generic_visit(n)


def lint_py(path, out):
    src = open(path).read()
    lines = src.splitlines(True)
    _text_checks(path, lines, out)
    try:
        tree = ast.parse(src, path)
    except SyntaxError as e:
        out.append(f"{path}:{e.lineno}: syntax error {e.msg}")
        return
    if os.path.basename(path) == "__init__.py":
        return
    v = _Names()
    v.visit(tree)
    # names used in string annotations / __all__ count as used
    strings = " ".join(n.value for n in ast.walk(tree) if isinstance(n, ast.Constant) and isinstance(n.value, str))
    for node in ast.walk(tree):
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                continue
            if "noqa" in lines[node.lineno - 1]:
                continue
            for a in node.names:
                name = (a.asname or a.name).split(".")[0]
                if name not in v.used and not re.search(rf"\b{re.escape(name)}\b", strings):
                    out.append(f"{path}:{node.lineno}: unused import {name}")


def main(argv=None):
    out: list[str] = []
    for p in sorted(glob.glob(os.path.join(ROOT, "csrc", "**", "*"), recursive=True)):
        if p.endswith((".h", ".cc", ".cpp", ".hip")):
            lint_cpp(os.path.relpath(p, ROOT), out)
    pys = glob.glob(os.path.join(ROOT, "*.py"))
    for d in ("minips_amd", "tools", "tests"):
        pys += glob.glob(os.path.join(ROOT, d, "**", "*.py"), recursive=True)
    for p in sorted(pys):
        lint_py(os.path.relpath(p, ROOT), out)
    for line in out:
        print(line)
    print(f"lint: {len(out)} finding(s)", file=sys.stderr)
    return 1 if out else 0


if __name__ == "__main__":
    os.chdir(ROOT)
    sys.exit(main())
