#!/usr/bin/env python3
"""Isolated timings of the GPT-2 (config 4) memory-bound kernels at the model's shapes (B*T = 8192
rows, d = 768, vocab 50304): achieved TB/s against the ~8 TB/s HBM3E peak. In the training step
these kernels share the GPU with the weight-gradient GEMMs of the side stream, so rocprof's
in-step durations overstate their own cost; this separates the two.

    python tools/bench_nn.py
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters  # us


def main():
    from minips_amd import _native, ops

    _native.kernels()
    dev = torch.device("cuda", 0)
    M, C, V = 8192, 768, 50304
    bf = dict(dtype=torch.bfloat16, device=dev)
    x = torch.randn(M, C, **bf)
    dy = torch.randn(M, C, **bf)
    dx = torch.randn(M, C, **bf)
    g = torch.randn(C, **bf)
    bta = torch.randn(C, **bf)
    y = torch.empty(M, C, **bf)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    dg = torch.zeros(C, device=dev)
    db = torch.zeros(C, device=dev)
    ops.layernorm_fwd(x, C, g, bta, 1e-5, y, mean, rstd)
    rows = []
    us = timeit(lambda: ops.layernorm_fwd(x, C, g, bta, 1e-5, y, mean, rstd))
    rows.append(("layernorm_fwd", us, 2 * M * C * 2 + 8 * M))
    us = timeit(lambda: ops.layernorm_bwd(x, dy, C, g, mean, rstd, dx, dg, db, accumulate=True))
    rows.append(("layernorm_bwd (accumulate dx)", us, 4 * M * C * 2 + 8 * M))
    us = timeit(lambda: ops.add_bf16(x, dy, y))
    rows.append(("add_bf16", us, 3 * M * C * 2))
    logits = torch.randn(M, V, **bf)
    labels = torch.randint(0, 50257, (M,), device=dev)
    loss = torch.zeros(1, device=dev)
    us = timeit(lambda: ops.softmax_xent(logits, 50257, labels, 1.0 / M, loss), iters=10)
    rows.append(("softmax_xent (in place)", us, 2 * M * V * 2))
    for name, us, nbytes in rows:
        print(f"{name:32s} {us:9.1f} us  {nbytes / us / 1e6:6.2f} TB/s")


if __name__ == "__main__":
    main()
