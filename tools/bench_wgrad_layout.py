#!/usr/bin/env python3
"""Weight-gradient layouts on the GPT-2 shapes: dW[N,K] += dy^T x with dy [M,N], x [M,K] (M = tokens).

  perm   ops.linear_wgrad: both operands K-major (the reduction index is the row of both), every
         fragment read transposed from LDS
  xT     x transposed first (x^T [K,M], a small copy), then A = dy (K-major) x B = x^T (row-major)
  dyT    dy transposed first, then A = dy^T (row-major) x B = x (K-major): the dgrad-style kernel

Times include the transpose. One MI355X:  python tools/bench_wgrad_layout.py
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    from minips_amd import _native, ops

    _native.kernels()
    dev = torch.device("cuda", 0)
    M = 8192
    shapes = [("lm_head", 50304, 768), ("qkv", 2304, 768), ("fc", 3072, 768), ("fc2", 768, 3072), ("proj", 768, 768)]
    for name, N, K in shapes:
        dy = (torch.randn(M, N, device=dev) * 0.1).to(torch.bfloat16)
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        ref = torch.zeros(N, K, device=dev)
        ops.linear_wgrad(dy, x, ref)
        flop = 2.0 * M * N * K
        res = {}
        dw = torch.zeros(N, K, device=dev)
        res["perm"] = timeit(lambda: ops.linear_wgrad(dy, x, dw))

        tiles = ((N + 127) // 128) * ((K + 127) // 128)
        sk = max(1, min(M // 640, (512 + tiles - 1) // tiles))  # the split-K rule of ops.linear_wgrad

        def xt():
            xT = x.t().contiguous()
            ops.gemm(dy, xT, dw, N, K, M, True, False, ops.EPI_ATOMIC_F32, split_k=sk)

        def dyt():
            dyT = dy.t().contiguous()
            ops.gemm(dyT, x, dw, N, K, M, False, True, ops.EPI_ATOMIC_F32, split_k=sk)

        for tag, fn in (("xT", xt), ("dyT", dyt)):
            dw.zero_()
            fn()
            err = float((dw - ref).abs().max() / ref.abs().max())
            res[tag] = timeit(fn)
            res[tag + "_err"] = err
        print(f"{name:8s} N={N:6d} K={K:5d}  perm {res['perm']:8.1f} us ({flop / res['perm'] / 1e6:6.0f} TF/s)  "
              f"xT {res['xT']:8.1f} us ({flop / res['xT'] / 1e6:6.0f})  dyT {res['dyT']:8.1f} us "
              f"({flop / res['dyT'] / 1e6:6.0f})  rel.err xT {res['xT_err']:.1e} dyT {res['dyT_err']:.1e}",
              flush=True)


if __name__ == "__main__":
    main()
