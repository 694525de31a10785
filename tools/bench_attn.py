#!/usr/bin/env python3
"""Fused causal attention microbenchmark (GPT-2 shape by default) vs torch SDPA on the same
device: time per call and TFLOP/s (causal FLOPs: fwd 2 products, bwd 5 products over T^2/2)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from minips_amd import ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--H", type=int, default=12)
    a = ap.parse_args()
    B, T, H = a.B, a.T, a.H
    d = H * 64
    dev = torch.device("cuda")
    qkv = torch.randn(B * T, 3 * d, device=dev).to(torch.bfloat16)
    dO = torch.randn(B * T, d, device=dev).to(torch.bfloat16)
    O = torch.empty(B * T, d + 8, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * T, device=dev)
    delta = torch.empty_like(lse)
    dqkv = torch.empty_like(qkv)
    fl = 4.0 * B * H * T * T / 2 * 64
    tf = timeit(lambda: ops.attn_fwd(qkv, B, T, H, 0.125, O, lse))
    tb = timeit(lambda: ops.attn_bwd(qkv, O, dO, lse, delta, B, T, H, 0.125, dqkv))
    print(f"ours  fwd {tf * 1e3:8.1f} us {fl / tf / 1e9:7.1f} TF/s   "
          f"bwd {tb * 1e3:8.1f} us {2.5 * fl / tb / 1e9:7.1f} TF/s")
    q, k, v = (qkv[:, i * d:(i + 1) * d].reshape(B, T, H, 64).transpose(1, 2).contiguous() for i in range(3))
    q.requires_grad_(True), k.requires_grad_(True), v.requires_grad_(True)
    go = dO.reshape(B, T, H, 64).transpose(1, 2).contiguous()
    F = torch.nn.functional.scaled_dot_product_attention
    try:
        tf2 = timeit(lambda: F(q, k, v, is_causal=True))
        out = F(q, k, v, is_causal=True)
        tb2 = timeit(lambda: torch.autograd.grad(out, (q, k, v), go, retain_graph=True))
        print(f"sdpa  fwd {tf2 * 1e3:8.1f} us {fl / tf2 / 1e9:7.1f} TF/s   bwd {tb2 * 1e3:8.1f} us "
              f"{2.5 * fl / tb2 / 1e9:7.1f} TF/s")
    except Exception as e:  # pragma: no cover
        print("sdpa unavailable:", e)


if __name__ == "__main__":
    main()
