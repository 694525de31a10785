#!/usr/bin/env python3
"""K-scan of one GEMM shape family: time vs K at fixed M, N, to split a kernel's cost into a
fixed part (prologue, epilogue, wave quantisation) and a per-K-step part (main loop).

    MINIPS_GEMM_TILE=256 python tools/gemm_kscan.py --M 16384 --N 1024 --layout nt
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from minips_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=16384)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--Ks", default="128,256,512,848,1024,2048,4096")
    ap.add_argument("--layout", default="nt", choices=["nt", "nn", "tn"])
    ap.add_argument("--split", type=int, default=1)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    M, N = a.M, a.N
    a_km, b_kn = {"nt": (False, False), "nn": (False, True), "tn": (True, True)}[a.layout]
    for K in [int(k) for k in a.Ks.split(",")]:
        A = torch.randn((K, M) if a_km else (M, K), device=dev).to(torch.bfloat16)
        B = torch.randn((K, N) if b_kn else (N, K), device=dev).to(torch.bfloat16)
        C = torch.zeros(M, N, device=dev, dtype=torch.float32 if a.layout == "tn" else torch.bfloat16)
        epi = ops.EPI_ATOMIC_F32 if a.layout == "tn" else ops.EPI_STORE_BF16
        f = lambda: ops.gemm(A, B, C, M, N, K, a_km, b_kn, epi, split_k=a.split)  # noqa: E731
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(15):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                f()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) / 5 * 1e3)
        t = sorted(ts)[len(ts) // 2]
        print(f"{a.tag:10s} M={M} N={N} K={K:5d} {a.layout} split={a.split} {t:8.1f} us "
              f"{2.0 * M * N * K / t / 1e6:7.1f} TF/s",
              flush=True)


if __name__ == "__main__":
    main()
