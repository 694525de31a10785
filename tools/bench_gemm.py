#!/usr/bin/env python3
"""Microbenchmark of the gfx950 MFMA GEMM on the model shapes vs torch.matmul (hipBLASLt).

Prints TFLOP/s per shape/layout for our kernel and the vendor library on identical random
bf16 data, timed with HIP events over interleaved rounds in one process.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from minips_amd import ops  # noqa: E402

SHAPES = [  # (name, M, N, K, layout)
    ("wd.fwd1", 16384, 1024, 848, "nt"), ("wd.fwd2", 16384, 512, 1032, "nt"), ("wd.fwd3", 16384, 256, 520, "nt"),
    ("wd.dgrad2", 16384, 512, 256, "nn"), ("wd.dgrad1", 16384, 1024, 512, "nn"), ("wd.dgrad0", 16384, 832, 1024, "nn"),
    ("wd.wgrad3", 256, 520, 16384, "tn"), ("wd.wgrad2", 512, 1032, 16384, "tn"), ("wd.wgrad1", 1024, 848, 16384, "tn"),
    ("sq4096", 4096, 4096, 4096, "nt"), ("gpt.qkv", 8192, 2304, 768, "nt"), ("gpt.fc", 8192, 3072, 768, "nt"),
]


def _shapes():
    """SHAPES, or GEMM_SHAPES='name:M:N:K:layout,...' from the environment."""
    env = os.environ.get("GEMM_SHAPES")
    if not env:
        return SHAPES
    out = []
    for item in env.split(","):
        name, M, N, K, lay = item.split(":")
        out.append((name, int(M), int(N), int(K), lay))
    return out


def run(rounds=20):
    dev = torch.device("cuda")
    for name, M, N, K, lay in _shapes():
        a_km, b_kn = {"nt": (False, False), "nn": (False, True), "tn": (True, True)}[lay]
        A = torch.randn((K, M) if a_km else (M, K), device=dev).to(torch.bfloat16)
        B = torch.randn((K, N) if b_kn else (N, K), device=dev).to(torch.bfloat16)
        C = torch.empty(M, N, device=dev, dtype=torch.float32 if lay == "tn" else torch.bfloat16)
        epi = ops.EPI_ATOMIC_F32 if lay == "tn" else ops.EPI_STORE_BF16
        split = 1
        if lay == "tn":
            tiles = ((M + 127) // 128) * ((N + 127) // 128)
            split = max(1, min(K // 640, (int(os.environ.get("MINIPS_WGRAD_BLOCKS", "512")) + tiles - 1) // tiles))
        At = A.t() if a_km else A
        Bt = B if b_kn else B.t()

        def ours():
            ops.gemm(A, B, C, M, N, K, a_km, b_kn, epi, split_k=split)

        def ref():
            torch.matmul(At, Bt)

        for f in (ours, ref):
            f()
        torch.cuda.synchronize()
        times = {"ours": [], "hipblaslt": []}
        for _ in range(rounds):
            for key, f in (("ours", ours), ("hipblaslt", ref)):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    f()
                e.record()
                e.synchronize()
                times[key].append(s.elapsed_time(e) / 5)
        fl = 2.0 * M * N * K
        med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
        print(f"{name:10s} M={M:6d} N={N:5d} K={K:6d} {lay}  ours {med['ours']*1e3:8.1f}us "
              f"{fl/med['ours']/1e9:7.1f} TF/s | hipBLASLt {med['hipblaslt']*1e3:8.1f}us "
              f"{fl/med['hipblaslt']/1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    run()
