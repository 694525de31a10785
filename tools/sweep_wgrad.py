#!/usr/bin/env python3
"""Split-K sweep of the weight-gradient GEMM (dW[N,K] += dY^T X) on the model shapes.

The kernel variant is chosen by env vars read once per process (MINIPS_GEMM_WGRAD_V2,
MINIPS_GEMM_TILE), so run one process per variant. Prints us/call per (shape, split).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from minips_amd import ops  # noqa: E402

SHAPES = [  # (name, rows M (reduction), dy cols N, x cols K)
    ("wd.w1", 16384, 1024, 848), ("wd.w2", 16384, 512, 1032), ("wd.w3", 16384, 256, 520),
    ("gpt.qkv", 8192, 2304, 768), ("gpt.fc", 8192, 3072, 768), ("gpt.fc2", 8192, 768, 3072),
    ("gpt.proj", 8192, 768, 768),
]


def main():
    dev = torch.device("cuda")
    splits = [int(x) for x in os.environ.get("SPLITS", "1,2,4,6,8,12,16,24").split(",")]
    tag = os.environ.get("TAG", "")
    for name, M, N, K in SHAPES:
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        dw = torch.zeros(N, K, device=dev)
        ref = (dy.float().t() @ x.float())
        res = []
        for sp in splits:
            if M // sp < 64:
                continue
            dw.zero_()
            ops.linear_wgrad(dy, x, dw, split_k=sp)
            torch.cuda.synchronize()
            err = float((dw - ref).abs().max() / ref.abs().max())
            ts = []
            for _ in range(7):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    ops.linear_wgrad(dy, x, dw, split_k=sp)
                e.record()
                e.synchronize()
                ts.append(s.elapsed_time(e) / 5 * 1e3)
            t = sorted(ts)[len(ts) // 2]
            res.append((t, sp, err))
        best = min(res)
        fl = 2.0 * M * N * K
        line = " ".join(f"s{sp}:{t:.1f}" for t, sp, _ in res)
        print(f"{tag:8s} {name:9s} best {best[0]:7.1f}us ({fl / best[0] / 1e6:6.1f} TF/s, split {best[1]}, "
              f"relerr {best[2]:.1e}) | {line}", flush=True)


if __name__ == "__main__":
    main()
