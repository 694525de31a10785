#!/usr/bin/env python3
"""Run a few model-shape GEMMs back to back (for rocprofv3 --pmc passes, one kernel per shape)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from minips_amd import ops  # noqa: E402

dev = torch.device("cuda")


def bf(*s):
    return torch.randn(*s, device=dev).to(torch.bfloat16)


X, W1, dH1 = bf(16384, 848), bf(1024, 848), bf(16384, 1024)
H = torch.empty(16384, 1024, device=dev, dtype=torch.bfloat16)
dX = torch.empty(16384, 848, device=dev, dtype=torch.bfloat16)
dW = torch.zeros(1024, 848, device=dev)
A4, B4 = bf(4096, 4096), bf(4096, 4096)
C4 = torch.empty(4096, 4096, device=dev, dtype=torch.bfloat16)
for _ in range(int(os.environ.get("REPS", "10"))):
    ops.linear_fwd(X, W1, None, "relu", out=H)                  # fwd1 (nt)
    ops.linear_dgrad(dH1, W1, out=dX)                           # dgrad0 (nn, tr-read B)
    ops.linear_wgrad(dH1, X, dW)                                # wgrad1 (tn, split-K)
    ops.gemm(A4, B4, C4, 4096, 4096, 4096, False, False, ops.EPI_STORE_BF16)  # sq4096
torch.cuda.synchronize()
print("done")
