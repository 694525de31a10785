#!/usr/bin/env python3
"""Microbenchmark of the W&D embedding backward (segment-sum of dX rows into unique rows) on the
real Criteo-shaped plan of one batch."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from minips_amd import ops  # noqa: E402
from minips_amd.data.synthetic import CriteoSynth  # noqa: E402


def main(B=16384):
    dev = torch.device("cuda")
    data = CriteoSynth(B, device=dev, seed=1)
    dense, keys, y = data.next()
    bounds = torch.tensor([0, 1 << 62], dtype=torch.int64, device=dev)
    uniq, inv, counts = ops.unique_bucketize(keys.reshape(-1), bounds, 26)
    U = int(counts.sum())
    dX = torch.randn(B, 26 * 32, device=dev).to(torch.bfloat16)
    dw = torch.randn(B, device=dev)
    g = torch.zeros(U, 36, device=dev)

    def timed(fn, n=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / n * 1e3

    full = timed(lambda: ops.wd_emb_backward(dX, dw, inv, 26, 32, g))
    csr = ops.emb_build_csr(inv, 26, U)
    build = timed(lambda: ops.emb_build_csr(inv, 26, U))
    seg = timed(lambda: ops.wd_emb_backward(dX, dw, inv, 26, 32, g, csr=csr))
    print(f"U={U} lookups={B * 26} MINIPS_SEG_CFG={os.environ.get('MINIPS_SEG_CFG', '0')}: build+sum {full:.1f} us, "
          f"csr build {build:.1f} us, zero+segment sum {seg:.1f} us")


if __name__ == "__main__":
    main()
