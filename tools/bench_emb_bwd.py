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
    g = torch.zeros(U, 33, device=dev)
    for _ in range(3):
        ops.wd_emb_backward(dX, dw, inv, 26, 32, g)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        ops.wd_emb_backward(dX, dw, inv, 26, 32, g)
    e.record()
    torch.cuda.synchronize()
    print(f"U={U} lookups={B * 26} emb_backward {s.elapsed_time(e) / 20 * 1e3:.1f} us "
          f"(MINIPS_EMB_BWD={os.environ.get('MINIPS_EMB_BWD', 'segment')})")


if __name__ == "__main__":
    main()
