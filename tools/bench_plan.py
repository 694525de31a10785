#!/usr/bin/env python3
"""Microbenchmark of key planning on a Criteo-shaped batch: the atomic-free per-column sort
(ops.plan_sorted) vs the hash dedupe + CSR build, and the sort's cost per radix pass."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from minips_amd import ops  # noqa: E402
from minips_amd.data.synthetic import CRITEO_KAGGLE_CARDS, CriteoSynth  # noqa: E402


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


def main(B=16384):
    dev = torch.device("cuda")
    cards = CRITEO_KAGGLE_CARDS
    F = len(cards)
    keys = CriteoSynth(B, device=dev, seed=1).next()[1]
    bases = torch.tensor([sum(cards[:f]) for f in range(F)], device=dev)
    bits = [max(1, (c - 1).bit_length()) for c in cards]
    R = sum(cards)
    t_sort = timed(lambda: ops.plan_sorted(keys, bases, bits, 402653189, R))
    bounds = torch.tensor([0, R], device=dev)

    def hashed():
        (uniq, inv, counts, U), z = ops.unique_bucketize_n(keys.reshape(-1), bounds, F, 402653189, R,
                                                           extra_zero_ints=2 * B * F, csr_counts=True)
        ops.emb_build_csr(inv, F, B * F, zeroed=z, counts_ready=True)

    t_hash = timed(hashed)
    print(f"B={B} F={F}: sort plan {t_sort:.1f} us | hash dedupe + CSR {t_hash:.1f} us")
    for nb in (4, 8, 16, 24, 32):
        t = timed(lambda: ops.plan_sorted(keys, bases, [nb] * F, 402653189, R))
        print(f"  all columns at {nb:2d} bits ({(nb + 3) // 4} passes): {t:.1f} us")


if __name__ == "__main__":
    main()
