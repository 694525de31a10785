#!/usr/bin/env python3
"""Average unique-key count U per Wide&Deep batch (bench.py's synthetic Criteo data, one GPU):
the byte counts of the embedding kernels in tools/kernel_roofline.py scale with it."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(batches=20):
    from minips_amd import ops
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.widedeep import WideDeepConfig

    dev = torch.device("cuda", 0)
    cfg = WideDeepConfig()
    data = CriteoSynth(16384, cards=cfg.cards, device=dev, seed=1)
    bounds = torch.tensor([0, sum(cfg.cards)], device=dev)
    us = []
    for _ in range(batches):
        _, keys, _ = data.next()
        _, _, _, U = ops.unique_bucketize_n(keys, bounds, keys.shape[1])
        us.append(int(U.item()))
    print(f"U mean {sum(us) / len(us):.0f} over {batches} batches of {keys.numel()} lookups (min {min(us)}, "
          f"max {max(us)})")


if __name__ == "__main__":
    main()
