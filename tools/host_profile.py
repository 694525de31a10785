#!/usr/bin/env python3
"""cProfile of the host side of the 1-GPU Wide&Deep step (bench.py's loop): where the ~0.3 ms of
Python + launch work per step goes. Prints the top functions by own time."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig
    from minips_amd.ps.comm import Comm

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = WideDeepConfig()
    model = WideDeep(cfg, Comm(device=dev))
    data = CriteoSynth(16384, cards=cfg.cards, device=dev, seed=1)
    cur = data.next()

    def step():
        nonlocal cur
        nxt = data.next()
        model.train_step(*cur, next_keys=nxt[1])
        cur = nxt

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(200):
        step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(int(os.environ.get("TOP", "35")))


if __name__ == "__main__":
    main()
