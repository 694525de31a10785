#!/usr/bin/env python3
"""Is the 1-GPU Wide&Deep step host-bound or GPU-bound? Issues N steps through bench.py's
LookaheadFeeder without any sync and reports the host issue time per step next to the wall
time per step (after the final synchronize). A step issues no host wait on one rank, so the host
runs ahead of the GPU when it is the faster side: issue < wall means GPU-bound."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(n=int(os.environ.get("STEPS", "300"))):
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.feeder import LookaheadFeeder
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig
    from minips_amd.ps.comm import Comm

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Comm(device=dev)
    cfg = WideDeepConfig()
    model = WideDeep(cfg, comm)
    feeder = LookaheadFeeder(model, CriteoSynth(16384, cards=cfg.cards, device=dev, seed=1), comm)
    for _ in range(10):
        feeder.step()
    torch.cuda.synchronize()
    for rep in range(3):
        t0 = time.perf_counter()
        for _ in range(n):
            feeder.step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"rep {rep}: host issue {(t1 - t0) / n * 1e3:.4f} ms/step, wall {(t2 - t0) / n * 1e3:.4f} ms/step",
              flush=True)


if __name__ == "__main__":
    main()
