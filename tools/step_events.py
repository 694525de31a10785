#!/usr/bin/env python3
"""Where the 1-GPU Wide&Deep step waits: HIP events on the compute stream at the step start, after
the sparse Get (its wait for the planning stream's plan + the row gather) and at the step end,
over bench.py's loop. A Get segment much longer than the gather kernel means the compute stream
sat waiting for the next batch's key planning."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(n=int(os.environ.get("STEPS", "200"))):
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
    marks = []
    orig_get = model.emb.get

    def get(keys, plan=None):
        out = orig_get(keys, plan=plan)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks[-1].append(ev)
        return out

    model.emb.get = get
    for i in range(n + 10):
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        marks.append([e0])
        feeder.step()
    e_end = torch.cuda.Event(enable_timing=True)
    e_end.record()
    torch.cuda.synchronize()
    marks = marks[10:]
    get_ms = [m[0].elapsed_time(m[1]) for m in marks]
    step_ms = [marks[i][0].elapsed_time(marks[i + 1][0]) for i in range(len(marks) - 1)]
    get_ms.sort()
    step_ms.sort()
    med = lambda v: v[len(v) // 2]  # noqa: E731
    print(f"step {med(step_ms):.4f} ms (median), step start -> Get done {med(get_ms):.4f} ms "
          f"(p10 {get_ms[len(get_ms) // 10]:.4f}, p90 {get_ms[9 * len(get_ms) // 10]:.4f})")


if __name__ == "__main__":
    main()
