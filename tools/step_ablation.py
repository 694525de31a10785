#!/usr/bin/env python3
"""What the 1-GPU Wide&Deep step pays for its data + key planning: times bench.py's loop
(LookaheadFeeder: next batch generated and planned on the planning stream every step) against
the same model stepping through a ring of pre-generated batches whose plans were computed up
front (no generation, no dedupe / CSR per step; distinct batches keep the row traffic real).
Diagnostic only -- the second number is not a valid benchmark."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, n):
    for _ in range(40):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


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
    data = CriteoSynth(16384, cards=cfg.cards, device=dev, seed=1)
    feeder = LookaheadFeeder(model, data, comm)
    full = _time(feeder.step, n)
    torch.cuda.synchronize()
    # a ring of pre-generated batches with their plans: realistic cache behaviour for the rows
    ring = []
    for _ in range(int(os.environ.get("RING", "48"))):
        dense, keys, labels = data.next()
        ring.append((dense, keys, labels, model.emb.plan(keys, csr=True)))
    torch.cuda.synchronize()
    plans = {id(b[1]): b[3] for b in ring}
    model._take_plan = lambda k: plans[id(k)]
    pos = [0]

    def step():
        d, k, y, _ = ring[pos[0] % len(ring)]
        pos[0] += 1
        model.train_step(d, k, y)

    fixed = _time(step, n)
    # the same ring, plus the planning stream's work of a real step (next batch generated and
    # planned, result discarded): isolates its interference from the feeder's hand-over
    ps = comm.plan_stream()

    def step_plus_planning():
        with torch.cuda.stream(ps):
            k = data.next()[1]
        model.emb.plan_async(k, csr=True, keys_on_plan_stream=True)
        step()

    both = _time(step_plus_planning, n)

    def step_plus_data():
        with torch.cuda.stream(ps):
            data.next()
        step()

    data_only = _time(step_plus_data, n)

    def step_then_planning():
        step()
        with torch.cuda.stream(ps):
            k = data.next()[1]
        model.emb.plan_async(k, csr=True, keys_on_plan_stream=True)

    after = _time(step_then_planning, n)
    import time as _t

    def host_plan_cost():  # host time of issuing one batch generation + plan (GPU idle-ish)
        torch.cuda.synchronize()
        t0 = _t.perf_counter()
        for _ in range(50):
            with torch.cuda.stream(ps):
                k = data.next()[1]
            model.emb.plan_async(k, csr=True, keys_on_plan_stream=True)
        t1 = _t.perf_counter()
        torch.cuda.synchronize()
        return (t1 - t0) / 50 * 1e3

    host_ms = host_plan_cost()

    def step_plus_bare_planning():  # the same kernels without plan_async's stream bookkeeping
        with torch.cuda.stream(ps):
            k = data.next()[1]
            model.emb._start_plan(k, csr=True, exchange=False)
        step()

    bare = _time(step_plus_bare_planning, n)
    print(f"feeder step {full:.4f} ms | pre-planned ring of {len(ring)} batches {fixed:.4f} ms | data + planning "
          f"cost {full - fixed:.4f} ms/step | ring + discarded planning {both:.4f} ms | ring + discarded batch "
          f"generation only {data_only:.4f} ms | planning issued after the step {after:.4f} ms | host issue of "
          f"one batch + plan {host_ms:.4f} ms | ring + planning kernels without record_stream/events "
          f"{bare:.4f} ms")


if __name__ == "__main__":
    main()
