#!/usr/bin/env python3
"""Diagnostics of the 1-GPU Wide&Deep step (bench.py's loop: LookaheadFeeder, next batch generated
and planned on the planning stream every step). One entry point:

    python tools/step_probe.py issue     host issue time per step vs wall time per step (no syncs
                                         inside: issue < wall means GPU-bound)
    python tools/step_probe.py cprofile  cProfile of the host side, top functions by own time
    python tools/step_probe.py events    HIP events: step start -> sparse Get done (a Get segment much
                                         longer than the gather kernel = the compute stream waited
                                         for the planning stream)
    python tools/step_probe.py ablation  feeder step vs a ring of pre-planned batches (+ the planning
                                         stream's work issued beside / after / without bookkeeping).
                                         Diagnostic only: the ring numbers are not valid benchmarks.
    python tools/step_probe.py curve     per-step GPU time (HIP events) of the first STEPS steps after
                                         the model build, averaged over step ranges; SPIN_MS > 0 first
                                         keeps the GPU busy with GEMMs for that long (clock-ramp test);
                                         REPEAT=k measures k curves in one process, PAUSE_S idle between
STEPS (env) sets the step count.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _setup():
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
    return comm, model, data, LookaheadFeeder(model, data, comm)


def _time(fn, n, warm=40):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def cmd_issue(n):
    _, _, _, feeder = _setup()
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


def cmd_cprofile(n):
    import cProfile
    import pstats

    _, _, _, feeder = _setup()
    for _ in range(5):
        feeder.step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        feeder.step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats(os.environ.get("SORT", "tottime")).print_stats(int(os.environ.get("TOP", "35")))
    if os.environ.get("CALLERS"):  # who calls the named functions (e.g. CALLERS=current_stream)
        st.print_callers(os.environ["CALLERS"])


def cmd_events(n):
    _, model, _, feeder = _setup()
    marks = []
    orig = model.emb.get_source if hasattr(model.emb, "get_source") else None
    orig_get = model.emb.get

    def mark(out):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks[-1].append(ev)
        return out

    model.emb.get = lambda keys, plan=None: mark(orig_get(keys, plan=plan))
    if orig is not None:  # one rank: the Get is folded into the assembly; mark after the source lookup
        model.emb.get_source = lambda keys, plan=None: mark(orig(keys, plan=plan))
    for _ in range(n + 10):
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        marks.append([e0])
        feeder.step()
    torch.cuda.synchronize()
    marks = marks[10:]
    get_ms = sorted(m[0].elapsed_time(m[1]) for m in marks if len(m) > 1)
    step_ms = sorted(marks[i][0].elapsed_time(marks[i + 1][0]) for i in range(len(marks) - 1))
    med = lambda v: v[len(v) // 2]  # noqa: E731
    print(f"step {med(step_ms):.4f} ms (median), step start -> Get done {med(get_ms):.4f} ms "
          f"(p10 {get_ms[len(get_ms) // 10]:.4f}, p90 {get_ms[9 * len(get_ms) // 10]:.4f})")


def cmd_ablation(n):
    comm, model, data, feeder = _setup()
    full = _time(feeder.step, n)
    ring = []
    for _ in range(int(os.environ.get("RING", "48"))):  # distinct batches keep the row traffic real
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

    ps = comm.plan_stream()

    def plus_planning():
        with torch.cuda.stream(ps):
            k = data.next()[1]
        model.emb.plan_async(k, csr=True, keys_on_plan_stream=True)
        step()

    def plus_data():
        with torch.cuda.stream(ps):
            data.next()
        step()

    def then_planning():
        step()
        with torch.cuda.stream(ps):
            k = data.next()[1]
        model.emb.plan_async(k, csr=True, keys_on_plan_stream=True)

    def plus_bare_planning():  # the same kernels without plan_async's stream bookkeeping
        with torch.cuda.stream(ps):
            k = data.next()[1]
            model.emb._start_plan(k, csr=True, exchange=False)
        step()

    fixed = _time(step, n)
    both, data_only, after, bare = (_time(f, n) for f in (plus_planning, plus_data, then_planning, plus_bare_planning))
    print(f"feeder step {full:.4f} ms | pre-planned ring of {len(ring)} batches {fixed:.4f} ms | data + planning "
          f"cost {full - fixed:.4f} ms/step | ring + discarded planning {both:.4f} ms | ring + discarded batch "
          f"generation only {data_only:.4f} ms | planning issued after the step {after:.4f} ms | ring + planning "
          f"kernels without record_stream/events {bare:.4f} ms")


def cmd_curve(n):
    _, _, _, feeder = _setup()
    spin = float(os.environ.get("SPIN_MS", "0"))
    if spin > 0:
        # SPIN_KIND=gemm: compute-bound (4096^3 bf16 GEMMs); mem: HBM-bound (1 GiB device copies)
        mem = os.environ.get("SPIN_KIND", "gemm") == "mem"
        a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
        if mem:
            src = torch.empty(1 << 28, device="cuda", dtype=torch.float32)
            dst = torch.empty_like(src)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < spin:
            for _ in range(8):
                if mem:
                    dst.copy_(src)
                else:
                    a @ a
            torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    # PRELOAD_MS: queue that much GPU work (GEMMs, no sync) right before step 0, so the host starts
    # the timed steps already ahead of the GPU (host-proximity test of the early-step curve)
    preload = float(os.environ.get("PRELOAD_MS", "0"))
    # CLOCK_PROBE=1: the effective shader clock after every step (ops_py clock_probe: s_memtime
    # cycles over s_memrealtime ticks), printed per step window beside the step times
    probes = None
    if os.environ.get("CLOCK_PROBE", "0") == "1":
        from minips_amd._native import kernels

        probes = torch.zeros(n, 2, dtype=torch.int64, device="cuda")
    pa = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16) if preload > 0 else None
    for rep in range(int(os.environ.get("REPEAT", "1"))):
        if rep:
            time.sleep(float(os.environ.get("PAUSE_S", "0.5")))  # idle, queue drained
        host = [0.0] * n
        if pa is not None:
            for _ in range(max(1, int(preload / 0.12))):  # ~0.12 ms per 4096^3 GEMM
                pa @ pa
        evs[0].record()
        for i in range(n):
            t = time.perf_counter()
            feeder.step()
            if probes is not None:  # one wave, ~10 us, in order after the step's main-stream work
                kernels().clock_probe(probes[i], 1000, 0)
            evs[i + 1].record()
            host[i] = (time.perf_counter() - t) * 1e3
        torch.cuda.synchronize()
        ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(n)]
        mhz = (probes[:, 0].double() / probes[:, 1].double() * 100.0).tolist() if probes is not None else None
        edges = [0, 1, 2, 5, 10, 20, 30, 50, 80, 120, 200, 300, 500, 1000, 1500]
        kind = os.environ.get('SPIN_KIND', 'gemm')
        print(f"spin {spin:.0f} ms ({kind}), preload {preload:.0f} ms before step 0; "
              f"reserved {torch.cuda.memory_reserved() / 2**30:.2f} GiB, "
              f"alloc retries {torch.cuda.memory_stats().get('num_alloc_retries', 0)}")
        for lo, hi in zip(edges, edges[1:]):
            if lo < n:
                seg, hseg = ms[lo:min(hi, n)], host[lo:min(hi, n)]
                clk = f", SCLK {sum(mhz[lo:min(hi, n)]) / len(seg):.0f} MHz" if mhz is not None else ""
                print(f"steps {lo:4d}-{min(hi, n) - 1:4d}: GPU {sum(seg) / len(seg):.4f} ms/step, host issue "
                      f"{sum(hseg) / len(hseg):.4f} ms/step{clk}", flush=True)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("cmd", choices=["issue", "cprofile", "events", "ablation", "curve"])
    a = ap.parse_args(argv)
    n = int(os.environ.get("STEPS", "300"))
    globals()["cmd_" + a.cmd](n)


if __name__ == "__main__":
    main()
