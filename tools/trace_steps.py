#!/usr/bin/env python3
"""Steady-state step breakdown from a rocprofv3 --kernel-trace CSV.

    python tools/trace_steps.py run_kernel_trace.csv [--anchor adam_kernel] [--skip 3]

The window runs from the ``skip``-th to the last occurrence of the anchor kernel (one per
training step), so initialisation and warm-up kernels drop out. Prints wall ms per step, the
union of busy intervals over all queues (GPU busy), per-queue busy time and the kernels sorted
by device time per step -- the numbers that tell an overlap problem (busy << wall) from a
kernel problem (busy ~ wall).
"""
from __future__ import annotations

import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", default="adam_kernel")
    ap.add_argument("--skip", type=int, default=3)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "0"))
          for r in rows]
    ks.sort()
    anchors = [s for s, e, n, q in ks if a.anchor in n]
    if len(anchors) < a.skip + 2:
        raise SystemExit(f"only {len(anchors)} '{a.anchor}' kernels in the trace")
    lo, hi = anchors[a.skip], anchors[-1]
    steps = len(anchors) - 1 - a.skip
    win = [(max(s, lo), min(e, hi), n, q) for s, e, n, q in ks if e > lo and s < hi]
    wall = (hi - lo) / steps / 1e6
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in sorted(win):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    per_q = collections.Counter()
    per_k = collections.Counter()
    calls = collections.Counter()
    for s, e, n, q in win:
        per_q[q] += e - s
        short = n.split("(")[0][:110]
        per_k[short] += e - s
        calls[short] += 1
    tot = sum(per_k.values())
    print(f"steps {steps}  wall {wall:.4f} ms/step  GPU busy (union) {busy / steps / 1e6:.4f} ms/step  "
          f"kernel sum {tot / steps / 1e6:.4f} ms/step")
    print("per queue busy ms/step: " + ", ".join(f"q{q}={t / steps / 1e6:.4f}" for q, t in sorted(per_q.items())))
    print(f"{'ms/step':>9} {'calls/step':>10} {'us/call':>8}  kernel")
    for n, t in per_k.most_common(a.top):
        c = calls[n]
        print(f"{t / steps / 1e6:9.4f} {c / steps:10.2f} {t / c / 1e3:8.1f}  {n}")


if __name__ == "__main__":
    main()
