#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv: total time and the top kernels (per call and
share), optionally divided by a step count."""
import csv
import sys


def main(path, steps=1, top=25):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total kernel time {tot / 1e6:.3f} ms ({tot / 1e6 / steps:.3f} ms per step over {steps} steps)")
    print(f"{'ms/step':>9} {'calls':>6} {'us/call':>9} {'share':>7}  kernel")
    for r in rows[:top]:
        t = float(r["TotalDurationNs"])
        c = int(r["Calls"])
        print(f"{t / 1e6 / steps:9.3f} {c:6d} {t / 1e3 / c:9.1f} {100 * t / tot:6.2f}%  {r['Name'][:100]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
