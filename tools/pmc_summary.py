#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection.csv rows per (kernel, counter); prints a table per kernel."""
import collections
import csv
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
for path in sys.argv[1:]:
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row.get("Kernel_Name", "?")[:90]
            tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
for k, c in tot.items():
    print(k)
    for name in sorted(c):
        print(f"    {name:30s} {c[name]:.4g}")
    if c.get("SQ_BUSY_CU_CYCLES") and c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
        print(f"    MFMA busy / CU busy            {c['SQ_VALU_MFMA_BUSY_CYCLES'] / c['SQ_BUSY_CU_CYCLES']:.3f}")
