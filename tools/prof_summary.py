#!/usr/bin/env python3
"""rocprofv3 output summaries (one entry point):

    python tools/prof_summary.py stats run_kernel_stats.csv [steps] [--top 25]
        total kernel time and the top kernels (per call and share), divided by a step count
    python tools/prof_summary.py pmc counter_collection.csv [...]
        counters summed per (kernel, counter), with MFMA busy / CU busy when both were collected
    python tools/prof_summary.py trace run_kernel_trace.csv [--anchor adam_kernel] [--skip 3]
        steady-state step breakdown: the window runs from the ``skip``-th to the last occurrence of
        the anchor kernel (one per step); prints wall ms per step, the union of busy intervals over
        all queues (GPU busy), per-queue busy time and the kernels by device time per step -- the
        numbers that tell an overlap problem (busy << wall) from a kernel problem (busy ~ wall)

    python tools/prof_summary.py lag run_kernel_trace.csv run_hip_api_trace.csv [--anchor K] [--skip 8]
        (rocprofv3 --kernel-trace --hip-runtime-trace) one steady step kernel by kernel with the HOST
        time its launch call returned next to the GPU start: ``slack`` = GPU start - launch return.
        A kernel with ~0 slack started as soon as the host issued it -- the host path, not a GPU
        dependency, set its start (the steady-step median slack per kernel is printed too)

    python tools/prof_summary.py markers run_marker_api_trace.csv [--steps N]
        roctx ranges (MINIPS_ROCTX=1 under ``rocprofv3 --marker-trace``): count and host time per
        range name (Get / Add / Clock / collectives / the owner's apply batches)

(A bare path as the first argument means ``stats``.) Per-kernel TFLOP/s and TB/s of the W&D step:
tools/kernel_roofline.py.
"""
from __future__ import annotations

import argparse
import collections
import csv
import sys



def _short(name: str) -> str:
    """Kernel name without its argument list (keeps '(anonymous namespace)::' qualifiers)."""
    n = name.replace("(anonymous namespace)::", "")
    return n.split("(")[0][:110]


def stats(path, steps=1, top=25):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total kernel time {tot / 1e6:.3f} ms ({tot / 1e6 / steps:.3f} ms per step over {steps} steps)")
    print(f"{'ms/step':>9} {'calls':>6} {'us/call':>9} {'share':>7}  kernel")
    for r in rows[:top]:
        t = float(r["TotalDurationNs"])
        c = int(r["Calls"])
        print(f"{t / 1e6 / steps:9.3f} {c:6d} {t / 1e3 / c:9.1f} {100 * t / tot:6.2f}%  {r['Name'][:100]}")


def pmc(paths):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for path in paths:
        with open(path) as f:
            for row in csv.DictReader(f):
                tot[row.get("Kernel_Name", "?")[:90]][row["Counter_Name"]] += float(row["Counter_Value"])
    for k, c in tot.items():
        print(k)
        for name in sorted(c):
            print(f"    {name:30s} {c[name]:.4g}")
        if c.get("SQ_BUSY_CU_CYCLES") and c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            print(f"    MFMA busy / CU busy            {c['SQ_VALU_MFMA_BUSY_CYCLES'] / c['SQ_BUSY_CU_CYCLES']:.3f}")


def pmc_table(paths, match=""):
    """Per-dispatch averages of every counter, one row per kernel (counter_collection.csv files of
    separate passes merge by kernel name): waves, VALU / LDS instructions per wave, LDS bank-conflict
    cycles per LDS instruction, HBM MB fetched / written per dispatch (FETCH_SIZE / WRITE_SIZE, KB)."""
    import re

    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for path in paths:
        with open(path) as f:
            for row in csv.DictReader(f):
                k = re.sub(r"void |minips_k::", "", re.sub(r"\(.*", "", row.get("Kernel_Name", "?")))[:56]
                if match and not re.search(match, k):
                    continue
                tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k][row["Counter_Name"]].add(row.get("Dispatch_Id", ""))
    print(f"{'kernel':56s} {'waves':>8} {'VALU/w':>8} {'LDS/w':>7} {'conf/LDS':>8} {'fetchMB':>8} {'writeMB':>8}")
    for k in sorted(tot):
        c, d = tot[k], disp[k]

        def per(name):
            n = len(d.get(name, ())) or 1
            return c.get(name, 0.0) / n

        waves = c.get("SQ_WAVES", 0.0)
        lds = c.get("SQ_INSTS_LDS", 0.0)
        print(f"{k:56s} {per('SQ_WAVES'):8.0f} {c.get('SQ_INSTS_VALU', 0.0) / max(waves, 1):8.1f} "
              f"{lds / max(waves, 1):7.1f} {c.get('SQ_LDS_BANK_CONFLICT', 0.0) / max(lds, 1):8.2f} "
              f"{per('FETCH_SIZE') / 1024:8.1f} {per('WRITE_SIZE') / 1024:8.1f}")


def trace(a):
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
        short = _short(n)
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
    if a.timeline:
        # one steady step, kernel by kernel: start offset and duration per queue, and the idle gap of
        # each queue before the kernel -- what the critical path waits on
        t0, t1 = anchors[a.skip + 1], anchors[a.skip + 2]
        print(f"\ntimeline of one step ({(t1 - t0) / 1e3:.1f} us), anchor {a.anchor}: "
              "start_us dur_us gap_us queue kernel")
        last_end = {}
        for s, e, n, q in ks:
            if s < t0 or s >= t1:
                continue
            gap = (s - last_end[q]) / 1e3 if q in last_end else 0.0
            last_end[q] = e
            print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {gap:7.1f}  q{q}  {_short(n)[:90]}")


def lag(a):
    kr = list(csv.DictReader(open(a.trace)))
    launch = {}
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(a.api)):
        fn = r.get("Function", r.get("Operation", ""))
        dur[fn].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        if "Launch" in fn:
            launch[r["Correlation_Id"]] = int(r["End_Timestamp"])
    print("host time per HIP API call (us): calls, median, p90, max, total ms -- a call that blocks the host")
    print("(e.g. a stream wait that waits for its event) shows a large p90 / max")
    for fn, v in sorted(dur.items(), key=lambda kv: -sum(kv[1]))[:16]:
        v.sort()
        print(f"  {len(v):7d} {v[len(v) // 2]:8.1f} {v[int(len(v) * 0.9)]:8.1f} {v[-1]:9.1f} {sum(v) / 1e3:9.2f}  {fn}")
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "0"),
                 launch.get(r.get("Correlation_Id"))) for r in kr)
    anchors = [s for s, e, n, q, h in ks if a.anchor in n]
    if len(anchors) < a.skip + 3:
        raise SystemExit(f"only {len(anchors)} '{a.anchor}' kernels in the trace")
    slack = collections.defaultdict(list)
    for s, e, n, q, h in ks:
        if anchors[a.skip] <= s < anchors[-1] and h is not None:
            slack[_short(n)].append((s - h) / 1e3)
    print(f"median slack (GPU start - host launch return, us) over steps {a.skip}..{len(anchors) - 1}:")
    for n, v in sorted(slack.items(), key=lambda kv: sorted(kv[1])[len(kv[1]) // 2]):
        print(f"  {sorted(v)[len(v) // 2]:9.1f}  (min {min(v):8.1f}, n {len(v):5d})  {n[:80]}")
    t0, t1 = anchors[a.skip + 1], anchors[a.skip + 2]
    print(f"\none step ({(t1 - t0) / 1e3:.1f} us), anchor {a.anchor}: start_us dur_us host_us slack_us queue kernel")
    for s, e, n, q, h in ks:
        if t0 <= s < t1:
            hs = f"{(h - t0) / 1e3:8.1f} {(s - h) / 1e3:8.1f}" if h is not None else f"{'-':>8} {'-':>8}"
            print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {hs}  q{q}  {_short(n)[:80]}")


def markers(a):
    """roctx ranges of a ``--marker-trace`` run (MINIPS_ROCTX=1): per range name its count, total
    and mean host time, per thread; ``--steps`` divides the totals into per-step figures."""
    rows = list(csv.DictReader(open(a.path)))
    if not rows:
        raise SystemExit("no marker records")
    keys = rows[0].keys()
    name_col = next((c for c in ("Message", "Marker_Name", "Name", "Function") if c in keys), None)
    if name_col is None:
        raise SystemExit(f"no name column among {list(keys)}")
    tid_col = "Thread_Id" if "Thread_Id" in keys else None
    agg = collections.defaultdict(lambda: [0, 0])
    threads = collections.defaultdict(set)
    for r in rows:
        try:
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        except (KeyError, ValueError):
            continue
        n = r[name_col]
        agg[n][0] += 1
        agg[n][1] += d
        if tid_col:
            threads[n].add(r[tid_col])
    steps = max(1, a.steps)
    print(f"{'calls/step':>10} {'ms/step':>9} {'us/call':>9} {'threads':>7}  range   ({len(rows)} records, "
          f"per step over {steps})")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{c / steps:10.2f} {t / steps / 1e6:9.4f} {t / c / 1e3:9.1f} {len(threads[n]):7d}  {n[:80]}")


def early(a):
    """Per kernel name: mean duration in the step windows [lo, hi) of a kernel trace (steps counted
    by the anchor kernel), to see which kernels carry the slow early steps; plus the step length."""
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), _short(r["Kernel_Name"])) for r in rows)
    anchors = [s for s, e, n in ks if a.anchor in n]
    wins = [tuple(int(x) for x in w.split("-")) for w in a.windows.split(",")]
    wins = [(lo, min(hi, len(anchors) - 1)) for lo, hi in wins if lo < len(anchors) - 1]
    agg = collections.defaultdict(dict)
    steplen = {}
    for lo, hi in wins:
        t0, t1 = anchors[lo], anchors[hi]
        steplen[(lo, hi)] = (t1 - t0) / (hi - lo) / 1e3
        d = collections.defaultdict(list)
        for s, e, n in ks:
            if t0 <= s < t1:
                d[n].append(e - s)
        for n, v in d.items():
            agg[n][(lo, hi)] = sum(v) / (hi - lo) / 1e3  # us per step
    hdr = " ".join(f"{f'{lo}-{hi}':>9}" for lo, hi in wins)
    print(f"us per step in step windows (anchor {a.anchor})\n{'':60s} {hdr}")
    print(f"{'step length':60s} " + " ".join(f"{steplen[w]:9.1f}" for w in wins))
    last = wins[-1]
    for n in sorted(agg, key=lambda n: -agg[n].get(last, 0.0))[: a.top]:
        print(f"{n[:60]:60s} " + " ".join(f"{agg[n].get(w, 0.0):9.1f}" for w in wins))


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv and argv[0] not in ("stats", "pmc", "pmctable", "trace", "lag", "markers", "early", "-h", "--help"):
        argv.insert(0, "stats")
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("stats")
    p.add_argument("path")
    p.add_argument("steps", nargs="?", type=int, default=1)
    p.add_argument("--top", type=int, default=25)
    sub.add_parser("pmc").add_argument("paths", nargs="+")
    pt = sub.add_parser("pmctable")
    pt.add_argument("paths", nargs="+")
    pt.add_argument("--match", default="", help="regex on the kernel name")
    p = sub.add_parser("trace")
    p.add_argument("trace")
    p.add_argument("--anchor", default="adam_kernel")
    p.add_argument("--skip", type=int, default=3)
    p.add_argument("--top", type=int, default=30)
    p.add_argument("--timeline", action="store_true", help="also list one steady step kernel by kernel")
    p = sub.add_parser("lag")
    p.add_argument("trace")
    p.add_argument("api")
    p.add_argument("--anchor", default="wd_head_kernel")
    p.add_argument("--skip", type=int, default=8)
    p = sub.add_parser("early")
    p.add_argument("trace")
    p.add_argument("--anchor", default="adam_kernel")
    p.add_argument("--windows", default="2-10,10-30,30-60,150-290")
    p.add_argument("--top", type=int, default=25)
    p = sub.add_parser("markers")
    p.add_argument("path")
    p.add_argument("--steps", type=int, default=1)
    a = ap.parse_args(argv)
    if a.cmd == "markers":
        markers(a)
    elif a.cmd == "stats":
        stats(a.path, a.steps, a.top)
    elif a.cmd == "pmc":
        pmc(a.paths)
    elif a.cmd == "pmctable":
        pmc_table(a.paths, a.match)
    elif a.cmd == "lag":
        lag(a)
    elif a.cmd == "early":
        early(a)
    else:
        trace(a)


if __name__ == "__main__":
    main()
