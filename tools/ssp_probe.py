#!/usr/bin/env python3
"""Bisect the 4-rank SSP(1) Wide&Deep loss spike (tests/test_multirank_gpu.py::
test_widedeep_ssp_world4_tracks_one_rank_bsp[onesided]) on one GPU: four ranks share cuda:0
over gloo, six steps on one global batch stream, as in the test. Each RUN repeats the world with
one transport combination and prints, per rank and step, the loss and two checksums taken right
after the step's reads: the dense parameters the forward used and the embedding rows it gathered.

    python tools/ssp_probe.py [--runs N] [--sparse onesided|collective] [--dense onesided|collective]
                              [--steps S] [--staleness s]

A step whose loss leaves the one-rank BSP reference by more than 0.1 is flagged SPIKE; the
checksums then show whether the dense read, the row read, or neither differed from the other
ranks' (every rank reads the same global state at a clock when the applies are complete).
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

CARDS = [1000, 50, 20000, 7, 300, 20, 5, 60, 90, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26]
WD_TOTAL = 4096


def _args() -> dict:  # (spawned ranks re-import this module: the options travel in the environment)
    import json

    return json.loads(os.environ["SSP_PROBE_ARGS"])


def _world_fn(rank, world):
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig
    from minips_amd.ps.comm import Comm

    a = _args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Comm(device=dev)
    per = WD_TOTAL // world
    cons = "ssp" if a["staleness"] >= 0 else "bsp"
    cfg = WideDeepConfig(cards=CARDS, consistency=cons, staleness=max(0, a["staleness"]), transport=a["sparse"],
                         dense_transport=a["dense"], max_batch=per)
    m = WideDeep(cfg, comm)
    g = torch.Generator().manual_seed(5)
    full = torch.randn(m.num_rows, cfg.row_width, generator=g) * 0.01
    full[:, cfg.emb_dim:] = 0
    m.emb.shard.copy_(full[m.emb.base: m.emb.base + m.emb.rows_local].to(dev))
    torch.cuda.synchronize()
    comm.barrier()
    data = CriteoSynth(WD_TOTAL, cards=CARDS, device=dev, seed=11)
    rows = []
    for _ in range(a["steps"]):
        dense, keys, y = data.next()
        sl = slice(rank * per, (rank + 1) * per)
        t = m.train_step(dense[sl], keys[sl], y[sl]).clone()
        b = m._buffers(per)
        # what the forward read: the dense parameters and the assembled input (rows + dense)
        p = m.dense.params if hasattr(m.dense, "params") else None
        ps = float(p.float().sum()) if p is not None else float("nan")
        xs = float(b["X"].float().abs().sum())
        comm.all_reduce_(t)
        rows.append((float(t) / WD_TOTAL, ps, xs))
    m.drain()
    torch.cuda.synchronize()
    return rows


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--runs", type=int, default=4)
    ap.add_argument("--sparse", default="onesided", choices=["onesided", "collective"])
    ap.add_argument("--dense", default="onesided", choices=["onesided", "collective"])
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--staleness", type=int, default=1)
    args = ap.parse_args()
    os.environ.setdefault("MINIPS_SHARE_DEVICE", "1")
    os.environ.setdefault("MINIPS_DIST_BACKEND", "gloo")
    import json

    from test_ps_gloo import run_world

    # the one-rank BSP reference of the same global batches
    os.environ["SSP_PROBE_ARGS"] = json.dumps(dict(vars(args), sparse="collective", dense="collective",
                                                   staleness=-1))
    ref = [r[0] for r in run_world(_world_fn, world=1)[0]]
    os.environ["SSP_PROBE_ARGS"] = json.dumps(vars(args))
    print(f"reference (1 rank BSP): {[round(x, 4) for x in ref]}", flush=True)
    spikes = 0
    for run in range(args.runs):
        out = run_world(_world_fn, world=4)
        bad = []
        for r in sorted(out):
            for s, (loss, ps, xs) in enumerate(out[r]):
                if abs(loss - ref[s]) > 0.1:
                    bad.append((r, s))
        spikes += bool(bad)
        print(f"run {run}: sparse={args.sparse} dense={args.dense} {'SPIKE ' + str(bad) if bad else 'ok'}", flush=True)
        for s in range(args.steps):
            line = "  ".join(f"r{r} {out[r][s][0]:.4f} p{out[r][s][1]:.3f} x{out[r][s][2]:.1f}" for r in sorted(out))
            print(f"  step {s}: {line}", flush=True)
    print(f"[ssp-probe] sparse={args.sparse} dense={args.dense}: {spikes}/{args.runs} runs spiked", flush=True)


if __name__ == "__main__":
    main()
