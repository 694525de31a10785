"""The reference's basic push/pull demo on GPU ranks through the Engine API
(apps/basic/basic_example.cpp:19-77): one table of kMaxKey = 1000 keys (SSP, staleness 1, Map
storage), 10 workers per rank, each doing 100 x {Get every key, Add 0.5 to every key, Clock}.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m minips_amd.apps.basic

The last line on rank 0 is a JSON summary: the final value of every key (0.5 x workers x
iterations when every Add landed exactly once), the SSP read bound check of every Get, timings.
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch


def run(engine, workers: int = 10, iters: int = 100, max_key: int = 1000, model: str = "ssp", staleness: int = 1,
        storage: str = "map", transport: str = "collective"):
    from ..engine import MLTask

    # rows start at 0 (the reference's Map/VectorStorage default-insert 0)
    extra = {} if storage == "map" else {"init_std": 0.0}
    tid = engine.create_table("sparse", num_rows=max_key, width=1, model=model, staleness=staleness,
                              storage=storage, transport=transport, optimizer="add", **extra)
    engine.barrier()
    dev = engine.comm.device
    total = workers * engine.world
    s = staleness if model == "ssp" else (0 if model == "bsp" else None)

    def worker(info):
        table = info.create_kv_client_table(tid)
        keys = torch.arange(max_key, device=dev)
        vals = torch.full((max_key, 1), 0.5, device=dev)
        low = []  # reads below the SSP bound (must stay empty)
        for i in range(iters):
            ret = table.get(keys)
            assert ret.shape[0] == keys.numel()
            v = float(ret[0, 0])
            # every worker's Adds of clocks < i - s are in (ssp_model.cpp:58-85)
            if s is not None and v < 0.5 * total * max(0, i - s) - 1e-6:
                low.append((i, v))
            table.add(keys, vals)
            table.clock()
        return low

    t0 = time.perf_counter()
    lows = engine.run(MLTask(fn=worker, workers_per_rank=workers, tables=[tid]))
    el = time.perf_counter() - t0
    engine.barrier()
    final = engine.table(tid).get_rows(torch.arange(max_key, device=dev)).reshape(-1).double()
    return dict(final_min=float(final.min()), final_max=float(final.max()), expected=0.5 * total * iters,
                bound_violations=sum(len(x) for x in lows), workers=total, ranks=engine.world,
                seconds=round(el, 3))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=10, help="workers per rank (reference: 10 per node)")
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--max_key", type=int, default=1000)
    ap.add_argument("--kModelType", dest="model", default="ssp", type=str.lower)
    ap.add_argument("--kStaleness", dest="staleness", type=int, default=1)
    ap.add_argument("--kStorageType", dest="storage", default="map", type=str.lower)
    ap.add_argument("--transport", default="collective", choices=["collective", "onesided"])
    a = ap.parse_args(argv)
    from ..engine import Engine

    engine = Engine()
    out = run(engine, a.workers, a.iters, a.max_key, a.model, a.staleness, a.storage, a.transport)
    engine.stop()
    if engine.rank == 0:
        print(json.dumps(out), flush=True)
    ok = out["bound_violations"] == 0 and out["final_min"] == out["final_max"] == out["expected"]
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
