"""The Engine API on GPU-rank tables (minips_amd/engine.py): create_table + run(MLTask) with
several workers per rank, each with its own clock in the native ProgressTracker; the reference's
basic app (apps/basic/basic_example.cpp:19-77) through it. The same 40 workers give identical
results as 1 rank x 40 workers and as 4 gloo ranks x 10 workers."""
import pytest
import torch

from test_ps_gloo import run_world


def _basic(rank, world, workers, storage="map", transport="collective", model="ssp", iters=30):
    from minips_amd.apps.basic import run
    from minips_amd.engine import Engine
    from minips_amd.ps.comm import Comm

    eng = Engine(Comm(device=torch.device("cpu")))
    out = run(eng, workers=workers, iters=iters, max_key=200, model=model, staleness=1, storage=storage,
              transport=transport)
    eng.stop()
    return out


class _Fn:
    def __init__(self, **kw):
        self.kw = kw

    def __call__(self, rank, world):
        return _basic(rank, world, **self.kw)


def _check(out, workers_total, iters=30):
    assert out["bound_violations"] == 0, out
    assert out["final_min"] == out["final_max"] == 0.5 * workers_total * iters, out


def test_basic_app_one_rank_forty_workers():
    out = _basic(0, 1, 40)
    _check(out, 40)
    assert out["ranks"] == 1 and out["workers"] == 40


def test_basic_app_four_ranks_ten_workers_identical():
    outs = run_world(_Fn(workers=10), world=4)
    one = _basic(0, 1, 40)
    for r, o in outs.items():
        _check(o, 40)
        assert (o["final_min"], o["final_max"], o["expected"]) == (one["final_min"], one["final_max"], one["expected"])


@pytest.mark.parametrize("model", ["ssp", "asp"])
def test_basic_app_onesided_free_running_workers(model):
    """One-sided tables: the workers of a rank run free, every Get gated on its own progress."""
    outs = run_world(_Fn(workers=5, storage="vector", transport="onesided", model=model), world=2)
    for o in outs.values():
        _check(o, 10)


def _wd_engine(rank, world):
    """W&D's tables built through Engine.create_table and trained in a task."""
    from minips_amd.data.synthetic import CriteoSynth
    from minips_amd.engine import Engine, MLTask
    from minips_amd.models.widedeep import WideDeep, WideDeepConfig
    from minips_amd.ps.comm import Comm

    eng = Engine(Comm(device=torch.device("cpu")))
    cards = [50, 7, 300, 20, 5, 60, 90, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28]
    m = WideDeep(WideDeepConfig(cards=cards), eng.comm, engine=eng)
    assert set(eng.tables.values()) == {m.emb, m.dense}
    data = CriteoSynth(64, cards=cards, seed=rank)

    def fn(info):
        return [float(m.train_step(*data.next())) / 64 for _ in range(8)]

    losses = eng.run(MLTask(fn=fn, tables=[]))[0]
    eng.stop()
    return losses


def test_widedeep_tables_through_engine():
    out = run_world(_wd_engine, world=2)
    for losses in out.values():
        assert losses[-1] < losses[0], losses
