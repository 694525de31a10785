"""bf16 embedding rows (SparseTable(value_dtype=torch.bfloat16)): fp32 gradients and row-wise
Adagrad state, bf16 storage with stochastically rounded applies. At 2 gloo ranks the table
tracks the fp32 table within bf16 rounding, and its shards checkpoint / restore exactly."""
import torch

from test_ps_gloo import run_world


def _bf16_vs_fp32(rank, world, prefix=None):
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.tables import SparseTable

    comm = Comm(device=torch.device("cpu"))
    kw = dict(num_rows=300, width=16, optimizer="rowwise_adagrad", lr=0.05, pull_dtype=torch.float32,
              init_std=0.0, route="range")
    tb = SparseTable(comm, value_dtype=torch.bfloat16, **kw)
    tf = SparseTable(comm, **kw)
    g = torch.Generator().manual_seed(rank)
    for step in range(6):
        keys = torch.randint(0, 300, (40,), generator=g)
        vals = torch.randn(40, 16, generator=g)
        for t in (tb, tf):
            rows, plan = t.get(keys)
            t.add_keys(keys, vals)
            t.clock()
    allk = torch.arange(300)
    a, b = tb.get_rows(allk), tf.get_rows(allk)
    out = dict(dtype=str(tb.shard.dtype), err=float((a - b).abs().max()), scale=float(b.abs().max()))
    if prefix:
        from minips_amd.ps.checkpoint import Checkpointer

        ck = Checkpointer(comm, prefix)
        ck.save({0: tb}, iteration=6, blocking=True)
        snap, applies = tb.shard.clone(), tb._applies
        tb.shard.zero_()
        tb._applies = 0
        ck.load({0: tb})
        out["restored"] = bool(torch.equal(tb.shard, snap))
        # the stochastic-rounding stream resumes where it was, not at step 0
        out["applies"] = (applies, tb._applies)
    return out


class _Fn:
    def __init__(self, prefix):
        self.prefix = prefix

    def __call__(self, rank, world):
        return _bf16_vs_fp32(rank, world, self.prefix)


def test_bf16_rows_track_fp32_and_checkpoint(tmp_path):
    out = run_world(_Fn(str(tmp_path) + "/ck_"), world=2)
    for r, o in out.items():
        assert o["dtype"] == "torch.bfloat16"
        assert o["err"] <= 2 ** -7 * o["scale"] * 2 + 1e-3, o  # within a couple of bf16 ulps
        assert o["restored"], o
        assert o["applies"][0] > 0 and o["applies"][0] == o["applies"][1], o
