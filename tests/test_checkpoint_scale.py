"""Checkpoint I/O that scales to the 10B-row config (reference per-rank shard
dump / restore, server/vector_storage.hpp:54-90): 8 gloo ranks save through a tiny staging ring,
then restore at 8 (same sharding) and at 3 ranks (reshard). Byte counters prove each rank reads
only the rows it owns (every payload byte read once in total across the ranks), and the host
staging never exceeds the ring size."""
import os

import pytest
import torch

from test_ps_gloo import run_world

RING = 4096  # bytes: forces many streamed chunks even for these small tables
N_DENSE, N_ROWS, W = 1003, 1001, 4


def _tables(comm):
    from minips_amd.ps.tables import DenseTable, HashSparseTable, SparseTable

    dense = DenseTable(comm, N_DENSE, optimizer="adam", pull_dtype=torch.float32)
    sparse = SparseTable(comm, num_rows=N_ROWS, width=W, optimizer="rowwise_adagrad", pull_dtype=torch.float32,
                         init_std=0.0, route="range")
    hashed = HashSparseTable(comm, width=W, capacity=64)
    return {0: dense, 1: sparse, 2: hashed}


def _hash_keys():
    return torch.tensor([3, 77, 1 << 40, (1 << 62) + 5, 123456789, 42, 9999999, 5 << 50, 17, 1 << 33])


def _fill(t):
    dense, sparse, hashed = t[0], t[1], t[2]
    dense.load_full(torch.arange(N_DENSE, dtype=torch.float32))
    dense.m.copy_(dense.master * 2)
    dense.v.copy_(dense.master * 3)
    rows = torch.arange(sparse.base, sparse.base + sparse.rows_local, dtype=torch.float32)
    sparse.shard.copy_(rows[:, None] * 10 + torch.arange(W, dtype=torch.float32))
    sparse.state.copy_(rows * 0.5)
    keys = _hash_keys()
    hashed.add_keys(keys, (keys % 1000).float()[:, None].expand(-1, W).contiguous())
    hashed.clock()


def _save8(rank, world, prefix):
    from minips_amd.ps.checkpoint import Checkpointer
    from minips_amd.ps.comm import Comm

    comm = Comm(device=torch.device("cpu"))
    t = _tables(comm)
    _fill(t)
    ck = Checkpointer(comm, prefix, ring_bytes=RING)
    ck.save(t, iteration=7, blocking=True)
    return ck.peak_staging_bytes, ck.last_mode


def _restore(rank, world, prefix):
    from minips_amd._native import runtime
    from minips_amd.ps.checkpoint import Checkpointer
    from minips_amd.ps.comm import Comm

    comm = Comm(device=torch.device("cpu"))
    t = _tables(comm)
    ck = Checkpointer(comm, prefix, ring_bytes=RING)
    read = {}
    for tid in (0, 1, 2):
        runtime().reset_shard_bytes_read()
        assert ck.load({tid: t[tid]}) == 7
        read[tid] = int(runtime().shard_bytes_read())
    dense_ok = torch.equal(t[0].full_master(), torch.arange(N_DENSE, dtype=torch.float32))
    lo, hi = t[0].restore_range()
    dense_state_ok = torch.equal(t[0].m[: hi - lo], torch.arange(lo, hi, dtype=torch.float32) * 2)
    keys = torch.arange(N_ROWS)
    got = t[1].get_rows(keys)
    sparse_ok = torch.equal(got, keys.float()[:, None] * 10 + torch.arange(W, dtype=torch.float32))
    s_lo, s_hi = t[1].restore_range()
    state_ok = torch.equal(t[1].state, torch.arange(s_lo, s_hi, dtype=torch.float32) * 0.5)
    hk = _hash_keys()
    hash_ok = torch.equal(t[2].get_rows(hk)[:, 0], 8 * (hk % 1000).float())  # all 8 savers added
    owned_hash = int(((t[2]._route_keys(hk) >= t[2].restore_range()[0]) &
                      (t[2]._route_keys(hk) < t[2].restore_range()[1])).sum())
    return dict(read=read, dense_ok=dense_ok, dense_state_ok=dense_state_ok, sparse_ok=sparse_ok,
                state_ok=state_ok, hash_ok=hash_ok, dense_rows=hi - lo, sparse_rows=s_hi - s_lo,
                owned_hash=owned_hash, peak=ck.peak_staging_bytes)


class _Save:
    def __init__(self, prefix):
        self.prefix = prefix

    def __call__(self, rank, world):
        return _save8(rank, world, self.prefix)


class _Restore:
    def __init__(self, prefix):
        self.prefix = prefix

    def __call__(self, rank, world):
        return _restore(rank, world, self.prefix)


@pytest.mark.parametrize("restore_world", [8, 3])
def test_reshard_reads_only_owned_rows(tmp_path, restore_world):
    prefix = str(tmp_path / "ck_")
    saved = run_world(_Save(prefix), world=8)
    for peak, mode in saved.values():
        assert peak <= RING, peak
    out = run_world(_Restore(prefix), world=restore_world)
    n_hash = _hash_keys().numel()
    probes = 2 * 8 * (8 * 12)  # binary-search probes: 2 searches x 8 files x <= 12 reads x 8 B (loose)
    tot = {0: 0, 1: 0, 2: 0}
    for rank, r in out.items():
        assert r["dense_ok"] and r["dense_state_ok"] and r["sparse_ok"] and r["state_ok"] and r["hash_ok"], (rank, r)
        assert r["peak"] <= RING, r["peak"]
        # dense (adam): master + m + v, fp32, exactly the owned element range
        assert r["read"][0] == r["dense_rows"] * 3 * 4, (rank, r)
        # sparse (row-wise adagrad): rows x (W params + 1 state) fp32, exactly the owned rows
        assert r["read"][1] == r["sparse_rows"] * (W + 1) * 4, (rank, r)
        # hash: the owned (key, row) pairs + binary-search probes, never other ranks' rows
        payload = r["owned_hash"] * (8 + W * 4)
        assert payload <= r["read"][2] <= payload + probes, (rank, r)
        for k in tot:
            tot[k] += r["read"][k]
    assert tot[0] == N_DENSE * 3 * 4  # every byte of the checkpoint read once in total
    assert tot[1] == N_ROWS * (W + 1) * 4
    assert tot[2] >= n_hash * (8 + W * 4)


def test_large_shard_streams_through_ring_gpu_policy():
    """Above the ring size a CPU shard is written straight from memory in ring-sized pieces (no
    whole-shard host copy): mode 'stream', peak staging 0; at or below it, one staged copy."""
    from minips_amd.ps.checkpoint import Checkpointer
    from minips_amd.ps.comm import Comm

    import tempfile

    comm = Comm(device=torch.device("cpu"))
    with tempfile.TemporaryDirectory() as d:
        t = _tables(comm)
        _fill(t)
        ck = Checkpointer(comm, os.path.join(d, "a_"), ring_bytes=RING)
        ck.save(t, iteration=1, blocking=True)
        assert ck.last_mode == "stream" and ck.peak_staging_bytes == 0
        ck2 = Checkpointer(comm, os.path.join(d, "b_"), ring_bytes=1 << 20)
        ck2.save(t, iteration=1, blocking=True)
        assert ck2.last_mode == "pinned" and 0 < ck2.peak_staging_bytes <= 1 << 20
        t2 = _tables(comm)
        assert Checkpointer(comm, os.path.join(d, "a_"), ring_bytes=RING).load(t2) == 1
        assert torch.equal(t2[1].shard, t[1].shard) and torch.equal(t2[0].v, t[0].v)


class _GptSave:
    def __init__(self, prefix):
        self.prefix = prefix

    def __call__(self, rank, world):
        from minips_amd.models.gpt2 import GPT2, GPT2Config
        from minips_amd.ps.checkpoint import Checkpointer
        from minips_amd.ps.comm import Comm

        comm = Comm(device=torch.device("cpu"))
        m = GPT2(GPT2Config(vocab=300, n_ctx=32, d=128, n_layer=2, n_head=2, lr=1e-3), comm)
        g = torch.Generator().manual_seed(2)
        tokens = torch.randint(0, 300, (8, 32), generator=g)
        per = 8 // world
        for _ in range(2):
            m.train_step(tokens[rank * per:(rank + 1) * per], torch.roll(tokens, -1, 1)[rank * per:(rank + 1) * per])
        Checkpointer(comm, self.prefix).save({0: m.table}, iteration=2, blocking=True)
        return m.table.full_master().tolist(), m.table.buckets is not None


class _GptLoad:
    def __init__(self, prefix, bucketed):
        self.prefix, self.bucketed = prefix, bucketed

    def __call__(self, rank, world):
        from minips_amd.models.gpt2 import GPT2, GPT2Config
        from minips_amd.ps.checkpoint import Checkpointer
        from minips_amd.ps.comm import Comm

        comm = Comm(device=torch.device("cpu"))
        m = GPT2(GPT2Config(vocab=300, n_ctx=32, d=128, n_layer=2, n_head=2, lr=1e-3, bucketed=self.bucketed), comm)
        assert Checkpointer(comm, self.prefix).load({0: m.table}) == 2
        return m.table.full_master().tolist(), m.table.step, m.table.m.abs().sum().item() > 0


@pytest.mark.parametrize("restore_world,bucketed", [(2, True), (3, False)])
def test_bucketed_dense_checkpoint_is_canonical(tmp_path, restore_world, bucketed):
    """A bucketed (bucket-major ownership) dense table checkpoints in the canonical contiguous
    layout: it restores at another world size, bucketed or not, to the same parameters."""
    prefix = str(tmp_path / "g_")
    saved = run_world(_GptSave(prefix), world=4)
    full0, was_bucketed = saved[0]
    assert was_bucketed
    out = run_world(_GptLoad(prefix, bucketed), world=restore_world)
    for r, (full, step, has_m) in out.items():
        assert full == full0 and step == 2 and has_m


def _save_text(rank, world, prefix):
    from minips_amd.ps.checkpoint import Checkpointer
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.tables import DenseTable, SparseTable

    comm = Comm(device=torch.device("cpu"))
    dense = DenseTable(comm, 1001, optimizer="add", value_dtype=torch.float64)
    dense.load_full(torch.arange(1001, dtype=torch.float64) / 3.0)  # needs 17 digits to round-trip
    sparse = SparseTable(comm, num_rows=N_ROWS, width=W, optimizer="rowwise_adagrad", pull_dtype=torch.float32,
                         init_std=0.0, route="range")
    rows = torch.arange(sparse.base, sparse.base + sparse.rows_local, dtype=torch.float32)
    sparse.shard.copy_(rows[:, None] * 10 + torch.arange(W, dtype=torch.float32) + 1)
    ck = Checkpointer(comm, prefix, ring_bytes=RING, text_limit=-1)  # text for every shard, streamed
    ck.save({0: dense, 1: sparse}, iteration=3, blocking=True)
    # plain lists: a tensor would travel as a shared-memory fd the exiting child may close first
    return dense.master.tolist(), sparse.shard.reshape(-1).tolist()


class _SaveText:
    def __init__(self, prefix):
        self.prefix = prefix

    def __call__(self, rank, world):
        return _save_text(rank, world, self.prefix)


def test_streamed_text_checkpoint_and_reference_names(tmp_path):
    """text_limit=-1: the reference text file is written for every shard from the ring chunks
    (RING forces many chunks; indices continue across them, fp64 keeps 17 digits), and the
    reference's flat names <prefix>server_params_<id> / server_progress_<id> / worker_config_<id>
    point into the committed iteration."""
    from minips_amd.ps.checkpoint import load_text_params

    prefix = str(tmp_path / "ck_")
    out = run_world(_SaveText(prefix), world=2)
    for r in range(2):
        dense_master = torch.tensor(out[r][0], dtype=torch.float64)
        sparse_flat = torch.tensor(out[r][1], dtype=torch.float32)
        got = load_text_params(f"{prefix}server_params_{r}", dense_master.numel()).to(torch.float64)
        assert torch.equal(got, dense_master)  # exact fp64 round trip through the text
        got1 = load_text_params(f"{prefix}server_params_{r}_t1", sparse_flat.numel()).float()
        assert torch.equal(got1, sparse_flat)
        assert os.path.islink(f"{prefix}server_params_{r}")
        assert os.path.realpath(f"{prefix}server_params_{r}").endswith(f"iter_3/server_params_{r}_t0")
        assert open(f"{prefix}server_progress_{r}").read().startswith("min_clock:")
        assert open(f"{prefix}worker_config_{r}").read().strip()
