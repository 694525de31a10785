"""Numerics of every gfx950 HIP kernel against a plain PyTorch fp32 reference of the same op
(the CPU implementations in minips_amd.ops are that reference)."""
import math

import pytest
import torch

from minips_amd import _native, ops

pytestmark = pytest.mark.gpu


def _bf(x):
    return x.to(torch.bfloat16)


@pytest.fixture(autouse=True)
def _require_kernels(dev):
    _native.kernels()  # a GPU run must load the native extension, never fall back


@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (200, 136, 96), (1024, 512, 848), (64, 1024, 32)])
@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
def test_gemm_layouts_f32(dev, M, N, K, layout):
    g = torch.Generator().manual_seed(M * 7 + N)
    a_km, b_kn = {"nt": (False, False), "nn": (False, True), "tn": (True, True)}[layout]
    # asymmetric data catches transposed writes
    A = torch.randn(K if a_km else M, M if a_km else K, generator=g)
    B = torch.randn(K if b_kn else N, N if b_kn else K, generator=g)
    if (a_km and M % 8) or (b_kn and N % 8):
        pytest.skip("layout needs M/N % 8")
    Ab, Bb = _bf(A), _bf(B)
    ref = torch.empty(M, N)
    ops.gemm(Ab, Bb, ref, M, N, K, a_km, b_kn, ops.EPI_STORE_F32)
    C = torch.full((M, N), float("nan"), device=dev)
    ops.gemm(Ab.to(dev), Bb.to(dev), C, M, N, K, a_km, b_kn, ops.EPI_STORE_F32)
    torch.testing.assert_close(C.cpu(), ref, rtol=2e-3, atol=2e-3 * K ** 0.5)


def test_gemm_identity_asymmetric(dev):
    # A = I with an asymmetric B: any row/col swap in the C write shows up exactly.
    n = 128
    A = torch.eye(n)
    B = torch.arange(n * n, dtype=torch.float32).view(n, n) % 97
    C = torch.zeros(n, n, device=dev)
    ops.gemm(_bf(A).to(dev), _bf(B).to(dev), C, n, n, n, False, True, ops.EPI_STORE_F32)
    torch.testing.assert_close(C.cpu(), _bf(B).float())


def test_gemm_epilogues(dev):
    g = torch.Generator().manual_seed(3)
    M, N, K = 384, 256, 160
    X = _bf(torch.randn(M, K, generator=g))
    W = _bf(torch.randn(N, K, generator=g) * 0.1)
    b = _bf(torch.randn(N, generator=g))
    for act in ("relu", "none", "gelu"):
        ref = ops.linear_fwd(X, W, b, act)
        out = ops.linear_fwd(X.to(dev), W.to(dev), b.to(dev), act)
        torch.testing.assert_close(out.float().cpu(), ref.float(), rtol=2e-2, atol=2e-2)
    # dgrad with relu mask + colsum
    dY = _bf(torch.randn(M, N, generator=g))
    mask = _bf(torch.randn(M, K, generator=g))
    cs_ref = torch.zeros(K)
    ref = ops.linear_dgrad(dY, W, mask=mask, colsum=cs_ref)
    cs = torch.zeros(K, device=dev)
    out = ops.linear_dgrad(dY.to(dev), W.to(dev), mask=mask.to(dev), colsum=cs)
    torch.testing.assert_close(out.float().cpu(), ref.float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(cs.cpu(), cs_ref, rtol=1e-3, atol=1e-2)
    # wgrad split-K accumulate
    dW_ref = torch.ones(N, K)
    ops.linear_wgrad(dY, X, dW_ref)
    dW = torch.ones(N, K, device=dev)
    ops.linear_wgrad(dY.to(dev), X.to(dev), dW, split_k=3)
    torch.testing.assert_close(dW.cpu(), dW_ref, rtol=2e-3, atol=2e-2)


def test_unique_bucketize(dev):
    g = torch.Generator().manual_seed(0)
    keys = torch.randint(0, 5000, (20000,), generator=g)
    bounds = torch.tensor([0, 1000, 2500, 4000, 5000])
    uniq, inv, counts = ops.unique_bucketize(keys.to(dev), bounds.to(dev))
    uniq, inv, counts = uniq.cpu(), inv.cpu(), counts.cpu()
    U = int(counts.sum())
    assert U == torch.unique(keys).numel()
    torch.testing.assert_close(uniq[inv], keys)  # inverse is exact
    u = uniq[:U]
    assert torch.unique(u).numel() == U
    start = 0
    for p in range(4):  # grouped by owner
        seg = u[start: start + int(counts[p])]
        assert ((seg >= bounds[p]) & (seg < bounds[p + 1])).all()
        start += int(counts[p])


def test_gather_scatter_adagrad(dev):
    g = torch.Generator().manual_seed(1)
    R, W = 1000, 36
    table = torch.randn(R, W, generator=g)
    keys = torch.randint(100, 100 + R, (300,), generator=g).unique()
    for dt in (torch.float32, torch.bfloat16):
        out = torch.empty(keys.numel(), W, dtype=dt, device=dev)
        ops.gather_rows(table.to(dev), keys.to(dev), 100, out)
        torch.testing.assert_close(out.float().cpu(), table[keys - 100].to(dt).float())
    src = torch.randn(500, W, generator=g)
    idx = torch.randint(0, 50, (500,), generator=g)
    acc = torch.zeros(50, W, device=dev)
    ops.scatter_add_rows(src.to(dev), idx.to(dev), acc)
    torch.testing.assert_close(acc.cpu(), torch.zeros(50, W).index_add_(0, idx, src), rtol=1e-5, atol=1e-5)
    # row-wise adagrad with split state
    grads = torch.randn(keys.numel(), 33, generator=g)
    t_ref, s_ref, s2_ref = table.clone(), torch.rand(R, generator=g), torch.rand(R, generator=g)
    t_gpu, s_gpu, s2_gpu = t_ref.to(dev), s_ref.to(dev), s2_ref.to(dev)
    ops.sparse_rowwise_adagrad(t_ref, s_ref, keys, 100, grads, 0.1, 1e-8, state2=s2_ref, split=32)
    ops.sparse_rowwise_adagrad(t_gpu, s_gpu, keys.to(dev), 100, grads.to(dev), 0.1, 1e-8, state2=s2_gpu, split=32)
    torch.testing.assert_close(t_gpu.cpu(), t_ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(s_gpu.cpu(), s_ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(s2_gpu.cpu(), s2_ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("D,split", [(36, 32), (64, 64), (20, 20), (48, 40)])
def test_rowwise_adagrad_vec4(dev, D, split):
    """16-byte rows take the 8-lanes-per-row float4 kernel: same result as the CPU reference,
    including the split (deep | wide) state and rows past 32 columns."""
    g = torch.Generator().manual_seed(D)
    R = 5000
    table = torch.randn(R, D, generator=g)
    keys = torch.randperm(R, generator=g)[:3001] + 7
    grads = torch.randn(keys.numel(), D, generator=g)
    s_ref, s2_ref = torch.rand(R, generator=g), torch.rand(R, generator=g)
    t_ref = table.clone()
    t_gpu, s_gpu, s2_gpu = table.to(dev), s_ref.to(dev), s2_ref.to(dev)
    kw = dict(state2=s2_ref, split=split) if split < D else {}
    ops.sparse_rowwise_adagrad(t_ref, s_ref, keys, 7, grads, 0.05, 1e-8, **kw)
    kw = dict(state2=s2_gpu, split=split) if split < D else {}
    ops.sparse_rowwise_adagrad(t_gpu, s_gpu, keys.to(dev), 7, grads.to(dev), 0.05, 1e-8, **kw)
    torch.testing.assert_close(t_gpu.cpu(), t_ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(s_gpu.cpu(), s_ref, rtol=1e-5, atol=1e-6)
    if split < D:
        torch.testing.assert_close(s2_gpu.cpu(), s2_ref, rtol=1e-5, atol=1e-6)


def test_dense_optimizers(dev):
    g = torch.Generator().manual_seed(2)
    n = 10003
    w, m, v, gr = (torch.randn(n, generator=g) for _ in range(4))
    v = v.abs()
    cpu = [t.clone() for t in (w, m, v)]
    gpu = [t.to(dev) for t in (w, m, v)]
    wb = torch.empty(n, dtype=torch.bfloat16, device=dev)
    ops.adam_apply(*cpu, gr, 1e-2, step=3, weight_decay=0.01)
    ops.adam_apply(*gpu, gr.to(dev), 1e-2, step=3, weight_decay=0.01, w_bf16=wb)
    for a, b in zip(gpu, cpu):
        torch.testing.assert_close(a.cpu(), b, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(wb.float().cpu(), cpu[0].to(torch.bfloat16).float())
    # zero_g: same update, and the gradient (odd length: float4 body + tail) comes back cleared
    gz, gpu2 = gr.to(dev), [t.to(dev) for t in (w, m, v)]
    ops.adam_apply(*gpu2, gz, 1e-2, step=3, weight_decay=0.01, zero_g=True)
    for a, b in zip(gpu2, cpu):
        torch.testing.assert_close(a.cpu(), b, rtol=1e-5, atol=1e-6)
    assert int((gz != 0).sum()) == 0
    acc = torch.rand(n, generator=g)
    w1, a1 = w.clone(), acc.clone()
    w2, a2 = w.to(dev), acc.to(dev)
    ops.adagrad_apply(w1, a1, gr, 0.1)
    ops.adagrad_apply(w2, a2, gr.to(dev), 0.1)
    torch.testing.assert_close(w2.cpu(), w1, rtol=1e-5, atol=1e-6)


def test_widedeep_kernels(dev):
    g = torch.Generator().manual_seed(4)
    B, F, D, nd, U = 96, 5, 32, 13, 40
    ldx = (F * D + nd + 7) // 8 * 8
    rows = _bf(torch.randn(U, 36, generator=g))
    inv = torch.randint(0, U, (B * F,), generator=g)
    dense = torch.randn(B, nd, generator=g)
    X_ref, w_ref = torch.empty(B, ldx, dtype=torch.bfloat16), torch.empty(B)
    ops.wd_assemble(dense, rows, inv, F, D, X_ref, w_ref)
    X, wl = torch.empty(B, ldx, dtype=torch.bfloat16, device=dev), torch.empty(B, device=dev)
    ops.wd_assemble(dense.to(dev), rows.to(dev), inv.to(dev), F, D, X, wl)
    torch.testing.assert_close(X.cpu(), X_ref)
    torch.testing.assert_close(wl.cpu(), w_ref, rtol=1e-5, atol=1e-5)
    # head
    Hd = 256
    H = _bf(torch.relu(torch.randn(B, Hd, generator=g)))
    w = _bf(torch.randn(Hd, generator=g) * 0.1)
    b0 = _bf(torch.tensor([0.1]))
    y = (torch.rand(B, generator=g) > 0.5).float()

    def run(d):
        outs = dict(dH=torch.empty(B, Hd, dtype=torch.bfloat16, device=d), dw=torch.zeros(Hd, device=d),
                    db=torch.zeros(1, device=d), dwide=torch.empty(B, device=d), loss=torch.zeros(1, device=d),
                    cs=torch.zeros(Hd, device=d))
        ops.wd_head(H.to(d), w.to(d), b0.to(d), w_ref.to(d), y.to(d), outs["dH"], outs["dw"], outs["db"],
                    outs["dwide"], outs["loss"], outs["cs"], 1.0 / B)
        return {k: v.cpu() for k, v in outs.items()}

    r, o = run("cpu"), run(dev)
    for k in r:
        torch.testing.assert_close(o[k].float(), r[k].float(), rtol=2e-2, atol=1e-4)
    # embedding backward
    dX = torch.randn(B, F * D, generator=g)
    dwide = torch.randn(B, generator=g)
    gr_ref = torch.zeros(U, 36)
    ops.wd_emb_backward(dX, dwide, inv, F, D, gr_ref)
    gr = torch.zeros(U, 36, device=dev)
    ops.wd_emb_backward(dX.to(dev), dwide.to(dev), inv.to(dev), F, D, gr)
    torch.testing.assert_close(gr.cpu(), gr_ref, rtol=1e-4, atol=1e-4)


def test_wd_assemble_tab_and_head_full_batch(dev):
    """The one-rank fused Get+assemble (rows read in place from the fp32 shard) is bit-identical
    to gather_rows(bf16) + wd_assemble; the head at the bench's batch (256 blocks, per-block
    partials folded by atomics) matches the fp32 reference."""
    g = torch.Generator().manual_seed(14)
    B, F, D, nd, rows_local, base = 2048, 26, 32, 13, 5000, 1000
    ldx = (F * D + nd + 1 + 63) // 64 * 64
    shard = torch.randn(rows_local, 36, generator=g)
    U = 1500
    uniq = torch.randperm(rows_local, generator=g)[:U] + base
    inv = torch.randint(0, U, (B * F,), generator=g)
    dense = torch.randn(B, nd, generator=g)
    d = lambda t: t.to(dev)  # noqa: E731
    rows = torch.empty(U, 36, dtype=torch.bfloat16, device=dev)
    ops.gather_rows(d(shard), d(uniq), base, rows)
    X1, w1 = torch.empty(B, ldx, dtype=torch.bfloat16, device=dev), torch.empty(B, device=dev)
    z1 = torch.ones(1, device=dev)
    ops.wd_assemble(d(dense), rows, d(inv), F, D, X1, w1, ones_col=F * D + nd, zero=z1)
    X2, w2 = torch.empty_like(X1), torch.empty_like(w1)
    z2 = torch.ones(1, device=dev)
    ops.wd_assemble_tab(d(dense), d(shard), d(uniq), base, d(inv), F, D, X2, w2, ones_col=F * D + nd, zero=z2)
    assert torch.equal(X1, X2)
    torch.testing.assert_close(w2, w1, rtol=1e-6, atol=1e-6)
    assert float(z2) == 0.0
    # CPU reference of the in-place form
    X3, w3 = torch.empty(B, ldx, dtype=torch.bfloat16), torch.empty(B)
    ops.wd_assemble_tab(dense, shard, uniq, base, inv, F, D, X3, w3, ones_col=F * D + nd)
    assert torch.equal(X3, X1.cpu())
    # head at the bench's batch
    Bh, Hd = 16384, 256
    H = _bf(torch.relu(torch.randn(Bh, Hd, generator=g)))
    w = _bf(torch.randn(Hd, generator=g) * 0.1)
    b0 = _bf(torch.tensor([0.1]))
    wide = torch.randn(Bh, generator=g)
    y = (torch.rand(Bh, generator=g) > 0.5).float()

    def run(dv, defer=False):
        o = dict(dH=torch.empty(Bh, Hd, dtype=torch.bfloat16, device=dv), dw=torch.full((Hd,), 0.5, device=dv),
                 db=torch.full((1,), 0.25, device=dv), dwide=torch.empty(Bh, device=dv),
                 loss=torch.zeros(1, device=dv), cs=torch.zeros(Hd, device=dv))
        ops.wd_head(H.to(dv), w.to(dv), b0.to(dv), wide.to(dv), y.to(dv), o["dH"], o["dw"], o["db"], o["dwide"],
                    o["loss"], o["cs"], 1.0 / Bh, defer_fold=defer)
        if defer:  # the batch sums folded by the separate kernel, on another stream
            side = torch.cuda.Stream(device=dv)
            side.wait_stream(torch.cuda.current_stream(dv))
            with torch.cuda.stream(side):
                ops.wd_head_fold(Bh, Hd, o["dw"], o["db"], o["loss"], o["cs"])
            torch.cuda.current_stream(dv).wait_stream(side)
        return {k: v.cpu() for k, v in o.items()}

    r, o = run("cpu"), run(dev)
    for k in r:
        torch.testing.assert_close(o[k].float(), r[k].float(), rtol=2e-2, atol=1e-4)
    # the deferred fold sums the 256 block rows in the in-kernel fold's order: bit-identical
    od = run(dev, defer=True)
    for k in o:
        assert torch.equal(od[k], o[k]), k


def test_lr_and_kmeans(dev):
    g = torch.Generator().manual_seed(5)
    B, nnz, U = 64, 10, 200
    rowptr = torch.arange(0, (B + 1) * nnz, nnz)
    cols = torch.randint(0, U, (B * nnz,), generator=g)
    vals = torch.rand(B * nnz, generator=g)
    labels = torch.where(torch.rand(B, generator=g) > 0.5, 1.0, -1.0)
    w = torch.randn(U, generator=g) * 0.1
    d_ref, c_ref = torch.zeros(U), torch.zeros(1)
    ops.lr_sparse_step(rowptr, cols, vals, labels, w, 0.5, d_ref, c_ref)
    d, c = torch.zeros(U, device=dev), torch.zeros(1, device=dev)
    ops.lr_sparse_step(rowptr.to(dev), cols.to(dev), vals.to(dev), labels.to(dev), w.to(dev), 0.5, d, c)
    torch.testing.assert_close(d.cpu(), d_ref, rtol=1e-4, atol=1e-5)
    assert float(c) == float(c_ref)
    X = torch.randn(500, 24, generator=g)
    C = torch.randn(5, 24, generator=g)
    a_ref = ops.kmeans_assign(X, C)
    a = ops.kmeans_assign(X.to(dev), C.to(dev))
    assert (a.cpu() == a_ref).float().mean() > 0.995


def test_embedding_bag(dev):
    g = torch.Generator().manual_seed(6)
    rows = torch.randn(100, 16, generator=g)
    idx = torch.randint(0, 100, (50,), generator=g)
    offsets = torch.tensor([0, 3, 3, 10, 25, 50])
    for mean in (False, True):
        ref = ops.embedding_bag_fwd(rows, idx, offsets, mean)
        out = ops.embedding_bag_fwd(rows.to(dev), idx.to(dev), offsets.to(dev), mean)
        torch.testing.assert_close(out.cpu(), ref, rtol=1e-5, atol=1e-5)
        go = torch.randn(5, 16, generator=g)
        gr_ref = ops.embedding_bag_bwd(go, idx, offsets, torch.zeros(100, 16), mean)
        gr = ops.embedding_bag_bwd(go.to(dev), idx.to(dev), offsets.to(dev), torch.zeros(100, 16, device=dev), mean)
        torch.testing.assert_close(gr.cpu(), gr_ref, rtol=1e-5, atol=1e-5)


def test_criteo_synth_kernel(dev):
    from minips_amd.data.synthetic import CRITEO_KAGGLE_CARDS, CriteoSynth

    d = CriteoSynth(4096, device=dev, seed=3)
    dense, keys, y = d.next()
    offs = d.offsets.cpu()
    cards = torch.tensor(CRITEO_KAGGLE_CARDS)
    k = keys.cpu() - offs
    assert (k >= 0).all() and (k < cards).all()
    assert abs(float(dense.mean())) < 0.05 and abs(float(dense.std()) - 1) < 0.05
    assert 0.2 < float(y.mean()) < 0.8
    # Zipf-like head: the most frequent id of the 10M-row feature covers a visible share
    col = keys[:, 2]
    assert torch.unique(col).numel() < 4096
    d2 = CriteoSynth(4096, device=dev, seed=3)
    torch.testing.assert_close(d2.next()[1], keys)  # reproducible


@pytest.mark.parametrize("D,dtype", [(32, torch.bfloat16), (64, torch.float32), (16, torch.bfloat16)])
def test_embedding_backward_segment_hot_rows(dev, D, dtype):
    """Segment-sum embedding backward incl. Zipf-hot rows (thousands of lookups: spanning many
    pieces, finished by the fix-up kernel over the pieces' partials); rows without lookups are
    not written (a plan's unique rows always have lookups)."""
    g = torch.Generator().manual_seed(D)
    B, F, U = 8192, 3, 5000
    inv = torch.randint(0, U - 100, (B * F,), generator=g)  # the last 100 rows get no lookups
    inv[: 6000] = 7                                         # a hot row: 6000 lookups
    inv[6000: 8500] = 11                                    # and one just above the split size
    dX = torch.randn(B, F * D + 8, generator=g).to(dtype)
    dwide = torch.randn(B, generator=g)
    ref = torch.zeros(U, D + 4)
    ops.wd_emb_backward(dX.float(), dwide, inv, F, D, ref)
    gr = torch.full((U, D + 4), float("nan"), device=dev)
    ops.wd_emb_backward(dX.to(dev), dwide.to(dev), inv.to(dev), F, D, gr)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-3
    hit = torch.zeros(U, dtype=torch.bool)
    hit[inv] = True
    torch.testing.assert_close(gr.cpu()[hit], ref[hit], rtol=1e-4, atol=tol * 8)
    assert bool(torch.isnan(gr.cpu()[~hit]).all())  # untouched


@pytest.mark.parametrize("D,out_dtype", [(32, torch.float32), (32, torch.bfloat16), (64, torch.bfloat16),
                                         (16, torch.float32)])
def test_embedding_backward_deterministic(dev, D, out_dtype):
    """The segment sum has one fixed summation order (no atomics): repeated runs are bit-identical,
    for fp32 and bf16 output rows (the multi-rank push payload), Criteo-shaped batches with hot rows
    that span many pieces; the wide column and the zero pad columns are written."""
    g = torch.Generator().manual_seed(40 + D)
    B, F = 16384, 26
    cards = [3, 50, 1000, 20000] * 6 + [7, 100000]
    keys = torch.stack([torch.randint(0, c, (B,), generator=g) for c in cards], 1)
    keys[:5000, 1] = 4  # a very hot row (5000 lookups)
    base = torch.tensor([sum(cards[:f]) for f in range(F)], dtype=torch.int64)
    bits = [max(1, (c - 1).bit_length()) for c in cards]
    res = ops.plan_sorted((keys + base).to(dev), base.to(dev), bits)
    inv, U = res[1], int(res[3].item())
    csr = (res[4], res[5])
    W = D + 4
    dX = (torch.randn(B, F * D, generator=g) * 0.1).to(torch.bfloat16).to(dev)
    dwide = torch.randn(B, generator=g).to(dev)
    outs = []
    for _ in range(3):
        gr = torch.full((B * F, W), float("nan"), dtype=out_dtype, device=dev)
        ops.wd_emb_backward(dX, dwide, inv, F, D, gr, csr=csr)
        outs.append(gr[:U].clone())
    for o in outs[1:]:
        assert torch.equal(o.view(torch.int16) if out_dtype == torch.bfloat16 else o.view(torch.int32),
                           outs[0].view(torch.int16) if out_dtype == torch.bfloat16 else outs[0].view(torch.int32))
    ref = torch.zeros(U, W)
    ops.wd_emb_backward(dX.cpu().float(), dwide.cpu(), inv.cpu(), F, D, ref)
    tol = 2e-2 if out_dtype == torch.bfloat16 else 2e-3
    torch.testing.assert_close(outs[0].float().cpu(), ref, rtol=tol, atol=tol)
    assert bool((outs[0][:, D + 1:] == 0).all())


@pytest.mark.parametrize("P,recv_dtype", [(8, torch.bfloat16), (3, torch.float32), (16, torch.bfloat16)])
def test_owner_rows_adagrad(dev, P, recv_dtype):
    """Owner side of a multi-rank push: owner_slots + owner_rows_adagrad (per owned row the <= P
    requesters' rows summed in requester order, row-wise Adagrad with the split state) against the
    scatter-add + sparse_rowwise_adagrad reference, bit-identical across runs, rows past the device
    count untouched."""
    g = torch.Generator().manual_seed(P)
    R, W, D1, base = 50000, 36, 32, 1000
    splits = [int(x) for x in torch.randint(500, 3000, (P,), generator=g)]
    # each requester pushes distinct keys; requesters overlap (hot keys pushed by everyone)
    segs = [torch.cat([torch.arange(5), torch.randperm(R - 5, generator=g)[: n - 5] + 5]) + base for n in splits]
    recv_keys = torch.cat(segs)
    uniq, own_inv = torch.unique(recv_keys, return_inverse=True)
    U, M = uniq.numel(), recv_keys.numel()
    own_uniq = torch.full((M,), -1, dtype=torch.int64)
    own_uniq[:U] = uniq
    recv = (torch.randn(M, W, generator=g) * 0.1).to(recv_dtype)
    table = torch.randn(R, W, generator=g)
    state, state2 = torch.rand(R, generator=g), torch.rand(R, generator=g)
    # reference: scatter-add, then the plain apply
    gsum = torch.zeros(U, W)
    gsum.index_add_(0, own_inv, recv.float())
    t_ref, s_ref, s2_ref = table.clone(), state.clone(), state2.clone()
    ops.sparse_rowwise_adagrad(t_ref, s_ref, uniq, base, gsum, 0.05, 1e-8, state2=s2_ref, split=D1)
    slots = ops.owner_slots(own_inv.to(dev), splits, M)
    cslots = ops.owner_slots(own_inv, splits, M)
    assert torch.equal(slots.cpu(), cslots)
    U_dev = torch.tensor([U], device=dev)
    runs = []
    for _ in range(2):
        t, s1, s2 = table.to(dev), state.to(dev), state2.to(dev)
        ops.owner_rows_adagrad(t, s1, own_uniq.to(dev), M, base, recv.to(dev), slots, P, 0.05, 1e-8, state2=s2,
                               split=D1, n_dev=U_dev)
        runs.append((t.cpu(), s1.cpu(), s2.cpu()))
    assert all(torch.equal(a, b) for a, b in zip(runs[0], runs[1]))
    torch.testing.assert_close(runs[0][0], t_ref, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(runs[0][1], s_ref, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(runs[0][2], s2_ref, rtol=1e-4, atol=1e-6)
    # the CPU reference of the fused op agrees too
    t_c, s_c, s2_c = table.clone(), state.clone(), state2.clone()
    ops.owner_rows_adagrad(t_c, s_c, own_uniq, M, base, recv, cslots, P, 0.05, 1e-8, state2=s2_c, split=D1,
                           n_dev=torch.tensor([U]))
    torch.testing.assert_close(t_c, t_ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("P,recv_dtype", [(2, torch.float32), (8, torch.bfloat16), (13, torch.bfloat16)])
def test_owner_push_adagrad_direct(dev, P, recv_dtype):
    """The direct-addressed owner apply (stamp table, no owner-side plan) is bit-identical to the
    planned fused apply (owner_slots + owner_rows_adagrad) over three consecutive pushes that share
    one stamp table -- entries of earlier pushes must retire by their stamp -- and agrees with its
    CPU reference."""
    g = torch.Generator().manual_seed(100 + P)
    R, W, D1, base = 40000, 36, 32, 700
    table = torch.randn(R, W, generator=g)
    state, state2 = torch.rand(R, generator=g), torch.rand(R, generator=g)
    t_a, s_a, s2_a = table.to(dev), state.to(dev), state2.to(dev)
    t_b, s_b, s2_b = table.to(dev), state.to(dev), state2.to(dev)
    t_c, s_c, s2_c = table.clone(), state.clone(), state2.clone()
    rs = torch.full((R * P * 2,), -1, dtype=torch.int32, device=dev)
    for push in range(3):
        splits = [int(x) for x in torch.randint(0 if push == 1 else 300, 2500, (P,), generator=g)]
        segs = [torch.cat([torch.arange(min(n, 4)), torch.randperm(R - 4, generator=g)[: max(0, n - 4)] + 4]) + base
                for n in splits]
        recv_keys = torch.cat(segs)
        M = recv_keys.numel()
        recv = (torch.randn(M, W, generator=g) * 0.1).to(recv_dtype)
        uniq, own_inv = torch.unique(recv_keys, return_inverse=True)
        U = uniq.numel()
        own_uniq = torch.full((max(M, 1),), -1, dtype=torch.int64)
        own_uniq[:U] = uniq
        slots = ops.owner_slots(own_inv.to(dev), splits, M)
        ops.owner_rows_adagrad(t_a, s_a, own_uniq.to(dev), M, base, recv.to(dev), slots, P, 0.05, 1e-8, state2=s2_a,
                               split=D1, n_dev=torch.tensor([U], device=dev))
        ops.owner_push_adagrad(t_b, s_b, recv_keys.to(dev), base, recv.to(dev), splits, rs, push, 0.05, 1e-8,
                               state2=s2_b, split=D1)
        ops.owner_push_adagrad(t_c, s_c, recv_keys, base, recv, splits, None, push, 0.05, 1e-8, state2=s2_c, split=D1)
    assert torch.equal(t_a.cpu(), t_b.cpu()) and torch.equal(s_a.cpu(), s_b.cpu())
    assert torch.equal(s2_a.cpu(), s2_b.cpu())
    torch.testing.assert_close(t_b.cpu(), t_c, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(s_b.cpu(), s_c, rtol=1e-5, atol=1e-6)


def test_device_counts_and_prebuilt_csr(dev):
    """unique_bucketize_n's device-side U bounds gather / row-wise Adagrad / the embedding
    backward without a host sync; the CSR prebuilt at planning time gives the same gradient."""
    g = torch.Generator().manual_seed(5)
    B, F, D = 4096, 4, 32
    keys = torch.randint(0, 3000, (B, F), generator=g)
    bounds = torch.tensor([0, 3000])
    uniq, inv, counts, U_dev = ops.unique_bucketize_n(keys.to(dev), bounds.to(dev), F)
    U = int(U_dev.item())
    assert U == int(counts.sum()) == torch.unique(keys).numel()
    n = keys.numel()
    table = torch.randn(3000, 36, generator=g)
    # gather bounded by the device count: rows past U untouched
    out = torch.full((n, 36), 7.0, device=dev)
    ops.gather_rows(table.to(dev), uniq, 0, out, n_dev=U_dev)
    torch.testing.assert_close(out[:U].cpu(), table[uniq[:U].cpu()])
    assert bool((out[U:] == 7.0).all())
    # embedding backward with the prebuilt CSR vs the reference
    dX = torch.randn(B, F * D, generator=g).to(torch.bfloat16)
    dwide = torch.randn(B, generator=g)
    ref = torch.zeros(U, D + 1)
    ops.wd_emb_backward(dX.float(), dwide, inv.cpu(), F, D, ref)
    csr = ops.emb_build_csr(inv, F, n)
    gr = torch.full((n, D + 1), float("nan"), device=dev)
    ops.wd_emb_backward(dX.to(dev), dwide.to(dev), inv, F, D, gr, csr=csr)
    torch.testing.assert_close(gr[:U].cpu(), ref, rtol=1e-4, atol=0.16)
    # row-wise Adagrad bounded by the device count: keys past U (garbage) never applied
    t_gpu = table.to(dev)
    st = torch.zeros(3000, device=dev)
    grads = torch.randn(n, 36, generator=g)
    ops.sparse_rowwise_adagrad(t_gpu, st, uniq, 0, grads.to(dev), 0.1, n_dev=U_dev)
    t_ref, s_ref = table.clone(), torch.zeros(3000)
    ops.sparse_rowwise_adagrad(t_ref, s_ref, uniq[:U].cpu(), 0, grads[:U], 0.1)
    torch.testing.assert_close(t_gpu.cpu(), t_ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("n,k,d", [(20000, 1000, 128), (3000, 37, 20)])
def test_kmeans_assign_mfma(dev, n, k, d):
    """MFMA (hi/lo-split bf16 GEMM + argmin) assignment vs the fp64 reference: the chosen centre
    is optimal up to fp32 rounding of the distance, and the distances match."""
    g = torch.Generator().manual_seed(k)
    X = torch.randn(n, d, generator=g)
    C = torch.randn(k, d, generator=g)
    dist_ref = torch.cdist(X.double(), C.double()) ** 2
    best_ref = dist_ref.min(1).values
    dist = torch.empty(n, device=dev)
    a = ops.kmeans_assign(X.to(dev), C.to(dev), dist=dist, mfma=True).cpu().long()
    chosen = dist_ref.gather(1, a.view(-1, 1)).view(-1)
    assert bool(((chosen - best_ref) <= 1e-4 * best_ref.abs() + 1e-4).all())
    torch.testing.assert_close(dist.cpu().double(), best_ref, rtol=1e-4, atol=1e-3)


def test_unique_bucketize_fused_routing(dev):
    """key -> key*A mod N routing fused into the dedupe kernel matches routing first on the CPU."""
    from minips_amd.ps.tables import _route_multiplier

    g = torch.Generator().manual_seed(8)
    N = 33_762_577
    A = _route_multiplier(N)
    keys = torch.randint(0, N, (4096, 26), generator=g)
    keys[:, 3] = keys[0, 3]  # a hot id
    bounds = torch.tensor([0, N // 4, N // 2, 3 * (N // 4), N])
    u, inv, c, U = ops.unique_bucketize_n(keys.to(dev), bounds.to(dev), 26, A, N)
    ur, invr, cr, Ur = ops.unique_bucketize_n(keys, bounds, 26, A, N)
    assert int(U) == int(Ur) and c.cpu().tolist() == cr.tolist()
    assert torch.equal(u.cpu()[inv.cpu()], (keys.reshape(-1) * A) % N)


@pytest.mark.parametrize("P", [1, 8])
def test_dedupe_fused_csr_counts(dev, P):
    """The dedupe's fused per-key lookup counts equal bincount(inverse), and the CSR built from
    them (counts_ready) groups exactly the lookups of each unique row."""
    g = torch.Generator().manual_seed(P)
    B, F = 4096, 26
    hot = torch.randint(0, 4, (B, F), generator=g)            # Zipf-like head: tiny cardinalities
    cold = torch.randint(0, 1 << 20, (B, F), generator=g)
    keys = torch.where(torch.rand(B, F, generator=g) < 0.5, hot, cold).to(dev)
    n = B * F
    bounds = torch.linspace(0, 1 << 20, P + 1).long().to(dev)
    bounds[-1] = 1 << 62
    (uniq, inv, counts, U_dev), zeroed = ops.unique_bucketize_n(keys, bounds, F, extra_zero_ints=2 * n,
                                                                csr_counts=True)
    U = int(U_dev.item())
    ref = torch.bincount(inv.cpu(), minlength=U)
    torch.testing.assert_close(zeroed[:U].cpu(), ref.to(torch.int32))
    assert int(zeroed[U:n].abs().sum()) == 0
    members, memrow = ops.emb_build_csr(inv, F, n, zeroed=zeroed, counts_ready=True)
    memrow_c, members_c = memrow.cpu().long(), members.cpu().long()
    assert bool((memrow_c[1:] >= memrow_c[:-1]).all())
    torch.testing.assert_close(inv.cpu()[members_c], memrow_c)
    assert sorted(members_c.tolist()) == list(range(n))


def test_sparse_lr_fp64_matches_cpu(dev):
    """Reference-precision LR (double tables, lr_example.cpp:182): the fp64 HIP path (f64 row
    kernels + lr_sparse_step<double>) matches the CPU fp64 oracle to fp64 rounding."""
    from minips_amd.data.synthetic import SparseLRSynth
    from minips_amd.models.lr import SparseLR, SparseLRConfig
    from minips_amd.ps.comm import Comm

    res = {}
    for d in (torch.device("cpu"), dev):
        m = SparseLR(SparseLRConfig(num_dims=3000, alpha=0.05, value_dtype=torch.float64), Comm(device=d))
        data = SparseLRSynth(256, num_dims=3000, nnz=16, device="cpu", seed=7)
        for _ in range(5):
            rp, c, v, y = data.next()
            m.train_step(rp.to(d), c.to(d), v.to(d), y.to(d))
        res[d.type] = m.table.shard.cpu()
    assert res["cuda"].dtype == torch.float64
    assert torch.allclose(res["cuda"], res["cpu"], rtol=1e-12, atol=1e-14)
    assert res["cpu"].abs().sum() > 0


def test_colsum_bf16(dev):
    """ops.colsum_add (bias gradient of a Linear) against the fp32 column sums."""
    g = torch.Generator().manual_seed(11)
    for M, N in ((16384, 512), (1000, 72), (3, 8)):
        x = torch.randn(M, N, generator=g).to(torch.bfloat16)
        out = torch.full((N,), 0.5)
        ref = out + x.float().sum(0)
        got = ops.colsum_add(x.to(dev), out.to(dev))
        torch.testing.assert_close(got.cpu(), ref, rtol=1e-4, atol=1e-3)
        again = ops.colsum_add(x.to(dev), out.to(dev))  # one summation order: bit-identical
        assert torch.equal(again.cpu(), got.cpu())


@pytest.mark.parametrize("B,cards,P", [(16384, [3, 1460, 10131227, 583, 24, 2202608], 1),
                                       (16384, [3, 1460, 10131227, 583, 24, 2202608], 8), (1000, [5, 70000], 3),
                                       (16384, [1 << 24], 1), (4096, [1 << 27, 7, 1], 16)])
def test_plan_sorted_matches_reference(dev, B, cards, P):
    """Atomic-free sort-based planning (plan.hip) vs the CPU reference of the same op: unique keys
    column-major / ascending, stably regrouped by owner for P > 1 owners (the owner bits ride above
    the key in the sort: 27 + 4 bits for 16 owners); uniq[inv] == routed keys; the lookup CSR with
    contiguous rows; per-owner counts."""
    g = torch.Generator().manual_seed(B + len(cards) + P)
    bases = [sum(cards[:f]) for f in range(len(cards))]
    cols = []
    for c, base in zip(cards, bases):
        zipf = torch.floor(torch.exp(torch.rand(B, generator=g, dtype=torch.float64) * math.log(c + 1)) - 1)
        cols.append(zipf.clamp(0, c - 1).to(torch.int64) + base)
    keys = torch.stack(cols, 1)
    R = sum(cards)
    mult = 402653189 if R % 402653189 else 201326611
    bits = [max(1, (c - 1).bit_length()) for c in cards]
    bounds = torch.tensor([R * p // P for p in range(P + 1)], dtype=torch.int64)
    ref = ops.plan_sorted(keys, torch.tensor(bases), bits, mult, R, bounds=bounds)
    got = [None if t is None else t.cpu() for t in ops.plan_sorted(keys.to(dev), torch.tensor(bases, device=dev),
                                                                   bits, mult, R, bounds=bounds.to(dev))]
    U = int(ref[3])
    assert int(got[3]) == U and int(got[2].sum()) == U
    torch.testing.assert_close(got[2], ref[2])                      # per-owner counts
    torch.testing.assert_close(got[0][:U], ref[0][:U])              # grouped by owner
    torch.testing.assert_close(got[1], ref[1])
    torch.testing.assert_close(got[0][got[1]], (keys.reshape(-1) * mult) % R)
    torch.testing.assert_close(got[4], ref[4])
    torch.testing.assert_close(got[5], ref[5])
    assert bool((got[1][got[4].long()] == got[5].long()).all())      # members belong to their row
    pos = ops.plan_sorted(keys.to(dev), torch.tensor(bases, device=dev), bits, mult, R, bounds=bounds.to(dev),
                          positions=True)[6].cpu()
    assert torch.equal(pos[got[4].long()], torch.arange(keys.numel(), dtype=torch.int32))  # inverse of members
    if P == 1:  # rowstart, and each lookup's table row (routed key) for the input assembly
        assert len(got) == 9 and len(ref) == 9
        torch.testing.assert_close(got[7][: U + 1], ref[7][: U + 1])
        torch.testing.assert_close(got[8], ref[8])
        torch.testing.assert_close(got[8].long(), (keys.reshape(-1) * mult) % R)


@pytest.mark.parametrize("num_rows,n,P,route", [(16_609_143, 200_000, 1, True), (1000, 5000, 3, False),
                                                (100_000_000, 425_984, 8, True), (77, 1, 2, False)])
def test_bitmap_plan_matches_sorted_unique(dev, num_rows, n, P, route):
    """The bitmap planner (csrc/kernels/bitmap.hip) gives exactly the CPU reference plan: sorted
    unique (routed) keys, inverse, per-owner counts and U, with duplicates and ragged owners."""
    from minips_amd.ps.tables import _route_multiplier, even_bounds

    g = torch.Generator().manual_seed(n)
    keys = torch.randint(0, num_rows, (n,), generator=g)
    keys[: n // 3] = keys[n // 3: 2 * (n // 3)]  # plenty of duplicates
    bounds = torch.tensor(even_bounds(num_rows, P), dtype=torch.int64)
    mult = _route_multiplier(num_rows) if route else 0
    cu, ci, cc, cU = ops.bitmap_plan(keys, bounds, num_rows, mult)
    gu, gi, gc, gU = ops.bitmap_plan(keys.to(dev), bounds.to(dev), num_rows, mult)
    U = int(cU.reshape(-1)[0])
    assert int(gU.reshape(-1)[0]) == U
    assert torch.equal(gu[:U].cpu(), cu[:U])
    assert torch.equal(gi.cpu(), ci)
    assert torch.equal(gc.cpu(), cc)
    assert torch.equal(cu[:U][ci], (keys * mult) % num_rows if route else keys)


@pytest.mark.parametrize("base,rows,M", [(4_200_000, 4_200_000, 300_000), (7, 1000, 5000)])
def test_owner_side_bitmap_dedupe_nonzero_base(dev, base, rows, M):
    """the owner-side dedupe of the keys all requesters asked for (SparseTable._finish_plan
    at N > 1) plans them relative to the owner's base with the bitmap planner; with synthetic
    recv_keys in [base, base + rows) it must give what the hash dedupe gives on the absolute keys
    (same unique set, an inverse that maps every key back, one owner holding all of them)."""
    g = torch.Generator().manual_seed(M)
    recv = torch.randint(base, base + rows, (M,), generator=g)
    recv[: M // 4] = recv[M // 4: M // 2]
    recv = recv.to(dev)
    local = torch.tensor([0, rows], dtype=torch.int64, device=dev)
    ou, oi, oc, oU = ops.bitmap_plan(recv - base, local, rows)
    ou = ou + base
    hu, hi, hc, hU = ops.unique_bucketize_n(recv, torch.tensor([0, (1 << 63) - 1], dtype=torch.int64, device=dev))
    U = int(oU.reshape(-1)[0])
    assert U == int(hU.reshape(-1)[0]) == int(oc[0])
    assert torch.equal(torch.sort(ou[:U]).values, torch.sort(hu[:U]).values)
    assert torch.equal(ou[oi], recv) and torch.equal(hu[hi], recv)


def test_bitmap_plan_counts_out_of_range_keys(dev):
    """a key outside the planner's key space is never written and never silently
    aliased: the device counter records it, and a table surfaces it at drain()."""
    from minips_amd.ps.comm import Comm
    from minips_amd.ps.tables import SparseTable

    oor = torch.zeros(1, dtype=torch.int64, device=dev)
    keys = torch.tensor([3, 5, 1000, -2, 5], dtype=torch.int64, device=dev)
    ops.bitmap_plan(keys, torch.tensor([0, 100], dtype=torch.int64, device=dev), 100, oor=oor)
    assert int(oor) == 2
    t = SparseTable(Comm(device=torch.device(dev)), 100, 4, optimizer="add", route="range", init_std=0.0)
    t.get(torch.tensor([1, 2, 500], device=dev))  # bitmap planner (small key space)
    with pytest.raises(ValueError, match="outside"):
        t.drain()


def test_dgrad_permuted_rows_and_sorted_emb_backward(dev):
    """The embedding dgrad written in the planner's member order (EPI_PERM_ROWS_BF16) holds exactly
    the rows of the plain dgrad, and the embedding backward over those sorted rows equals the
    gather path (and the fp32 CPU reference within bf16 rounding)."""
    B, F, D, H = 1024, 26, 32, 256
    g = torch.Generator().manual_seed(5)
    inv = torch.randint(0, 900, (B * F,), generator=g)
    inv[::7] = 3  # a hot row
    U = int(inv.max()) + 1
    dH = (torch.randn(B, H, generator=g) * 0.1).to(torch.bfloat16).to(dev)
    Wt = (torch.randn(H, F * D + 8, generator=g) * 0.1).to(torch.bfloat16).to(dev)
    dwide = torch.randn(B, generator=g).to(dev)
    inv_d = inv.to(dev)
    members, memrow = ops.emb_build_csr(inv_d, F, U)
    pos = ops.emb_csr_positions(members)
    assert torch.equal(pos.cpu()[members.cpu().long()], torch.arange(B * F, dtype=torch.int32))
    dX = ops.linear_dgrad(dH, Wt, n_cols=F * D)
    dXs = ops.linear_dgrad(dH, Wt, n_cols=F * D, perm=pos, seg=D)
    assert dXs.shape == (B * F, D)
    assert torch.equal(dXs[pos.long()], dX.reshape(B * F, D))
    W = D + 4
    ga = torch.zeros(U, W, device=dev)
    gb = torch.zeros(U, W, device=dev)
    ops.wd_emb_backward(dX, dwide, inv_d, F, D, ga, csr=(members, memrow))
    ops.wd_emb_backward(dXs, dwide, inv_d, F, D, gb, csr=(members, memrow, pos), sorted_rows=True)
    torch.testing.assert_close(gb, ga, rtol=1e-5, atol=1e-5)
    ref = torch.zeros(U, W)
    ops.wd_emb_backward(dX.cpu(), dwide.cpu(), inv, F, D, ref)
    torch.testing.assert_close(gb.cpu()[:, : D + 1], ref[:, : D + 1], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("D,split", [(64, None), (32, 24), (16, None)])
def test_bf16_rows_apply_matches_fp32_within_rounding(dev, D, split):
    """bf16 table rows (bf16rows.hip): the gather equals the rows, and one row-wise Adagrad apply
    with stochastic rounding lands within one bf16 ulp of the fp32 reference apply."""
    R, n = 5000, 1200
    g = torch.Generator().manual_seed(D)
    rows = (torch.randn(R, D, generator=g) * 0.05).to(torch.bfloat16)
    keys = torch.randperm(R, generator=g)[:n] + 100
    grads = torch.randn(n, D, generator=g)
    t = rows.to(dev)
    st = torch.zeros(R, device=dev)
    st2 = torch.zeros(R, device=dev) if split else None
    out = torch.empty(n, D, dtype=torch.float32, device=dev)
    ops.gather_rows(t, keys.to(dev), 100, out)
    assert torch.equal(out.cpu(), rows[keys - 100].float())
    ops.sparse_apply_bf16("rowwise_adagrad", t, st, keys.to(dev), 100, grads.to(dev), 0.05, 1e-8, state2=st2,
                          split=split, step=1, seed=3)
    ref = rows.float().clone()
    rs = torch.zeros(R)
    rs2 = torch.zeros(R) if split else None
    ops.sparse_rowwise_adagrad(ref, rs, keys, 100, grads, 0.05, 1e-8, state2=rs2, split=split)
    torch.testing.assert_close(st.cpu(), rs)
    ulp = ref.abs().clamp_min(1e-30) * 2.0 ** -7  # one bf16 ulp of the fp32 result (upper bound)
    assert bool(((t.cpu().float() - ref).abs() <= ulp + 1e-12).all())


def test_bf16_rows_stochastic_rounding_is_unbiased(dev):
    """Updates far below half a bf16 ulp: round-to-nearest would never move the weights, the
    stochastic rounding of the bf16 apply moves them by the right amount on average."""
    R, D, steps = 4096, 16, 200
    t = torch.ones(R, D, dtype=torch.bfloat16, device=dev)
    keys = torch.arange(R, device=dev)
    g = torch.full((R, D), 1e-4, device=dev)  # bf16 ulp at 1.0 is 2^-7 = 7.8e-3
    for s in range(steps):
        ops.sparse_apply_bf16("add", t, None, keys, 0, g, 0.0, scale=1.0, step=s, seed=11)
    mean = float(t.float().mean())
    assert abs(mean - (1.0 + steps * 1e-4)) < 2e-3, mean  # RNE would stay at exactly 1.0


def test_launch_list_replays_on_new_data(dev):
    """A native LaunchList (ops.recording) replays its GEMMs, split-K slab GEMM, column sum and
    cross-stream fork on the current contents of the recorded buffers: after the inputs change, a
    replay gives what the op-by-op issue gives (fp32 CPU reference of the same ops)."""
    from minips_amd.models.layers import SideStream
    from minips_amd.utils import streams

    g = torch.Generator().manual_seed(9)
    M, N, K = 512, 256, 192
    X = _bf(torch.randn(M, K, generator=g)).to(dev)
    W = _bf(torch.randn(N, K, generator=g) * 0.1).to(dev)
    H = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    cs = torch.zeros(N, device=dev)
    dW = torch.zeros(N, K, device=dev)
    slab = torch.empty(4 * N * K, device=dev)
    side = SideStream(dev)
    nsplit = []

    def fn():
        ops.linear_fwd(X, W, None, "relu", out=H)
        with side.fork():
            ops.colsum_add(H, cs)
            ops.gemm(H, X, dW, N, K, M, True, True, ops.EPI_ATOMIC_F32, split_k=2)
            nsplit.append((ops._REC.lst if ops._REC is not None else _native.kernels()).gemm_slab(
                H, X, slab, N, K, M, True, True, 4))
        side.join()

    lst = _native.kernels().LaunchList(streams.current_raw(0), side._raw)
    with ops.recording(lst):
        fn()
    assert lst.size() >= 6 and nsplit[0] >= 1
    for _ in range(2):  # new inputs, then a replay
        X.copy_(_bf(torch.randn(M, K, generator=g)))
        cs.zero_()
        dW.zero_()
        lst.run(streams.current_raw(0), side._raw)
        torch.cuda.synchronize()
        Xc, Wc = X.float().cpu(), W.float().cpu()
        Hr = torch.relu(Xc @ Wc.t())
        torch.testing.assert_close(H.float().cpu(), Hr, rtol=2e-2, atol=2e-2)
        Hb = H.float().cpu()
        torch.testing.assert_close(cs.cpu(), Hb.sum(0), rtol=1e-3, atol=1e-2)
        ref = Hb.t() @ Xc
        torch.testing.assert_close(dW.cpu(), ref, rtol=1e-3, atol=5e-2)
        planes = slab[: nsplit[0] * N * K].view(nsplit[0], N, K).sum(0).cpu()
        torch.testing.assert_close(planes, ref, rtol=1e-3, atol=5e-2)
