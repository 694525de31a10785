"""Numerics of the dense-model gfx950 kernels (LayerNorm, softmax-xent, causal softmax,
GELU, residual add, DLRM interaction, lookup, batched/strided GEMM, GELU epilogues) against
the plain-PyTorch fp32 reference of the same op, plus GPU-vs-CPU model steps (MLP, DLRM)."""
import pytest
import torch

from minips_amd import _native, ops

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _require_kernels(dev):
    _native.kernels()


def _bf(x):
    return x.to(torch.bfloat16)


def _close(a, b, tol):
    torch.testing.assert_close(a.float().cpu(), b.float().cpu(), rtol=tol, atol=tol)


def test_layernorm(dev):
    g = torch.Generator().manual_seed(1)
    M, C, ld = 300, 768, 776
    x = _bf(torch.randn(M, ld, generator=g) * 2 + 0.5)
    gamma, beta = _bf(torch.randn(C, generator=g)), _bf(torch.randn(C, generator=g))
    outs = {}
    for d in ("cpu", dev):
        y = torch.zeros(M, ld, dtype=torch.bfloat16, device=d)
        mean, rstd = torch.empty(M, device=d), torch.empty(M, device=d)
        ops.layernorm_fwd(x.to(d), C, gamma.to(d), beta.to(d), 1e-5, y, mean, rstd)
        dy = _bf(torch.randn(M, ld, generator=torch.Generator().manual_seed(2))).to(d)
        dx = torch.zeros(M, ld, dtype=torch.bfloat16, device=d)
        dg, db = torch.zeros(C, device=d), torch.zeros(C, device=d)
        ops.layernorm_bwd(x.to(d), dy, C, gamma.to(d), mean, rstd, dx, dg, db)
        outs[str(d)] = (y, mean, rstd, dx, dg, db)
    c, gp = outs["cpu"], outs[str(dev)]
    _close(gp[0][:, :C], c[0][:, :C], 3e-2)
    _close(gp[1], c[1], 1e-4)
    _close(gp[2], c[2], 1e-3)
    _close(gp[3][:, :C], c[3][:, :C], 5e-2)
    _close(gp[4], c[4], 0.3)
    _close(gp[5], c[5], 0.3)


@pytest.mark.parametrize("V,ld,M", [(10, 16, 64), (10, 16, 70000), (33, 48, 300), (64, 64, 500), (65, 72, 100),
                                    (1000, 1000, 64), (50257, 50264, 64),
                                    (50257, 50304, 700)])
def test_softmax_xent(dev, V, ld, M):
    """V <= 64 runs the one-thread-per-row kernel (M = 70000: grid-stride rows), larger V the
    block-per-row kernel; both against the fp32 reference."""
    g = torch.Generator().manual_seed(V)
    z = _bf(torch.randn(M, ld, generator=g) * 3)
    y = torch.randint(0, V, (M,), generator=g)
    res = {}
    for d in ("cpu", dev):
        lg = z.clone().to(d)
        loss, corr = torch.zeros(1, device=d), torch.zeros(1, device=d)
        ops.softmax_xent(lg, V, y.to(d), 0.5, loss, corr)
        res[str(d)] = (lg[:, :V], loss, corr)
    c, gp = res["cpu"], res[str(dev)]
    _close(gp[0], c[0], 1e-2)
    _close(gp[1], c[1], 1e-3 * M)
    # a hit is "label logit == row max" on the GPU, argmax (first index) on the CPU: bf16 ties differ
    assert abs(float(gp[2]) - float(c[2])) <= 1 + M // 1000


@pytest.mark.parametrize("T", [64, 128, 1024])
def test_causal_softmax(dev, T):
    g = torch.Generator().manual_seed(T)
    BH = 3
    S = torch.randn(BH, T, T, generator=g) * 4
    dP = torch.randn(BH, T, T, generator=g)
    res = {}
    for d in ("cpu", dev):
        P = torch.empty(BH, T, T, dtype=torch.bfloat16, device=d)
        ops.causal_softmax_fwd(S.to(d), T, P)
        dS = torch.empty(BH, T, T, dtype=torch.bfloat16, device=d)
        ops.causal_softmax_bwd(P, dP.to(d), T, 0.125, dS)
        res[str(d)] = (P, dS)
    _close(res[str(dev)][0], res["cpu"][0], 1e-2)
    _close(res[str(dev)][1], res["cpu"][1], 2e-2)


def test_gelu_add(dev):
    g = torch.Generator().manual_seed(5)
    u, dh, b = (_bf(torch.randn(4097, generator=g) * 2) for _ in range(3))
    res = {}
    for d in ("cpu", dev):
        du = torch.empty(4097, dtype=torch.bfloat16, device=d)
        ops.gelu_bwd(dh.to(d), u.to(d), du)
        s = torch.empty_like(du)
        ops.add_bf16(u.to(d), b.to(d), s)
        res[str(d)] = (du, s)
    _close(res[str(dev)][0], res["cpu"][0], 2e-2)
    _close(res[str(dev)][1], res["cpu"][1], 1e-2)


@pytest.mark.parametrize("D,B", [(64, 96), (64, 97), (32, 50), (16, 1003)])
def test_dlrm_interaction_and_lookup(dev, D, B):
    """The MFMA interaction kernels (one wave per sample, 16x16x32 bf16 tiles; B not a multiple of
    the 4 waves of a block) against the fp32 reference, for the DLRM (D = 64) and DLRM-10B (D = 16)
    widths."""
    g = torch.Generator().manual_seed(8 + D)
    NV, F = 27, 26
    U = 500
    ld = (D + NV * (NV - 1) // 2 + 7) // 8 * 8
    rows = _bf(torch.randn(U, D, generator=g))
    inv = torch.randint(0, U, (B * F,), generator=g)
    bottom = _bf(torch.relu(torch.randn(B, D, generator=g)) - 0.2)
    dout = _bf(torch.randn(B, ld, generator=g))
    res = {}
    for d in ("cpu", dev):
        V = torch.zeros(B, NV * D, dtype=torch.bfloat16, device=d)
        ops.lookup_rows(rows.to(d), inv.to(d), F, D, V)
        V[:, F * D:] = bottom.to(d)
        out = torch.zeros(B, ld, dtype=torch.bfloat16, device=d)
        ops.dlrm_interact_fwd(V, NV, D, out, dense_idx=F)
        dV = torch.empty(B, NV * D, device=d)
        dd = torch.empty(B, D, dtype=torch.bfloat16, device=d)
        ops.dlrm_interact_bwd(V, NV, D, dout.to(d), dV, dd, dense_idx=F)
        res[str(d)] = (V, out, dV, dd)
    for a, b, tol in zip(res[str(dev)], res["cpu"], (0, 3e-2, 2e-2, 3e-2)):
        _close(a, b, max(tol, 1e-6))


def test_gemm_strided_batched_and_gelu(dev):
    g = torch.Generator().manual_seed(11)
    # batched: 2 outer x 3 inner "heads" of [T, hd] blocks interleaved inside [*, 3*hd] rows
    Bo, H, T, hd = 2, 3, 128, 64
    Q = _bf(torch.randn(Bo * T, H * hd, generator=g))
    Kt = _bf(torch.randn(Bo * T, H * hd, generator=g))
    strides = [T * H * hd, hd, T * H * hd, hd, H * T * T, T * T]
    res = {}
    for d in ("cpu", dev):
        S = torch.zeros(Bo * H, T, T, device=d)
        ops.gemm_batched(Q.to(d), Kt.to(d), S, T, T, hd, False, False, ops.EPI_STORE_F32, Bo * H, H, H * hd, H * hd,
                         T, strides, alpha=0.125)
        res[str(d)] = S
    _close(res[str(dev)], res["cpu"], 2e-2)
    # GELU aux epilogue and its gradient epilogue
    M, N, K = 256, 384, 136
    X, W = _bf(torch.randn(M, K, generator=g)), _bf(torch.randn(N, K, generator=g) * 0.1)
    dY = _bf(torch.randn(M, N, generator=g))
    out = {}
    for d in ("cpu", dev):
        C = torch.empty(M, N, dtype=torch.bfloat16, device=d)
        U = torch.empty(M, N, dtype=torch.bfloat16, device=d)
        ops.gemm(X.to(d), W.to(d), C, M, N, K, False, False, ops.EPI_BIAS_GELU_AUX_BF16, mask=U)
        dX = torch.empty(M, N, dtype=torch.bfloat16, device=d)
        ops.gemm(dY.to(d), torch.eye(N, dtype=torch.bfloat16, device=d), dX, M, N, N, False, True,
                 ops.EPI_GELU_GRAD_BF16, mask=U)
        # the derivative-saving form: aux = gelu'(u), then dX = dY * aux
        C2 = torch.empty(M, N, dtype=torch.bfloat16, device=d)
        Dg = torch.empty(M, N, dtype=torch.bfloat16, device=d)
        ops.gemm(X.to(d), W.to(d), C2, M, N, K, False, False, ops.EPI_BIAS_GELU_DAUX_BF16, mask=Dg)
        dX2 = torch.empty(M, N, dtype=torch.bfloat16, device=d)
        ops.gemm(dY.to(d), torch.eye(N, dtype=torch.bfloat16, device=d), dX2, M, N, N, False, True,
                 ops.EPI_MUL_AUX_BF16, mask=Dg)
        out[str(d)] = (C, U, dX, C2, Dg, dX2)
    for a, b in zip(out[str(dev)], out["cpu"]):
        _close(a, b, 3e-2)
    # both backward forms agree (gelu' of a bf16 u vs a bf16 gelu'(u): bf16 rounding apart)
    _close(out[str(dev)][5], out[str(dev)][2], 3e-2)


# ------------------------------------------------------------------------------ models
def test_mlp_gpu_matches_cpu(dev):
    from minips_amd.data.synthetic import MnistSynth
    from minips_amd.models.mlp import MLP, MLPConfig
    from minips_amd.ps.comm import Comm

    data = MnistSynth(256, device="cpu", seed=3)
    batches = [data.next() for _ in range(4)]
    losses = {}
    for d in ("cpu", dev):
        m = MLP(MLPConfig(), Comm(device=torch.device(d)))
        ls = []
        for x, y in batches:
            loss, _ = m.train_step(x.to(d), y.to(d))
            ls.append(float(loss) / 256)
        m.drain()
        losses[str(d)] = ls
    for a, b in zip(losses[str(dev)], losses["cpu"]):
        assert abs(a - b) < 2e-2 * max(1.0, abs(b)), losses


def test_dlrm_gpu_matches_cpu(dev):
    from minips_amd.models.dlrm import DLRM, DLRMConfig
    from minips_amd.ps.comm import Comm

    g = torch.Generator().manual_seed(4)
    batches = []
    for _ in range(4):
        dense = torch.randn(256, 13, generator=g)
        keys = torch.randint(0, 20000, (256, 26), generator=g)
        y = (dense[:, 0] > 0).float()
        batches.append((dense, keys, y))
    emb = torch.randn(20000, 64, generator=g) * 0.05
    losses = {}
    for d in ("cpu", dev):
        m = DLRM(DLRMConfig(num_rows=20000, consistency="bsp"), Comm(device=torch.device(d)))
        m.emb.shard.copy_(emb.to(d))
        ls = []
        for dense, keys, y in batches:
            ls.append(float(m.train_step(dense.to(d), keys.to(d), y.to(d))) / 256)
        m.drain()
        losses[str(d)] = ls
    for a, b in zip(losses[str(dev)], losses["cpu"]):
        assert abs(a - b) < 2e-2, losses


def test_lr_kmeans_gpu_matches_cpu(dev):
    from minips_amd.data.synthetic import SparseLRSynth
    from minips_amd.models.kmeans import KMeans, KMeansConfig
    from minips_amd.models.lr import SparseLR, SparseLRConfig
    from minips_amd.ps.comm import Comm

    data = SparseLRSynth(256, num_dims=4000, nnz=16, seed=7)
    batches = [data.next() for _ in range(6)]
    g = torch.Generator().manual_seed(0)
    true = torch.randn(6, 12, generator=g) * 5
    init = true + torch.randn(6, 12, generator=g)
    Xs = [true[torch.randint(0, 6, (512,), generator=g)] + torch.randn(512, 12, generator=g) * 0.5 for _ in range(4)]
    res = {}
    for d in ("cpu", dev):
        comm = Comm(device=torch.device(d))
        m = SparseLR(SparseLRConfig(num_dims=4000, alpha=0.05), comm)
        acc = [float(m.train_step(*(t.to(d) for t in b))) for b in batches]
        m.drain()
        km = KMeans(KMeansConfig(K=6, dims=12), comm, init_centres=init)
        sse = [float(km.train_step(X.to(d))) for X in Xs]
        km.drain()
        res[str(d)] = (acc, m.table.shard.cpu(), sse, km.centres().cpu())
    c, gp = res["cpu"], res[str(dev)]
    assert max(abs(a - b) for a, b in zip(gp[0], c[0])) <= 2
    torch.testing.assert_close(gp[1], c[1], rtol=1e-4, atol=1e-5)
    for a, b in zip(gp[2], c[2]):
        assert abs(a - b) < 1e-3 * b
    torch.testing.assert_close(gp[3], c[3], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("B,T,H", [(2, 64, 2), (1, 256, 3), (2, 200, 2), (1, 1024, 1)])
def test_flash_attention(dev, B, T, H):
    g = torch.Generator().manual_seed(T + H)
    d = H * 64
    qkv = _bf(torch.randn(B * T, 3 * d, generator=g))
    dO = _bf(torch.randn(B * T, d, generator=g))
    scale = 0.125
    res = {}
    for dv in ("cpu", dev):
        O = torch.zeros(B * T, d + 8, dtype=torch.bfloat16, device=dv)
        lse = torch.empty(B * H * T, device=dv)
        ops.attn_fwd(qkv.to(dv), B, T, H, scale, O, lse)
        dq = torch.zeros(B * T, 3 * d, dtype=torch.bfloat16, device=dv)
        delta = torch.empty(B * H * T, device=dv)
        # backward from the CPU forward output so both sides see the same O
        Oc = res["cpu"][0].to(dv) if "cpu" in res else O
        ops.attn_bwd(qkv.to(dv), Oc, dO.to(dv), lse, delta, B, T, H, scale, dq)
        res[str(dv)] = (O, lse, dq)
    c, gp = res["cpu"], res[str(dev)]
    _close(gp[0][:, :d], c[0][:, :d], 2e-2)
    _close(gp[1], c[1], 2e-3)
    err = (gp[2].float().cpu() - c[2].float()).abs().max() / c[2].float().abs().max()
    assert err < 2e-2, float(err)


@pytest.mark.parametrize("mode", ["kmeans++", "kmeans_parallel"])
def test_kmeans_init_gpu(dev, mode):
    """GPU seeding: every D^2 pass runs the kmeans_assign kernels (MFMA form for the k-means||
    candidate assignment); every well-separated blob receives a centre."""
    from minips_amd.models.kmeans import init_centres, sampled_sse

    g = torch.Generator().manual_seed(0)
    K, D = 64, 32
    true = torch.randn(K, D, generator=g) * 8
    X = true[torch.randint(0, K, (20000,), generator=g)] + torch.randn(20000, D, generator=g) * 0.2
    C = init_centres(X.to(dev), K, mode, seed=5)
    torch.cuda.synchronize()
    C = C.cpu()
    assert C.shape == (K, D) and torch.isfinite(C).all()
    hit = torch.cdist(true, C).argmin(0).unique().numel()
    assert hit >= K - 2, hit  # D^2 seeding leaves at most a couple of blobs doubled up
    assert sampled_sse(X.to(dev), C.to(dev), n=500) < 50.0


def test_uniform_synth_dlrm_batches(dev):
    """The fused DLRM batch generator: keys uniform in [0, rows) (10B rows: above 2^32), dense
    N(0,1), label = dense[:, 0] > 0, a new batch every call, reproducible from the seed."""
    from minips_amd.data.synthetic import DLRMSynth

    for rows in (1000, 10_000_000_000):
        a = DLRMSynth(16384, 26, rows, 13, device=dev, seed=3)
        d1, k1, l1 = a.next()
        d2, k2, _ = a.next()
        assert k1.shape == (16384, 26) and d1.shape == (16384, 13) and l1.shape == (16384,)
        assert int(k1.min()) >= 0 and int(k1.max()) < rows
        assert abs(float(k1.double().mean()) / rows - 0.5) < 0.01
        assert not torch.equal(k1, k2) and not torch.equal(d1, d2)
        assert abs(float(d1.mean())) < 0.02 and abs(float(d1.std()) - 1.0) < 0.02
        assert torch.equal(l1, (d1[:, 0] > 0).float())
        b = DLRMSynth(16384, 26, rows, 13, device=dev, seed=3)
        assert torch.equal(b.next()[1], k1)
    assert int(k1.max()) > (1 << 32)  # the 10B-row table is addressed beyond 32 bits
