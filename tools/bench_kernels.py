#!/usr/bin/env python3
"""Isolated kernel microbenchmarks on the model shapes (one MI355X), one entry point:

    python tools/bench_kernels.py gemm [--set wd|gpt2] [--shapes name:M:N:K:layout,...]
                                        ours vs torch.matmul (hipBLASLt), TFLOP/s per shape
    python tools/bench_kernels.py kscan --M 16384 --N 1024 --layout nt
                                        time vs K at fixed M, N: fixed cost vs per-K-step cost
    python tools/bench_kernels.py pmc   model-shape GEMMs back to back (for rocprofv3 --pmc passes)
    python tools/bench_kernels.py one --shape name:M:N:K:layout [--lib]   one shape, repeated (--pmc target)
    python tools/bench_kernels.py attn  fused causal attention vs torch SDPA
    python tools/bench_kernels.py nn    GPT-2 memory-bound kernels (LayerNorm, add, softmax-xent): TB/s
    python tools/bench_kernels.py emb   W&D embedding backward on a real Criteo-shaped plan
    python tools/bench_kernels.py plan  key planning: per-column sort vs hash dedupe + CSR
    torchrun --nproc-per-node N tools/bench_kernels.py rccl [--min-mb 0.25 --max-mb 256]
                                        RCCL bytes vs time per collective of the PS data plane
                                        (reduce-scatter, all-gather, all-to-all, all-to-all-v),
                                        bus GB/s against the 7 x 153 GB/s xGMI links of one GPU;
                                        NCCL_ALGO / NCCL_PROTO / NCCL_* from the environment

GEMM layouts: nt = forward (A [M,K], B [N,K]), nn = dgrad (B [K,N]), tn = wgrad (A [K,M],
B [K,N], fp32 out; through ops.linear_wgrad, i.e. the model's split-K choice, unless
GEMM_TN_MODEL=0). In the training steps these kernels share the GPU with side streams, so rocprof's
in-step durations overstate their own cost; this separates the two.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from minips_amd import ops  # noqa: E402

WD_SHAPES = [  # (name, M, N, K, layout)
    ("wd.fwd1", 16384, 1024, 896, "nt"), ("wd.fwd2", 16384, 512, 1032, "nt"), ("wd.fwd3", 16384, 256, 520, "nt"),
    ("wd.dgrad2", 16384, 512, 256, "nn"), ("wd.dgrad1", 16384, 1024, 512, "nn"), ("wd.dgrad0", 16384, 832, 1024, "nn"),
    ("wd.wgrad3", 256, 520, 16384, "tn"), ("wd.wgrad2", 512, 1032, 16384, "tn"), ("wd.wgrad1", 1024, 896, 16384, "tn"),
    ("sq4096", 4096, 4096, 4096, "nt"),
]
# every GEMM of one GPT-2 small step (B*T = 8192, d = 768, vocab 50304): forward, dgrad, wgrad
GPT2_SHAPES = [
    ("g.qkv.f", 8192, 2304, 768, "nt"), ("g.proj.f", 8192, 768, 768, "nt"), ("g.fc.f", 8192, 3072, 768, "nt"),
    ("g.fc2.f", 8192, 768, 3072, "nt"), ("g.lm.f", 8192, 50304, 768, "nt"),
    ("g.qkv.d", 8192, 768, 2304, "nn"), ("g.proj.d", 8192, 768, 768, "nn"), ("g.fc.d", 8192, 768, 3072, "nn"),
    ("g.fc2.d", 8192, 3072, 768, "nn"), ("g.lm.d", 8192, 768, 50304, "nn"),
    ("g.qkv.w", 2304, 768, 8192, "tn"), ("g.proj.w", 768, 768, 8192, "tn"), ("g.fc.w", 3072, 768, 8192, "tn"),
    ("g.fc2.w", 768, 3072, 8192, "tn"), ("g.lm.w", 50304, 768, 8192, "tn"),
]
LAYOUTS = {"nt": (False, False), "nn": (False, True), "tn": (True, True)}


def dev():
    return torch.device("cuda")


def timed(fn, iters=20, warm=3):
    """Mean time per call in us (HIP events around `iters` back-to-back calls)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def median_rounds(fns, rounds=20, per=5):
    """Interleaved rounds of several callables; median us per call of each."""
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    times = {k: [] for k in fns}
    for _ in range(rounds):
        for k, f in fns.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(per):
                f()
            e.record()
            e.synchronize()
            times[k].append(s.elapsed_time(e) / per * 1e3)
    return {k: sorted(v)[len(v) // 2] for k, v in times.items()}


def gemm_operands(M, N, K, lay):
    a_km, b_kn = LAYOUTS[lay]
    A = torch.randn((K, M) if a_km else (M, K), device=dev()).to(torch.bfloat16)
    B = torch.randn((K, N) if b_kn else (N, K), device=dev()).to(torch.bfloat16)
    C = torch.zeros(M, N, device=dev(), dtype=torch.float32 if lay == "tn" else torch.bfloat16)
    return A, B, C


def ours_gemm(A, B, C, M, N, K, lay, split=1):
    a_km, b_kn = LAYOUTS[lay]
    if lay == "tn" and os.environ.get("GEMM_TN_MODEL", "1") == "1":
        return lambda: ops.linear_wgrad(A, B, C)  # the model's wgrad path (split-K choice, slabs + reduce)
    epi = ops.EPI_ATOMIC_F32 if lay == "tn" else ops.EPI_STORE_BF16
    return lambda: ops.gemm(A, B, C, M, N, K, a_km, b_kn, epi, split_k=split)


def cmd_gemm(a):
    if a.shapes:
        shapes = [(n, int(m), int(nn), int(k), lay) for n, m, nn, k, lay in (s.split(":") for s in a.shapes.split(","))]
    else:
        shapes = GPT2_SHAPES if a.set == "gpt2" else WD_SHAPES
    tot = {k: 0.0 for k in ["ours"] + (["hipblaslt"] if a.lib else [])}
    for name, M, N, K, lay in shapes:
        a_km, b_kn = LAYOUTS[lay]
        A, B, C = gemm_operands(M, N, K, lay)
        At, Bt = (A.t() if a_km else A), (B if b_kn else B.t())
        fns = {"ours": ours_gemm(A, B, C, M, N, K, lay, a.split)}
        if a.lib:
            fns["hipblaslt"] = lambda: torch.matmul(At, Bt)
        med = median_rounds(fns)
        for k in tot:
            tot[k] += med[k]
        fl = 2.0 * M * N * K
        cols = " | ".join(f"{k} {med[k]:8.1f}us {fl / med[k] / 1e6:7.1f} TF/s" for k in tot)
        print(f"{name:10s} M={M:6d} N={N:5d} K={K:6d} {lay}  {cols}", flush=True)
    print("sum: " + " | ".join(f"{k} {v:.1f} us" for k, v in tot.items()))


def cmd_one(a):
    """One shape, `reps` back-to-back launches of ours (or the library with --lib): a rocprofv3 --pmc target."""
    name, M, N, K, lay = a.shape.split(":")
    M, N, K = int(M), int(N), int(K)
    A, B, C = gemm_operands(M, N, K, lay)
    a_km, b_kn = LAYOUTS[lay]
    if a.lib:
        At, Bt = (A.t() if a_km else A), (B if b_kn else B.t())
        Cf = torch.zeros(M, N, device=dev())
        f = (lambda: torch.addmm(Cf, At, Bt, out_dtype=torch.float32, out=Cf)) if lay == "tn" else \
            (lambda: torch.matmul(At, Bt))
    else:
        f = ours_gemm(A, B, C, M, N, K, lay, a.split)
    for _ in range(a.reps):
        f()
    torch.cuda.synchronize()
    print("done", name)


def cmd_kscan(a):
    M, N = a.M, a.N
    for K in [int(k) for k in a.Ks.split(",")]:
        A, B, C = gemm_operands(M, N, K, a.layout)
        t = median_rounds({"k": ours_gemm(A, B, C, M, N, K, a.layout, a.split)}, rounds=15)["k"]
        print(f"{a.tag:10s} M={M} N={N} K={K:5d} {a.layout} split={a.split} {t:8.1f} us "
              f"{2.0 * M * N * K / t / 1e6:7.1f} TF/s", flush=True)


def cmd_wgrad(a):
    """The W&D weight-gradient GEMMs in their step form (split-K into fp32 slab planes, ops.linear_wgrad
    defer path -> gemm_slab) over split counts; MINIPS_GEMM_TILE forces the tile (128 / 200 / 256).
    Also the plane bytes the Adam then folds (nsplit x N x K x 4)."""
    from minips_amd._native import kernels

    B = a.batch
    for name, N, K in (("W3", 256, 512), ("W2", 512, 1024), ("W1", 1024, 896)):
        dy = torch.randn(B, N, device=dev()).to(torch.bfloat16)
        x = torch.randn(B, K, device=dev()).to(torch.bfloat16)
        for split in [int(v) for v in a.splits.split(",")]:
            slab = torch.empty(split * N * K, device=dev())
            ns = [0]

            def f():
                ns[0] = kernels().gemm_slab(dy, x, slab, N, K, B, True, True, split)

            t = median_rounds({"k": f}, rounds=15)["k"]
            print(f"{name} N={N:5d} K={K:5d} M={B} split={split:3d} (ran {ns[0]:3d}) {t:7.1f} us "
                  f"{2.0 * B * N * K / t / 1e6:7.1f} TF/s  planes {ns[0] * N * K * 4 / 1e6:6.1f} MB", flush=True)


def cmd_pmc(a):
    def bf(*s):
        return torch.randn(*s, device=dev()).to(torch.bfloat16)

    X, W1, dH1 = bf(16384, 896), bf(1024, 896), bf(16384, 1024)
    H = torch.empty(16384, 1024, device=dev(), dtype=torch.bfloat16)
    dX = torch.empty(16384, 896, device=dev(), dtype=torch.bfloat16)
    dW = torch.zeros(1024, 896, device=dev())
    A4, B4 = bf(4096, 4096), bf(4096, 4096)
    C4 = torch.empty(4096, 4096, device=dev(), dtype=torch.bfloat16)
    for _ in range(a.reps):
        ops.linear_fwd(X, W1, None, "relu", out=H)                  # fwd1 (nt)
        ops.linear_dgrad(dH1, W1, out=dX)                           # dgrad0 (nn, tr-read B)
        ops.linear_wgrad(dH1, X, dW)                                # wgrad1 (tn, split-K)
        ops.gemm(A4, B4, C4, 4096, 4096, 4096, False, False, ops.EPI_STORE_BF16)  # sq4096
    torch.cuda.synchronize()
    print("done")


def cmd_attn(a):
    B, T, H = a.B, a.T, a.H
    d = H * 64
    qkv = torch.randn(B * T, 3 * d, device=dev()).to(torch.bfloat16)
    dO = torch.randn(B * T, d, device=dev()).to(torch.bfloat16)
    O = torch.empty(B * T, d + 8, device=dev(), dtype=torch.bfloat16)
    lse = torch.empty(B * H * T, device=dev())
    delta = torch.empty_like(lse)
    dqkv = torch.empty_like(qkv)
    fl = 4.0 * B * H * T * T / 2 * 64  # causal: 2 products over T^2/2 forward, 5 backward
    tf = timed(lambda: ops.attn_fwd(qkv, B, T, H, 0.125, O, lse))
    tb = timed(lambda: ops.attn_bwd(qkv, O, dO, lse, delta, B, T, H, 0.125, dqkv))
    print(f"ours  fwd {tf:8.1f} us {fl / tf / 1e6:7.1f} TF/s   bwd {tb:8.1f} us {2.5 * fl / tb / 1e6:7.1f} TF/s")
    q, k, v = (qkv[:, i * d:(i + 1) * d].reshape(B, T, H, 64).transpose(1, 2).contiguous() for i in range(3))
    q.requires_grad_(True), k.requires_grad_(True), v.requires_grad_(True)
    go = dO.reshape(B, T, H, 64).transpose(1, 2).contiguous()
    F = torch.nn.functional.scaled_dot_product_attention
    try:
        tf2 = timed(lambda: F(q, k, v, is_causal=True))
        out = F(q, k, v, is_causal=True)
        tb2 = timed(lambda: torch.autograd.grad(out, (q, k, v), go, retain_graph=True))
        print(f"sdpa  fwd {tf2:8.1f} us {fl / tf2 / 1e6:7.1f} TF/s   "
              f"bwd {tb2:8.1f} us {2.5 * fl / tb2 / 1e6:7.1f} TF/s")
    except Exception as e:  # pragma: no cover
        print("sdpa unavailable:", e)


def cmd_nn(a):
    M, C, V = 8192, 768, 50304
    bf = dict(dtype=torch.bfloat16, device=dev())
    x, dy, dx = torch.randn(M, C, **bf), torch.randn(M, C, **bf), torch.randn(M, C, **bf)
    g, bta = torch.randn(C, **bf), torch.randn(C, **bf)
    y = torch.empty(M, C, **bf)
    mean, rstd = torch.empty(M, device=dev()), torch.empty(M, device=dev())
    dg, db = torch.zeros(C, device=dev()), torch.zeros(C, device=dev())
    ops.layernorm_fwd(x, C, g, bta, 1e-5, y, mean, rstd)
    rows = [
        ("layernorm_fwd", timed(lambda: ops.layernorm_fwd(x, C, g, bta, 1e-5, y, mean, rstd), 50),
         2 * M * C * 2 + 8 * M),
        ("layernorm_bwd (accumulate dx)",
         timed(lambda: ops.layernorm_bwd(x, dy, C, g, mean, rstd, dx, dg, db, accumulate=True), 50),
         4 * M * C * 2 + 8 * M),
        ("add_bf16", timed(lambda: ops.add_bf16(x, dy, y), 50), 3 * M * C * 2),
    ]
    logits = torch.randn(M, V, **bf)
    labels = torch.randint(0, 50257, (M,), device=dev())
    loss = torch.zeros(1, device=dev())
    rows.append(("softmax_xent (in place)",
                 timed(lambda: ops.softmax_xent(logits, 50257, labels, 1.0 / M, loss), 10), 2 * M * V * 2))
    for name, us, nbytes in rows:
        print(f"{name:32s} {us:9.1f} us  {nbytes / us / 1e6:6.2f} TB/s")


def cmd_emb(a):
    from minips_amd.data.synthetic import CriteoSynth

    B = a.batch
    dense, keys, y = CriteoSynth(B, device=dev(), seed=1).next()
    bounds = torch.tensor([0, 1 << 62], dtype=torch.int64, device=dev())
    uniq, inv, counts = ops.unique_bucketize(keys.reshape(-1), bounds, 26)
    U = int(counts.sum())
    dX = torch.randn(B, 26 * 32, device=dev()).to(torch.bfloat16)
    dw = torch.randn(B, device=dev())
    g = torch.zeros(U, 36, device=dev())
    full = timed(lambda: ops.wd_emb_backward(dX, dw, inv, 26, 32, g))
    csr = ops.emb_build_csr(inv, 26, U)
    build = timed(lambda: ops.emb_build_csr(inv, 26, U))
    seg = timed(lambda: ops.wd_emb_backward(dX, dw, inv, 26, 32, g, csr=csr))
    print(f"U={U} lookups={B * 26}: build+sum {full:.1f} us, csr build {build:.1f} us, zero+segment sum {seg:.1f} us")


def cmd_embstep(a):
    """The one-rank W&D step's non-GEMM critical chain on its real shapes, each kernel alone:
    the embedding backward (deterministic segment sums, fp32 rows), the row-wise Adagrad of the
    unique rows on the full 33.76M x 36 shard, and the input assembly read in place from the shard.
    Planned by the real planner (plan_sorted, one owner). Median us and effective TB/s."""
    from minips_amd.data.synthetic import CRITEO_KAGGLE_CARDS, CriteoSynth

    B, cards = a.batch, CRITEO_KAGGLE_CARDS
    F, D, W = len(cards), 32, 36
    R = sum(cards)
    dense, keys, _ = CriteoSynth(B, device=dev(), seed=1).next()
    bases = torch.tensor([sum(cards[:f]) for f in range(F)], device=dev())
    bits = [max(1, (c - 1).bit_length()) for c in cards]
    mult = 402653189 if R % 402653189 else 201326611
    res = ops.plan_sorted(keys, bases, bits, mult, R)
    uniq, inv, U_dev, members, memrow, rowstart, rowidx = res[0], res[1], res[3], res[4], res[5], res[7], res[8]
    U = int(U_dev.item())
    table = torch.randn(R, W, device=dev()) * 0.01
    state, state2 = torch.zeros(R, device=dev()), torch.zeros(R, device=dev())
    dX = (torch.randn(B, F * D, device=dev()) * 0.01).to(torch.bfloat16)
    dw = torch.randn(B, device=dev()) * 0.01
    g = torch.zeros(B * F, W, device=dev())
    X = torch.empty(B, 896, device=dev(), dtype=torch.bfloat16)
    wide = torch.empty(B, device=dev())
    n = B * F
    t_emb = timed(lambda: ops.wd_emb_backward(dX, dw, inv, F, D, g, csr=(members, memrow)))
    # the step's form: the dX dgrad wrote the lookups' rows in member order (positions), one row per
    # lookup read contiguously
    dXs = dX.view(n, D)[members.long()].contiguous()
    t_embs = timed(lambda: ops.wd_emb_backward(dXs, dw, inv, F, D, g, csr=(members, memrow), sorted_rows=True))
    t_ada = timed(lambda: ops.sparse_rowwise_adagrad(table, state, uniq, 0, g, 0.01, 1e-8, state2=state2, split=D,
                                                     n_dev=U_dev))
    t_asm = timed(lambda: ops.wd_assemble_tab(dense, table, uniq, 0, inv, F, D, X, wide, ones_col=F * D + 13,
                                              rowidx=rowidx))
    mb_emb = (n * D * 2 + n * 8 + B * 4 + U * W * 4) / 1e6
    mb_ada = (U * W * 4 * 3 + U * 16) / 1e6
    mb_asm = (n * 4 + n * 128 + B * 896 * 2) / 1e6
    print(f"U={U} lookups={n}")
    for name, t, mb in (("emb backward", t_emb, mb_emb), ("emb backward (sorted)", t_embs, mb_emb),
                        ("rowwise adagrad", t_ada, mb_ada),
                        ("assemble (in place)", t_asm, mb_asm)):
        print(f"{name:22s} {t:8.1f} us  {mb:7.1f} MB  {mb / t:6.2f} TB/s")


def cmd_plan(a):
    from minips_amd.data.synthetic import CRITEO_KAGGLE_CARDS, CriteoSynth

    B, cards = a.batch, CRITEO_KAGGLE_CARDS
    F = len(cards)
    keys = CriteoSynth(B, device=dev(), seed=1).next()[1]
    bases = torch.tensor([sum(cards[:f]) for f in range(F)], device=dev())
    bits = [max(1, (c - 1).bit_length()) for c in cards]
    R = sum(cards)
    t_sort = timed(lambda: ops.plan_sorted(keys, bases, bits, 402653189, R))
    bounds = torch.tensor([0, R], device=dev())

    def hashed():
        (uniq, inv, counts, U), z = ops.unique_bucketize_n(keys.reshape(-1), bounds, F, 402653189, R,
                                                           extra_zero_ints=2 * B * F, csr_counts=True)
        ops.emb_build_csr(inv, F, B * F, zeroed=z, counts_ready=True)

    print(f"B={B} F={F}: sort plan {t_sort:.1f} us | hash dedupe + CSR {timed(hashed):.1f} us")
    for nb in (4, 8, 16, 24, 32):
        t = timed(lambda: ops.plan_sorted(keys, bases, [nb] * F, 402653189, R))
        print(f"  all columns at {nb:2d} bits ({(nb + 3) // 4} passes): {t:.1f} us")


XGMI_LINKS, XGMI_LINK_GBPS = 7, 153.0  # per MI355X: 7 links to the other 7 GPUs of the node


def cmd_rccl(a):
    """Bytes vs time of the PS data plane's collectives over RCCL (one process per GPU, torchrun).
    For each message size (per-rank payload): median time of ``iters`` calls, algorithm bandwidth
    (payload / time) and bus bandwidth -- the bytes each GPU moves over its links: (N-1)/N of the
    payload for reduce-scatter / all-gather / all-to-all -- as a fraction of the 7-link bound. The
    all-to-all-v uses a Zipf-like split (owner r gets ~1/(r+1) of the rows), the shape of an
    unrouted sparse push; the routed tables' splits are near-uniform (plain all-to-all)."""
    import json
    import statistics
    import time

    import torch.distributed as dist

    from minips_amd.ps.comm import init_distributed

    comm = init_distributed()
    N, rank, dev = comm.world, comm.rank, comm.device
    if N < 2:
        raise SystemExit("rccl: launch with torchrun --nproc-per-node N (N >= 2)")
    env = {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_")) and "DEBUG" not in k}
    sizes, mb = [], a.min_mb
    while mb <= a.max_mb:
        sizes.append(mb)
        mb *= 2
    bound = XGMI_LINKS * XGMI_LINK_GBPS
    bf = torch.bfloat16 if dev.type == "cuda" else torch.float32  # (gloo plumbing runs: no bf16)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def run(op, n_bytes):
        if op == "reduce_scatter":  # fp32 gradients, n_bytes per rank in, n_bytes / N out
            n = max(N, (n_bytes // 4) // N * N)
            inp, out = torch.ones(n, device=dev), torch.empty(n // N, device=dev)
            fn, moved = (lambda: dist.reduce_scatter_tensor(out, inp)), n * 4 * (N - 1) / N
        elif op == "all_gather":  # bf16 parameters, n_bytes per rank out
            n = max(N, (n_bytes // 2) // N * N)
            out, inp = torch.empty(n, dtype=bf, device=dev), torch.ones(n // N, dtype=bf,
                                                                                    device=dev)
            fn, moved = (lambda: dist.all_gather_into_tensor(out, inp)), n * 2 * (N - 1) / N
        elif op == "all_to_all":  # bf16 rows, equal splits
            n = max(N, (n_bytes // 2) // N * N)
            inp, out = torch.ones(n, dtype=bf, device=dev), torch.empty(n, dtype=bf, device=dev)
            fn, moved = (lambda: dist.all_to_all_single(out, inp)), n * 2 * (N - 1) / N
        else:  # all_to_all_v: row splits ~ 1 / (owner + 1), 72-byte rows (W&D bf16 push rows)
            rows = max(N, n_bytes // 72)
            w = [1.0 / (r + 1) for r in range(N)]
            send = [int(rows * x / sum(w)) for x in w]
            send[0] += rows - sum(send)
            # every rank sends the same split vector, so rank r receives send[r] rows from each peer
            recv = [send[rank]] * N
            inp = torch.ones(sum(send), 36, dtype=bf, device=dev)
            out = torch.empty(sum(recv), 36, dtype=bf, device=dev)
            fn = lambda: dist.all_to_all_single(out, inp, recv, send)  # noqa: E731
            moved = (sum(send) - send[rank]) * 72
        for _ in range(a.warmup):
            fn()
        sync()
        ts = []
        for _ in range(a.iters):
            dist.barrier()
            sync()
            t0 = time.perf_counter()
            fn()
            sync()
            ts.append(time.perf_counter() - t0)
        t = torch.tensor([statistics.median(ts)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item()), moved

    ops_ = a.ops.split(",")
    if rank == 0:
        print(f"# RCCL over {N} ranks, 7-link bound {bound:.0f} GB/s per GPU, env {json.dumps(env)}", flush=True)
        print(f"{'op':16s} {'MB/rank':>9s} {'us':>10s} {'algo GB/s':>10s} {'bus GB/s':>9s} {'of bound':>8s}")
    for op in ops_:
        for mb in sizes:
            n_bytes = int(mb * 2**20)
            t, moved = run(op, n_bytes)
            if rank == 0:
                bus = moved / t / 1e9
                print(f"{op:16s} {mb:9.2f} {t * 1e6:10.1f} {n_bytes / t / 1e9:10.1f} {bus:9.1f} {bus / bound:8.1%}",
                      flush=True)
    dist.barrier()
    dist.destroy_process_group()


def cmd_bubble(a):
    """GPU-side cost of a cross-stream fork on the stream forked FROM: N x (a 256-workgroup spin
    kernel of ~3 us on the compute stream [+ an event record there] [+ the side stream's wait on
    it] [+ a tiny kernel on the side stream]), per-iteration time from events around the loop.
    The difference to the bare loop is the bubble a fork puts on the compute stream."""
    from minips_amd._native import kernels
    k = kernels()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    raw, sraw = s.cuda_stream, side.cuda_stream
    fev = [k.FastEvent() for _ in range(8)]
    tev = [torch.cuda.Event() for _ in range(8)]
    n, ticks = 300, int(a.ticks)

    def run(kind):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0.record(s)
        for i in range(n):
            k.wire_spin(ticks, 256, raw)
            if kind == "spin":
                continue
            if kind.startswith("torch"):
                e = tev[i % 8]
                e.record(s)
                if kind == "torch+wait":
                    side.wait_event(e)
                continue
            e = fev[i % 8]
            e.record(raw)
            if kind in ("fast+wait", "fast+wait+side"):
                e.wait(sraw)
            if kind == "fast+wait+side":
                k.wire_spin(10, 1, sraw)
        t1.record(s)
        torch.cuda.synchronize()
        return t0.elapsed_time(t1) * 1e3 / n

    for rep in range(2):
        base = run("spin")
        print(f"rep {rep}: spin only {base:7.2f} us/iter (spin {ticks} ticks = {ticks / 100:.1f} us)")
        for kind in ("fast", "fast+wait", "fast+wait+side", "torch", "torch+wait"):
            t = run(kind)
            print(f"       + {kind:16s} {t:7.2f} us/iter  (+{t - base:5.2f})")


def cmd_issue(a):
    """HOST issue cost per call (no sync between calls) of the step's building blocks on one GPU:
    c10d collectives over a one-rank RCCL group (the Python + ProcessGroupNCCL + RCCL enqueue path
    each rank pays per call on an N-rank job), one of our kernel bindings, a torch elementwise op,
    and event record / wait -- the units a step's host budget is spent in."""
    import time

    import torch.distributed as dist

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29731", world_size=1, rank=0,
                                device_id=dev)
    from minips_amd import ops

    n = 1 << 16
    f = torch.ones(n, device=dev)
    o = torch.empty(n, device=dev)
    bfv = torch.ones(n, dtype=torch.bfloat16, device=dev)
    bo = torch.empty(n, dtype=torch.bfloat16, device=dev)
    keys = torch.arange(4096, device=dev)
    table = torch.randn(8192, 36, device=dev)
    rows = torch.empty(4096, 36, dtype=torch.bfloat16, device=dev)
    ev = torch.cuda.Event()
    s2 = torch.cuda.Stream(dev)
    from minips_amd.utils import streams

    fev = streams.FastEvent()
    cur = torch.cuda.current_stream(dev)
    pin = torch.zeros(8, dtype=torch.int64, pin_memory=True)
    # the native RCCL data plane (csrc/comm/rccl_comm.h) behind minips_amd.ps.comm.Comm: the binding
    # alone and the whole Comm method a table calls
    from minips_amd.ps.comm import Comm

    comm = Comm(device=dev, force_collectives=True)
    rc = comm._rc()
    cnt, cnt_o = torch.ones(1, dtype=torch.int64, device=dev), torch.empty(1, dtype=torch.int64, device=dev)
    rows2 = torch.empty(4096, 36, dtype=torch.bfloat16, device=dev)
    cases = {
        "native rccl all_to_all_v (binding)": lambda: rc.all_to_all_v(bo, bfv, [n], [n]),
        "native rccl all_to_all (counts)": lambda: rc.all_to_all(cnt_o, cnt),
        "native rccl reduce_scatter": lambda: rc.reduce_scatter(o, f),
        "native rccl all_gather": lambda: rc.all_gather(bo, bfv),
        "Comm.all_to_all_v (rows, native)": lambda: comm.all_to_all_v(rows2, rows, [4096], [4096]),
        "Comm.reduce_scatter (native)": lambda: comm.reduce_scatter(o, f),
        "Comm.all_gather (native)": lambda: comm.all_gather(bo, bfv),
        "c10d all_to_all_single (equal)": lambda: dist.all_to_all_single(bo, bfv),
        "c10d all_to_all_single (splits)": lambda: dist.all_to_all_single(bo, bfv, [n], [n]),
        "c10d reduce_scatter_tensor": lambda: dist.reduce_scatter_tensor(o, f),
        "c10d all_gather_into_tensor": lambda: dist.all_gather_into_tensor(bo, bfv),
        "c10d all_reduce": lambda: dist.all_reduce(f),
        "ops.gather_rows (binding)": lambda: ops.gather_rows(table, keys, 0, rows),
        "torch add_ (elementwise)": lambda: o.add_(f),
        "torch.empty": lambda: torch.empty(n, device=dev),
        "event record + wait": lambda: (ev.record(), s2.wait_event(ev)),
        "FastEvent record + wait": lambda: (fev.record(cur), fev.wait(s2)),
        "torch.cuda.Event() create + record": lambda: torch.cuda.Event().record(),
        "stream.wait_stream": lambda: s2.wait_stream(cur),
        "tensor.record_stream": lambda: f.record_stream(s2),
        "streams.current()": lambda: streams.current(dev),
        "pinned empty(16)": lambda: torch.empty(16, dtype=torch.int64, pin_memory=True),
        "tensor.tolist() (pinned, 8)": lambda: pin.tolist(),
        "slice view": lambda: f[128:4096],
    }
    print(f"{'call':40s} {'host us/call':>12s}")
    for name, fn in cases.items():
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            fn()
        t = (time.perf_counter() - t0) / a.iters
        torch.cuda.synchronize()
        print(f"{name:40s} {t * 1e6:12.2f}", flush=True)
    dist.destroy_process_group()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("gemm")
    p.add_argument("--set", default=os.environ.get("GEMM_SET", "wd"), choices=["wd", "gpt2"])
    p.add_argument("--no-lib", dest="lib", action="store_false", help="gemm: skip the hipBLASLt column")
    p.add_argument("--shapes", default=os.environ.get("GEMM_SHAPES", ""))
    p.add_argument("--split", type=int, default=1, help="split-K of the nt / nn shapes (slab + reduce)")
    p = sub.add_parser("one")
    p.add_argument("--shape", default="g.lm.d:8192:768:50304:nn")
    p.add_argument("--split", type=int, default=1)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--lib", action="store_true", help="torch.matmul / addmm(out_dtype=fp32) instead of ours")
    p = sub.add_parser("kscan")
    p.add_argument("--M", type=int, default=16384)
    p.add_argument("--N", type=int, default=1024)
    p.add_argument("--Ks", default="128,256,512,848,1024,2048,4096")
    p.add_argument("--layout", default="nt", choices=list(LAYOUTS))
    p.add_argument("--split", type=int, default=1)
    p.add_argument("--tag", default="")
    p = sub.add_parser("pmc")
    p.add_argument("--reps", type=int, default=10)
    p = sub.add_parser("attn")
    p.add_argument("--B", type=int, default=8)
    p.add_argument("--T", type=int, default=1024)
    p.add_argument("--H", type=int, default=12)
    sub.add_parser("nn")
    for name in ("emb", "plan", "embstep"):
        sub.add_parser(name).add_argument("--batch", type=int, default=16384)
    p = sub.add_parser("rccl")
    p.add_argument("--min-mb", type=float, default=0.25)
    p.add_argument("--max-mb", type=float, default=256.0)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--ops", default="reduce_scatter,all_gather,all_to_all,all_to_all_v")
    sub.add_parser("issue").add_argument("--iters", type=int, default=200)
    sub.add_parser("bubble").add_argument("--ticks", type=int, default=2000)
    p = sub.add_parser("wgrad")
    p.add_argument("--batch", type=int, default=16384)
    p.add_argument("--splits", default="2,4,6,8,10,12,16,24,32")
    a = ap.parse_args(argv)
    from minips_amd import _native

    _native.kernels()
    globals()["cmd_" + a.cmd](a)


if __name__ == "__main__":
    main()
