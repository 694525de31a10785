"""Data-plane ops of minips_amd.

Every op has ONE device implementation: GPU tensors go to the hand-written gfx950 HIP
kernels in ``minips_amd._kernels`` (and raise if that extension is missing -- there is no
silent eager fallback on a GPU). CPU tensors run a plain PyTorch reference of the same math;
that path exists for the CPU/gloo plumbing configuration (BASELINE config 1) and as the fp32
oracle the GPU numerics tests compare against.
"""
from __future__ import annotations

import math

import torch

from .._native import kernels

EPI_STORE_F32 = 0
EPI_ATOMIC_F32 = 1
EPI_BIAS_RELU_BF16 = 2
EPI_BIAS_BF16 = 3
EPI_STORE_BF16 = 4
EPI_RELU_MASK_BF16 = 5
EPI_BIAS_GELU_BF16 = 6
EPI_BIAS_GELU_AUX_BF16 = 7  # C = gelu(u), mask(aux) = u  (pre-activation saved for backward)
EPI_GELU_GRAD_BF16 = 8      # C = acc * gelu'(mask)
EPI_PERM_ROWS_BF16 = 9      # C rows of `seg` columns permuted by `perm` (embedding dgrad in planner order)
EPI_BIAS_GELU_DAUX_BF16 = 13  # C = gelu(u), mask(aux) = gelu'(u)  (the derivative saved for backward)
EPI_MUL_AUX_BF16 = 14       # C = acc * mask(aux)
_L2E = 1.4426950408889634


def _gelu_grad(u):
    k, c = 0.7978845608, 0.044715
    t = torch.tanh(k * (u + c * u ** 3))
    return 0.5 * (1 + t) + 0.5 * u * (1 - t * t) * k * (1 + 3 * c * u * u)


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# ----------------------------------------------------------------------------- GEMM
_NO_STRIDES: list = []
_REC = None  # the active ops.recording, if any


class recording:
    """Inside ``with ops.recording(lst):`` the GEMM-family ops (gemm, linear_fwd / dgrad / wgrad,
    colsum_add) run through ``lst``, a native LaunchList (csrc/bindings/ops_py.cpp): each launches
    as usual AND is appended, validated, for ``lst.run()`` to replay with no Python or binding cost.
    ``sink_adds`` collects the slab-sink registrations the replay must repeat (linear_wgrad defer)."""

    def __init__(self, lst):
        self.lst = lst
        self.sink_adds: list = []

    def __enter__(self):
        global _REC
        self.prev, _REC = _REC, self
        return self

    def __exit__(self, *exc):
        global _REC
        _REC = self.prev
        return False


def gemm(A, B, C, M, N, K, a_km=False, b_kn=False, epi=EPI_STORE_F32, bias=None, mask=None, colsum=None,
         alpha=1.0, split_k=1, perm=None, seg=0, tile=0):
    """C[M,N] (op)= A.B.  A is [M][K] (a_km=False) or [K][M]; B is [N][K] (b_kn=False) or [K][N].
    EPI_PERM_ROWS_BF16: C is [M*N/seg, seg] and output (row, col) goes to row perm[row*N/seg + col//seg].
    ``tile`` (GPU): 128 / 200 (256x128) / 256 forces the workgroup tile, 0 lets the launcher pick."""
    if _gpu(A):
        if _REC is not None:
            _REC.lst.gemm(A, B, C, M, N, K, a_km, b_kn, epi, bias, mask, colsum, float(alpha), int(split_k), perm,
                          int(seg), int(tile))
            return C
        # (all positional: pybind's keyword / default-argument path costs ~1 us per call)
        kernels().gemm(A, B, C, M, N, K, a_km, b_kn, epi, bias, mask, colsum, float(alpha), int(split_k), 1, 1, 0, 0,
                       0, _NO_STRIDES, perm, int(seg), int(tile))
        return C
    a = (A[:K, :M].t() if a_km else A[:M, :K]).float()
    b = (B[:K, :N] if b_kn else B[:N, :K].t()).float()
    acc = (a @ b) * alpha
    if epi == EPI_STORE_F32:
        C[:M, :N] = acc
    elif epi == EPI_ATOMIC_F32:
        C[:M, :N] += acc
    elif epi == EPI_BIAS_GELU_AUX_BF16:
        if bias is not None:
            acc = acc + bias[:N].float()
        mask[:M, :N] = acc.to(torch.bfloat16)
        C[:M, :N] = torch.nn.functional.gelu(acc, approximate="tanh").to(torch.bfloat16)
    elif epi == EPI_GELU_GRAD_BF16:
        C[:M, :N] = (acc * _gelu_grad(mask[:M, :N].float())).to(torch.bfloat16)
    elif epi == EPI_BIAS_GELU_DAUX_BF16:
        if bias is not None:
            acc = acc + bias[:N].float()
        mask[:M, :N] = _gelu_grad(acc).to(torch.bfloat16)
        C[:M, :N] = torch.nn.functional.gelu(acc, approximate="tanh").to(torch.bfloat16)
    elif epi == EPI_MUL_AUX_BF16:
        C[:M, :N] = (acc * mask[:M, :N].float()).to(torch.bfloat16)
    elif epi in (EPI_BIAS_RELU_BF16, EPI_BIAS_BF16, EPI_BIAS_GELU_BF16):
        if bias is not None:
            acc = acc + bias[:N].float()
        if epi == EPI_BIAS_RELU_BF16:
            acc = torch.relu(acc)
        elif epi == EPI_BIAS_GELU_BF16:
            acc = torch.nn.functional.gelu(acc, approximate="tanh")
        C[:M, :N] = acc.to(torch.bfloat16)
    elif epi == EPI_STORE_BF16:
        C[:M, :N] = acc.to(torch.bfloat16)
    elif epi == EPI_PERM_ROWS_BF16:
        C.view(-1, seg)[perm[: M * (N // seg)].long()] = acc.to(torch.bfloat16).reshape(-1, seg)
    elif epi == EPI_RELU_MASK_BF16:
        out = torch.where(mask[:M, :N].float() > 0, acc, torch.zeros_like(acc)).to(torch.bfloat16)
        C[:M, :N] = out
        if colsum is not None:
            colsum[:N] += out.float().sum(0)
    else:
        raise ValueError(f"unknown epilogue {epi}")
    return C


def gemm_batched(A, B, C, M, N, K, a_km, b_kn, epi, batch, inner, lda, ldb, ldc, strides, alpha=1.0, bias=None):
    """``batch`` GEMMs over flat buffers; operand z starts at (z//inner)*s_outer + (z%inner)*s_inner
    (strides = [sa_o, sa_i, sb_o, sb_i, sc_o, sc_i] in elements), leading dims lda/ldb/ldc."""
    if _gpu(A):
        if _REC is not None:
            raise RuntimeError("ops.recording: batched GEMMs are not recordable")
        kernels().gemm(A, B, C, M, N, K, a_km, b_kn, epi, bias, None, None, float(alpha), 1, int(batch), int(inner),
                       int(lda), int(ldb), int(ldc), [int(x) for x in strides])
        return C
    Af, Bf, Cf = A.reshape(-1), B.reshape(-1), C.reshape(-1)
    for z in range(batch):
        zo, zi = divmod(z, inner)
        oa, ob, oc = (zo * strides[0] + zi * strides[1], zo * strides[2] + zi * strides[3],
                      zo * strides[4] + zi * strides[5])
        ar, ac = (K, M) if a_km else (M, K)
        br, bc = (K, N) if b_kn else (N, K)
        a = Af[oa: oa + (ar - 1) * lda + ac].as_strided((ar, ac), (lda, 1))
        b = Bf[ob: ob + (br - 1) * ldb + bc].as_strided((br, bc), (ldb, 1))
        c = Cf[oc: oc + (M - 1) * ldc + N].as_strided((M, N), (ldc, 1))
        gemm(a, b, c, M, N, K, a_km, b_kn, epi, bias=bias, alpha=alpha)
    return C


_FWD_EPI = {"relu": EPI_BIAS_RELU_BF16, "none": EPI_BIAS_BF16, "gelu": EPI_BIAS_GELU_BF16}


def linear_fwd(x, w, bias=None, act="relu", out=None):
    """y = act(x w^T + b) in bf16 (x [M,K], w [N,K])."""
    M, K = x.shape[0], w.shape[1]
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
    return gemm(x, w, out, M, N, K, False, False, _FWD_EPI[act], bias=bias)


def colsum_add(x, out):
    """out[:N] += x.sum(0) in fp32 (x bf16 [M, N]): a Linear's bias gradient from its dy."""
    if _gpu(x):
        (kernels() if _REC is None else _REC.lst).colsum_bf16(x, out)
        return out
    out[: x.shape[1]] += x.float().sum(0)
    return out


def linear_dgrad(dy, w, mask=None, colsum=None, out_f32=False, n_cols=None, out=None, perm=None, seg=0, tile=0):
    """dx = dy w (dy [M,N], w [N,K]) -> bf16 masked by (mask > 0) (+colsum), or fp32. ``perm`` /
    ``seg``: dx's row segments of ``seg`` columns go to rows perm[...] of out [M*K/seg, seg] (the
    embedding gradient written straight into the key planner's row-sorted order). ``tile``: gemm's."""
    M, N = dy.shape
    K = w.shape[1] if n_cols is None else n_cols
    if perm is not None:
        if out is None:
            out = torch.empty(M * K // seg, seg, dtype=torch.bfloat16, device=dy.device)
        return gemm(dy, w, out, M, K, N, False, True, EPI_PERM_ROWS_BF16, perm=perm, seg=seg, tile=tile)
    if out is None:
        out = torch.empty(M, K, dtype=torch.float32 if out_f32 else torch.bfloat16, device=dy.device)
    epi = EPI_STORE_F32 if out_f32 else (EPI_RELU_MASK_BF16 if mask is not None else EPI_STORE_BF16)
    return gemm(dy, w, out, M, K, N, False, True, epi, mask=mask, colsum=colsum, tile=tile)


# Split-K weight gradients: about one 128x128 workgroup per CU pair (512 blocks), but a minimum number
# of reduction rows per split (profiles/r2/gpt2_wgrad_sweep.txt: shorter slices lose to their fixed
# prologue/epilogue cost). 640 rows is the isolated-kernel optimum (a wgrad on the critical path, e.g.
# the MLP); a wgrad forked onto a side stream beside the dgrad chain (SideStream sets overlap_mode)
# favours throughput: fewer, longer splits with less slab traffic -- 1024 rows measured best there
# (W&D 0.461 ms vs 0.490 at 2048; tools/gpu_round.sh ab, profiles/r2/gemm_round2.txt). A block-count floor
# for overlapped wgrads with few tiles measured worse (W&D 0.528 -> 0.539 ms at 128 blocks) and is gone;
# so are the 256x256 wgrad tile and the phase-split v3 wgrad (profiles/r4/ab_gpt2_knobs.txt).
_WGRAD_BLOCKS = 512
_WGRAD_MIN_ROWS = 640
_WGRAD_MIN_ROWS_OVERLAP = 1024
_overlap_state = __import__("threading").local()


def overlap_mode(on: bool) -> bool:
    """Mark GEMMs issued from now on as overlapped side-stream work (returns the previous mode)."""
    prev = getattr(_overlap_state, "on", False)
    _overlap_state.on = on
    return prev


def linear_wgrad(dy, x, dw, split_k=None, blocks=None, defer=None, tile=0):
    """dw[N,K] += dy^T x (dy [M,N], x [M,K]); fp32 accumulate. ``blocks``: the workgroup target of
    the split-K choice (default _WGRAD_BLOCKS; a model may tune its own). ``defer``: a
    DenseTable slab sink (DenseTable.slab_sink()): the K slices stay in fp32 slab planes that the
    table's next Adam folds in (no reduce kernel); dw must be a contiguous [N, K] region of the
    table's gradient, which the sum then never passes through. ``tile``: gemm's tile hint."""
    M, N = dy.shape
    K = x.shape[1]
    if split_k is None:
        tiles = ((N + 127) // 128) * ((K + 127) // 128)
        overlapped = getattr(_overlap_state, "on", False)
        min_rows = _WGRAD_MIN_ROWS_OVERLAP if overlapped else _WGRAD_MIN_ROWS
        target = _WGRAD_BLOCKS if blocks is None else int(blocks)
        split_k = max(1, min(M // min_rows, (target + tiles - 1) // tiles))
    if (defer is not None and _gpu(dy) and split_k > 1 and K % 4 == 0 and dw.dim() == 2
            and dw.stride(1) == 1 and dw.stride(0) == K and defer.accepts(dw)):
        slab = defer.slab(dw, split_k)
        nsplit = (kernels() if _REC is None else _REC.lst).gemm_slab(dy, x, slab, N, K, M, True, True, int(split_k))
        defer.add(dw, slab, nsplit)
        if _REC is not None:
            _REC.sink_adds.append((defer, dw, slab, nsplit))
        return dw
    return gemm(dy, x, dw, N, K, M, True, True, EPI_ATOMIC_F32, split_k=split_k, tile=tile)


# ----------------------------------------------------------------------------- sparse keys
def unique_bucketize(keys: torch.Tensor, bounds: torch.Tensor, F: int = 1):
    """Dedupe ``keys`` and group the unique keys by owner shard.

    Returns (uniq [n] with the first sum(counts) valid, inverse [n], counts [P]) where
    ``bounds`` [P+1] are the shard key boundaries and uniq[inverse[i]] == keys[i]. ``F`` > 1
    declares the flat keys as a [B, F] batch (the GPU kernel then dedupes feature-major tiles).
    """
    uniq, inv, counts, _ = unique_bucketize_n(keys, bounds, F)
    return uniq, inv, counts


def unique_bucketize_n(keys: torch.Tensor, bounds: torch.Tensor, F: int = 1, route_mult: int = 0,
                       route_n: int = 0, extra_zero_ints: int = 0, csr_counts: bool = False):
    """unique_bucketize plus the total unique count U as a 1-element device tensor, so that
    consumers (gather_rows / sparse_* with ``n_dev``, wd_emb_backward with ``U_dev``) bound
    their work on the GPU without a host round trip. ``route_mult`` != 0 first maps every key to
    key * route_mult mod route_n (fused into the GPU kernel). ``csr_counts`` (GPU, with
    extra_zero_ints >= n): the first n ints of the zeroed block receive each unique key's lookup
    count, for emb_build_csr(..., counts_ready=True)."""
    if _gpu(keys):
        out = kernels().unique_bucketize(keys.contiguous(), bounds.contiguous(), int(F), int(route_mult),
                                         int(route_n), int(extra_zero_ints), bool(csr_counts))
        if extra_zero_ints:  # (..., zeroed int32 workspace cleared by the same memset)
            return tuple(out[:4]), out[4]
        return tuple(out)
    keys = keys.reshape(-1)
    if route_mult:
        keys = (keys * route_mult) % route_n
    u, inv = torch.unique(keys, sorted=True, return_inverse=True)
    owner = torch.bucketize(u, bounds[1:-1], right=True)
    counts = torch.bincount(owner, minlength=bounds.numel() - 1)
    # sorted unique keys are already grouped by owner (ranges are contiguous)
    out = torch.empty_like(keys)
    out[: u.numel()] = u
    return out, inv, counts, torch.tensor([u.numel()], dtype=torch.int64)


def bitmap_plan(keys: torch.Tensor, bounds: torch.Tensor, num_rows: int, route_mult: int = 0, oor=None):
    """unique_bucketize_n for a bounded key space: keys (after the optional routing
    key * route_mult mod num_rows) in [0, num_rows). GPU: an N-bit map + popcount ranks
    (csrc/kernels/bitmap.hip), no hash table; the unique keys come out sorted, so the CPU
    reference (torch.unique) produces the identical plan. Returns (uniq, inverse, counts, U).
    ``oor`` (device int64 [1], optional): accumulates the number of keys outside the key space
    (they would alias row 0); the caller checks it at a host sync point (no sync here)."""
    if _gpu(keys):
        return tuple(kernels().bitmap_plan(keys.reshape(-1).contiguous(), bounds.contiguous(), int(num_rows),
                                           int(route_mult), int(num_rows) if route_mult else 0, oor))
    flat = keys.reshape(-1)
    k = (flat * route_mult) % num_rows if route_mult else flat
    bad = (k < 0) | (k >= num_rows)
    if bool(bad.any()):
        if oor is None:
            raise ValueError(f"keys outside [0, {num_rows})")
        oor += int(bad.sum())
    return unique_bucketize_n(flat, bounds, 1, int(route_mult), int(num_rows) if route_mult else 0)


def plan_sorted(keys, col_base, col_bits, route_mult=0, route_n=0, bits_dev=None, bounds=None, positions=False):
    """Key planning of a [B, F] batch whose columns hold disjoint key ranges (column f's keys in
    [col_base[f], col_base[f] + 2**col_bits[f])): per-column radix sort, no global atomics
    (plan.hip). ``col_bits``: a list of ints (or one int for every column); ``bounds`` [P+1]: the
    owners' routed-key ranges (None: one owner). Returns (uniq [n] (first U valid, routed; column-
    major, inside a column by (owner, key) -- ascending keys for one owner -- then stably grouped by
    owner), inv [n], counts [P], U_dev [1], members [n] int32, memrow [n] int32) -- the
    unique_bucketize_n outputs plus the lookup CSR of emb_build_csr (rows contiguous, in that
    column-major order)."""
    if bounds is None:
        bounds = torch.tensor([0, (1 << 62)], dtype=torch.int64, device=keys.device)
    if _gpu(keys):
        bits = [int(col_bits)] * keys.shape[1] if isinstance(col_bits, int) else [int(b) for b in col_bits]
        if bits_dev is None:  # (tables pass their cached device copy: no H2D copy per plan)
            bits_dev = torch.tensor(bits, dtype=torch.int32, device=keys.device)
        return tuple(kernels().plan_sorted(keys.contiguous(), col_base.contiguous(), bits_dev, bits,
                                           int(route_mult), int(route_n), bounds.contiguous(), bool(positions)))
    B, F = keys.shape
    P = bounds.numel() - 1
    uniq_l, inv_l = [], []
    base = 0
    for f in range(F):
        u, i = torch.unique(keys[:, f], sorted=True, return_inverse=True)
        if P > 1:  # inside a column the keys sort by (owner shard of the routed key, key)
            r = (u * route_mult) % route_n if route_mult else u
            o = torch.sort(torch.bucketize(r, bounds[1:-1], right=True), stable=True).indices
            rank = torch.empty_like(o)
            rank[o] = torch.arange(o.numel())
            u, i = u[o], rank[i]
        uniq_l.append(u)
        inv_l.append(i + base)
        base += u.numel()
    U = base
    uniq = torch.cat(uniq_l)
    if route_mult:
        uniq = (uniq * route_mult) % route_n
    owner = torch.bucketize(uniq, bounds[1:-1], right=True)
    perm_order = torch.sort(owner, stable=True).indices      # regrouped position -> u
    perm = torch.empty(U, dtype=torch.int64)
    perm[perm_order] = torch.arange(U)                         # u -> regrouped position
    out = torch.empty(B * F, dtype=torch.int64)
    out[:U] = uniq[perm_order]
    inv_u = torch.stack(inv_l, 1).reshape(-1)                  # column-major u of each lookup
    order = torch.sort(inv_u, stable=True).indices             # lookups grouped by u (ascending)
    counts = torch.bincount(owner, minlength=P).to(torch.int64)
    res = (out, perm[inv_u], counts, torch.tensor([U], dtype=torch.int64), order.to(torch.int32),
           perm[inv_u[order]].to(torch.int32))
    pos = None
    if positions:  # members = order: pos[order[m]] = m
        pos = torch.empty(B * F, dtype=torch.int32)
        pos[order] = torch.arange(B * F, dtype=torch.int32)
    if P == 1:  # row u's lookups are members [rowstart[u], rowstart[u + 1]): (.., positions or None, rowstart,
        # rowidx or None) -- rowidx: each lookup's table row (routed key) when routed keys fit int32
        rs = torch.full((B * F + 1,), B * F, dtype=torch.int32)
        rs[0] = 0
        rs[1: U + 1] = torch.cumsum(torch.bincount(inv_u, minlength=U), 0).to(torch.int32)
        ri = uniq[inv_u].to(torch.int32) if route_mult and 0 < route_n <= 0x7FFFFFFF else None
        return res + (pos, rs, ri)
    return res + (pos,) if positions else res


def gather_rows(table, keys, base, out, n_dev=None):
    """out[i] = table[keys[i] - base] for i < n (n = keys.numel(), or the device count n_dev)."""
    if _gpu(keys):
        kernels().gather_rows(table, keys, int(base), out, n_dev)
        return out
    if n_dev is not None:
        keys = keys[: int(n_dev.reshape(-1)[0])]
    rows = table[(keys - base), : out.shape[1]]
    out[: keys.numel()] = rows.to(out.dtype)
    return out


def lookup_rows(rows, inv, F, D, out):
    """out[b, f*D:(f+1)*D] = rows[inv[b*F+f], :D] (bf16; out may be a row-major column slice)."""
    if _gpu(rows):
        kernels().lookup_rows(rows, inv, int(F), int(D), out)
        return out
    B = out.shape[0]
    out[:, : F * D] = rows[inv, :D].reshape(B, F * D).to(out.dtype)
    return out


def scatter_add_rows(src, idx, acc):
    """acc[idx[i]] += src[i] (src fp32 or bf16, acc fp32; or both fp64)."""
    if _gpu(src):
        kernels().scatter_add_rows(src, idx, acc)
        return acc
    acc.index_add_(0, idx, src.to(acc.dtype))
    return acc


def _sr_bf16(x: torch.Tensor, gen: torch.Generator | None = None) -> torch.Tensor:
    """Stochastic rounding of fp32 to bf16 (CPU reference of bf16rows.hip): add 16 random bits
    below the bf16 mantissa, truncate."""
    b = x.contiguous().view(torch.int32)
    r = torch.randint(0, 1 << 16, b.shape, dtype=torch.int32, generator=gen)
    finite = (b & 0x7F800000) != 0x7F800000
    b = torch.where(finite, b + r, b)
    return (b & -65536).view(torch.float32).to(torch.bfloat16)


def sparse_apply_bf16(opt, table, state, keys, base, grads, lr, eps=1e-8, scale=1.0, state2=None, split=None,
                      step=0, seed=0, n_dev=None):
    """fp32 gradient rows into a bf16 table with stochastic rounding (opt "rowwise_adagrad" |
    "add" (w += scale * g))."""
    D = table.shape[1]
    D1 = D if split is None else split
    code = 0 if opt == "rowwise_adagrad" else 1
    if _gpu(table):
        kernels().sparse_apply_bf16(code, table, state, state2, int(D1), keys, int(base), grads, float(lr), float(eps),
                                    float(scale), int(step) & 0xFFFFFFFF, int(seed) & 0xFFFFFFFF, n_dev)
        return
    if n_dev is not None:
        n = int(n_dev.reshape(-1)[0])
        keys, grads = keys[:n], grads[:n]
    rows = keys - base
    w = table[rows].float()
    g = grads[:, :D].float()
    if code == 0:
        s1 = state[rows] + (g[:, :D1] ** 2).mean(1)
        state[rows] = s1
        w[:, :D1] -= lr * g[:, :D1] / (s1.sqrt() + eps).unsqueeze(1)
        if D1 < D:
            s2 = state2[rows] + (g[:, D1:] ** 2).mean(1)
            state2[rows] = s2
            w[:, D1:] -= lr * g[:, D1:] / (s2.sqrt() + eps).unsqueeze(1)
    else:
        w += scale * g
    table[rows] = _sr_bf16(w, torch.Generator().manual_seed((int(seed) * 1000003 + int(step)) & 0x7FFFFFFF))


def sparse_rowwise_adagrad(table, state, keys, base, grads, lr, eps=1e-8, state2=None, split=None, n_dev=None,
                           zero_g=False):
    """Row-wise Adagrad on table rows keys - base. ``zero_g``: the kernel clears the gradient rows
    after reading them (a persistent, pre-zeroed push buffer stays zero for the next push)."""
    D = grads.shape[1]
    D1 = D if split is None else split
    if _gpu(table):
        kernels().sparse_rowwise_adagrad(table, state, state2, D1, keys, int(base), grads, float(lr), float(eps),
                                         n_dev, bool(zero_g))
        return
    if n_dev is not None:
        n = int(n_dev.reshape(-1)[0])
        keys, grads = keys[:n], grads[:n]
    rows = keys - base
    g1 = grads[:, :D1]
    s1 = state[rows] + (g1 * g1).mean(1)
    state[rows] = s1
    table[rows, :D1] -= lr * g1 / (s1.sqrt() + eps).unsqueeze(1)
    if D1 < D:
        g2 = grads[:, D1:]
        s2 = state2[rows] + (g2 * g2).mean(1)
        state2[rows] = s2
        table[rows, D1:D] -= lr * g2 / (s2.sqrt() + eps).unsqueeze(1)


def owner_slots(own_inv, splits, cap):
    """Owner side of a multi-rank push: the received rows come grouped by requester (``splits``,
    host ints); returns int32 slots [cap * P] with slots[u * P + s] = the received row requester s
    sent for owned unique row u (own_inv[i] = u), -1 where s sent none."""
    P = len(splits)
    if _gpu(own_inv):
        return kernels().owner_slots(own_inv, [int(c) for c in splits], int(cap))
    slots = torch.full((max(int(cap), 1) * P,), -1, dtype=torch.int32)
    seg = torch.repeat_interleave(torch.arange(P), torch.tensor([int(c) for c in splits], dtype=torch.int64))
    slots[own_inv * P + seg] = torch.arange(own_inv.numel(), dtype=torch.int32)
    return slots


def owner_push_adagrad(table, state, keys, base, recv, splits, rs, stamp, lr, eps=1e-8, state2=None, split=None):
    """Owner apply of one push without an owner-side dedupe: received key i (requester segments
    ``splits``, each requester's keys distinct) carries gradient row recv[i]; every touched row gets
    the row-wise Adagrad of the sum of its received rows in requester order -- owner_rows_adagrad's
    arithmetic. ``rs``: a persistent int32 [rows * P * 2] {stamp, row} table (GPU), ``stamp`` this
    push's number (increasing, >= 0)."""
    D = recv.shape[1]
    D1 = D if split is None else split
    if _gpu(table):
        kernels().owner_push_adagrad(table, state, state2, int(D1), keys, int(base), recv.contiguous(),
                                     [int(c) for c in splits], rs, int(stamp), float(lr), float(eps))
        return
    M = keys.numel()
    if M == 0:
        return
    uniq, inv = torch.unique(keys, sorted=True, return_inverse=True)
    P = len(splits)
    seg = torch.repeat_interleave(torch.arange(P), torch.tensor([int(c) for c in splits], dtype=torch.int64))
    slots = torch.full((uniq.numel() * P,), -1, dtype=torch.int32)
    slots[inv * P + seg] = torch.arange(M, dtype=torch.int32)
    owner_rows_adagrad(table, state, uniq, uniq.numel(), base, recv, slots, P, lr, eps, state2=state2, split=split)


def owner_rows_adagrad(table, state, keys, n, base, recv, slots, P, lr, eps=1e-8, state2=None, split=None, n_dev=None):
    """Row-wise Adagrad of owned rows keys[:n] (n_dev: device bound) with the gradient of row u =
    sum over s in 0..P-1 of recv[slots[u * P + s]] (bf16 / fp32 rows, fp32 sum in requester order)
    -- ops.sparse_rowwise_adagrad of the owner-side segment sums, in one pass."""
    D = recv.shape[1]
    D1 = D if split is None else split
    if _gpu(table):
        kernels().owner_rows_adagrad(table, state, state2, int(D1), keys, int(n), n_dev, int(base), recv, int(P), slots,
                                     float(lr), float(eps))
        return
    if n_dev is not None:
        n = min(int(n), int(n_dev.reshape(-1)[0]))
    sl = slots[: n * P].view(n, P).long()
    g = torch.zeros(n, D, dtype=torch.float32)
    for s in range(P):  # requester order (the GPU sum's order)
        m = sl[:, s]
        hit = m >= 0
        g[hit] += recv[m[hit]].float()
    sparse_rowwise_adagrad(table, state, keys[:n], base, g, lr, eps, state2=state2, split=split)


def sparse_sgd(table, keys, base, grads, scale, n_dev=None):
    if _gpu(table):
        kernels().sparse_sgd(table, keys, int(base), grads, float(scale), n_dev)
        return
    if n_dev is not None:
        n = int(n_dev.reshape(-1)[0])
        keys, grads = keys[:n], grads[:n]
    table.index_add_(0, keys - base, scale * grads, alpha=1.0) if grads.shape[1] == table.shape[1] else \
        table[:, : grads.shape[1]].index_add_(0, keys - base, scale * grads)


def embedding_bag_fwd(rows, idx, offsets, mean=False, out=None):
    B = offsets.numel() - 1
    if out is None:
        out = torch.empty(B, rows.shape[1], dtype=torch.float32, device=rows.device)
    if _gpu(rows):
        kernels().embedding_bag_fwd(rows, idx, offsets, bool(mean), out)
        return out
    mode = "mean" if mean else "sum"
    out.copy_(torch.nn.functional.embedding_bag(idx, rows, offsets[:-1], mode=mode, include_last_offset=False))
    return out


def embedding_bag_bwd(grad_out, idx, offsets, grad_rows, mean=False):
    if _gpu(grad_out):
        kernels().embedding_bag_bwd(grad_out, idx, offsets, bool(mean), grad_rows)
        return grad_rows
    lens = (offsets[1:] - offsets[:-1])
    bag = torch.repeat_interleave(torch.arange(lens.numel(), device=idx.device), lens)
    g = grad_out[bag]
    if mean:
        g = g / lens[bag].clamp_min(1).unsqueeze(1).to(g.dtype)
    grad_rows.index_add_(0, idx, g)
    return grad_rows


# ----------------------------------------------------------------------------- Wide&Deep
def wd_assemble(dense, rows, inv, F, D, X, wide_logit, ones_col=-1, zero=None):
    """X = [emb_0..emb_{F-1} | dense | 1 at ones_col | 0-pad] (bf16);
    wide_logit[b] = sum_f rows[inv, D]. ``zero`` (fp32 [1], optional) is set to 0 on the way
    (the step's loss accumulator: no separate fill kernel)."""
    if _gpu(X):
        kernels().wd_assemble(dense, rows, inv, int(F), int(D), X, wide_logit, int(ones_col), zero)
        return X, wide_logit
    if zero is not None:
        zero.zero_()
    B = X.shape[0]
    r = rows[inv].view(B, F, rows.shape[1]).float()
    X.zero_()
    X[:, : F * D] = r[:, :, :D].reshape(B, F * D).to(torch.bfloat16)
    X[:, F * D: F * D + dense.shape[1]] = dense.to(torch.bfloat16)
    if ones_col >= 0:
        X[:, ones_col] = 1.0
    wide_logit.copy_(r[:, :, D].sum(1))
    return X, wide_logit


def wd_assemble_tab(dense, table, index, base, inv, F, D, X, wide_logit, ones_col=-1, zero=None, rowidx=None):
    """wd_assemble with the rows read in place: the row of unique u is table[index[u] - base]
    (fp32), rounded to bf16 exactly as gather_rows(out bf16) does. ``rowidx`` (plan_sorted, one
    owner): lookup j's row + base directly (the same rows, one index load per lookup)."""
    if _gpu(X):
        kernels().wd_assemble_tab(dense, table, index, int(base), inv, int(F), int(D), X, wide_logit, int(ones_col),
                                  zero, rowidx)
        return X, wide_logit
    U = int(inv.max()) + 1 if inv.numel() else 0
    rows = table[index[:U] - base].to(torch.bfloat16)
    return wd_assemble(dense, rows, inv, F, D, X, wide_logit, ones_col, zero)


def wd_head(H, w, b0, wide_logit, labels, dH, dw, db, dwide, loss_sum, dH_colsum=None, grad_scale=1.0,
            defer_fold=False):
    """Last layer + BCE forward/backward. ``defer_fold`` (GPU): the batch sums into dw / db /
    loss_sum / dH_colsum are left as per-block partials for wd_head_fold (a later kernel, e.g. on
    the weight-gradient stream, off the dgrad chain); on the CPU they are added here and the fold
    is a no-op."""
    if _gpu(H):
        kernels().wd_head(H, w, b0, wide_logit, labels, dH, dw, db, dwide, loss_sum, dH_colsum, float(grad_scale),
                          bool(defer_fold))
        return
    h = H.float()
    z = h @ w.float() + b0.float() + wide_logit
    y = (labels > 0.5).float()
    p = torch.sigmoid(z)
    dz = (p - y) * grad_scale
    dwide.copy_(dz)
    db += dz.sum()
    loss_sum += (torch.clamp_min(z, 0) - z * y + torch.log1p(torch.exp(-z.abs()))).sum()
    g = torch.where(h > 0, dz.unsqueeze(1) * w.float().unsqueeze(0), torch.zeros_like(h)).to(torch.bfloat16)
    dH.copy_(g)
    dw += (dz.unsqueeze(1) * h).sum(0)
    if dH_colsum is not None:
        dH_colsum += g.float().sum(0)


def wd_head_fold(B, Hd, dw, db, loss_sum, dH_colsum=None):
    """The totals of the device's last wd_head(defer_fold=True) (same B, Hd), on the current
    stream (recordable into a LaunchList). No-op on the CPU (wd_head added them)."""
    if _gpu(dw):
        (kernels() if _REC is None else _REC.lst).wd_head_fold(int(B), int(Hd), dw, db, loss_sum, dH_colsum)


def emb_csr_positions(members):
    """pos[members[m]] = m (int32): the member-order row of every lookup (the dgrad's permutation)."""
    if _gpu(members):
        return kernels().emb_csr_positions(members)
    pos = torch.empty_like(members)
    pos[members.long()] = torch.arange(members.numel(), dtype=members.dtype)
    return pos


def emb_build_csr(inv, F, U, zeroed=None, counts_ready=False):
    """Lookups grouped by unique row: (members, memrow) int32 [n] with memrow sorted and
    members[i] the lookup id (b*F + f) of the i-th entry. Depends on ``inv`` only, so the PS
    builds it while planning a batch (off the critical path). ``zeroed``: an already-zero int32
    block of >= 2U (from unique_bucketize_n's extra_zero_ints) saves the counter memset."""
    if _gpu(inv):
        return tuple(kernels().emb_build_csr(inv, int(F), int(max(U, 1)), zeroed, bool(counts_ready)))
    order = torch.sort(inv, stable=True).indices
    return order.to(torch.int32), inv[order].to(torch.int32)


def wd_emb_backward(dX, dwide, inv, F, D, grad_rows, x_off=0, csr=None, sorted_rows=False):
    """grad_rows[u, :D] = sum of dX[b, x_off + f*D : ...] over the lookups (b, f) with
    inv[b*F+f] == u; column D likewise sums dwide[b] when given, columns D+1.. are 0. On the GPU
    (D 16 / 32 / 64) every row that has lookups (every unique row of a plan) is written exactly
    once, in a fixed summation order -- the same bits on every run; rows without lookups are left
    untouched -- and ``grad_rows`` may be fp32 or bf16 (the multi-rank push payload);
    the CPU reference adds into grad_rows, so callers pass a zeroed buffer. ``sorted_rows``: dX is
    [B*F, D] in the CSR's member order (row m = lookup csr[0][m]; linear_dgrad(perm=csr[2]) writes it)."""
    if _gpu(dX):
        members, memrow = (csr[0], csr[1]) if csr is not None else (None, None)
        kernels().wd_emb_backward(dX, dwide, inv, int(F), int(D), grad_rows, int(x_off), members, memrow,
                                  bool(sorted_rows))
        return grad_rows
    if sorted_rows:  # back to lookup order
        un = torch.empty_like(dX)
        un[csr[0].long()] = dX
        dX, x_off = un.reshape(-1, F * D), 0
    B = dX.shape[0]
    g = dX[:, x_off: x_off + F * D].float().reshape(B * F, D)
    acc = grad_rows if grad_rows.dtype == torch.float32 else grad_rows.float()
    acc[:, :D].index_add_(0, inv, g)
    if dwide is not None:
        acc[:, D].index_add_(0, inv, dwide.repeat_interleave(F))
    if acc is not grad_rows:
        grad_rows.copy_(acc)
    return grad_rows


# ----------------------------------------------------------------------------- optimizers
def adam_apply(w, m, v, g, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step=1, grad_scale=1.0,
               w_bf16=None, step_dev=None, zero_g=False, slabs=()):
    """Fused Adam(W). ``step_dev`` (int32 [1] device tensor): the bias-correction step is read on the
    device, so a captured (HIP graph) clock stays correct on replay. ``zero_g``: the kernel also
    clears ``g`` after reading it (the gradient accumulator of the next clock; no fill kernel).
    ``slabs``: (slab, nsplit, plane, offset) split-K gradient planes folded into g[offset:offset+plane]."""
    if _gpu(w):
        kernels().adam_apply(w, m, v, g, float(lr), float(beta1), float(beta2), float(eps), float(weight_decay),
                             int(step), float(grad_scale), w_bf16, step_dev, bool(zero_g),
                             [(s, int(n), int(p), int(o)) for s, n, p, o in slabs])
        return
    g_in = g
    if slabs:
        g = g.clone()
        for s, n, p, o in slabs:
            g[o: o + p] += s[: n * p].view(n, p).sum(0)
    if step_dev is not None:
        step = int(step_dev.reshape(-1)[0])
    gg = g * grad_scale
    m.mul_(beta1).add_((1 - beta1) * gg)
    v.mul_(beta2).add_((1 - beta2) * gg * gg)
    bc1, bc2 = 1 - beta1 ** step, 1 - beta2 ** step
    w.sub_(lr * ((m / bc1) / ((v / bc2).sqrt() + eps) + weight_decay * w))
    if w_bf16 is not None:
        w_bf16.copy_(w.to(torch.bfloat16))
    if zero_g:
        g_in.zero_()


def slab_pack(g, out, slabs=()):
    """out = g + the split-K planes ``slabs`` ((slab, nsplit, plane, offset), as adam_apply) folded
    into their regions; g cleared -- a several-rank dense clock's reduce-scatter input in one pass."""
    if _gpu(g):
        kernels().slab_pack(g, out, [(s, int(n), int(p), int(o)) for s, n, p, o in slabs])
        return out
    out.copy_(g)
    for s, n, p, o in slabs:
        out[o: o + p] += s[: n * p].view(n, p).sum(0)
    g.zero_()
    return out


def sgd_apply(w, g, lr, grad_scale=1.0, w_bf16=None):
    if _gpu(w):
        kernels().sgd_apply(w, g, float(lr), float(grad_scale), w_bf16)
        return
    w.sub_(lr * grad_scale * g)
    if w_bf16 is not None:
        w_bf16.copy_(w.to(torch.bfloat16))


def adagrad_apply(w, acc, g, lr, eps=1e-10, grad_scale=1.0, w_bf16=None):
    if _gpu(w):
        kernels().adagrad_apply(w, acc, g, float(lr), float(eps), float(grad_scale), w_bf16)
        return
    gg = g * grad_scale
    acc.add_(gg * gg)
    w.sub_(lr * gg / (acc.sqrt() + eps))
    if w_bf16 is not None:
        w_bf16.copy_(w.to(torch.bfloat16))


def cast_f32_bf16(x, y):
    if _gpu(x):
        kernels().cast_f32_bf16(x, y)
        return y
    y.copy_(x.to(torch.bfloat16))
    return y


# ----------------------------------------------------------------------------- LR / K-Means
def lr_sparse_step(rowptr, cols, vals, labels, w, alpha, delta=None, correct=None):
    """Sparse LR gradient (lr_example.cpp:291-312): delta[col] += alpha*x*(y - sigmoid(w.x))."""
    if _gpu(w):
        kernels().lr_sparse_step(rowptr, cols, vals, labels, w, float(alpha), delta, correct)
        return
    B = labels.numel()
    lens = rowptr[1:] - rowptr[:-1]
    row = torch.repeat_interleave(torch.arange(B, device=w.device), lens)
    dot = torch.zeros(B, dtype=w.dtype, device=w.device).index_add_(0, row, w[cols] * vals)
    p = torch.sigmoid(dot)
    y = labels.clamp_min(0)
    err = alpha * (y - p)
    if delta is not None:
        delta.index_add_(0, cols, err[row] * vals)
    if correct is not None:
        correct += ((p > 0.5) == (y > 0.5)).float().sum()


def kmeans_assign_csr(rowptr, cols, vals, C, assign=None, dist=None):
    """Nearest centre of every sparse point (CSR rowptr [n+1], cols / vals [nnz]) among the dense
    centres C [k, d] fp32 (kmeans_helper.hpp:45-66); optional squared distances. int32 assign."""
    n = rowptr.numel() - 1
    if assign is None:
        assign = torch.empty(n, dtype=torch.int32, device=C.device)
    if _gpu(C):
        cnorm = torch.empty(C.shape[0], dtype=torch.float32, device=C.device)
        kernels().kmeans_assign_csr(rowptr, cols, vals, C, cnorm, assign, dist)
        return assign
    lens = rowptr[1:] - rowptr[:-1]
    row = torch.repeat_interleave(torch.arange(n, device=C.device), lens)
    ok = cols < C.shape[1]
    xn = torch.zeros(n, dtype=torch.float32).index_add_(0, row, vals * vals)
    dots = torch.zeros(n, C.shape[0], dtype=torch.float32)
    dots.index_add_(0, row[ok], vals[ok, None] * C[:, cols[ok]].t())
    d2 = xn[:, None] - 2 * dots + (C * C).sum(1)[None]
    best, idx = d2.min(1)
    assign.copy_(idx.to(torch.int32))
    if dist is not None:
        dist.copy_(best.clamp_min(0))
    return assign


def kmeans_csr_accum(rowptr, cols, vals, assign, sums):
    """sums[assign[i], col] += val for every non-zero of every point."""
    if _gpu(sums):
        kernels().kmeans_csr_accum(rowptr, cols, vals, assign, sums)
        return sums
    n = rowptr.numel() - 1
    row = torch.repeat_interleave(torch.arange(n, device=sums.device), rowptr[1:] - rowptr[:-1])
    ok = cols < sums.shape[1]
    sums.index_put_((assign.to(torch.int64)[row[ok]], cols[ok]), vals[ok], accumulate=True)
    return sums


_KMEANS_CHUNK = 16384  # rows of S = X.C^T per GEMM (keeps the fp32 score block L2/MALL-sized)


def kmeans_assign(X, C, assign=None, dist=None, mfma=None):
    """Nearest centre of every row of X (fp32 [n, d]) among C (fp32 [k, d]); optional squared
    distance. GPU: the MFMA form (hi/lo-split bf16 GEMM for x.c, argmin kernel) unless the
    problem is tiny (or mfma=False: the one-wave-per-point fp32 kernel)."""
    if assign is None:
        assign = torch.empty(X.shape[0], dtype=torch.int32, device=X.device)
    if _gpu(X):
        n, d = X.shape
        k = C.shape[0]
        if mfma is None:
            mfma = n * k >= 1 << 16 and k >= 16
        if not mfma:
            kernels().kmeans_assign(X, C, assign, dist)
            return assign
        ld = (3 * d + 7) // 8 * 8
        Xc, Cc = X.contiguous(), C.contiguous()
        Cs = torch.empty(k, ld, dtype=torch.bfloat16, device=X.device)
        cn = torch.empty(k, dtype=torch.float32, device=X.device)
        kernels().kmeans_split3(Cc, Cs, 1, cn)
        xn = torch.empty(n, dtype=torch.float32, device=X.device)
        for r0 in range(0, n, _KMEANS_CHUNK):
            r1 = min(n, r0 + _KMEANS_CHUNK)
            Xs = torch.empty(r1 - r0, ld, dtype=torch.bfloat16, device=X.device)
            kernels().kmeans_split3(Xc[r0:r1], Xs, 0, xn[r0:r1])
            S = torch.empty(r1 - r0, k, dtype=torch.float32, device=X.device)
            gemm(Xs, Cs, S, r1 - r0, k, ld, False, False, EPI_STORE_F32)
            kernels().kmeans_argmin(S, cn, xn[r0:r1], assign[r0:r1], None if dist is None else dist[r0:r1])
        return assign
    d = torch.cdist(X.double(), C.double()) ** 2
    best, idx = d.min(1)
    assign.copy_(idx.to(torch.int32))
    if dist is not None:
        dist.copy_(best.to(dist.dtype))
    return assign


# ----------------------------------------------------------------------------- dense models
def layernorm_fwd(x, C, gamma, beta, eps, y, mean, rstd):
    if _gpu(x):
        kernels().layernorm_fwd(x, int(C), gamma, beta, float(eps), y, mean, rstd)
        return y
    xf = x[:, :C].float()
    mu = xf.mean(1)
    var = (xf * xf).mean(1) - mu * mu
    rs = torch.rsqrt(var.clamp_min(0) + eps)
    y[:, :C] = ((xf - mu[:, None]) * rs[:, None] * gamma.float() + beta.float()).to(torch.bfloat16)
    mean.copy_(mu)
    rstd.copy_(rs)
    return y


def layernorm_bwd(x, dy, C, gamma, mean, rstd, dx, dgamma, dbeta, accumulate=False):
    if _gpu(x):
        kernels().layernorm_bwd(x, dy, int(C), gamma, mean, rstd, dx, dgamma, dbeta, bool(accumulate))
        return dx
    xh = (x[:, :C].float() - mean[:, None]) * rstd[:, None]
    d = dy[:, :C].float()
    g = d * gamma.float()
    a = g.mean(1, keepdim=True)
    b = (g * xh).mean(1, keepdim=True)
    v = rstd[:, None] * (g - a - xh * b)
    if accumulate:
        v = v + dx[:, :C].float()
    dx[:, :C] = v.to(torch.bfloat16)
    dgamma += (d * xh).sum(0)
    dbeta += d.sum(0)
    return dx


def softmax_xent(logits, V, labels, scale, loss_sum, correct=None):
    """In place: logits[:, :V] <- (softmax - onehot) * scale (bf16); loss_sum += sum CE."""
    if _gpu(logits):
        kernels().softmax_xent(logits, int(V), labels, float(scale), loss_sum, correct)
        return logits
    z = logits[:, :V].float()
    lse = torch.logsumexp(z, 1)
    loss_sum += (lse - z.gather(1, labels[:, None]).squeeze(1)).sum()
    if correct is not None:
        correct += (z.argmax(1) == labels).float().sum()
    p = torch.softmax(z, 1)
    p[torch.arange(z.shape[0]), labels] -= 1.0
    logits[:, :V] = (p * scale).to(torch.bfloat16)
    return logits


def causal_softmax_fwd(S, T, P):
    if _gpu(S):
        kernels().causal_softmax_fwd(S, int(T), P)
        return P
    s = S.reshape(-1, T, T).float()
    mask = torch.ones(T, T, dtype=torch.bool).triu(1)
    P.view(-1, T, T).copy_(torch.softmax(s.masked_fill(mask, float("-inf")), -1).to(P.dtype))
    return P


def causal_softmax_bwd(P, dP, T, scale, dS):
    if _gpu(P):
        kernels().causal_softmax_bwd(P, dP, int(T), float(scale), dS)
        return dS
    p = P.reshape(-1, T, T).float()
    dp = dP.reshape(-1, T, T).float()
    mask = torch.ones(T, T, dtype=torch.bool).triu(1)
    dp = dp.masked_fill(mask, 0.0)
    ds = p * (dp - (p * dp).sum(-1, keepdim=True)) * scale
    dS.view(-1, T, T).copy_(ds.to(dS.dtype))
    return dS


def gelu_bwd(dh, u, du):
    if _gpu(u):
        kernels().gelu_bwd(dh, u, du)
        return du
    du.copy_((dh.float() * _gelu_grad(u.float())).to(du.dtype))
    return du


def add_bf16(a, b, out):
    if _gpu(a):
        kernels().add_bf16(a, b, out)
        return out
    out.copy_((a.float() + b.float()).to(out.dtype))
    return out


def _attn_heads(x, B, T, H, col0):
    hd = 64
    return x[:, col0: col0 + H * hd].float().reshape(B, T, H, hd).transpose(1, 2)


def attn_fwd(qkv, B, T, H, scale, O, lse):
    """Fused causal attention (head dim 64): O[:, h*64:] = softmax(mask(Q K^T scale)) V per head,
    lse [B*H*T] = log2-sum-exp2 of the scaled scores (log2 units, for the backward)."""
    if _gpu(qkv):
        kernels().attn_fwd(qkv, int(B), int(T), int(H), float(scale), O, lse)
        return O
    d = H * 64
    q, k, v = (_attn_heads(qkv, B, T, H, c) for c in (0, d, 2 * d))
    s = (q @ k.transpose(-1, -2)) * scale
    s = s.masked_fill(torch.ones(T, T, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    lse.view(B, H, T).copy_(torch.logsumexp(s, -1) * (1.0 / math.log(2.0)))
    o = torch.softmax(s, -1) @ v
    O[:, :d] = o.transpose(1, 2).reshape(B * T, d).to(O.dtype)
    return O


def attn_bwd(qkv, O, dO, lse, delta, B, T, H, scale, dqkv):
    """Backward of attn_fwd: writes dQ|dK|dV into dqkv [B*T, 3*H*64]; delta is [B*H*T] scratch."""
    if _gpu(qkv):
        kernels().attn_bwd(qkv, O, dO, lse, delta, int(B), int(T), int(H), float(scale), dqkv)
        return dqkv
    d = H * 64
    q, k, v = (_attn_heads(qkv, B, T, H, c) for c in (0, d, 2 * d))
    o = _attn_heads(O, B, T, H, 0)
    do = _attn_heads(dO, B, T, H, 0)
    s = (q @ k.transpose(-1, -2)) * scale
    mask = torch.ones(T, T, dtype=torch.bool, device=s.device).triu(1)
    p = torch.exp2(s * (1.0 / math.log(2.0)) - lse.view(B, H, T, 1)).masked_fill(mask, 0.0)
    dl = (do * o).sum(-1, keepdim=True)
    delta.view(B, H, T).copy_(dl.squeeze(-1))
    dv = p.transpose(-1, -2) @ do
    ds = p * (do @ v.transpose(-1, -2) - dl)
    dq = ds @ k * scale
    dk = ds.transpose(-1, -2) @ q * scale
    for i, t in enumerate((dq, dk, dv)):
        dqkv[:, i * d: (i + 1) * d] = t.transpose(1, 2).reshape(B * T, d).to(dqkv.dtype)
    return dqkv


_U64 = (1 << 64) - 1


def _mix64_int(x: int) -> int:
    x ^= x >> 33
    x = (x * 0xFF51AFD7ED558CCD) & _U64
    x ^= x >> 33
    x = (x * 0xC4CEB9FE1A85EC53) & _U64
    x ^= x >> 33
    return x


def hash_slots(tab_keys, q, slots, vals, init_scale, seed, counters, n_dev=None):
    """Lookup-or-insert of q in the open-addressing table (EMPTY = -1), linear probing from
    mix64(key); new rows are zero or uniform[-a, a) from mix64(key*golden + seed + c). With
    ``n_dev`` (device int64 count) only q[:n_dev] is resolved; the rest get slot -1."""
    if _gpu(q):
        kernels().hash_slots(tab_keys, q, slots, vals, float(init_scale), int(seed), counters, n_dev)
        return slots
    if n_dev is not None:
        n = int(n_dev.reshape(-1)[0])
        slots[n:] = -1
        q, slots = q[:n], slots[:n]
    cap = tab_keys.numel()
    W = vals.shape[1]
    tk = tab_keys.tolist()
    out = []
    for k in q.tolist():
        s = _mix64_int(k & _U64) & (cap - 1)
        found = -1
        for _ in range(cap):
            if tk[s] == k:
                found = s
                break
            if tk[s] == -1:
                tk[s] = k
                tab_keys[s] = k
                if init_scale != 0.0:
                    row = []
                    for c in range(W):
                        h = _mix64_int(((k & _U64) * 0x9E3779B97F4A7C15 + seed + c) & _U64)
                        row.append(init_scale * (2.0 * float(h >> 40) / 16777216.0 - 1.0))
                    vals[s] = torch.tensor(row, dtype=vals.dtype)
                else:
                    vals[s] = 0
                counters[0] += 1
                found = s
                break
            s = (s + 1) & (cap - 1)
        if found < 0:
            counters[1] += 1
        out.append(found)
    slots[: len(out)] = torch.tensor(out, dtype=torch.int64)
    return slots


def hash_rehash(old_keys, old_vals, old_state, new_keys, new_vals, new_state, counters):
    if _gpu(old_keys):
        kernels().hash_rehash(old_keys, old_vals, old_state, new_keys, new_vals, new_state, counters)
        return
    occ = (old_keys != -1).nonzero().reshape(-1)
    slots = torch.empty(occ.numel(), dtype=torch.int64)
    hash_slots(new_keys, old_keys[occ], slots, new_vals, 0.0, 0, counters)
    new_vals[slots] = old_vals[occ]
    if old_state is not None:
        new_state[slots] = old_state[occ]


def embed_fwd(wte, wpe, tok, T, out):
    """out[m, :C] = wte[tok[m]] + wpe[m % T] (bf16)."""
    if _gpu(wte):
        kernels().embed_fwd(wte, wpe, tok.reshape(-1), int(T), out)
        return out
    t = tok.reshape(-1)
    C = wte.shape[1]
    pos = torch.arange(t.numel()) % T
    out[:, :C] = (wte[t].float() + wpe[pos].float()).to(out.dtype)
    return out


def embed_bwd(dx, tok, T, dwte, dwpe):
    """dwte[tok[m]] += dx[m, :C]; dwpe[m % T] += dx[m, :C] (fp32 accumulators)."""
    if _gpu(dx):
        kernels().embed_bwd(dx, tok.reshape(-1), int(T), dwte, dwpe)
        return
    t = tok.reshape(-1)
    C = dwte.shape[1]
    d = dx[:, :C].float()
    dwte.index_add_(0, t, d)
    dwpe.index_add_(0, torch.arange(t.numel()) % T, d)


def dlrm_interact_fwd(V, NV, D, out, dense_idx=0):
    """V [B, NV, D] bf16 -> out[b] = [V[b,dense_idx] | V_i . V_j for i > j (lower triangle, row-major)]."""
    if _gpu(V):
        kernels().dlrm_interact_fwd(V, int(NV), int(D), int(dense_idx), out)
        return out
    v = V.reshape(-1, NV, D).float()
    z = v @ v.transpose(1, 2)
    ii, jj = torch.tril_indices(NV, NV, -1)
    out[:, :D] = V.reshape(-1, NV, D)[:, dense_idx]
    out[:, D: D + ii.numel()] = z[:, ii, jj].to(out.dtype)
    return out


def dlrm_interact_bwd(V, NV, D, dout, dV, d_dense, dense_idx=0):
    """dV fp32 [B, NV*D]; d_dense bf16 [B, D] = dV[:, dense_idx] * (V[:, dense_idx] > 0)."""
    if _gpu(V):
        kernels().dlrm_interact_bwd(V, int(NV), int(D), int(dense_idx), dout, dV, d_dense)
        return dV
    v = V.reshape(-1, NV, D).float()
    B = v.shape[0]
    ii, jj = torch.tril_indices(NV, NV, -1)
    dz = torch.zeros(B, NV, NV)
    g = dout[:, D: D + ii.numel()].float()
    dz[:, ii, jj] = g
    dz[:, jj, ii] = g
    d = dz @ v
    d[:, dense_idx] += dout[:, :D].float()
    dV.view(B, NV, D).copy_(d)
    d_dense.copy_(torch.where(v[:, dense_idx] > 0, d[:, dense_idx], torch.zeros_like(d[:,
                                                                                       dense_idx])).to(d_dense.dtype))
    return dV


def kaiming_uniform_(w: torch.Tensor, fan_in: int, gen=None):
    bound = 1.0 / math.sqrt(fan_in)
    return w.uniform_(-bound, bound, generator=gen)
