"""Every GEMM kernel variant against the fp32 reference, incl. M/N/K tails, split-K and batched
mode. The tile/kernel choice is read from the environment once per process, so each variant runs
in its own subprocess (one at a time): the LDS-DMA v2 kernel at its three tiles (256x256 with 16
waves, 256x128, 128x128) and the register-staged v1 (the > 2 GiB operand fallback)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHECK = r'''
import torch
from minips_amd import ops
dev = torch.device("cuda", 0)
bf = lambda x: x.to(torch.bfloat16)
worst = 0.0
for (M, N, K) in [(256, 256, 64), (520, 264, 200), (1000, 776, 848), (64, 1024, 1032), (300, 2048, 72),
                  (4160, 4200, 72)]:  # (>= 16 x 16 tiles: the grouped wide-grid order)
    for layout in ("nt", "nn", "tn"):
        a_km, b_kn = {"nt": (False, False), "nn": (False, True), "tn": (True, True)}[layout]
        if (a_km and M % 8) or (b_kn and N % 8):
            continue
        g = torch.Generator().manual_seed(M + N + K)
        A = bf(torch.randn(K if a_km else M, M if a_km else K, generator=g))
        B = bf(torch.randn(K if b_kn else N, N if b_kn else K, generator=g))
        ref = (A.float().t() if a_km else A.float()) @ (B.float() if b_kn else B.float().t())
        for split in ((1, 3) if layout == "tn" else (1,)):
            C = torch.zeros(M, N, device=dev) if split > 1 else torch.full((M, N), float("nan"), device=dev)
            epi = ops.EPI_ATOMIC_F32 if split > 1 else ops.EPI_STORE_F32
            ops.gemm(A.to(dev), B.to(dev), C, M, N, K, a_km, b_kn, epi, split_k=split)
            err = float((C.cpu() - ref).abs().max()) / (K ** 0.5)
            assert err < 3e-3, (M, N, K, layout, split, err)
            worst = max(worst, err)
# wgrad through linear_wgrad (default split choice), accumulating into a non-zero dW
dy = bf(torch.randn(4096, 520))
x = bf(torch.randn(4096, 264))
dW = torch.ones(520, 264, device=dev)
ops.linear_wgrad(dy.to(dev), x.to(dev), dW)
ref = 1.0 + dy.float().t() @ x.float()
assert float((dW.cpu() - ref).abs().max()) < 0.2, float((dW.cpu() - ref).abs().max())
# back-to-back split-K wgrads on one stream (slab workspace reuse), many splits, M/N tails
for it, (Mw, Nw, Kw, sp) in enumerate([(8192, 1024, 848, 8), (8192, 520, 264, 16), (2048, 264, 136, 5),
                                       (8192, 1024, 848, 8), (4096, 256, 1032, 2)]):
    g = torch.Generator().manual_seed(it)
    dy = bf(torch.randn(Mw, Nw, generator=g)); x = bf(torch.randn(Mw, Kw, generator=g))
    dW = torch.full((Nw, Kw), 0.5, device=dev)
    ops.linear_wgrad(dy.to(dev), x.to(dev), dW, split_k=sp)
    ref = 0.5 + dy.float().t() @ x.float()
    e = float((dW.cpu() - ref).abs().max()) / (Mw ** 0.5)
    assert e < 3e-3, (it, Mw, Nw, Kw, sp, e)
# batched (attention-style strided) GEMM
Bt, Mb, Nb, Kb = 3, 200, 136, 64
A = bf(torch.randn(Bt, Mb, Kb)); B = bf(torch.randn(Bt, Nb, Kb))
C = torch.empty(Bt, Mb, Nb, device=dev)
ops.gemm_batched(A.to(dev), B.to(dev), C, Mb, Nb, Kb, False, False, ops.EPI_STORE_F32, Bt, 1, Kb, Kb, Nb,
                 (Mb * Kb, 0, Nb * Kb, 0, Mb * Nb, 0))
ref = A.float() @ B.float().transpose(1, 2)
assert float((C.cpu() - ref).abs().max()) < 0.05
print("ok", worst)
'''


@pytest.mark.parametrize("env", [
    {"MINIPS_GEMM_TILE": "256"},                                # v2 256x256 everywhere
    {"MINIPS_GEMM_TILE": "200"},                                # v2 256x128 everywhere
    {"MINIPS_GEMM_TILE": "128"},                                # v2 128x128 everywhere
    {"MINIPS_GEMM_TILE": "1"},                                  # the register-staged v1 (> 2 GiB operands)
    {},                                                         # defaults (tile by wave quantisation)
])
def test_gemm_variant(env):
    e = dict(os.environ, **env)
    r = subprocess.run([sys.executable, "-c", CHECK], cwd=ROOT, env=e, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, (env, r.stdout[-2000:], r.stderr[-3000:])
