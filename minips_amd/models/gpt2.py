"""GPT-2-small trained through the GPU parameter server (BASELINE config 4): every dense
parameter lives in ONE DenseTable whose fp32 master + Adam state are sharded over the PS ranks
(reduce-scatter of gradients, fused Adam on the owned shard, all-gather of the bf16 pull).

Architecture (GPT-2 small): vocab 50257 (padded to 50304 rows), context 1024, d_model 768,
12 layers x 12 heads, pre-LayerNorm blocks, GELU(tanh) MLP 768 -> 3072 -> 768, tied LM head.

Compute path (all gfx950 kernels from minips_amd.ops, no autograd):
  embed_fwd                   x0 = wte[tok] + wpe[pos]
  layernorm_fwd               into a bias-folded activation (ones column at 768)
  gemm (bias epilogue)        qkv = ln1 W_qkv^T
  attn_fwd                    fused causal flash attention (MFMA, online softmax; Q/K/V read in
                              place from qkv, O written into the bias-folded proj input, only
                              the per-query log-sum-exp kept for the backward)
  gemm + add_bf16             x_mid = x + O W_o^T
  gemm (GELU-aux epilogue)    g = gelu(ln2 W_fc^T), gelu'(u) saved for the fc2 dgrad
  gemm + add_bf16             x_next = x_mid + g W_proj^T
  gemm                        logits = ln_f(x) wte^T (bf16)
  softmax_xent                row logsumexp and (softmax - onehot) / (B T) in place (one pass)
The backward mirrors it with dgrad/wgrad GEMMs (GELU-grad epilogue), attn_bwd (recomputes P per
tile; dQ and dK/dV sweeps), layernorm_bwd (accumulating into the residual gradient) and embed_bwd.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .. import ops
from ..ps.comm import Comm
from ..ps.tables import DenseTable
from .layers import SideStream, Linear, ParamLayout, align, ext_activation


@dataclass
class GPT2Config:
    vocab: int = 50257
    n_ctx: int = 1024
    d: int = 768
    n_layer: int = 12
    n_head: int = 12
    lr: float = 3e-4
    weight_decay: float = 0.0
    consistency: str = "bsp"
    staleness: int = 0
    seed: int = 0
    # multi-rank: per-layer gradient buckets (~28 MB each at GPT-2 small) reduced + applied +
    # re-gathered as soon as the layer's backward finished (DenseTable bucket_ready)
    bucketed: bool = True
    # one rank: the clock on the table's side stream too, each layer's bucket applied (Adam) as
    # soon as its backward finished, overlapping the rest of the backward (DenseTable overlap_w1;
    # GPT2_OVERLAP_W1 off: one Adam over the whole table after the backward)
    overlap_w1: bool = True

    @property
    def vocab_pad(self):
        return align(self.vocab, 64)


_WGRAD_DEFER_GPT2 = False
# the LM-head dgrad (K = the 50304-row vocabulary, only 8192 x 768 outputs): split-K into fp32 slabs
# + one bf16 reduce; 8 splits measured best (764 vs 906 / 970 us at 4 / 12, profiles/r4/gemm_lm_head_splits.txt;
# in the round-5 step 13.25-13.28 ms vs 13.29-13.32 / 13.26 / 13.33-13.34 at 4 / 6 / 12,
# profiles/r5/ab_gpt2_lm_split.txt).
# All three LM-head GEMMs (logits, dgrad, wte wgrad) run on gemm.hip (round 5: the hipBLASLt path is gone)
_LM_DGRAD_SPLIT = 8
# the wte weight gradient (50304 x 768 outputs, K = 8192 tokens) on 256x256 tiles: 746 vs 835 us
# isolated at the launcher's 128x128 choice (its wave quantisation, 591 vs 2358 tiles, favours 128;
# the 256 tile moves half the L2->LDS bytes per MFMA), hipBLASLt 635; in the step 12.89-12.91 vs
# 13.19-13.22 ms (635 vs 620 K tokens/s; profiles/r6/lm_head_tiles.txt)
_LM_WGRAD_TILE = 256
# MLP: the fc forward saves gelu'(u) (its tanh is computed there anyway) and the fc2 dgrad multiplies
# by it; GPT2_GELU_D off saves u and re-evaluates tanh in the dgrad epilogue
_GELU_D = True
# per-layer weight gradients: split-K gemm.hip (the hipBLASLt form, GPT2_WGRAD=lib, measured
# 13.0-13.1 vs 12.78 ms/step in round 3 and was removed in round 4)


class GPT2:
    def __init__(self, cfg: GPT2Config, comm: Comm):
        assert cfg.d == 64 * cfg.n_head, "the attention kernels are specialised for head dim 64"
        self.cfg, self.comm = cfg, comm
        d = cfg.d
        L = ParamLayout()
        self.layout = L
        L.add("wte", (cfg.vocab_pad, d))
        L.add("wpe", (cfg.n_ctx, d))
        self.blocks = []
        for i in range(cfg.n_layer):
            blk = dict(
                ln1_g=L.add(f"h{i}.ln1_g", (d,)), ln1_b=L.add(f"h{i}.ln1_b", (d,)),
                qkv=Linear(L, f"h{i}.qkv", d, 3 * d),
                proj=Linear(L, f"h{i}.proj", d, d),
                ln2_g=L.add(f"h{i}.ln2_g", (d,)), ln2_b=L.add(f"h{i}.ln2_b", (d,)),
                fc=Linear(L, f"h{i}.fc", d, 4 * d),
                fc2=Linear(L, f"h{i}.fc2", 4 * d, d),
            )
            self.blocks.append(blk)
        L.add("lnf_g", (d,))
        L.add("lnf_b", (d,))
        starts = [L.entries[f"h{i}.ln1_g"][0] for i in range(cfg.n_layer)] if cfg.bucketed else None
        self.table = DenseTable(comm, L.size, optimizer="adam", lr=cfg.lr, consistency=cfg.consistency,
                                staleness=cfg.staleness, weight_decay=cfg.weight_decay, betas=(0.9, 0.95),
                                buckets=starts, overlap_w1=cfg.overlap_w1)
        self._layer_bucket = [self.table.bucket_for_layer(x) for x in starts] if starts else None
        g = torch.Generator().manual_seed(cfg.seed)
        full = torch.zeros(L.size)
        L.view(full, "wte")[: cfg.vocab].normal_(0.0, 0.02, generator=g)
        L.view(full, "wpe").normal_(0.0, 0.01, generator=g)
        proj_std = 0.02 / math.sqrt(2 * cfg.n_layer)
        for blk in self.blocks:
            for name in ("ln1_g", "ln2_g"):
                L.view(full, blk[name]).fill_(1.0)
            blk["qkv"].init(full, g, std=0.02)
            blk["fc"].init(full, g, std=0.02)
            blk["proj"].init(full, g, std=proj_std)
            blk["fc2"].init(full, g, std=proj_std)
        L.view(full, "lnf_g").fill_(1.0)
        self.table.load_full(full)
        self._bufs = {}
        self._side = SideStream(comm.device)

    @property
    def n_params(self):
        c = self.cfg
        return c.vocab * c.d + c.n_ctx * c.d + c.n_layer * (12 * c.d * c.d + 13 * c.d) + 2 * c.d

    # ------------------------------------------------------------------------------ buffers
    def _buffers(self, B, T):
        key = (B, T)
        if key not in self._bufs:
            c, dev = self.cfg, self.comm.device
            M, d, H = B * T, c.d, c.n_head
            bf = dict(dtype=torch.bfloat16, device=dev)
            f32 = dict(dtype=torch.float32, device=dev)
            nl = c.n_layer
            self._bufs[key] = dict(
                x=[torch.empty(M, d, **bf) for _ in range(nl + 1)],       # residual stream per layer input
                xm=[torch.empty(M, d, **bf) for _ in range(nl)],          # after attention
                h1=[ext_activation(M, d, dev) for _ in range(nl)],        # ln1 out (+ ones column)
                h2=[ext_activation(M, d, dev) for _ in range(nl)],
                st1=[(torch.empty(M, **f32), torch.empty(M, **f32)) for _ in range(nl)],
                st2=[(torch.empty(M, **f32), torch.empty(M, **f32)) for _ in range(nl)],
                qkv=[torch.empty(M, 3 * d, **bf) for _ in range(nl)],
                lse=[torch.empty(B * H * T, **f32) for _ in range(nl)],  # attention log-sum-exp
                ao=[ext_activation(M, d, dev) for _ in range(nl)],        # attention out (+ ones)
                u=[torch.empty(M, 4 * d, **bf) for _ in range(nl)],       # pre-GELU
                g=[ext_activation(M, 4 * d, dev) for _ in range(nl)],     # GELU out (+ ones)
                # ln_f output: only the LM head reads it (no bias column), contiguous rows
                hf=torch.empty(M, d, **bf), stf=(torch.empty(M, **f32), torch.empty(M, **f32)),
                logits=torch.empty(M, c.vocab_pad, **bf),
                delta=torch.empty(B * H * T, **f32),
                tmp=torch.empty(M, d, **bf), dx=torch.empty(M, d, **bf), dh=torch.empty(M, d, **bf),
                dqkv=torch.empty(M, 3 * d, **bf), dao=torch.empty(M, d, **bf), du=torch.empty(M, 4 * d, **bf),
                loss=torch.zeros(1, **f32),
            )
        return self._bufs[key]

    # ------------------------------------------------------------------------------ step
    def train_step(self, tokens, targets):
        """tokens/targets [B, T] int64. Returns the summed token cross-entropy (device scalar)."""
        c = self.cfg
        B, T = tokens.shape
        assert T <= c.n_ctx and T % 8 == 0
        M, d = B * T, c.d
        scale = 1.0 / math.sqrt(d // c.n_head)
        b = self._buffers(B, T)
        L = self.layout
        P = self.table.get()
        G = self.table.grad
        v = lambda buf, name: L.view(buf, name)  # noqa: E731
        x = b["x"]
        ops.embed_fwd(v(P, "wte"), v(P, "wpe"), tokens, T, x[0])
        for i, blk in enumerate(self.blocks):
            m1, r1 = b["st1"][i]
            ops.layernorm_fwd(x[i], d, v(P, blk["ln1_g"]), v(P, blk["ln1_b"]), 1e-5, b["h1"][i], m1, r1)
            blk["qkv"].forward(P, b["h1"][i], b["qkv"][i], "none")
            ops.attn_fwd(b["qkv"][i], B, T, c.n_head, scale, b["ao"][i], b["lse"][i])
            blk["proj"].forward(P, b["ao"][i], b["tmp"], "none")
            ops.add_bf16(x[i], b["tmp"], b["xm"][i])
            m2, r2 = b["st2"][i]
            ops.layernorm_fwd(b["xm"][i], d, v(P, blk["ln2_g"]), v(P, blk["ln2_b"]), 1e-5, b["h2"][i], m2, r2)
            blk["fc"].forward(P, b["h2"][i], b["g"][i], "gelu_daux" if _GELU_D else "gelu_aux", aux=b["u"][i])
            blk["fc2"].forward(P, b["g"][i], b["tmp"], "none")
            ops.add_bf16(b["xm"][i], b["tmp"], x[i + 1])
        mf, rf = b["stf"]
        hf = b["hf"]
        ops.layernorm_fwd(x[-1], d, v(P, "lnf_g"), v(P, "lnf_b"), 1e-5, hf, mf, rf)
        wte = v(P, "wte")
        logits = b["logits"]
        b["loss"].zero_()
        # plain GEMM + the block-per-row softmax-xent (row reduction + gradient in place, one kernel);
        # (round 3's softmax partials in the GEMM epilogue measured 13.87 vs 14.14 ms/step: removed)
        ops.gemm(hf[:, :d], wte, logits, M, c.vocab_pad, d, False, False, ops.EPI_STORE_BF16)
        ops.softmax_xent(logits, c.vocab, targets.reshape(-1), 1.0 / (M * self.comm.world), b["loss"])
        # ---- backward. Weight gradients fork onto a side stream beside the dgrad chain; before the
        # chain overwrites a buffer a forked wgrad reads (dx, du, dqkv), it waits for that wgrad.
        side = self._side
        dh = b["dh"]
        with side.fork():
            ops.linear_wgrad(logits, hf[:, :d], v(G, "wte"), tile=_LM_WGRAD_TILE)
        # long K (the vocabulary), few outputs: split-K into fp32 slabs + one bf16 reduce
        ops.gemm(logits, wte, dh, M, d, c.vocab_pad, False, True, ops.EPI_STORE_BF16, split_k=_LM_DGRAD_SPLIT)
        dx = b["dx"]
        ops.layernorm_bwd(x[-1], dh, d, v(P, "lnf_g"), mf, rf, dx, v(G, "lnf_g"), v(G, "lnf_b"))
        ev_du = ev_dqkv = None
        # GPT2_WGRAD_DEFER on: the per-layer weight gradients' split-K planes folded by their
        # bucket's Adam instead of reduce kernels -- measured neutral here (12.66-12.68 vs 12.48-12.64
        # ms/step; profiles/r4/ab_gpt2_knobs.txt), so the reduces stay by default
        sink = self.table.slab_sink() if _WGRAD_DEFER_GPT2 and hasattr(self.table, "slab_sink") else None
        for i in range(c.n_layer - 1, -1, -1):
            blk = self.blocks[i]
            # MLP branch
            with side.fork():
                blk["fc2"].wgrad(G, dx, b["g"][i], sink)
            ev_dx = side.mark()
            side.wait(ev_du)  # du: read by the previous layer's fc wgrad
            if _GELU_D:
                blk["fc2"].dgrad(P, dx, b["du"], gelu_d=b["u"][i])
            else:
                blk["fc2"].dgrad(P, dx, b["du"], gelu_u=b["u"][i])
            with side.fork():
                blk["fc"].wgrad(G, b["du"], b["h2"][i], sink)
            ev_du = side.mark()
            blk["fc"].dgrad(P, b["du"], dh)
            m2, r2 = b["st2"][i]
            side.wait(ev_dx)  # dx accumulates next
            ops.layernorm_bwd(b["xm"][i], dh, d, v(P, blk["ln2_g"]), m2, r2, dx, v(G, blk["ln2_g"]),
                              v(G, blk["ln2_b"]), accumulate=True)
            # attention branch
            with side.fork():
                blk["proj"].wgrad(G, dx, b["ao"][i], sink)
            ev_dx = side.mark()
            blk["proj"].dgrad(P, dx, b["dao"])
            side.wait(ev_dqkv)  # dqkv: read by the previous layer's qkv wgrad
            ops.attn_bwd(b["qkv"][i], b["ao"][i], b["dao"], b["lse"][i], b["delta"], B, T, c.n_head, scale, b["dqkv"])
            with side.fork():
                blk["qkv"].wgrad(G, b["dqkv"], b["h1"][i], sink)
            ev_dqkv = side.mark()
            blk["qkv"].dgrad(P, b["dqkv"], dh)
            m1, r1 = b["st1"][i]
            side.wait(ev_dx)
            ops.layernorm_bwd(x[i], dh, d, v(P, blk["ln1_g"]), m1, r1, dx, v(G, blk["ln1_g"]), v(G, blk["ln1_b"]),
                              accumulate=True)
            if self._layer_bucket is not None:  # layer i's gradients are final: send its bucket
                self.table.bucket_ready(self._layer_bucket[i], events=(side.mark(),))
        side.join()  # embed_bwd accumulates into the wte gradient the LM-head wgrad wrote
        ops.embed_bwd(dx, tokens, T, v(G, "wte"), v(G, "wpe"))
        self.table.add()
        self.table.clock()
        return b["loss"]

    def drain(self):
        self.table.drain()
