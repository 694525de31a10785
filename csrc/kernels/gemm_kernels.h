// bf16 MFMA GEMM kernel templates for gfx950 (included by gemm.hip and the per-layout
// translation units gemm_l*.hip, which instantiate one operand layout each so the build runs in
// parallel).
//
// bf16 MFMA GEMM for gfx950 with fused epilogues (worker forward/backward of the MLP
// towers: Wide&Deep deep tower, DLRM bottom/top MLPs, the 3-layer MLP, GPT-2 projections).
//
//   C[M,N] = A . B   (fp32 accumulate on v_mfma_f32_16x16x32_bf16)
//   A stored MK ([M][K], k contiguous)  or KM ([K][M], m contiguous)
//   B stored NK ([N][K], a Linear weight) or KN ([K][N], n contiguous)
//   forward   Y = act(X W^T + b):        A=X  (MK), B=W  (NK)
//   dgrad     dX = (dY W) * mask:        A=dY (MK), B=W  (KN)
//   wgrad     dW += dY^T X  (split-K):   A=dY (KM), B=X  (KN)
//
// Tiling: 128x128x32 block tile, 256 threads = 4 waves in 2x2, each wave 64x64 = 4x4 MFMA
// 16x16 tiles (64 accumulator VGPRs). Operands are staged global -> registers -> LDS with a
// one-tile register prefetch (the next tile's loads are in flight during the MFMAs). MK/NK
// tiles live in LDS as [row][k] and are read with ds_read_b128; KM/KN tiles live as
// [k][row] and are read with the gfx950 transposing ds_read_b64_tr_b16, so no operand is
// ever transposed in memory. When both operands are tr-read (wgrad) the k order inside a
// 32-wide step is permuted identically on both sides so that each 32-lane half reads 8
// consecutive LDS rows (bank-conflict free with the 288-B row pitch).
// Block ids are remapped so that consecutive tiles of one row panel share an XCD (T1).
#pragma once
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"

namespace minips_k {

typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128;

template <int BK>
struct Lds {
  static constexpr int ROW = BK + 8;   // [row][k] pitch in bf16 (80 B at BK=32, 144 B at BK=64)
  static constexpr int TR = BM + 16;   // [k][row] pitch in bf16 (288 B)
  static constexpr int TILE = (BM * ROW > BK * TR) ? BM * ROW : BK * TR;
  static constexpr int CHUNKS = BM * BK / 8 / 256;  // 16-byte chunks per thread per operand tile
};

__device__ __forceinline__ v4s ds_read_tr16(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}

// Loads one BMxBK (or BKxBM) tile into registers: CHUNKS x 16 B per thread.
template <int BK, bool KMAJOR>
__device__ __forceinline__ void load_tile(const bf16_t* __restrict__ G, int ld, int row0, int k0, int rows, int K,
                                          int tid, uint4 (&r)[Lds<BK>::CHUNKS]) {
#pragma unroll
  for (int h = 0; h < Lds<BK>::CHUNKS; ++h) {
    int c = tid + h * 256;
    int row, k;
    if (!KMAJOR) {
      row = c / (BK / 8);
      k = (c % (BK / 8)) * 8;
    } else {
      k = c >> 4;
      row = (c & 15) * 8;
    }
    int gr = row0 + row, gk = k0 + k;
    bool ok = (gr < rows) && (gk < K);
    const bf16_t* src = !KMAJOR ? G + (int64_t)gr * ld + gk : G + (int64_t)gk * ld + gr;
    r[h] = ok ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
  }
}

template <int BK, bool KMAJOR>
__device__ __forceinline__ void store_tile(bf16_t* S, int tid, const uint4 (&r)[Lds<BK>::CHUNKS]) {
#pragma unroll
  for (int h = 0; h < Lds<BK>::CHUNKS; ++h) {
    int c = tid + h * 256;
    if (!KMAJOR) {
      *reinterpret_cast<uint4*>(S + (c / (BK / 8)) * Lds<BK>::ROW + (c % (BK / 8)) * 8) = r[h];
    } else {
      *reinterpret_cast<uint4*>(S + (c >> 4) * Lds<BK>::TR + (c & 15) * 8) = r[h];
    }
  }
}

// Fragment of the 16x16x32 operand for k sub-step `ks` (k in [32ks, 32ks+32)): 8 bf16 along
// k for row `row_base + lane&15` (A) / column (B).
template <int BK, bool KMAJOR, bool PERM>
__device__ __forceinline__ v8s read_frag(const bf16_t* S, int row_base, int ks, int lane) {
  int g = lane >> 4;
  if (!KMAJOR) {
    int row = row_base + (lane & 15);
    const bf16_t* p = S + row * Lds<BK>::ROW + 32 * ks;
    if (!PERM) return *reinterpret_cast<const v8s*>(p + 8 * g);
    v4s lo = *reinterpret_cast<const v4s*>(p + 4 * g);
    v4s hi = *reinterpret_cast<const v4s*>(p + 16 + 4 * g);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  } else {
    int i = lane & 15, q = i >> 2, p = i & 3;
    int r0 = 32 * ks + (PERM ? 4 * g : 8 * g);
    int r1 = 32 * ks + (PERM ? 16 + 4 * g : 8 * g + 4);
    v4s lo = ds_read_tr16(S + (r0 + q) * Lds<BK>::TR + row_base + 4 * p);
    v4s hi = ds_read_tr16(S + (r1 + q) * Lds<BK>::TR + row_base + 4 * p);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

struct EpiArgs {
  void* C;
  int ldc;
  const bf16_t* bias;    // [N] bf16 (pulled params are bf16)
  const bf16_t* mask;    // [M][ldmask] (relu mask source)
  int ldmask;
  float* colsum;         // [N] column sums of the (masked) output
  float alpha;
  // batched GEMM: z = blockIdx.y, offsets (z / inner) * s_outer + (z % inner) * s_inner
  int inner;
  int64_t sa_o, sa_i, sb_o, sb_i, sc_o, sc_i;
  int64_t sc_split;  // split-K slab mode: C += blockIdx.z * sc_split (0 = all splits share C)
  const int* perm;   // kEpiPermRowsBf16: segment positions [M][N / seg]
  int seg;
  // kEpiWdHead: the W&D output head folded into the last hidden layer's GEMM (see wd_head_epilogue)
  const float* head_wide = nullptr;   // [M] wide-part logits
  const float* head_label = nullptr;  // [M] labels (> 0.5 = positive)
  float* head_dwide = nullptr;        // [M] dLoss/dlogit (the wide part's gradient)
  float* head_loss = nullptr;         // [1] += sum of the BCE-with-logits losses
  float head_scale = 0.f;             // gradient scale (1 / global batch)
  float* head_dh_colsum = nullptr;    // [N] (stride head_dh_colsum_ld) += column sums of dH (optional)
  int head_dh_colsum_ld = 1;
  const bf16_t* head_bias = nullptr;  // [N] the hidden layer's bias (nullptr: folded into K)
  float* head_slab = nullptr;         // [workgroups + groups][2N + 2] partial rows of the fold
  unsigned* head_ticket = nullptr;    // 1 + groups tickets (zero before and after a launch)
  int colsum_ld = 1;                  // kEpiReluMaskBf16: colsum[col * colsum_ld] (a column of a matrix)
  // kEpiFoldF32: C is this K slice's slab plane; the tile's last slice adds every plane into
  // fold_out (ldc fold_ldc); fold_cnt[tile] counts the slices that arrived (the last one re-zeroes it)
  float* fold_out = nullptr;
  int fold_ldc = 0;
  unsigned* fold_cnt = nullptr;
  int fold_nsplit = 1;
  // split-K launches (gridDim.z > 1, gridDim.y == 1): deal (K slice, tile) pairs to the XCDs in
  // contiguous runs, tile fastest, so an XCD's workgroups share one K slice's operand rows through
  // its L2 (the plain tile remap gives each XCD whole tile rows over every slice: each XCD then
  // streams the full other operand)
  int zmap = 0;
};

// Destination of an output row segment (kEpiPermRowsBf16: the permuted row of its segment).
template <int EPI>
__device__ __forceinline__ int64_t out_offset(const EpiArgs& ep, int N, int row, int col) {
  if (EPI == kEpiPermRowsBf16) {
    const int s = col / ep.seg;
    return (int64_t)ep.perm[(int64_t)row * (N / ep.seg) + s] * ep.seg + (col - s * ep.seg);
  }
  return (int64_t)row * ep.ldc + col;
}

// Fused epilogue of one wave's (16 MR) x 64 accumulator block at rows mb.., cols nb...
template <int EPI, int MR>
__device__ __forceinline__ void epilogue_at(const v4f (&acc)[MR][4], const EpiArgs& ep, int M, int N, int mb, int nb,
                                            int lane) {
  const int col_l = lane & 15, row_q = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = nb + j * 16 + col_l;
    const bool col_ok = col < N;
    float bias = 0.f;
    if (EPI == kEpiBiasReluBf16 || EPI == kEpiBiasBf16 || EPI == kEpiBiasGeluBf16 || EPI == kEpiBiasGeluAuxBf16 ||
        EPI == kEpiBiasGeluDAuxBf16)
      bias = (ep.bias && col_ok) ? bf2f(ep.bias[col]) : 0.f;
    float csum = 0.f;
#pragma unroll
    for (int i = 0; i < MR; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mb + i * 16 + row_q + r;
        if (!(col_ok && row < M)) continue;
        float v = acc[i][j][r] * ep.alpha;
        const int64_t off = out_offset<EPI>(ep, N, row, col);
        if (EPI == kEpiStoreF32) {
          ((float*)ep.C)[off] = v;
        } else if (EPI == kEpiAccumF32) {
          ((float*)ep.C)[off] += v;
        } else if (EPI == kEpiAtomicF32) {
          atomicAdd(((float*)ep.C) + off, v);
        } else if (EPI == kEpiBiasReluBf16) {
          ((bf16_t*)ep.C)[off] = f2bf(fmaxf(v + bias, 0.f));
        } else if (EPI == kEpiBiasBf16) {
          ((bf16_t*)ep.C)[off] = f2bf(v + bias);
        } else if (EPI == kEpiBiasGeluBf16) {
          float x = v + bias;
          float t = tanhf(0.7978845608f * (x + 0.044715f * x * x * x));
          ((bf16_t*)ep.C)[off] = f2bf(0.5f * x * (1.f + t));
        } else if (EPI == kEpiStoreBf16 || EPI == kEpiPermRowsBf16 || EPI == kEpiXentStatsBf16) {
          ((bf16_t*)ep.C)[off] = f2bf(v);  // (kEpiXentStatsBf16: the launcher takes the staged path)
        } else if (EPI == kEpiBiasGeluAuxBf16) {
          const float x = v + bias;
          const float t = tanhf(0.7978845608f * (x + 0.044715f * x * x * x));
          ((bf16_t*)ep.C)[off] = f2bf(0.5f * x * (1.f + t));
          const_cast<bf16_t*>(ep.mask)[(int64_t)row * ep.ldmask + col] = f2bf(x);
        } else if (EPI == kEpiBiasGeluDAuxBf16) {
          const float x = v + bias;
          const float k = 0.7978845608f, c3 = 0.044715f;
          const float t = tanhf(k * (x + c3 * x * x * x));
          ((bf16_t*)ep.C)[off] = f2bf(0.5f * x * (1.f + t));
          const_cast<bf16_t*>(ep.mask)[(int64_t)row * ep.ldmask + col] =
              f2bf(0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * c3 * x * x));
        } else if (EPI == kEpiMulAuxBf16) {
          ((bf16_t*)ep.C)[off] = f2bf(v * bf2f(ep.mask[(int64_t)row * ep.ldmask + col]));
        } else if (EPI == kEpiGeluGradBf16) {
          const float u = bf2f(ep.mask[(int64_t)row * ep.ldmask + col]);
          const float k = 0.7978845608f, c3 = 0.044715f;
          const float t = tanhf(k * (u + c3 * u * u * u));
          const float gp = 0.5f * (1.f + t) + 0.5f * u * (1.f - t * t) * k * (1.f + 3.f * c3 * u * u);
          ((bf16_t*)ep.C)[off] = f2bf(v * gp);
        } else if (EPI == kEpiReluMaskBf16) {
          float m = bf2f(ep.mask[(int64_t)row * ep.ldmask + col]);
          float o = m > 0.f ? v : 0.f;
          bf16_t ob = f2bf(o);
          ((bf16_t*)ep.C)[off] = ob;
          csum += bf2f(ob);
        }
      }
    }
    if (EPI == kEpiReluMaskBf16 && ep.colsum) {
      csum += __shfl_xor(csum, 16, 64);
      csum += __shfl_xor(csum, 32, 64);
      if (lane < 16 && col_ok) atomicAdd(ep.colsum + (int64_t)col * ep.colsum_ld, csum);
    }
  }
}

// LDS-staged epilogue of one wave's (16 MR) x 64 accumulator block at rows mb.., cols nb.. (v2/v3).
// The accumulator fragments hold 4 rows x 1 column per lane (16 lanes per row), so storing them
// directly writes 2-byte (bf16) / 4-byte values in 32-64 B pieces: ~64 store instructions per
// wave per 64x64 block and partial cache lines. Instead each 16-row slice goes through a private
// per-wave LDS scratch [16][68] fp32 (row pitch 272 B: the ds_write_b32 fragment pattern is
// conflict-free), is read back row-contiguous and leaves as whole 128-B (bf16) / 256-B (fp32)
// row segments: 16-byte stores (8 bf16 or 4 fp32 per lane), 16-byte mask/aux accesses, one
// 256-B atomic wave-instruction per row for the split-K fp32 epilogue. Scalar tail path when a
// row segment is not 16-byte aligned or runs past N. `scr` = this wave's 16*68 floats of LDS,
// free once every wave has left the main loop (its final barrier).
constexpr int kScrPitch = 68;
constexpr int kScrFloats = 16 * kScrPitch;

template <int EPI>
__device__ __forceinline__ float epi_apply(float v, float bias, float m, bf16_t* aux_out) {
  if (EPI == kEpiBiasReluBf16) return fmaxf(v + bias, 0.f);
  if (EPI == kEpiBiasBf16) return v + bias;
  if (EPI == kEpiBiasGeluBf16 || EPI == kEpiBiasGeluAuxBf16 || EPI == kEpiBiasGeluDAuxBf16) {
    const float x = v + bias;
    if (EPI == kEpiBiasGeluAuxBf16) *aux_out = f2bf(x);
    const float k = 0.7978845608f, c3 = 0.044715f;
    const float t = tanhf(k * (x + c3 * x * x * x));
    if (EPI == kEpiBiasGeluDAuxBf16)
      *aux_out = f2bf(0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * c3 * x * x));
    return 0.5f * x * (1.f + t);
  }
  if (EPI == kEpiMulAuxBf16) return v * m;
  if (EPI == kEpiGeluGradBf16) {
    const float k = 0.7978845608f, c3 = 0.044715f;
    const float t = tanhf(k * (m + c3 * m * m * m));
    const float gp = 0.5f * (1.f + t) + 0.5f * m * (1.f - t * t) * k * (1.f + 3.f * c3 * m * m);
    return v * gp;
  }
  if (EPI == kEpiReluMaskBf16) return m > 0.f ? v : 0.f;
  return v;  // kEpiStoreBf16 / kEpiPermRowsBf16 / kEpiXentStatsBf16 / kEpiStoreF32
}

template <int EPI, int MR>
__device__ __forceinline__ void epilogue_lds(const v4f (&acc)[MR][4], const EpiArgs& ep, int M, int N, int mb, int nb,
                                             int lane, float* __restrict__ scr) {
  constexpr bool F32OUT = EPI == kEpiStoreF32 || EPI == kEpiAtomicF32 || EPI == kEpiAccumF32 || EPI == kEpiFoldF32;
  constexpr bool HAS_BIAS = EPI == kEpiBiasReluBf16 || EPI == kEpiBiasBf16 || EPI == kEpiBiasGeluBf16 ||
                            EPI == kEpiBiasGeluAuxBf16 || EPI == kEpiBiasGeluDAuxBf16;
  constexpr bool READ_MASK = EPI == kEpiReluMaskBf16 || EPI == kEpiGeluGradBf16 || EPI == kEpiMulAuxBf16;
  constexpr bool WRITE_AUX = EPI == kEpiBiasGeluAuxBf16 || EPI == kEpiBiasGeluDAuxBf16;
  const int col_l = lane & 15, row_q = (lane >> 4) * 4;
  // vector paths need 16-byte aligned row segments
  const bool c_vec = (EPI == kEpiPermRowsBf16 ? (ep.seg & 7) == 0 : (ep.ldc & (F32OUT ? 3 : 7)) == 0) &&
                     ((reinterpret_cast<uintptr_t>(ep.C) & 15) == 0);
  const bool m_vec = ((ep.ldmask & 7) == 0) && ((reinterpret_cast<uintptr_t>(ep.mask) & 15) == 0);
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // the bias depends on the column only: this lane's 8 columns are loaded once (one 16-byte
  // load when aligned), not per 16-row slice
  float bias[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (HAS_BIAS && ep.bias) {
    const int col = nb + (lane & 7) * 8;
    if (col + 8 <= N && (reinterpret_cast<uintptr_t>(ep.bias + col) & 15) == 0) {
      const uint4 bu = *reinterpret_cast<const uint4*>(ep.bias + col);
      const uint32_t w[4] = {bu.x, bu.y, bu.z, bu.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bias[2 * e] = __uint_as_float(w[e] << 16);
        bias[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) bias[e] = (col + e < N) ? bf2f(ep.bias[col + e]) : 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < MR; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) scr[(row_q + r) * kScrPitch + j * 16 + col_l] = acc[i][j][r] * ep.alpha;
    __builtin_amdgcn_wave_barrier();
    const int row0 = mb + i * 16;
    if (EPI == kEpiAtomicF32) {
      // one row per wave-instruction: 64 lanes x 4 B = 256 contiguous bytes
      const int col = nb + lane;
#pragma unroll 4
      for (int rr = 0; rr < 16; ++rr) {
        const int row = row0 + rr;
        if (row < M && col < N) atomicAdd(((float*)ep.C) + (int64_t)row * ep.ldc + col, scr[rr * kScrPitch + lane]);
      }
    } else if (F32OUT) {
#pragma unroll
      for (int ro = 0; ro < 4; ++ro) {
        const int rr = ro * 4 + (lane >> 4), c4 = (lane & 15) * 4;
        const int row = row0 + rr, col = nb + c4;
        if (row >= M) continue;
        float4 v = *reinterpret_cast<const float4*>(scr + rr * kScrPitch + c4);
        float* dst = ((float*)ep.C) + (int64_t)row * ep.ldc + col;
        if constexpr (EPI == kEpiFoldF32) {
          // write-through (sc1) stores: the folding workgroup reads them on another CU / XCD
          // after one agent-scope acquire, no release fence (cdna_hip_programming.md G16, R1)
          if (c_vec && col + 4 <= N) {
            const __amdgpu_buffer_rsrc_t rc =
                __builtin_amdgcn_make_buffer_rsrc(ep.C, (short)0, 0x7ffffff0, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), rc,
                                                   (int)(((int64_t)row * ep.ldc + col) * 4), 0, 16);
          } else {
            const float vv[4] = {v.x, v.y, v.z, v.w};
            for (int e = 0; e < 4; ++e)
              if (col + e < N) __hip_atomic_store(dst + e, vv[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          continue;
        }
        if (c_vec && col + 4 <= N) {
          if (EPI == kEpiAccumF32) {
            const float4 o = *reinterpret_cast<const float4*>(dst);
            v.x += o.x;
            v.y += o.y;
            v.z += o.z;
            v.w += o.w;
          }
          *reinterpret_cast<float4*>(dst) = v;
        } else {
          const float vv[4] = {v.x, v.y, v.z, v.w};
          for (int e = 0; e < 4; ++e)
            if (col + e < N) dst[e] = EPI == kEpiAccumF32 ? dst[e] + vv[e] : vv[e];
        }
      }
    } else {
#pragma unroll
      for (int ro = 0; ro < 2; ++ro) {
        const int rr = ro * 8 + (lane >> 3), c8 = (lane & 7) * 8;
        const int row = row0 + rr, col = nb + c8;
        const bool row_ok = row < M;
        const float4 lo = *reinterpret_cast<const float4*>(scr + rr * kScrPitch + c8);
        const float4 hi = *reinterpret_cast<const float4*>(scr + rr * kScrPitch + c8 + 4);
        float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        const bool full = col + 8 <= N;
        float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const int64_t moff = (int64_t)row * ep.ldmask + col;
        if (READ_MASK && row_ok) {
          if (m_vec && full) {
            const uint4 mu = *reinterpret_cast<const uint4*>(ep.mask + moff);
            const uint32_t w[4] = {mu.x, mu.y, mu.z, mu.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              m[2 * e] = __uint_as_float(w[e] << 16);
              m[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
            }
          } else {
            for (int e = 0; e < 8; ++e)
              if (col + e < N) m[e] = bf2f(ep.mask[moff + e]);
          }
        }
        bf16_t aux[8];
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = epi_apply<EPI>(v[e], bias[e], m[e], &aux[e]);
        uint32_t pk[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) pk[e] = pack_bf2(o[2 * e], o[2 * e + 1]);
        if (EPI == kEpiReluMaskBf16 && ep.colsum && row_ok) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            csum[2 * e] += __uint_as_float(pk[e] << 16);
            csum[2 * e + 1] += __uint_as_float(pk[e] & 0xffff0000u);
          }
        }
        if (EPI == kEpiXentStatsBf16) {
          // softmax partial of this wave's 64 columns of `row` from the ROUNDED logits (the
          // gradient pass exponentiates the same bf16 values): the row's 8 lanes each fold their
          // 8 columns, then merge over lane bits 0..2 (all lanes take part in the shuffles)
          constexpr float kL2E = 1.4426950408889634f;
          float y[8], mx = -1.0e30f, sm = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float xv = (e & 1) ? __uint_as_float(pk[e >> 1] & 0xffff0000u) : __uint_as_float(pk[e >> 1] << 16);
            y[e] = col + e < ep.seg ? xv * kL2E : -1.0e30f;
            mx = fmaxf(mx, y[e]);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) sm += col + e < ep.seg ? __builtin_amdgcn_exp2f(y[e] - mx) : 0.f;
#pragma unroll
          for (int o = 1; o < 8; o <<= 1) {
            const float m2 = __shfl_xor(mx, o, 64), s2 = __shfl_xor(sm, o, 64);
            const float mn = fmaxf(mx, m2);
            sm = sm * __builtin_amdgcn_exp2f(mx - mn) + s2 * __builtin_amdgcn_exp2f(m2 - mn);
            mx = mn;
          }
          if ((lane & 7) == 0 && row_ok && nb < N)
            reinterpret_cast<float2*>(ep.colsum)[(int64_t)row * ep.ldmask + nb / 64] = make_float2(mx, sm);
        }
        if (!row_ok) continue;
        // (kEpiPermRowsBf16 with seg % 8 == 0: a lane's 8 columns never cross a segment)
        bf16_t* dst = ((bf16_t*)ep.C) + out_offset<EPI>(ep, N, row, col);
        if (c_vec && full) {
          *reinterpret_cast<uint4*>(dst) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        } else if (EPI == kEpiPermRowsBf16) {
          for (int e = 0; e < 8; ++e)
            if (col + e < N)
              ((bf16_t*)ep.C)[out_offset<EPI>(ep, N, row, col + e)] =
                  (bf16_t)((e & 1) ? (pk[e >> 1] >> 16) : (pk[e >> 1] & 0xffffu));
        } else {
          for (int e = 0; e < 8; ++e)
            if (col + e < N) dst[e] = (bf16_t)((e & 1) ? (pk[e >> 1] >> 16) : (pk[e >> 1] & 0xffffu));
        }
        if (WRITE_AUX) {
          bf16_t* adst = const_cast<bf16_t*>(ep.mask) + moff;
          if (m_vec && full) {
            uint32_t a[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) a[e] = (uint32_t)aux[2 * e] | ((uint32_t)aux[2 * e + 1] << 16);
            *reinterpret_cast<uint4*>(adst) = make_uint4(a[0], a[1], a[2], a[3]);
          } else {
            for (int e = 0; e < 8; ++e)
              if (col + e < N) adst[e] = aux[e];
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // this slice's reads retire before the next slice's writes
  }
  if (EPI == kEpiReluMaskBf16 && ep.colsum) {
    // lanes with equal (lane & 7) hold the same 8 columns: fold rows over lane bits 3..5
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float c = csum[e];
      c += __shfl_xor(c, 8, 64);
      c += __shfl_xor(c, 16, 64);
      c += __shfl_xor(c, 32, 64);
      const int col = nb + (lane & 7) * 8 + e;
      if (lane < 8 && col < N) atomicAdd(ep.colsum + (int64_t)col * ep.colsum_ld, c);
    }
  }
}

// One wave's 64x64 accumulator block (rows m0 + 64*wm.., cols n0 + 64*wn..).
template <int EPI>
__device__ __forceinline__ void epilogue(const v4f (&acc)[4][4], const EpiArgs& ep, int M, int N, int m0, int n0,
                                         int wm, int wn, int lane) {
  epilogue_at<EPI, 4>(acc, ep, M, N, m0 + wm * 64, n0 + wn * 64, lane);
}

template <int BK, bool A_KM, bool B_KN, int EPI>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                        int M, int N, int K, int lda, int ldb, int k_chunk,
                                                        EpiArgs ep) {
  constexpr bool PERM = A_KM && B_KN;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2][2][Lds<BK>::TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware remap (T1): hardware deals blocks round-robin over 8 XCDs; give each XCD a
  // contiguous run of tiles so neighbouring tiles (same A panel) share its L2.
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  if (nwg >= 16) {
    int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    bid = base + (bid >> 3);
  }
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kb = blockIdx.z * k_chunk;
  {
    const int z = blockIdx.y, zo = z / ep.inner, zi = z - zo * ep.inner;
    A += zo * ep.sa_o + zi * ep.sa_i;
    B += zo * ep.sb_o + zi * ep.sb_i;
    const int64_t co = zo * ep.sc_o + zi * ep.sc_i + (int64_t)blockIdx.z * ep.sc_split;
    const bool f32 = EPI == kEpiStoreF32 || EPI == kEpiAtomicF32 || EPI == kEpiAccumF32 || EPI == kEpiFoldF32;
    ep.C = f32 ? (void*)((float*)ep.C + co) : (void*)((bf16_t*)ep.C + co);
  }
  const int ke = min(K, kb + k_chunk);

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  // One register set: tile t+1's global loads are issued before tile t's MFMAs and written
  // to the other LDS buffer after them (T14 split). (A 2-deep register ring measured slower:
  // the extra 32-64 VGPRs halve occupancy, which hides more latency than the ring.)
  uint4 ra[Lds<BK>::CHUNKS], rb[Lds<BK>::CHUNKS];
  int cur = 0;
  if (kb < ke) {
    load_tile<BK, A_KM>(A, lda, m0, kb, M, ke, tid, ra);
    load_tile<BK, B_KN>(B, ldb, n0, kb, N, ke, tid, rb);
    store_tile<BK, A_KM>(smem[0][0], tid, ra);
    store_tile<BK, B_KN>(smem[0][1], tid, rb);
  }
  __syncthreads();
  for (int k0 = kb; k0 < ke; k0 += BK) {
    const bool has_next = k0 + BK < ke;
    if (has_next) {
      load_tile<BK, A_KM>(A, lda, m0, k0 + BK, M, ke, tid, ra);
      load_tile<BK, B_KN>(B, ldb, n0, k0 + BK, N, ke, tid, rb);
    }
    const bf16_t* SA = smem[cur][0];
    const bf16_t* SB = smem[cur][1];
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      v8s af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<BK, A_KM, PERM>(SA, wm * 64 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag<BK, B_KN, PERM>(SB, wn * 64 + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, af[i]),
                                                              __builtin_bit_cast(v8bf, bfr[j]), acc[i][j], 0, 0, 0);
    }
    if (has_next) {
      store_tile<BK, A_KM>(smem[cur ^ 1][0], tid, ra);
      store_tile<BK, B_KN>(smem[cur ^ 1][1], tid, rb);
    }
    __syncthreads();
    cur ^= 1;
  }

  epilogue<EPI>(acc, ep, M, N, m0, n0, wm, wn, lane);
}


// ================================================================ v2: LDS-DMA staging
// Same 128x128 tile / 2x2 waves / fragment math as above, but operands go global -> LDS with
// buffer_load_dwordx4 ... lds (no register staging, no VGPRs for the tile in flight), BK = 64
// always, 2 LDS stages (64 KiB -> 2 workgroups per CU). Lane-linear LDS images (a DMA wave
// instruction writes 1 KiB contiguously) are made bank-conflict-free by XOR-swizzling the
// 16-byte chunk index on the SOURCE address side:
//   [row][64 k] images (MK / NK operands, ds_read_b128): chunk' = chunk ^ ((row >> 1) & 7)
//     -> the 16 rows of a 16-lane read group cover all 64 banks
//   [k][128 m] images (KM / KN operands, ds_read_b64_tr_b16): chunk' = chunk ^ swz(k),
//     swz(k) = 2 * ((k & 3) | (((k >> 2) ^ (k >> 3)) & 1) << 2)
//     -> the 8 k-rows read by a 32-lane half land on 8 distinct 32-byte bank groups, for both
//        the plain and the permuted (wgrad) k order
// Out-of-range chunks (M/N/K tails) get an offset past the buffer's num_records, so the DMA
// writes zeros. One barrier after the stage's DMA retires (counted vmcnt, raw s_barrier: the
// next stage stays in flight), one before its buffer is refilled.
constexpr int BK2 = 64;
constexpr uint32_t kOobOffset = 0x80000000u;
#ifndef MINIPS_GEMM_SETPRIO
#define MINIPS_GEMM_SETPRIO 0  // T5 setprio pair: measured -1..-4 % here (tools/gpu_ab.sh)
#endif
constexpr bool kSetPrio = MINIPS_GEMM_SETPRIO != 0;
#ifndef MINIPS_GEMM_LDS_EPILOGUE
#define MINIPS_GEMM_LDS_EPILOGUE 1  // staged epilogue (epilogue_lds); 0: direct fragment stores
#endif
constexpr bool kLdsEpilogue = MINIPS_GEMM_LDS_EPILOGUE != 0;

__device__ __forceinline__ int swz_k(int k) { return 2 * ((k & 3) | ((((k >> 2) ^ (k >> 3)) & 1) << 2)); }

// One operand tile of ROWS x 64 k (MK/NK image [ROWS][64]) or 64 k x ROWS (KM/KN image
// [64][ROWS]) = ROWS/8 DMA wave-instructions of 1 KiB, split over the workgroup's waves.
template <bool KMAJOR, int ROWS, int NWAVES>
__device__ __forceinline__ void dma_tile(__amdgpu_buffer_rsrc_t rsrc, int ld, int row0, int k0, int rows, int kend,
                                         bf16_t* S, int wave, int lane) {
  constexpr int INSTR = ROWS / 8, PER = INSTR / NWAVES;
  static_assert(INSTR % NWAVES == 0, "tile must split evenly over the waves");
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int gi = wave * PER + j;  // 1-KiB piece index
    uint32_t voff;
    if (!KMAJOR) {
      const int R = 8 * gi + (lane >> 3);
      const int c = (lane & 7) ^ ((R >> 1) & 7);
      const int gr = row0 + R, gk = k0 + 8 * c;
      voff = (gr < rows && gk < kend) ? (uint32_t)(((int64_t)gr * ld + gk) * 2) : kOobOffset;
    } else {
      constexpr int CH = ROWS / 8;           // 16-byte chunks per k-row
      constexpr int RPI = 64 / CH;           // k-rows per 1-KiB piece
      const int kr = RPI * gi + lane / CH;
      const int c = (lane % CH) ^ swz_k(kr);  // flips chunk bits 1..3 only: stays in its 256-B half
      const int gk = k0 + kr, gm = row0 + 8 * c;
      voff = (gk < kend && gm < rows) ? (uint32_t)(((int64_t)gk * ld + gm) * 2) : kOobOffset;
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(S + gi * 512), 16, voff,
                                             0, 0, 0);
  }
}

template <bool KMAJOR, bool PERM, int ROWS>
__device__ __forceinline__ v8s frag2(const bf16_t* S, int row_base, int ks, int lane) {
  const int g = lane >> 4;
  if (!KMAJOR) {
    const int R = row_base + (lane & 15);
    const int c = (4 * ks + g) ^ ((R >> 1) & 7);
    return *reinterpret_cast<const v8s*>(S + R * BK2 + 8 * c);
  } else {
    const int i = lane & 15, q = i >> 2, p = i & 3;
    const int r0 = 32 * ks + (PERM ? 4 * g : 8 * g) + q;
    const int r1 = 32 * ks + (PERM ? 16 + 4 * g : 8 * g + 4) + q;
    const int ch = (row_base >> 3) + (p >> 1), sub = 4 * (p & 1);
    const v4s lo = ds_read_tr16(S + r0 * ROWS + 8 * (ch ^ swz_k(r0)) + sub);
    const v4s hi = ds_read_tr16(S + r1 * ROWS + 8 * (ch ^ swz_k(r1)) + sub);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// W&D output head as the epilogue of the last hidden layer's forward GEMM (kEpiWdHead): one
// workgroup owns TM rows and ALL N (<= TN) columns of H3 = relu(H2ext W3ext^T), so a row's head
// logit z = H3[row] . w4 + b4 + wide[row] is a reduction across the workgroup's WN waves (one LDS
// exchange). Then dz = (sigmoid(z) - label) * scale, dH3 = (H3 > 0) * bf16(dz * w4) goes out
// through the staged bf16 epilogue, dw4 / db4 / loss / dwide are accumulated here -- H3 itself
// never reaches HBM and the separate head kernel (H3 read + dH3 write, one wave per 4 samples)
// disappears. Numerics as wd_head: H3 rounded to bf16 before the dot product and the mask.
// ep.bias = w4 bf16 [N + 1] (b4 at N), ep.colsum = dw4 fp32 [N + 1] (db4 at N).
template <int TM, int TN>
__device__ __forceinline__ void wd_head_epilogue(v4f (&acc)[4][4], const EpiArgs& ep, int M, int N, int m0, int wm,
                                                 int wn, int lane, float* __restrict__ lds) {
  constexpr int WN = TN / 64, NW = (TM / 64) * WN;
  const int col_l = lane & 15, row_q = (lane >> 4) * 4;
  const int mb = m0 + wm * 64, nb = wn * 64;
  float* zp = lds + NW * kScrFloats;  // [TM][WN] wave partials of z, past the per-wave scratch
  float wv[4], bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = nb + j * 16 + col_l;
    wv[j] = col < N ? bf2f(ep.bias[col]) : 0.f;
    bv[j] = (ep.head_bias && col < N) ? bf2f(ep.head_bias[col]) : 0.f;
  }
  float zr[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float h = __uint_as_float(pack_bf2(fmaxf(acc[i][j][r] * ep.alpha + bv[j], 0.f), 0.f) << 16);
        acc[i][j][r] = h;
        a += h * wv[j];
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) a += __shfl_xor(a, o, 64);
      zr[i][r] = a;
    }
  if (col_l == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) zp[(wm * 64 + i * 16 + row_q + r) * WN + wn] = zr[i][r];
  }
  __syncthreads();
  const float b4 = bf2f(ep.bias[N]);
  float dz[4][4], dbl = 0.f, lossl = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = wm * 64 + i * 16 + row_q + r, row = m0 + rl;
      float d = 0.f;
      if (row < M) {
        float z = b4 + ep.head_wide[row];
#pragma unroll
        for (int w = 0; w < WN; ++w) z += zp[rl * WN + w];
        const float label = ep.head_label[row] > 0.5f ? 1.f : 0.f;
        d = (sigmoidf_(z) - label) * ep.head_scale;
        if (wn == 0 && col_l == 0) {
          ep.head_dwide[row] = d;
          dbl += d;
          lossl += fmaxf(z, 0.f) - z * label + log1pf(__expf(-fabsf(z)));
        }
      }
      dz[i][r] = d;
    }
  float cs[4] = {0.f, 0.f, 0.f, 0.f}, cg[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float h = acc[i][j][r];
        cs[j] += dz[i][r] * h;
        const float gv = h > 0.f ? dz[i][r] * wv[j] : 0.f;
        acc[i][j][r] = gv;
        cg[j] += __uint_as_float(pack_bf2(gv, 0.f) << 16);  // the stored (bf16) dH's column sums
      }
  EpiArgs st = ep;
  st.alpha = 1.f;
  epilogue_lds<kEpiStoreBf16, 4>(acc, st, M, N, mb, nb, lane, lds + (threadIdx.x >> 6) * kScrFloats);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    cs[j] += __shfl_xor(cs[j], 16, 64);
    cs[j] += __shfl_xor(cs[j], 32, 64);
    cg[j] += __shfl_xor(cg[j], 16, 64);
    cg[j] += __shfl_xor(cg[j], 32, 64);
  }
  if (wn == 0) {
    dbl = warp_sum(dbl);
    lossl = warp_sum(lossl);
  }
  if (!ep.head_slab) {  // (no fold workspace: same-address atomics, one per column per workgroup)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = nb + j * 16 + lane;
      if (lane < 16 && col < N) atomicAdd(ep.colsum + col, cs[j]);
      if (ep.head_dh_colsum && lane < 16 && col < N)
        atomicAdd(ep.head_dh_colsum + (int64_t)col * ep.head_dh_colsum_ld, cg[j]);
    }
    if (wn == 0 && lane == 0) {
      atomicAdd(ep.colsum + N, dbl);
      atomicAdd(ep.head_loss, lossl);
    }
    return;
  }
  // Two-level fold of the workgroups' partial rows {dw4 [N] | dH colsum [N] | db4 | loss}, every
  // hand-off write-through (cdna_hip_programming.md Guideline 16 R1: sc1 stores, drain, relaxed
  // ticket, one acquire by the folder): 256 workgroups x 2N same-address atomics were what made
  // this fused head slower than the GEMM + wd_head pair (51 vs 41 us, round 3).
  static_assert(TM == 64 && TN == 256, "the fold's partial row is laid out for one 64 x 256 tile per row band");
  constexpr int G = 16;  // workgroups per group
  const int NP = 2 * N + 2;
  const int nb_ = (int)gridDim.x, ngroups = (nb_ + G - 1) / G, blk = blockIdx.x, grp = blk / G;
  float* prow = ep.head_slab + (int64_t)blk * NP;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = nb + j * 16 + lane;
    if (lane < 16 && col < N) {
      __hip_atomic_store(prow + col, cs[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(prow + N + col, cg[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (wn == 0 && lane == 0) {
    __hip_atomic_store(prow + 2 * N, dbl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(prow + 2 * N + 1, lossl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  int* flag = reinterpret_cast<int*>(zp + TM * WN);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int gn = min(G, nb_ - grp * G);
    const unsigned t = __hip_atomic_fetch_add(ep.head_ticket + 1 + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == (unsigned)gn - 1;
    if (last) {
      __hip_atomic_store(ep.head_ticket + 1 + grp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  {
    const int g0 = grp * G, gn = min(G, nb_ - g0);
    float* grow = ep.head_slab + (int64_t)(nb_ + grp) * NP;
    for (int c = threadIdx.x; c < NP; c += blockDim.x) {
      float v[G];
#pragma unroll
      for (int k = 0; k < G; ++k) v[k] = k < gn ? ep.head_slab[(int64_t)(g0 + k) * NP + c] : 0.f;
      float tot = 0.f;
#pragma unroll
      for (int k = 0; k < G; ++k) tot += v[k];
      __hip_atomic_store(grow + c, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ep.head_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == (unsigned)ngroups - 1;
    if (last) {
      __hip_atomic_store(ep.head_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  for (int c = threadIdx.x; c < NP; c += blockDim.x) {
    float v[G];
#pragma unroll
    for (int k = 0; k < G; ++k) v[k] = k < ngroups ? ep.head_slab[(int64_t)(nb_ + k) * NP + c] : 0.f;
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < G; ++k) tot += v[k];
    if (c < N) ep.colsum[c] += tot;
    else if (c < 2 * N) {
      if (ep.head_dh_colsum) ep.head_dh_colsum[(int64_t)(c - N) * ep.head_dh_colsum_ld] += tot;
    } else if (c == 2 * N) ep.colsum[N] += tot;
    else *ep.head_loss += tot;
  }
}

// kEpiFoldF32 tail of a split-K workgroup (after its slab plane was stored write-through): one
// relaxed agent-scope ticket per tile; the K slice drawing the last ticket acquires (agent scope:
// this CU's L1 drops the planes' lines) and adds the tile's nsplit planes into ep.fold_out.
// Correct for any placement of a tile's slices over CUs / XCDs (cdna_hip_programming.md G16 R1).
template <int TM, int TN>
__device__ __forceinline__ void splitk_fold(const EpiArgs& ep, int M, int N, int m0, int n0, int tile, int ks,
                                            unsigned* __restrict__ flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its plane stores
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ep.fold_cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned last = t == (unsigned)ep.fold_nsplit - 1;
    if (last) {
      __hip_atomic_store(ep.fold_cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  const int64_t plane = ep.sc_split;
  const float* p0 = (const float*)ep.C - (int64_t)ks * plane;
  constexpr int PER_ROW = TN / 4;
  for (int i = threadIdx.x; i < TM * PER_ROW; i += blockDim.x) {
    const int rr = i / PER_ROW, c4 = (i - rr * PER_ROW) * 4;
    const int row = m0 + rr, col = n0 + c4;
    if (row >= M || col >= N) continue;
    const float* p = p0 + (int64_t)row * ep.ldc + col;
    float4 a = *reinterpret_cast<const float4*>(p);
    int z = 1;
    for (; z + 3 < ep.fold_nsplit; z += 4) {
      const float4 b0 = *reinterpret_cast<const float4*>(p + z * plane);
      const float4 b1 = *reinterpret_cast<const float4*>(p + (z + 1) * plane);
      const float4 b2 = *reinterpret_cast<const float4*>(p + (z + 2) * plane);
      const float4 b3 = *reinterpret_cast<const float4*>(p + (z + 3) * plane);
      a.x += (b0.x + b1.x) + (b2.x + b3.x);
      a.y += (b0.y + b1.y) + (b2.y + b3.y);
      a.z += (b0.z + b1.z) + (b2.z + b3.z);
      a.w += (b0.w + b1.w) + (b2.w + b3.w);
    }
    for (; z < ep.fold_nsplit; ++z) {
      const float4 b = *reinterpret_cast<const float4*>(p + z * plane);
      a.x += b.x;
      a.y += b.y;
      a.z += b.z;
      a.w += b.w;
    }
    float* o = ep.fold_out + (int64_t)row * ep.fold_ldc + col;
    o[0] += a.x;
    o[1] += a.y;
    o[2] += a.z;
    o[3] += a.w;
  }
}

// TM x TN output tile, (TM/64) x (TN/64) waves of 64x64 each (4, 8 or 16 waves). 128x128
// keeps 2 workgroups per CU; the 256-wide tiles halve the L2->LDS bytes per MFMA (the loads,
// not the MFMAs, bound this kernel at these sizes) and run one 16- or 8-wave workgroup per CU.
template <int TM, int TN, bool A_KM, bool B_KN, int EPI>
__global__ __launch_bounds__(TM * TN / 64) void gemm_v2_kernel(const bf16_t* __restrict__ A,
                                                               const bf16_t* __restrict__ B, int M, int N, int K,
                                                               int lda, int ldb, int k_chunk, EpiArgs ep) {
  constexpr bool PERM = A_KM && B_KN;
  constexpr int WN = TN / 64, NWAVES = (TM / 64) * (TN / 64);
  constexpr int VM_STAGE = (TM / 8 + TN / 8) / NWAVES;  // DMA instructions per thread per stage
  __shared__ __attribute__((aligned(1024))) bf16_t smem[2][(TM + TN) * BK2];
  static_assert(sizeof(smem) >= sizeof(float) * NWAVES * kScrFloats, "epilogue scratch must fit the staging LDS");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = (N + TN - 1) / TN, tiles_m = (M + TM - 1) / TM;
  const int nwg = tiles_m * tiles_n;
  int bid = blockIdx.x, ks = blockIdx.z;
  if (ep.zmap && gridDim.z > 1 && gridDim.y == 1) {
    // dispatch order is x fastest: L = x + nwg * z; XCD-contiguous runs over w = slice * nwg + tile
    const int W = nwg * (int)gridDim.z, L = bid + nwg * ks;
    const int xcd = L & 7, q = W >> 3, r = W & 7;
    const int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
    ks = w / nwg;
    bid = w - ks * nwg;
  } else if (nwg >= 16) {
    int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    bid = base + (bid >> 3);
  }
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * TM, n0 = tn * TN;
  {
    const int z = blockIdx.y, zo = z / ep.inner, zi = z - zo * ep.inner;
    A += zo * ep.sa_o + zi * ep.sa_i;
    B += zo * ep.sb_o + zi * ep.sb_i;
    const int64_t co = zo * ep.sc_o + zi * ep.sc_i + (int64_t)ks * ep.sc_split;
    const bool f32 = EPI == kEpiStoreF32 || EPI == kEpiAtomicF32 || EPI == kEpiAccumF32 || EPI == kEpiFoldF32;
    ep.C = f32 ? (void*)((float*)ep.C + co) : (void*)((bf16_t*)ep.C + co);
  }
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0x7ffffff0, 0x00020000);
  const int kb = ks * k_chunk;
  const int ke = min(K, kb + k_chunk);
  const int nt = ke > kb ? (ke - kb + BK2 - 1) / BK2 : 0;

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  if (nt > 0) {
    dma_tile<A_KM, TM, NWAVES>(ra, lda, m0, kb, M, ke, smem[0], wave, lane);
    dma_tile<B_KN, TN, NWAVES>(rb, ldb, n0, kb, N, ke, smem[0] + TM * BK2, wave, lane);
  }
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) {
      const int k1 = kb + (t + 1) * BK2;
      dma_tile<A_KM, TM, NWAVES>(ra, lda, m0, k1, M, ke, smem[cur ^ 1], wave, lane);
      dma_tile<B_KN, TN, NWAVES>(rb, ldb, n0, k1, N, ke, smem[cur ^ 1] + TM * BK2, wave, lane);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_STAGE) : "memory");  // this stage retired, the next in flight
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bf16_t* SA = smem[cur];
    const bf16_t* SB = smem[cur] + TM * BK2;
#pragma unroll
    for (int ks = 0; ks < BK2 / 32; ++ks) {
      v8s af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag2<A_KM, PERM, TM>(SA, wm * 64 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag2<B_KN, PERM, TN>(SB, wn * 64 + j * 16, ks, lane);
      if (kSetPrio) __builtin_amdgcn_s_setprio(1);  // T5: keeps the cluster between the barriers
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, af[i]),
                                                              __builtin_bit_cast(v8bf, bfr[j]), acc[i][j], 0, 0, 0);
      if (kSetPrio) __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done reading `cur` before it is refilled
    asm volatile("" ::: "memory");
  }
  if constexpr (EPI == kEpiWdHead)
    wd_head_epilogue<TM, TN>(acc, ep, M, N, m0, wm, wn, lane, reinterpret_cast<float*>(&smem[0][0]));
  else if (kLdsEpilogue || EPI == kEpiFoldF32)
    epilogue_lds<EPI, 4>(acc, ep, M, N, m0 + wm * 64, n0 + wn * 64, lane,
                         reinterpret_cast<float*>(&smem[0][0]) + wave * kScrFloats);
  else
    epilogue<EPI>(acc, ep, M, N, m0, n0, wm, wn, lane);
  if constexpr (EPI == kEpiFoldF32)  // (the flag word lies past every wave's epilogue scratch)
    splitk_fold<TM, TN>(ep, M, N, m0, n0, bid, ks,
                        reinterpret_cast<unsigned*>(reinterpret_cast<float*>(&smem[0][0]) + NWAVES * kScrFloats));
}

// ================================================================ v6: 256x256, 4 waves of 128x128
// The LDS-read bound of the 64x64-per-wave tiles: a wave reads 64 A + 64 B fragment rows per k for
// 64x64 MACs, so a 16-wave 256x256 workgroup pulls 256 KiB of fragments out of LDS per 64-deep
// K-step -- 2048 LDS cycles at 128 B/clk, the same as its 2048 MFMA cycles (SQ_WAIT_INST_LDS
// dominates the LM-head profile, profiles/r4/pmc_lm_dgrad_v2_v5.txt). Here ONE wave per SIMD owns
// a 128x128 block (8 x 8 MFMA 16x16x32 tiles, 256 fp32 accumulators: the AGPR half of the
// 512-entry register file at one wave per SIMD), reading 128 + 128 fragment rows per k for 4x the
// MACs: 128 KiB per K-step, half the MFMA time. Staging is v2's: BK = 64, two LDS-DMA stages of
// 64 KiB (swizzled images, zero-filled tails), one counted vmcnt + barrier per stage; inside a
// K-step the fragments of k-half 1 are read while k-half 0's 64 MFMAs run. XCD-contiguous tile
// order as v2; staged epilogue (epilogue_lds, two 128x64 halves per wave).
template <bool A_KM, bool B_KN, int EPI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_v6_kernel(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ B, int M, int N, int K, int lda, int ldb, int k_chunk,
    EpiArgs ep) {
  constexpr bool PERM = A_KM && B_KN;
  constexpr int TM = 256, TN = 256, NWAVES = 4;
  constexpr int VM_STAGE = (TM / 8 + TN / 8) / NWAVES;  // DMA instructions per thread per stage (16)
  __shared__ __attribute__((aligned(1024))) bf16_t smem[2][(TM + TN) * BK2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (N + TN - 1) / TN, tiles_m = (M + TM - 1) / TM;
  const int nwg = tiles_m * tiles_n;
  int bid = blockIdx.x, ks = blockIdx.z;
  if (ep.zmap && gridDim.z > 1 && gridDim.y == 1) {
    const int W = nwg * (int)gridDim.z, L = bid + nwg * ks;
    const int xcd = L & 7, q = W >> 3, r = W & 7;
    const int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
    ks = w / nwg;
    bid = w - ks * nwg;
  } else if (nwg >= 16) {
    int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    bid = base + (bid >> 3);
  }
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * TM, n0 = tn * TN;
  {
    const int z = blockIdx.y, zo = z / ep.inner, zi = z - zo * ep.inner;
    A += zo * ep.sa_o + zi * ep.sa_i;
    B += zo * ep.sb_o + zi * ep.sb_i;
    const int64_t co = zo * ep.sc_o + zi * ep.sc_i + (int64_t)ks * ep.sc_split;
    const bool f32 = EPI == kEpiStoreF32 || EPI == kEpiAtomicF32 || EPI == kEpiAccumF32 || EPI == kEpiFoldF32;
    ep.C = f32 ? (void*)((float*)ep.C + co) : (void*)((bf16_t*)ep.C + co);
  }
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0x7ffffff0, 0x00020000);
  const int kb = ks * k_chunk;
  const int ke = min(K, kb + k_chunk);
  const int nt = ke > kb ? (ke - kb + BK2 - 1) / BK2 : 0;

  v4f acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  if (nt > 0) {
    dma_tile<A_KM, TM, NWAVES>(ra, lda, m0, kb, M, ke, smem[0], wave, lane);
    dma_tile<B_KN, TN, NWAVES>(rb, ldb, n0, kb, N, ke, smem[0] + TM * BK2, wave, lane);
  }
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) {
      const int k1 = kb + (t + 1) * BK2;
      dma_tile<A_KM, TM, NWAVES>(ra, lda, m0, k1, M, ke, smem[cur ^ 1], wave, lane);
      dma_tile<B_KN, TN, NWAVES>(rb, ldb, n0, k1, N, ke, smem[cur ^ 1] + TM * BK2, wave, lane);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_STAGE) : "memory");  // this stage retired, the next in flight
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bf16_t* SA = smem[cur];
    const bf16_t* SB = smem[cur] + TM * BK2;
    v8s af[2][8], bfr[2][8];
#pragma unroll
    for (int i = 0; i < 8; ++i) af[0][i] = frag2<A_KM, PERM, TM>(SA, wm * 128 + i * 16, 0, lane);
#pragma unroll
    for (int j = 0; j < 8; ++j) bfr[0][j] = frag2<B_KN, PERM, TN>(SB, wn * 128 + j * 16, 0, lane);
#pragma unroll
    for (int h = 0; h < BK2 / 32; ++h) {
      if (h + 1 < BK2 / 32) {  // the next k-half's fragments while this half's MFMAs run
#pragma unroll
        for (int i = 0; i < 8; ++i) af[(h + 1) & 1][i] = frag2<A_KM, PERM, TM>(SA, wm * 128 + i * 16, h + 1, lane);
#pragma unroll
        for (int j = 0; j < 8; ++j) bfr[(h + 1) & 1][j] = frag2<B_KN, PERM, TN>(SB, wn * 128 + j * 16, h + 1, lane);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(v8bf, af[h & 1][i]), __builtin_bit_cast(v8bf, bfr[h & 1][j]), acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done reading `cur` before it is refilled
    asm volatile("" ::: "memory");
  }
  float* scr = reinterpret_cast<float*>(&smem[0][0]) + wave * kScrFloats;
#pragma unroll
  for (int jh = 0; jh < 2; ++jh) {
    v4f half[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) half[i][j] = acc[i][4 * jh + j];
    epilogue_lds<EPI, 8>(half, ep, M, N, m0 + wm * 128, n0 + wn * 128 + 64 * jh, lane, scr);
  }
}

// ================================================================ v3: 256x256, 8 waves, phase-split K-step
// 256x256 output tile, 8 waves as 2 (M) x 4 (N), each wave 128x64 = 8x4 MFMA 16x16 tiles (128
// accumulator registers), BK = 64, operands staged by LDS-DMA (same swizzled images as v2) as
// 128-row HALF tiles: [buf][A0 | A1 | B0 | B1], 16 KiB each, 2 buffers = 128 KiB (1 WG / CU).
// A K-step is split so that halves free up early and the DMA runs two K-steps ahead:
//   phase 0: read ALL of this wave's A fragments (16 x ds_read_b128: 8 m-tiles x 2 k) and the
//            B fragments of n-tile 0, 16 MFMAs; barrier -> the A halves of this buffer are free
//   phase 1: stage A of K-step t+2 into this buffer; B n-tile 1, 16 MFMAs
//   phase 2, 3: B n-tiles 2, 3, 16 MFMAs each
//   end:     counted vmcnt (A(t+2) stays in flight) + barrier -> B halves free, buffer t+1 landed
// and B of K-step t+1 is staged at phase 0 of t (into the other buffer, last read in t-1). So A
// has ~7 phases and B ~4 phases (~1.5 / 0.9 us) of load latency budget instead of one K-step.
// Raw s_barrier + explicit waits only: __syncthreads() would drain the DMA (vmcnt(0)).
constexpr int kV3Half = 128 * BK2;

template <bool A_KM, bool B_KN, int EPI, bool EARLY_A = true>
__global__ __launch_bounds__(512) void gemm_v3_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                      int M, int N, int K, int lda, int ldb, int k_chunk,
                                                      EpiArgs ep) {
  constexpr bool PERM = A_KM && B_KN;
  __shared__ __attribute__((aligned(1024))) bf16_t smem[2][4 * kV3Half];
  static_assert(sizeof(smem) >= sizeof(float) * 8 * kScrFloats, "epilogue scratch must fit the staging LDS");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = (N + 255) / 256, tiles_m = (M + 255) / 256;
  const int nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  if (nwg >= 16) {
    int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    bid = base + (bid >> 3);
  }
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * 256, n0 = tn * 256;
  {
    const int z = blockIdx.y, zo = z / ep.inner, zi = z - zo * ep.inner;
    A += zo * ep.sa_o + zi * ep.sa_i;
    B += zo * ep.sb_o + zi * ep.sb_i;
    const int64_t co = zo * ep.sc_o + zi * ep.sc_i + (int64_t)blockIdx.z * ep.sc_split;
    const bool f32 = EPI == kEpiStoreF32 || EPI == kEpiAtomicF32 || EPI == kEpiAccumF32 || EPI == kEpiFoldF32;
    ep.C = f32 ? (void*)((float*)ep.C + co) : (void*)((bf16_t*)ep.C + co);
  }
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0x7ffffff0, 0x00020000);
  const int kb = blockIdx.z * k_chunk;
  const int ke = min(K, kb + k_chunk);
  const int nt = ke > kb ? (ke - kb + BK2 - 1) / BK2 : 0;

  v4f acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  // 2 DMA instructions per thread per half tile -> 4 per operand per K-step
  auto stage_a = [&](int t, int buf) {
    const int k = kb + t * BK2;
    dma_tile<A_KM, 128, 8>(ra, lda, m0, k, M, ke, smem[buf], wave, lane);
    dma_tile<A_KM, 128, 8>(ra, lda, m0 + 128, k, M, ke, smem[buf] + kV3Half, wave, lane);
  };
  auto stage_b = [&](int t, int buf) {
    const int k = kb + t * BK2;
    dma_tile<B_KN, 128, 8>(rb, ldb, n0, k, N, ke, smem[buf] + 2 * kV3Half, wave, lane);
    dma_tile<B_KN, 128, 8>(rb, ldb, n0 + 128, k, N, ke, smem[buf] + 3 * kV3Half, wave, lane);
  };

  if (nt > 0) {
    stage_a(0, 0);
    stage_b(0, 0);
  }
  if (EARLY_A && nt > 1) {
    stage_a(1, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // A(0), B(0) landed; A(1) in flight
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  for (int t = 0; t < nt; ++t) {
    const int buf = t & 1;
    const bf16_t* SA = smem[buf] + wr * kV3Half;
    const bf16_t* SB = smem[buf] + (2 + (wc >> 1)) * kV3Half;
    const int bcol = (wc & 1) * 64;
    // ---- phase 0: every A fragment of the K-step + B n-tile 0
    if (t + 1 < nt) {
      if (!EARLY_A) stage_a(t + 1, buf ^ 1);  // plain double buffering: both operands one K-step ahead
      stage_b(t + 1, buf ^ 1);
    }
    v8s af[8][2], bfr[2];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) af[i][ks] = frag2<A_KM, PERM, 128>(SA, i * 16, ks, lane);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) bfr[ks] = frag2<B_KN, PERM, 128>(SB, bcol, ks, lane);
    if (kSetPrio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, af[i][ks]),
                                                            __builtin_bit_cast(v8bf, bfr[ks]), acc[i][0], 0, 0, 0);
    if (kSetPrio) __builtin_amdgcn_s_setprio(0);
    if (EARLY_A) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave's A reads of this buffer retired
      asm volatile("" ::: "memory");
      // ---- phases 1..3: B n-tiles 1..3 (A from registers); A of K-step t+2 streams in
      if (t + 2 < nt) stage_a(t + 2, buf);
    }
#pragma unroll
    for (int j = 1; j < 4; ++j) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) bfr[ks] = frag2<B_KN, PERM, 128>(SB, bcol + j * 16, ks, lane);
      if (kSetPrio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 8; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, af[i][ks]),
                                                              __builtin_bit_cast(v8bf, bfr[ks]), acc[i][j], 0, 0, 0);
      if (kSetPrio) __builtin_amdgcn_s_setprio(0);
    }
    // ---- end of K-step: operands of t+1 landed (A(t+2) may stay in flight), B halves free
    if (EARLY_A && t + 2 < nt) {
      asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  if (kLdsEpilogue)
    epilogue_lds<EPI, 8>(acc, ep, M, N, m0 + wr * 128, n0 + wc * 64, lane,
                         reinterpret_cast<float*>(&smem[0][0]) + wave * kScrFloats);
  else
    epilogue_at<EPI, 8>(acc, ep, M, N, m0 + wr * 128, n0 + wc * 64, lane);
}

// ================================================================ v4: 256x256, 8 waves, quarter-staged A
// The v3 tile with a staging schedule that keeps every DMA 4-7 phases ahead of its first read
// (v2 / v3 leave one K-step, ~1 us, to cover an HBM miss):
//   * 8 waves as 2 (M) x 4 (N), each wave 128 x 64 = 8 x 4 MFMA 16x16x32 tiles (128 acc VGPRs);
//     a K-step (BK = 64) runs as 4 PHASES, phase q = the wave's rows [32q, 32q + 32) of its A half
//     against all 4 of its B n-tiles (2 k sub-steps): 16 MFMAs per wave per phase;
//   * the wave's B fragments of the K-step (4 n-tiles x 2 k) are read ONCE, in phase 0, and stay
//     in registers -- so the whole B tile of the buffer is free after phase 0;
//   * A lives in LDS as 8 quarter images (half h, quarter q: 32 rows x 64 k, 4 KiB each), and
//     quarter q of a buffer is free after phase q;
//   * so K-step t + 2 (same buffer as t) streams in WHILE t computes: A quarter q at phase q + 1,
//     the B halves at phases 1 / 2, and A quarter 3 at phase 0 of t + 1; one counted
//     vmcnt (7 = the DMAs of K-step t + 2 this wave issued during t) + one barrier per K-step
//     retire K-step t + 1, and one barrier per phase orders the quarter reuse (WAR);
//   * the next quarter's A fragments are read during the current phase's MFMAs (two register sets).
// Images: MK quarter [32][64] with the v2 swizzle; KM quarter [64 k][32 rows] (64-byte rows) with
// chunk' = chunk ^ swz_q(k), which keeps the 32-lane halves of the transposing reads on disjoint
// bank groups for the plain and the permuted (wgrad) k order. B: the v2 128-row half images.
// Tile order: grouped (4 row tiles x tiles_n) inside each XCD's contiguous run of tiles, so the
// 32 workgroups one XCD runs at a time share 4 A panels and 8 B panels through its L2.
constexpr int kQuarter = 32 * BK2;  // bf16 elements of one A quarter image

__device__ __forceinline__ int swz_q(int k) { return 2 * (((k >> 2) ^ (k >> 3)) & 1); }

// Piece p (0..3, 1 KiB) of the A quarter image at S holding rows [row0, row0 + 32) x k [k0, k0 + 64).
template <bool KMAJOR>
__device__ __forceinline__ void dma_quarter(__amdgpu_buffer_rsrc_t rsrc, int ld, int row0, int k0, int rows, int kend,
                                            bf16_t* S, int p, int lane) {
  uint32_t voff;
  if (!KMAJOR) {
    const int R = 8 * p + (lane >> 3);
    const int c = (lane & 7) ^ ((R >> 1) & 7);
    const int gr = row0 + R, gk = k0 + 8 * c;
    voff = (gr < rows && gk < kend) ? (uint32_t)(((int64_t)gr * ld + gk) * 2) : kOobOffset;
  } else {
    const int kr = 16 * p + (lane >> 2);
    const int c = (lane & 3) ^ swz_q(kr);
    const int gk = k0 + kr, gm = row0 + 8 * c;
    voff = (gk < kend && gm < rows) ? (uint32_t)(((int64_t)gk * ld + gm) * 2) : kOobOffset;
  }
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(S + p * 512), 16, voff, 0,
                                           0, 0);
}

// 16x16x32 A fragment of rows [16 i, 16 i + 16) of a quarter image, k sub-step ks.
template <bool KMAJOR, bool PERM>
__device__ __forceinline__ v8s frag_quarter(const bf16_t* S, int i, int ks, int lane) {
  if (!KMAJOR) return frag2<false, PERM, 32>(S, 16 * i, ks, lane);
  const int g = lane >> 4, l = lane & 15, q = l >> 2, p = l & 3;
  const int r0 = 32 * ks + (PERM ? 4 * g : 8 * g) + q;
  const int r1 = 32 * ks + (PERM ? 16 + 4 * g : 8 * g + 4) + q;
  const int ch = 2 * i + (p >> 1), sub = 4 * (p & 1);
  const v4s lo = ds_read_tr16(S + r0 * 32 + 8 * (ch ^ swz_q(r0)) + sub);
  const v4s hi = ds_read_tr16(S + r1 * 32 + 8 * (ch ^ swz_q(r1)) + sub);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

#ifndef MINIPS_GEMM_V4_PRIO
#define MINIPS_GEMM_V4_PRIO 1
#endif
#ifndef MINIPS_GEMM_V4_GROUP
#define MINIPS_GEMM_V4_GROUP 4
#endif

// Tile (tm, tn) of block `bid`: XCD-contiguous runs (T1, bijective), row-grouped inside a run.
__device__ __forceinline__ void v4_tile(int bid, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int nwg = tiles_m * tiles_n;
  if (nwg >= 16) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    bid = base + (bid >> 3);
  }
  constexpr int G = MINIPS_GEMM_V4_GROUP;
  const int per_group = G * tiles_n, group = bid / per_group;
  const int first = group * G, gsz = min(tiles_m - first, G), in = bid - group * per_group;
  tm = first + in % gsz;
  tn = in / gsz;
}

template <bool A_KM, bool B_KN, int EPI>
__global__ __launch_bounds__(512) void gemm_v4_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                      int M, int N, int K, int lda, int ldb, int k_chunk, EpiArgs ep) {
  constexpr bool PERM = A_KM && B_KN;
  constexpr int kA = 256 * BK2;  // A region of a buffer (8 quarters); B follows
  __shared__ __attribute__((aligned(1024))) bf16_t smem[2][2 * 256 * BK2];
  static_assert(sizeof(smem) >= sizeof(float) * 8 * kScrFloats, "epilogue scratch must fit the staging LDS");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = (N + 255) / 256, tiles_m = (M + 255) / 256;
  int tm, tn;
  v4_tile(blockIdx.x, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  {
    const int z = blockIdx.y, zo = z / ep.inner, zi = z - zo * ep.inner;
    A += zo * ep.sa_o + zi * ep.sa_i;
    B += zo * ep.sb_o + zi * ep.sb_i;
    const int64_t co = zo * ep.sc_o + zi * ep.sc_i + (int64_t)blockIdx.z * ep.sc_split;
    const bool f32 = EPI == kEpiStoreF32 || EPI == kEpiAtomicF32 || EPI == kEpiAccumF32 || EPI == kEpiFoldF32;
    ep.C = f32 ? (void*)((float*)ep.C + co) : (void*)((bf16_t*)ep.C + co);
  }
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0x7ffffff0, 0x00020000);
  const int kb = blockIdx.z * k_chunk;
  const int ke = min(K, kb + k_chunk);
  const int nt = ke > kb ? (ke - kb + BK2 - 1) / BK2 : 0;

  v4f acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  // this wave's piece of A quarter q (both 128-row halves: waves 0-3 -> half 0, 4-7 -> half 1)
  auto a_quarter = [&](int t, int q, int buf) {
    const int h = wave >> 2;
    dma_quarter<A_KM>(ra, lda, m0 + h * 128 + q * 32, kb + t * BK2, M, ke, smem[buf] + (h * 4 + q) * kQuarter,
                      wave & 3, lane);
  };
  auto b_half = [&](int t, int hh, int buf) {
    dma_tile<B_KN, 128, 8>(rb, ldb, n0 + hh * 128, kb + t * BK2, N, ke, smem[buf] + kA + hh * 128 * BK2, wave, lane);
  };

  if (nt > 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) a_quarter(0, q, 0);
    b_half(0, 0, 0);
    b_half(0, 1, 0);
  }
  if (nt > 1) {
#pragma unroll
    for (int q = 0; q < 4; ++q) a_quarter(1, q, 1);
    b_half(1, 0, 1);
    b_half(1, 1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // K-step 0 landed, K-step 1 in flight
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  for (int t = 0; t < nt; ++t) {
    const int buf = t & 1;
    const bf16_t* SA = smem[buf] + wr * 4 * kQuarter;
    const bf16_t* SB = smem[buf] + kA + (wc >> 1) * 128 * BK2;
    const int bcol = (wc & 1) * 64;
    const bool more2 = t + 2 < nt;
    v8s bfr[4][2], af[2][2][2];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // ---- DMA of this phase (into regions every wave finished reading before the last barrier)
      if (q == 0) {
        if (t >= 1 && t + 1 < nt) a_quarter(t + 1, 3, buf ^ 1);
      } else if (more2) {
        a_quarter(t + 2, q - 1, buf);
        if (q < 3) b_half(t + 2, q - 1, buf);
      }
      // ---- fragments: all B + A quarter 0 at phase 0, then A quarter q + 1 ahead of its phase
      if (q == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) bfr[j][ks] = frag2<B_KN, PERM, 128>(SB, bcol + 16 * j, ks, lane);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) af[0][i][ks] = frag_quarter<A_KM, PERM>(SA, i, ks, lane);
      }
      if (q < 3) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            af[(q + 1) & 1][i][ks] = frag_quarter<A_KM, PERM>(SA + (q + 1) * kQuarter, i, ks, lane);
      }
      if (MINIPS_GEMM_V4_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[2 * q + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(v8bf, af[q & 1][i][ks]), __builtin_bit_cast(v8bf, bfr[j][ks]), acc[2 * q + i][j], 0,
                0, 0);
      if (MINIPS_GEMM_V4_PRIO) __builtin_amdgcn_s_setprio(0);
      if (q < 3) {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave's reads of quarter q (and of B at q = 0) retired
        asm volatile("" ::: "memory");
      }
    }
    // ---- end of the K-step: K-step t + 1 landed (K-step t + 2's 7 DMAs may stay in flight)
    if (t + 1 < nt) {
      if (more2) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // the staging LDS becomes the epilogue scratch
  asm volatile("" ::: "memory");
  epilogue_lds<EPI, 8>(acc, ep, M, N, m0 + wr * 128, n0 + wc * 64, lane,
                       reinterpret_cast<float*>(&smem[0][0]) + wave * kScrFloats);
}

// ================================================================ v5: 256x256, 8 waves, ping-pong
// The 256x256 / BK = 64 / 8-wave tile (2 (M) x 4 (N) waves of 128 x 64) with the two 4-wave row
// groups STAGGERED by one barrier: every phase is {ds_reads + DMA issue | barrier | 16 MFMAs |
// barrier} and group 1 runs one barrier behind group 0, so at any moment one group issues its
// LDS reads and DMAs while the other runs its MFMA cluster (the ping-pong that keeps the matrix
// cores fed at one workgroup per CU). A K-step is 4 phases over the wave's quadrants:
//   q0: A rows 0-63 (8 frags) + B n-tiles 0-1 (4) -> acc[0..3][0..1]
//   q1: B n-tiles 2-3 (4)                          -> acc[0..3][2..3]
//   q2: A rows 64-127 (8)                          -> acc[4..7][0..1]
//   q3: -                                          -> acc[4..7][2..3]
// LDS: [buf][A0 | A1 | B0 | B1] half tiles of 16 KiB (the v2 swizzled images), 2 buffers = 128 KiB.
// A half g is staged and read by row group g only (two 64-row DMA parts, or one 128-row part for
// KM operands); the B halves by all 8 waves. Staging of K-step t+1 runs through the phases of K-step
// t (B0 at q3 of t-1, B1 at q0, A lo at q1, A hi at q2: each region is refilled >= 1 barrier after
// every wave's reads of it retired), and two counted waits retire it: vmcnt at q3 (everything but
// A hi and the next step's B0) and vmcnt at q1 of t+1 (A hi, read at q2). Every read follows the
// issuing waves' wait by at least one barrier of the reading group, counted with the stagger.
template <bool A_KM, bool B_KN, int EPI>
__global__ __launch_bounds__(512) void gemm_v5_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                      int M, int N, int K, int lda, int ldb, int k_chunk, EpiArgs ep) {
  constexpr bool PERM = A_KM && B_KN;
  constexpr int kHalf = 128 * BK2;  // bf16 elements of one half-tile image
  __shared__ __attribute__((aligned(1024))) bf16_t smem[2][4 * kHalf];
  static_assert(sizeof(smem) >= sizeof(float) * 8 * kScrFloats, "epilogue scratch must fit the staging LDS");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3, gw = wave & 3;
  // wave-uniform in a scalar register: the stagger's extra s_barrier must be a scalar branch
  const bool group1 = __builtin_amdgcn_readfirstlane(tid) >= 256;
  const int tiles_n = (N + 255) / 256, tiles_m = (M + 255) / 256;
  int tm, tn;
  v4_tile(blockIdx.x, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  {
    const int z = blockIdx.y, zo = z / ep.inner, zi = z - zo * ep.inner;
    A += zo * ep.sa_o + zi * ep.sa_i;
    B += zo * ep.sb_o + zi * ep.sb_i;
    const int64_t co = zo * ep.sc_o + zi * ep.sc_i + (int64_t)blockIdx.z * ep.sc_split;
    const bool f32 = EPI == kEpiStoreF32 || EPI == kEpiAtomicF32 || EPI == kEpiAccumF32 || EPI == kEpiFoldF32;
    ep.C = f32 ? (void*)((float*)ep.C + co) : (void*)((bf16_t*)ep.C + co);
  }
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0x7ffffff0, 0x00020000);
  const int kb = blockIdx.z * k_chunk;
  const int ke = min(K, kb + k_chunk);
  const int nt = ke > kb ? (ke - kb + BK2 - 1) / BK2 : 0;

  v4f acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  // DMA issue per thread: B half 2, A part 2 (MK: 64 rows) or 4 (KM: the whole 128-row half)
  auto stage_b = [&](int t, int h, int buf) {
    dma_tile<B_KN, 128, 8>(rb, ldb, n0 + h * 128, kb + t * BK2, N, ke, smem[buf] + (2 + h) * kHalf, wave, lane);
  };
  auto stage_a = [&](int t, int part, int buf) {
    bf16_t* S = smem[buf] + wr * kHalf;
    if constexpr (!A_KM)
      dma_tile<false, 64, 4>(ra, lda, m0 + wr * 128 + part * 64, kb + t * BK2, M, ke, S + part * 64 * BK2, gw, lane);
    else if (part == 0)
      dma_tile<true, 128, 4>(ra, lda, m0 + wr * 128, kb + t * BK2, M, ke, S, gw, lane);
  };
  auto bar = [] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // vmcnt of the q1 wait (A hi of this K-step) / the q3 wait (the next K-step but its A hi),
  // steady state: DMAs issued after the one to retire (MK: 2 per stage; KM: A is one 4-DMA stage
  // at q1 and nothing at q2, so the q1 wait has nothing to retire and q3 waits for all but B0)
  constexpr int kVmQ1 = A_KM ? 8 : 6;
  constexpr int kVmQ3 = A_KM ? 2 : 4;

  if (nt > 0) {
    stage_b(0, 0, 0);
    stage_b(0, 1, 0);
    stage_a(0, 0, 0);
    stage_a(0, 1, 0);
  }
  if (nt > 1) {
    stage_b(1, 0, 1);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // K-step 0 landed, B0 of K-step 1 in flight
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();
  if (group1) bar();  // the stagger: group 1 runs one barrier behind group 0

  const int bcol = (wc & 1) * 64;
  for (int t = 0; t < nt; ++t) {
    const int buf = t & 1, nb = buf ^ 1;
    const bool more1 = t + 1 < nt, more2 = t + 2 < nt;
    const bf16_t* SA = smem[buf] + wr * kHalf;
    const bf16_t* SB = smem[buf] + (2 + (wc >> 1)) * kHalf;
    v8s af[4][2], bf0[2][2], bf1[2][2];
    // ---- q0
    if (more1) stage_b(t + 1, 1, nb);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) af[i][ks] = frag2<A_KM, PERM, 128>(SA, 16 * i, ks, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) bf0[j][ks] = frag2<B_KN, PERM, 128>(SB, bcol + 16 * j, ks, lane);
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, af[i][ks]),
                                                              __builtin_bit_cast(v8bf, bf0[j][ks]), acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // ---- q1
    if (more1) {
      stage_a(t + 1, 0, nb);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kVmQ1) : "memory");  // A hi of this K-step landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) bf1[j][ks] = frag2<B_KN, PERM, 128>(SB, bcol + 32 + 16 * j, ks, lane);
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(v8bf, af[i][ks]), __builtin_bit_cast(v8bf, bf1[j][ks]), acc[i][2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // ---- q2
    if (more1) stage_a(t + 1, 1, nb);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) af[i][ks] = frag2<A_KM, PERM, 128>(SA, 64 + 16 * i, ks, lane);
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(v8bf, af[i][ks]), __builtin_bit_cast(v8bf, bf0[j][ks]), acc[4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // ---- q3: B0 of K-step t + 2 into this buffer (every wave's B reads of it retired at q1)
    if (more2) {
      stage_b(t + 2, 0, buf);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kVmQ3) : "memory");  // K-step t+1 landed but A hi
    } else if (more1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kVmQ3 - 2) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 + i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(v8bf, af[i][ks]), __builtin_bit_cast(v8bf, bf1[j][ks]), acc[4 + i][2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar();
  }
  if (!group1) bar();  // group 0 catches up the stagger barrier
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  bar();  // the staging LDS becomes the epilogue scratch
  epilogue_lds<EPI, 8>(acc, ep, M, N, m0 + wr * 128, n0 + wc * 64, lane,
                       reinterpret_cast<float*>(&smem[0][0]) + wave * kScrFloats);
}

// v4 selection (MINIPS_GEMM_V4 at start-up, gemm_set_v4_mode() at run time for in-process A/B):
// 0 off, 1 where the 256x256 tile is picked, 2 every shape; v5 (ping-pong): 3 where the 256x256
// tile is picked, 4 every shape
inline int& gemm_v4_mode_ref() {
  static int mode = [] {
    const char* e = std::getenv("MINIPS_GEMM_V4");
    return e ? std::atoi(e) : 0;
  }();
  return mode;
}
inline int gemm_v4_mode() { return gemm_v4_mode_ref(); }

inline int gemm_impl() {
  static const int v = [] {
    const char* e = std::getenv("MINIPS_GEMM_IMPL");
    return e ? std::atoi(e) : 2;
  }();
  return v;
}

template <bool A_KM, bool B_KN, int EPI>
int launch(const bf16_t* A, const bf16_t* B, int M, int N, int K, int lda, int ldb, int split_k,
                  const EpiArgs& ep, int batch, hipStream_t s) {
  int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  // v2 (LDS-DMA) needs every byte offset within one batch element below 2 GiB (32-bit voffset)
  const int64_t a_ext = (int64_t)((A_KM ? K : M) - 1) * lda + (A_KM ? M : K);
  const int64_t b_ext = (int64_t)((B_KN ? K : N) - 1) * ldb + (B_KN ? N : K);
  // measured (tools/bench_kernels.py gemm): v2 wins on forward / dgrad; the split-K wgrad (both operands
  // tr-read) stays on the register-staged BK=32 kernel, which is faster there
  // wgrad kernel (MINIPS_GEMM_WGRAD): v2 (default: LDS-DMA, tr-read operands, staged epilogue), v1
  // (register-staged BK=32, round-1 default), or v3 (256x256 phase-split tiles, split-K chosen by
  // ops.linear_wgrad for ~one workgroup per CU)
  static const int wgrad_mode = [] {
    const char* e = std::getenv("MINIPS_GEMM_WGRAD");
    if (!e) return 2;  // v2 + LDS-staged epilogue measured best in the W&D step (tools/gpu_wgrad_ab2.sh)
    return std::string(e) == "v3" ? 3 : (std::string(e) == "v2" ? 2 : 1);
  }();
  const bool wgrad = A_KM && B_KN;
  const bool v2_ok = a_ext * 2 < 0x7ff00000ll && b_ext * 2 < 0x7ff00000ll;
  if (EPI == kEpiFoldF32 && !v2_ok) throw std::runtime_error("gemm: the split-K fold needs operands < 2 GiB (v2)");
  if ((EPI == kEpiFoldF32 || (gemm_impl() == 2 && (!wgrad || wgrad_mode >= 2))) && v2_ok) {
    const int kper = (K + split_k - 1) / split_k;
    const int kc = (kper + BK2 - 1) / BK2 * BK2;
    const int nsplit = (K + kc - 1) / kc;
    // Tile choice by wave quantisation: a 256x256 workgroup fills a CU alone (128 KiB LDS), two
    // 128x128 ones share it; take the 256 tile when its last round of workgroups is at least as
    // full as the 128 tile's (it moves half the L2->LDS bytes per MFMA), else 128x128
    // (tools/bench_kernels.py gemm: gpt.fc 1536 vs 384 tiles -> 128 wins; W&D dgrad0 256 tiles -> 256 wins).
    static const int force_tile = [] {
      const char* e = std::getenv("MINIPS_GEMM_TILE");
      return e ? std::atoi(e) : 0;
    }();
    const int64_t work = (int64_t)batch * nsplit;
    const int64_t t256 = work * ((M + 255) / 256) * ((N + 255) / 256);
    const int64_t t128 = work * (int64_t)tiles;
    const double eff256 = (double)t256 / (double)(((t256 + 255) / 256) * 256);
    const double eff128 = (double)t128 / (double)(((t128 + 511) / 512) * 512);
    // MINIPS_WGRAD_TILE=256: split-K weight gradients (both operands K-major) on the 256x256 tile
    // (ops.linear_wgrad then sizes its splits for that tile)
    static const int wgrad_tile = [] {
      const char* e = std::getenv("MINIPS_WGRAD_TILE");
      return e ? std::atoi(e) : 0;
    }();
    const int pick = force_tile ? force_tile
                     : (wgrad && wgrad_tile) ? wgrad_tile
                     : ((wgrad && wgrad_mode == 3) || eff256 >= eff128 ? 256 : 128);
    // v3 (experimental, MINIPS_GEMM_V3=1): measured within +-3 % of v2 on the forward shapes and
    // 10-25 % slower on the tr-read (dgrad/wgrad) shapes (tools/gpu_v3.sh), so v2 stays the default
    static const bool v3 = [] {
      const char* e = std::getenv("MINIPS_GEMM_V3");
      return e && std::atoi(e) != 0;
    }();
    static const bool v3_early = [] {
      const char* e = std::getenv("MINIPS_GEMM_V3_EARLY");
      return !e || std::atoi(e) != 0;
    }();
    const bool use_v3 = EPI != kEpiFoldF32 && (v3 || (wgrad && wgrad_mode == 3));
    const int v4 = EPI == kEpiFoldF32 ? 0 : gemm_v4_mode();  // the fold tail lives in v2 only
    if (EPI != kEpiWdHead && EPI != kEpiFoldF32 && (v4 == 6 || (v4 == 5 && pick == 256))) {
      dim3 grid(((M + 255) / 256) * ((N + 255) / 256), batch, nsplit);
      EpiArgs e6 = ep;
      e6.zmap = 1;
      hipLaunchKernelGGL((gemm_v6_kernel<A_KM, B_KN, EPI>), grid, dim3(256), 0, s, A, B, M, N, K, lda, ldb, kc, e6);
    } else if (EPI != kEpiWdHead && (v4 == 4 || (v4 == 3 && pick == 256))) {
      dim3 grid(((M + 255) / 256) * ((N + 255) / 256), batch, nsplit);
      hipLaunchKernelGGL((gemm_v5_kernel<A_KM, B_KN, EPI>), grid, dim3(512), 0, s, A, B, M, N, K, lda, ldb, kc, ep);
    } else if (v4 == 2 || (v4 == 1 && pick == 256)) {  // 2: v4 for every shape
      dim3 grid(((M + 255) / 256) * ((N + 255) / 256), batch, nsplit);
      hipLaunchKernelGGL((gemm_v4_kernel<A_KM, B_KN, EPI>), grid, dim3(512), 0, s, A, B, M, N, K, lda, ldb, kc, ep);
    } else if (pick == 256 && use_v3) {
      dim3 grid(((M + 255) / 256) * ((N + 255) / 256), batch, nsplit);
      if (v3_early)
        hipLaunchKernelGGL((gemm_v3_kernel<A_KM, B_KN, EPI, true>), grid, dim3(512), 0, s, A, B, M, N, K, lda, ldb, kc,
                           ep);
      else
        hipLaunchKernelGGL((gemm_v3_kernel<A_KM, B_KN, EPI, false>), grid, dim3(512), 0, s, A, B, M, N, K, lda, ldb,
                           kc, ep);
    } else {
      // MINIPS_GEMM_ZMAP: split-K slice-major XCD runs (EpiArgs::zmap)
      static const int zmap = [] {
        const char* e = std::getenv("MINIPS_GEMM_ZMAP");
        return e ? std::atoi(e) : 1;
      }();
      EpiArgs e2 = ep;
      e2.zmap = zmap;
      if (pick == 256) {
        dim3 grid(((M + 255) / 256) * ((N + 255) / 256), batch, nsplit);
        hipLaunchKernelGGL((gemm_v2_kernel<256, 256, A_KM, B_KN, EPI>), grid, dim3(1024), 0, s, A, B, M, N, K, lda,
                           ldb, kc, e2);
      } else if (pick == 200) {  // 256 x 128
        dim3 grid(((M + 255) / 256) * ((N + 127) / 128), batch, nsplit);
        hipLaunchKernelGGL((gemm_v2_kernel<256, 128, A_KM, B_KN, EPI>), grid, dim3(512), 0, s, A, B, M, N, K, lda,
                           ldb, kc, e2);
      } else {
        dim3 grid(tiles, batch, nsplit);
        hipLaunchKernelGGL((gemm_v2_kernel<128, 128, A_KM, B_KN, EPI>), grid, dim3(256), 0, s, A, B, M, N, K, lda,
                           ldb, kc, e2);
      }
    }
    return nsplit;
  }
  if (EPI == kEpiXentStatsBf16 || EPI == kEpiFoldF32)
    throw std::runtime_error("gemm: the xent-stats / split-K fold epilogues need the v2 kernel");
  // BK=64 halves the barriers per FLOP; short K chunks keep BK=32 (less tail waste).
  const int kper = (K + split_k - 1) / split_k;
  static const int forced = [] {
    const char* e = std::getenv("MINIPS_GEMM_BK");
    return e ? std::atoi(e) : 0;
  }();
  // measured: BK=64 wins on the forward/dgrad shapes, BK=32 on the split-K wgrad (tr-read) shapes
  const bool bk64 = forced ? forced == 64 : (kper >= 256 && !(A_KM && B_KN));
  const int BKs = bk64 ? 64 : 32;
  int kc = (kper + BKs - 1) / BKs * BKs;
  int nsplit = (K + kc - 1) / kc;
  dim3 grid(tiles, batch, nsplit);
  if (bk64)
    hipLaunchKernelGGL((gemm_bf16_kernel<64, A_KM, B_KN, EPI>), grid, dim3(256), 0, s, A, B, M, N, K, lda, ldb, kc, ep);
  else
    hipLaunchKernelGGL((gemm_bf16_kernel<32, A_KM, B_KN, EPI>), grid, dim3(256), 0, s, A, B, M, N, K, lda, ldb, kc, ep);
  return nsplit;
}

#define MINIPS_EPI_CASE(AKM, BKN, E)                                          \
  case E:                                                                     \
    nsplit = launch<AKM, BKN, E>(A, B, M, N, K, lda, ldb, split_k, ep, batch, s); \
    break;
#define MINIPS_GEMM_EPI_DISPATCH(AKM, BKN)                                        \
  switch (epi) {                                                                 \
    MINIPS_EPI_CASE(AKM, BKN, kEpiStoreF32)                                      \
    MINIPS_EPI_CASE(AKM, BKN, kEpiAtomicF32)                                     \
    MINIPS_EPI_CASE(AKM, BKN, kEpiBiasReluBf16)                                  \
    MINIPS_EPI_CASE(AKM, BKN, kEpiBiasBf16)                                      \
    MINIPS_EPI_CASE(AKM, BKN, kEpiBiasGeluBf16)                                  \
    MINIPS_EPI_CASE(AKM, BKN, kEpiStoreBf16)                                     \
    MINIPS_EPI_CASE(AKM, BKN, kEpiReluMaskBf16)                                  \
    MINIPS_EPI_CASE(AKM, BKN, kEpiBiasGeluAuxBf16)                               \
    MINIPS_EPI_CASE(AKM, BKN, kEpiGeluGradBf16)                                  \
    MINIPS_EPI_CASE(AKM, BKN, kEpiPermRowsBf16)                                  \
    MINIPS_EPI_CASE(AKM, BKN, kEpiAccumF32)                                      \
    MINIPS_EPI_CASE(AKM, BKN, kEpiBiasGeluDAuxBf16)                              \
    MINIPS_EPI_CASE(AKM, BKN, kEpiMulAuxBf16)                                    \
    MINIPS_EPI_CASE(AKM, BKN, kEpiFoldF32)                                       \
    case kEpiXentStatsBf16:                                                      \
      if constexpr (!AKM && !BKN) {                                              \
        nsplit = launch<false, false, kEpiXentStatsBf16>(A, B, M, N, K, lda, ldb, split_k, ep, batch, s); \
        break;                                                                   \
      }                                                                          \
      [[fallthrough]];                                                           \
    default:                                                                     \
      throw std::runtime_error("gemm: unknown epilogue " + std::to_string(epi)); \
  }


// One operand layout's epilogue dispatch (gemm_l<AKM><BKN>.hip); returns the K splits launched.
template <bool AKM, bool BKN>
int gemm_dispatch(int epi, const bf16_t* A, const bf16_t* B, int M, int N, int K, int lda, int ldb, int split_k,
                  const EpiArgs& ep, int batch, hipStream_t s);
template <>
int gemm_dispatch<false, false>(int epi, const bf16_t* A, const bf16_t* B, int M, int N, int K, int lda, int ldb,
                            int split_k, const EpiArgs& ep, int batch, hipStream_t s);
template <>
int gemm_dispatch<false, true>(int epi, const bf16_t* A, const bf16_t* B, int M, int N, int K, int lda, int ldb,
                            int split_k, const EpiArgs& ep, int batch, hipStream_t s);
template <>
int gemm_dispatch<true, true>(int epi, const bf16_t* A, const bf16_t* B, int M, int N, int K, int lda, int ldb,
                            int split_k, const EpiArgs& ep, int batch, hipStream_t s);
template <>
int gemm_dispatch<true, false>(int epi, const bf16_t* A, const bf16_t* B, int M, int N, int K, int lda, int ldb,
                            int split_k, const EpiArgs& ep, int batch, hipStream_t s);

}  // namespace minips_k
