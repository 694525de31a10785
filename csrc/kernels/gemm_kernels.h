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
  int colsum_ld = 1;                  // kEpiReluMaskBf16: colsum[col * colsum_ld] (a column of a matrix)
  // split-K launches (gridDim.z > 1, gridDim.y == 1): deal (K slice, tile) pairs to the XCDs in
  // contiguous runs, tile fastest, so an XCD's workgroups share one K slice's operand rows through
  // its L2 (the plain tile remap gives each XCD whole tile rows over every slice: each XCD then
  // streams the full other operand)
  int zmap = 0;
  // host-side tile hint (128, 256 or 200 = 256x128; 0: the wave-quantisation choice) -- a GEMM
  // that runs beside another stream's workgroups may want the smaller tile (see launch)
  int tile = 0;
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
        } else if (EPI == kEpiStoreBf16 || EPI == kEpiPermRowsBf16) {
          ((bf16_t*)ep.C)[off] = f2bf(v);
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
  return v;  // kEpiStoreBf16 / kEpiPermRowsBf16 / kEpiStoreF32
}

template <int EPI, int MR>
__device__ __forceinline__ void epilogue_lds(const v4f (&acc)[MR][4], const EpiArgs& ep, int M, int N, int mb, int nb,
                                             int lane, float* __restrict__ scr) {
  constexpr bool F32OUT = EPI == kEpiStoreF32 || EPI == kEpiAtomicF32 || EPI == kEpiAccumF32;
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
    const bool f32 = EPI == kEpiStoreF32 || EPI == kEpiAtomicF32 || EPI == kEpiAccumF32;
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
  // (a grouped order for wide grids -- ~tiles_m / 8 row tiles walked column by column per XCD, so
  // the LM head's tiles share B panels in L2 -- measured slower: 676 -> 730 us on the logits GEMM)
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * TM, n0 = tn * TN;
  {
    const int z = blockIdx.y, zo = z / ep.inner, zi = z - zo * ep.inner;
    A += zo * ep.sa_o + zi * ep.sa_i;
    B += zo * ep.sb_o + zi * ep.sb_i;
    const int64_t co = zo * ep.sc_o + zi * ep.sc_i + (int64_t)ks * ep.sc_split;
    const bool f32 = EPI == kEpiStoreF32 || EPI == kEpiAtomicF32 || EPI == kEpiAccumF32;
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
  if (kLdsEpilogue)
    epilogue_lds<EPI, 4>(acc, ep, M, N, m0 + wm * 64, n0 + wn * 64, lane,
                         reinterpret_cast<float*>(&smem[0][0]) + wave * kScrFloats);
  else
    epilogue<EPI>(acc, ep, M, N, m0, n0, wm, wn, lane);
}

// MINIPS_GEMM_TILE (test / A-B knob, read once): 0 = auto, 128 / 200 (256x128) / 256 = force that v2
// tile, 1 = force the register-staged v1 kernel (otherwise only used past the 2 GiB LDS-DMA offset limit)
inline int gemm_force_tile() {
  static const int v = [] {
    const char* e = std::getenv("MINIPS_GEMM_TILE");
    return e ? std::atoi(e) : 0;
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
  const bool wgrad = A_KM && B_KN;
  const bool v2_ok = a_ext * 2 < 0x7ff00000ll && b_ext * 2 < 0x7ff00000ll;
  const int force = gemm_force_tile();
  // v2 (LDS-DMA, tr-read operands, LDS-staged epilogue) on every layout, split-K wgrads included:
  // measured best in the W&D step (tools/gpu_wgrad_ab2.sh) and on every tools/bench_kernels.py gemm shape
  if (force != 1 && v2_ok) {
    const int kper = (K + split_k - 1) / split_k;
    const int kc = (kper + BK2 - 1) / BK2 * BK2;
    const int nsplit = (K + kc - 1) / kc;
    // Tile choice by wave quantisation: a 256x256 workgroup fills a CU alone (128 KiB LDS), two
    // 128x128 ones share it; take the 256 tile when its last round of workgroups is at least as
    // full as the 128 tile's (it moves half the L2->LDS bytes per MFMA), else 128x128
    // (tools/bench_kernels.py gemm: gpt.fc 1536 vs 384 tiles -> 128 wins; W&D dgrad0 256 tiles -> 256 wins).
    const int64_t work = (int64_t)batch * nsplit;
    const int64_t t256 = work * ((M + 255) / 256) * ((N + 255) / 256);
    const int64_t t128 = work * (int64_t)tiles;
    const double eff256 = (double)t256 / (double)(((t256 + 255) / 256) * 256);
    const double eff128 = (double)t128 / (double)(((t128 + 511) / 512) * 512);
    const int pick = force ? force : ep.tile ? ep.tile : (eff256 >= eff128 ? 256 : 128);
    // (round 4's 8-wave 256x256 variants -- phase-split v3, quarter-staged v4, ping-pong v5 -- and
    // round 5's 4-wave 128x128-per-wave v6 and 4-deep ring of 32-deep K-steps v7 measured slower
    // than v2 on the model shapes and are gone: profiles/r4/gemm_*_v5.txt, profiles/r5/gemm_v7_ring.txt)
    EpiArgs e2 = ep;
    e2.zmap = 1;  // split-K slice-major XCD runs (EpiArgs::zmap)
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
    return nsplit;
  }
  // v1: BK=64 halves the barriers per FLOP; short K chunks and the split-K wgrad (tr-read) shapes
  // keep BK=32 (less tail waste; measured)
  const int kper = (K + split_k - 1) / split_k;
  const bool bk64 = kper >= 256 && !wgrad;
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
