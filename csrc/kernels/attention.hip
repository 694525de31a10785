// Fused causal self-attention for gfx950 (GPT-2: head dim 64), flash-style: the T x T score
// matrix never reaches HBM.
//
//   attn_fwd    O = softmax(mask(Q K^T * scale)) V, plus the per-query log-sum-exp (log2 units)
//   attn_prep   delta[q] = sum_d dO[q,d] O[q,d]
//   attn_bwd_dq dQ = scale * dS K                  (workgroup = 128 queries, sweeps key tiles)
//   attn_bwd_dkv dV = P^T dO, dK = scale * dS^T Q   (workgroup = 128 keys, sweeps query tiles)
//   with P = exp2(S*scale*log2e - lse), dS = P * (dP - delta), dP = dO V^T recomputed per tile.
//
// Q/K/V are read in place from the fused qkv activation [B*T][3*d] (head h at columns h*64,
// d + h*64, 2d + h*64); O/dO/dQKV are row-major [B*T][ld] with head h at column h*64.
//
// MFMA v_mfma_f32_16x16x32_bf16 everywhere. The "key on the lane" trick: the forward and the
// dQ kernel compute S^T = K Q^T (M = keys, N = queries), so each accumulator lane holds four keys
// of one query: the online-softmax statistics of a query live in the 4 lanes that share
// lane&15 (two xor-shuffles), and the accumulators of two adjacent 16-key tiles ARE the B
// operand of the next product over keys (P^T for O^T = V^T P^T, dS^T for dQ^T = K^T dS^T) in
// the permuted k order {4g..4g+3, 16+4g..16+4g+3}; the A operand of that product (V^T, K^T) is
// read from the row-major LDS tile with the transposing ds_read_b64_tr_b16 in the same order.
// The dK/dV kernel computes S = Q K^T (M = queries, N = keys) for the same reason: P and dS are
// then the B operands of dV^T = dO^T P and dK^T = Q^T dS. No LDS round trip of P or dS at all;
// dQ is produced by its own sweep instead of float atomics (deterministic, 7 products per tile
// pair instead of 5).
// K/V (or Q/dO) tiles are double-buffered in LDS with a one-tile register prefetch.
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"

namespace minips_k {
namespace {

typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
constexpr int HD = 64;        // head dim
constexpr int TILE = 64;      // keys (fwd, dq) or queries (dkv) per LDS tile
constexpr int WROWS = 32;     // queries (fwd, dq) or keys (dkv) per wave
constexpr int BROWS = 128;    // per workgroup (4 waves)
constexpr int LP = HD + 8;    // LDS pitch in bf16 (144 B)
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNegBig = -1.0e30f;

__device__ __forceinline__ v4f mfma(v8s a, v8s b, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b), c, 0, 0, 0);
}
__device__ __forceinline__ v4s tr16(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}
// Operand fragment of a row-major [row][64] LDS tile: 8 consecutive k (= columns 32ks + 8g ..)
// of row row_base + (lane & 15).
__device__ __forceinline__ v8s frag_rows(const bf16_t* S, int row_base, int ks, int lane) {
  return *reinterpret_cast<const v8s*>(S + (row_base + (lane & 15)) * LP + 32 * ks + 8 * (lane >> 4));
}
// Transposed operand fragment of the same tile: rows are the k dimension (32ks + permuted
// {4g..4g+3, 16+4g..16+4g+3}), columns col_base + (lane & 15) the m/n dimension.
__device__ __forceinline__ v8s frag_cols(const bf16_t* S, int col_base, int ks, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const v4s lo = tr16(S + (32 * ks + 4 * g + q) * LP + col_base + 4 * p);
  const v4s hi = tr16(S + (32 * ks + 16 + 4 * g + q) * LP + col_base + 4 * p);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// Same fragment straight from global memory (row-major, leading dim ld), zero past `rows`.
__device__ __forceinline__ v8s frag_global(const bf16_t* G, int64_t ld, int row, int rows, int ks, int lane) {
  if (row >= rows) return v8s{0, 0, 0, 0, 0, 0, 0, 0};
  return *reinterpret_cast<const v8s*>(G + (int64_t)row * ld + 32 * ks + 8 * (lane >> 4));
}
// Two accumulator tiles (16 k-rows each) -> one bf16 B/A fragment in the permuted k order.
__device__ __forceinline__ v8s pack_frag(const v4f& lo, const v4f& hi) {
  v8s r;
  const uint32_t a = pack_bf2(lo[0], lo[1]), b = pack_bf2(lo[2], lo[3]);
  const uint32_t c = pack_bf2(hi[0], hi[1]), d = pack_bf2(hi[2], hi[3]);
  r[0] = (short)(a & 0xffff);
  r[1] = (short)(a >> 16);
  r[2] = (short)(b & 0xffff);
  r[3] = (short)(b >> 16);
  r[4] = (short)(c & 0xffff);
  r[5] = (short)(c >> 16);
  r[6] = (short)(d & 0xffff);
  r[7] = (short)(d >> 16);
  return r;
}

// 64 x 64 bf16 tile (rows r0.., leading dim ld) -> 2 x 16 B per thread.
struct TileRegs {
  uint4 v[2];
};
__device__ __forceinline__ void tile_load(const bf16_t* G, int64_t ld, int r0, int rows, int tid, TileRegs& t) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = tid + h * 256, r = c >> 3, col = (c & 7) * 8;
    t.v[h] = (r0 + r < rows) ? *reinterpret_cast<const uint4*>(G + (int64_t)(r0 + r) * ld + col)
        : make_uint4(0, 0, 0, 0);
  }
}
__device__ __forceinline__ void tile_store(bf16_t* S, int tid, const TileRegs& t) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = tid + h * 256;
    *reinterpret_cast<uint4*>(S + (c >> 3) * LP + (c & 7) * 8) = t.v[h];
  }
}

// Four 16-row accumulator tiles stored as bf16 rows of a row-major matrix:
// acc[i][n] holds element [16i + 4g + qq][16n + (lane & 15)] of the transposed result (d x rows)
// -> out[row = 16n + lane&15][col = 16i + 4g .. +3] (8-byte store per tile).
__device__ __forceinline__ void store_transposed(bf16_t* out, int64_t ld, int row0, int rows, const v4f (&acc)[4][2],
                                                 float scale, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const int row = row0 + 16 * n + (lane & 15);
    if (row >= rows) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint2 u;
      u.x = pack_bf2(acc[i][n][0] * scale, acc[i][n][1] * scale);
      u.y = pack_bf2(acc[i][n][2] * scale, acc[i][n][3] * scale);
      *reinterpret_cast<uint2*>(out + (int64_t)row * ld + 16 * i + 4 * g) = u;
    }
  }
}

// ------------------------------------------------------------------------------ forward
// OCC = waves per SIMD the register allocation must allow (amdgpu_waves_per_eu): the compiler left
// to itself gave the forward 188 and the dK/dV kernel 290 registers (2 and 1 waves per SIMD: every
// exp / LDS / barrier latency exposed); capped at 3 and 2 waves they fit without scratch
template <int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void attn_fwd_kernel(
    const bf16_t* __restrict__ qkv, int ldq, int T, int H,
                                                       int dmodel, float sl2, bf16_t* __restrict__ O, int ldo,
                                                       float* __restrict__ lse) {
  __shared__ __attribute__((aligned(16))) bf16_t sm[2][2][TILE * LP];  // [buf][K|V]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  // 1-D grid, block -> (query block, head) with the heaviest (latest) query blocks of every head
  // dispatched first (causal work grows with the query index).
  const int nq = (T + BROWS - 1) / BROWS, BH = gridDim.x / nq;
  const int z = blockIdx.x % BH, b = z / H, h = z - b * H;
  const int q0 = (nq - 1 - (int)blockIdx.x / BH) * BROWS;
  const bf16_t* Qg = qkv + (int64_t)b * T * ldq + h * HD;
  const bf16_t* Kg = Qg + dmodel;
  const bf16_t* Vg = Qg + 2 * dmodel;
  const int qw = q0 + w * WROWS;
  const bool active = qw < T;

  v8s qf[2][2];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qf[n][ks] = frag_global(Qg, ldq, qw + 16 * n + (lane & 15), T, ks, lane);
  v4f o[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int n = 0; n < 2; ++n) o[i][n] = v4f{0.f, 0.f, 0.f, 0.f};
  float m[2] = {kNegBig, kNegBig}, l[2] = {0.f, 0.f};

  const int kend = min(T, q0 + BROWS);
  const int ntiles = (kend + TILE - 1) / TILE;
  TileRegs rk, rv;
  tile_load(Kg, ldq, 0, T, tid, rk);
  tile_load(Vg, ldq, 0, T, tid, rv);
  tile_store(sm[0][0], tid, rk);
  tile_store(sm[0][1], tid, rv);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1, k0 = t * TILE;
    const bool has_next = t + 1 < ntiles;
    if (has_next) {
      tile_load(Kg, ldq, k0 + TILE, T, tid, rk);
      tile_load(Vg, ldq, k0 + TILE, T, tid, rv);
    }
    if (active && k0 <= qw + WROWS - 1) {
      const bf16_t* SK = sm[cur][0];
      const bf16_t* SV = sm[cur][1];
      v4f s[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          s[i][n] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) s[i][n] = mfma(frag_rows(SK, 16 * i, ks, lane), qf[n][ks], s[i][n]);
        }
      const bool diag = k0 + TILE - 1 > qw;  // some key of the tile may be after some query
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int q = qw + 16 * n + (lane & 15);
        float mx = kNegBig;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            float v = s[i][n][qq] * sl2;
            if (diag && k0 + 16 * i + 4 * g + qq > q) v = kNegBig;
            s[i][n][qq] = v;
            mx = fmaxf(mx, v);
          }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mn = fmaxf(m[n], mx);
        const float alpha = __builtin_amdgcn_exp2f(m[n] - mn);
        m[n] = mn;
        float ls = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const float p = __builtin_amdgcn_exp2f(s[i][n][qq] - mn);
            s[i][n][qq] = p;
            ls += p;
          }
        l[n] = l[n] * alpha + ls;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i][n] *= alpha;
      }
      // O^T[d][q] += V^T[d][key] P^T[key][q]
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        v8s pf[2];
#pragma unroll
        for (int n = 0; n < 2; ++n) pf[n] = pack_frag(s[2 * ks][n], s[2 * ks + 1][n]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const v8s vf = frag_cols(SV, 16 * i, ks, lane);
#pragma unroll
          for (int n = 0; n < 2; ++n) o[i][n] = mfma(vf, pf[n], o[i][n]);
        }
      }
    }
    if (has_next) {
      tile_store(sm[cur ^ 1][0], tid, rk);
      tile_store(sm[cur ^ 1][1], tid, rv);
    }
    __syncthreads();
  }
  if (!active) return;
  float inv[2];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    float lt = l[n];
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    inv[n] = 1.f / lt;
    const int q = qw + 16 * n + (lane & 15);
    if (g == 0 && q < T) lse[(int64_t)z * T + q] = m[n] + log2f(lt);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int n = 0; n < 2; ++n) o[i][n] *= inv[n];
  store_transposed(O + (int64_t)b * T * ldo + h * HD, ldo, qw, T, o, 1.f, lane);
}

// ------------------------------------------------------------------------------ delta
// delta[z*T + t] = sum_d dO[b*T+t][h*64+d] * O[b*T+t][h*64+d]; 8 lanes per (row, head).
__global__ void attn_prep_kernel(const bf16_t* __restrict__ O, int ldo, const bf16_t* __restrict__ dO, int lddo,
                                 int64_t rows, int T, int H, float* __restrict__ delta) {
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t item = gid >> 3;  // (row, head)
  const int sub = gid & 7;
  float acc = 0.f;
  int64_t row = 0;
  int h = 0;
  if (item < rows * H) {
    row = item / H;
    h = (int)(item - row * H);
    const uint4 a = *reinterpret_cast<const uint4*>(O + row * ldo + h * HD + sub * 8);
    const uint4 c = *reinterpret_cast<const uint4*>(dO + row * lddo + h * HD + sub * 8);
    const uint32_t* pa = (const uint32_t*)&a;
    const uint32_t* pc = (const uint32_t*)&c;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      acc += __uint_as_float(pa[q] << 16) * __uint_as_float(pc[q] << 16) +
             __uint_as_float(pa[q] & 0xffff0000u) * __uint_as_float(pc[q] & 0xffff0000u);
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (item < rows * H && sub == 0) {
    const int64_t b = row / T, t = row - b * T;
    delta[(b * H + h) * T + t] = acc;
  }
}

// ------------------------------------------------------------------------------ dQ
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const bf16_t* __restrict__ qkv, int ldq,
                                                          const bf16_t* __restrict__ dO,
                                                          int lddo, const float* __restrict__ lse,
                                                          const float* __restrict__ delta, int T, int H, int dmodel,
                                                          float sl2, float scale, bf16_t* __restrict__ dqkv, int lddq) {
  __shared__ __attribute__((aligned(16))) bf16_t sm[2][2][TILE * LP];  // [buf][K|V]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int nq = (T + BROWS - 1) / BROWS, BH = gridDim.x / nq;
  const int z = blockIdx.x % BH, b = z / H, h = z - b * H;
  const int q0 = (nq - 1 - (int)blockIdx.x / BH) * BROWS;
  const bf16_t* Qg = qkv + (int64_t)b * T * ldq + h * HD;
  const bf16_t* Kg = Qg + dmodel;
  const bf16_t* Vg = Qg + 2 * dmodel;
  const bf16_t* dOg = dO + (int64_t)b * T * lddo + h * HD;
  const int qw = q0 + w * WROWS;
  const bool active = qw < T;

  v8s qf[2][2], df[2][2];
  float ls[2], dl[2];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const int q = qw + 16 * n + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qf[n][ks] = frag_global(Qg, ldq, q, T, ks, lane);
      df[n][ks] = frag_global(dOg, lddo, q, T, ks, lane);
    }
    ls[n] = q < T ? lse[(int64_t)z * T + q] : 0.f;
    dl[n] = q < T ? delta[(int64_t)z * T + q] : 0.f;
  }
  v4f dq[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int n = 0; n < 2; ++n) dq[i][n] = v4f{0.f, 0.f, 0.f, 0.f};

  const int kend = min(T, q0 + BROWS);
  const int ntiles = (kend + TILE - 1) / TILE;
  TileRegs rk, rv;
  tile_load(Kg, ldq, 0, T, tid, rk);
  tile_load(Vg, ldq, 0, T, tid, rv);
  tile_store(sm[0][0], tid, rk);
  tile_store(sm[0][1], tid, rv);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1, k0 = t * TILE;
    const bool has_next = t + 1 < ntiles;
    if (has_next) {
      tile_load(Kg, ldq, k0 + TILE, T, tid, rk);
      tile_load(Vg, ldq, k0 + TILE, T, tid, rv);
    }
    if (active && k0 <= qw + WROWS - 1) {
      const bf16_t* SK = sm[cur][0];
      const bf16_t* SV = sm[cur][1];
      v4f s[4][2], dp[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          s[i][n] = v4f{0.f, 0.f, 0.f, 0.f};
          dp[i][n] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            s[i][n] = mfma(frag_rows(SK, 16 * i, ks, lane), qf[n][ks], s[i][n]);
            dp[i][n] = mfma(frag_rows(SV, 16 * i, ks, lane), df[n][ks], dp[i][n]);
          }
        }
      const bool diag = k0 + TILE - 1 > qw;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int q = qw + 16 * n + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            float p = __builtin_amdgcn_exp2f(s[i][n][qq] * sl2 - ls[n]);
            if (diag && k0 + 16 * i + 4 * g + qq > q) p = 0.f;
            s[i][n][qq] = p * (dp[i][n][qq] - dl[n]);  // dS^T
          }
      }
      // dQ^T[d][q] += K^T[d][key] dS^T[key][q]
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        v8s sf[2];
#pragma unroll
        for (int n = 0; n < 2; ++n) sf[n] = pack_frag(s[2 * ks][n], s[2 * ks + 1][n]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const v8s kf = frag_cols(SK, 16 * i, ks, lane);
#pragma unroll
          for (int n = 0; n < 2; ++n) dq[i][n] = mfma(kf, sf[n], dq[i][n]);
        }
      }
    }
    if (has_next) {
      tile_store(sm[cur ^ 1][0], tid, rk);
      tile_store(sm[cur ^ 1][1], tid, rv);
    }
    __syncthreads();
  }
  if (!active) return;
  store_transposed(dqkv + (int64_t)b * T * lddq + h * HD, lddq, qw, T, dq, scale, lane);
}

// ------------------------------------------------------------------------------ dK, dV
template <int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void attn_bwd_dkv_kernel(
    const bf16_t* __restrict__ qkv, int ldq,
                                                           const bf16_t* __restrict__ dO, int lddo,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta, int T, int H, int dmodel,
                                                           float sl2, float scale, bf16_t* __restrict__ dqkv,
                                                               int lddq) {
  __shared__ __attribute__((aligned(16))) bf16_t sm[2][2][TILE * LP];  // [buf][Q|dO]
  __shared__ float srow[2][2][TILE];                                    // [buf][lse|delta]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int BH = gridDim.x / ((T + BROWS - 1) / BROWS);
  const int z = blockIdx.x % BH, b = z / H, h = z - b * H;
  const int k0b = ((int)blockIdx.x / BH) * BROWS;  // lowest key blocks (most query tiles) launch first
  const bf16_t* Qg = qkv + (int64_t)b * T * ldq + h * HD;
  const bf16_t* Kg = Qg + dmodel;
  const bf16_t* Vg = Qg + 2 * dmodel;
  const bf16_t* dOg = dO + (int64_t)b * T * lddo + h * HD;
  const float* lz = lse + (int64_t)z * T;
  const float* dz = delta + (int64_t)z * T;
  const int kw = k0b + w * WROWS;
  const bool active = kw < T;

  v8s kf[2][2], vf[2][2];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      kf[n][ks] = frag_global(Kg, ldq, kw + 16 * n + (lane & 15), T, ks, lane);
      vf[n][ks] = frag_global(Vg, ldq, kw + 16 * n + (lane & 15), T, ks, lane);
    }
  v4f dk[4][2], dv[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int n = 0; n < 2; ++n) dk[i][n] = dv[i][n] = v4f{0.f, 0.f, 0.f, 0.f};

  const int t0 = k0b / TILE, ntiles = (T + TILE - 1) / TILE;
  TileRegs rq, rd;
  float rl = 0.f, rdl = 0.f;
  auto load_rows = [&](int qt) {
    tile_load(Qg, ldq, qt * TILE, T, tid, rq);
    tile_load(dOg, lddo, qt * TILE, T, tid, rd);
    if (tid < TILE) {
      const int q = qt * TILE + tid;
      rl = q < T ? lz[q] : 0.f;
      rdl = q < T ? dz[q] : 0.f;
    }
  };
  auto store_rows = [&](int buf) {
    tile_store(sm[buf][0], tid, rq);
    tile_store(sm[buf][1], tid, rd);
    if (tid < TILE) {
      srow[buf][0][tid] = rl;
      srow[buf][1][tid] = rdl;
    }
  };
  if (t0 < ntiles) {
    load_rows(t0);
    store_rows(0);
  }
  __syncthreads();
  for (int t = t0; t < ntiles; ++t) {
    const int cur = (t - t0) & 1, qb = t * TILE;
    const bool has_next = t + 1 < ntiles;
    if (has_next) load_rows(t + 1);
    if (active && qb + TILE - 1 >= kw) {
      const bf16_t* SQ = sm[cur][0];
      const bf16_t* SD = sm[cur][1];
      v4f s[4][2], dp[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          s[i][n] = v4f{0.f, 0.f, 0.f, 0.f};
          dp[i][n] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            s[i][n] = mfma(frag_rows(SQ, 16 * i, ks, lane), kf[n][ks], s[i][n]);    // S[q][key]
            dp[i][n] = mfma(frag_rows(SD, 16 * i, ks, lane), vf[n][ks], dp[i][n]);  // dP[q][key]
          }
        }
      const bool diag = qb < kw + WROWS - 1;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int r = 16 * i + 4 * g + qq, q = qb + r;
          const float lq = srow[cur][0][r], dq = srow[cur][1][r];
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            float p = __builtin_amdgcn_exp2f(s[i][n][qq] * sl2 - lq);
            if ((diag && kw + 16 * n + (lane & 15) > q) || q >= T) p = 0.f;
            s[i][n][qq] = p;                          // P[q][key]
            dp[i][n][qq] = p * (dp[i][n][qq] - dq);   // dS[q][key]
          }
        }
      // dV^T[d][key] += dO^T[d][q] P[q][key] ; dK^T[d][key] += Q^T[d][q] dS[q][key]
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        v8s pf[2], sf[2];
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          pf[n] = pack_frag(s[2 * ks][n], s[2 * ks + 1][n]);
          sf[n] = pack_frag(dp[2 * ks][n], dp[2 * ks + 1][n]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const v8s dof = frag_cols(SD, 16 * i, ks, lane);
          const v8s qtf = frag_cols(SQ, 16 * i, ks, lane);
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            dv[i][n] = mfma(dof, pf[n], dv[i][n]);
            dk[i][n] = mfma(qtf, sf[n], dk[i][n]);
          }
        }
      }
    }
    if (has_next) store_rows(cur ^ 1);
    __syncthreads();
  }
  if (!active) return;
  bf16_t* base = dqkv + (int64_t)b * T * lddq + h * HD;
  store_transposed(base + dmodel, lddq, kw, T, dk, scale, lane);
  store_transposed(base + 2 * dmodel, lddq, kw, T, dv, 1.f, lane);
}

void check_attn(int T, int H, int dmodel, int ldq, int ldo) {
  if (dmodel != H * HD) throw std::runtime_error("attention: head dim must be 64");
  if (T <= 0 || ldq % 8 || ldo % 8) throw std::runtime_error("attention: leading dims must be multiples of 8");
}

}  // namespace

void attn_fwd(const bf16_t* qkv, int ldq, int B, int T, int H, int dmodel, float scale, bf16_t* O, int ldo, float* lse,
              hipStream_t s) {
  check_attn(T, H, dmodel, ldq, ldo);
  const int grid = ((T + BROWS - 1) / BROWS) * B * H;  // decoded as (block of T, head) in the kernels
  // 3 waves per SIMD (the register cap of the template argument; 2 = the uncapped allocation, slower)
  hipLaunchKernelGGL(attn_fwd_kernel<3>, grid, 256, 0, s, qkv, ldq, T, H, dmodel, scale * kLog2e, O, ldo, lse);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void attn_bwd(const bf16_t* qkv, int ldq, const bf16_t* O, int ldo, const bf16_t* dO, int lddo, const float* lse,
              float* delta, int B, int T, int H, int dmodel, float scale, bf16_t* dqkv, int lddq, hipStream_t s) {
  check_attn(T, H, dmodel, ldq, lddq);
  const int64_t rows = (int64_t)B * T;
  hipLaunchKernelGGL(attn_prep_kernel, (int)((rows * H * 8 + 255) / 256), 256, 0, s, O, ldo, dO, lddo, rows, T, H,
                     delta);
  MINIPS_HIP_CHECK(hipGetLastError());
  const int grid = ((T + BROWS - 1) / BROWS) * B * H;
  hipLaunchKernelGGL(attn_bwd_dq_kernel, grid, 256, 0, s, qkv, ldq, dO, lddo, lse, delta, T, H, dmodel, scale * kLog2e,
                     scale, dqkv, lddq);
  MINIPS_HIP_CHECK(hipGetLastError());
  // 2 waves per SIMD (1 = the uncapped allocation, slower)
  hipLaunchKernelGGL(attn_bwd_dkv_kernel<2>, grid, 256, 0, s, qkv, ldq, dO, lddo, lse, delta, T, H, dmodel,
                     scale * kLog2e, scale, dqkv, lddq);
  MINIPS_HIP_CHECK(hipGetLastError());
}

}  // namespace minips_k
