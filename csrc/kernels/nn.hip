// Dense-model worker kernels (MLP, GPT-2-small, DLRM) for gfx950:
//   layernorm_fwd/bwd      row LayerNorm, bf16 activations, fp32 statistics, fp32 param grads
//   softmax_xent           fused softmax + cross-entropy forward/backward over [M, V] logits
//                          (MLP classes, GPT-2 vocab 50257): one block per row, 3 L2-resident passes
//   causal_softmax_fwd/bwd attention probabilities with the causal mask, one wave per row
//   gelu_bwd               dU = dH * gelu'(U)
//   add_bf16               residual adds
//   dlrm_interact_fwd/bwd  DLRM pairwise dot-product interaction (27 vectors x 64) per sample
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"

namespace minips_k {

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = warp_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float block_max(float v, float* red) {
  v = warp_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = -3.4e38f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t = fmaxf(t, red[i]);
  return t;
}

// ---------------------------------------------------------------------------- LayerNorm
// One wave per row; lane l owns columns k*256 + 4l .. +3 (k < 4), so C <= 1024, C % 4 == 0 and the
// row lives in registers between the statistics and the output pass (8-byte vector loads).
constexpr int kLnK = 4;

__device__ __forceinline__ void ld4(const bf16_t* p, float v[4]) {
  const uint2 u = *(const uint2*)p;
  v[0] = __uint_as_float(u.x << 16);
  v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16);
  v[3] = __uint_as_float(u.y & 0xffff0000u);
}
__device__ __forceinline__ void st4(bf16_t* p, const float v[4]) {
  uint2 u;
  u.x = pack_bf2(v[0], v[1]);
  u.y = pack_bf2(v[2], v[3]);
  *(uint2*)p = u;
}

__global__ __launch_bounds__(256) void layernorm_fwd_kernel(const bf16_t* __restrict__ x, int ldx, int64_t M, int C,
                                                            const bf16_t* __restrict__ gamma,
                                                            const bf16_t* __restrict__ beta, float eps,
                                                            bf16_t* __restrict__ y, int ldy,
                                                                float* __restrict__ mean_out,
                                                            float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  float gm[kLnK][4], bt[kLnK][4];
#pragma unroll
  for (int k = 0; k < kLnK; ++k) {
    const int c = k * 256 + lane * 4;
    if (c < C) {
      ld4(gamma + c, gm[k]);
      ld4(beta + c, bt[k]);
    }
  }
  for (int64_t r = wave; r < M; r += nw) {
    float v[kLnK][4];
    float s = 0.f, ss = 0.f;
#pragma unroll
    for (int k = 0; k < kLnK; ++k) {
      const int c = k * 256 + lane * 4;
      if (c < C) {
        ld4(x + r * ldx + c, v[k]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          s += v[k][q];
          ss += v[k][q] * v[k][q];
        }
      }
    }
    s = warp_sum(s);
    ss = warp_sum(ss);
    const float mu = s / C;
    const float rs = rsqrtf(fmaxf(ss / C - mu * mu, 0.f) + eps);
#pragma unroll
    for (int k = 0; k < kLnK; ++k) {
      const int c = k * 256 + lane * 4;
      if (c < C) {
        float o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (v[k][q] - mu) * rs * gm[k][q] + bt[k][q];
        st4(y + r * ldy + c, o);
      }
    }
    if (lane == 0) {
      mean_out[r] = mu;
      rstd_out[r] = rs;
    }
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma. dgamma/dbeta: every lane
// accumulates its own columns in registers over the wave's rows (no atomics). One wave per block,
// no LDS: the wave's column partials go straight to its partial row and layernorm_colsum adds the
// partials into dgamma/dbeta. (Round 4's 4-wave LDS-combining variant needed 32 KB of LDS, so
// beside a 256x256 GEMM workgroup (128 KB) only one of its blocks fit a CU; in GPT-2's backward it
// runs next to the side stream's weight-gradient GEMMs and lost: profiles/r4/ab_gpt2_ln_bwd.txt.)
__global__ __launch_bounds__(64) void layernorm_bwd_wave_kernel(const bf16_t* __restrict__ x, int ldx,
                                                                const bf16_t* __restrict__ dy, int lddy, int64_t M,
                                                                int C, const bf16_t* __restrict__ gamma,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ rstd,
                                                                bf16_t* __restrict__ dx, int lddx,
                                                                float* __restrict__ partial, bool accumulate_dx) {
  const int lane = threadIdx.x;
  float gm[kLnK][4], ag[kLnK][4], ab[kLnK][4];
#pragma unroll
  for (int k = 0; k < kLnK; ++k) {
    const int c = k * 256 + lane * 4;
    if (c < C) ld4(gamma + c, gm[k]);
#pragma unroll
    for (int q = 0; q < 4; ++q) ag[k][q] = ab[k][q] = 0.f;
  }
  for (int64_t r = blockIdx.x; r < M; r += gridDim.x) {
    const float mu = mean[r], rs = rstd[r];
    float xh[kLnK][4], g[kLnK][4];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int k = 0; k < kLnK; ++k) {
      const int c = k * 256 + lane * 4;
      if (c < C) {
        float d[4];
        ld4(x + r * ldx + c, xh[k]);
        ld4(dy + r * lddy + c, d);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          xh[k][q] = (xh[k][q] - mu) * rs;
          g[k][q] = d[q] * gm[k][q];
          a += g[k][q];
          b += g[k][q] * xh[k][q];
          ag[k][q] += d[q] * xh[k][q];
          ab[k][q] += d[q];
        }
      }
    }
    a = warp_sum(a) / C;
    b = warp_sum(b) / C;
#pragma unroll
    for (int k = 0; k < kLnK; ++k) {
      const int c = k * 256 + lane * 4;
      if (c < C) {
        float o[4], prev[4];
        if (accumulate_dx) ld4(dx + r * lddx + c, prev);
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = rs * (g[k][q] - a - xh[k][q] * b) + (accumulate_dx ? prev[q] : 0.f);
        st4(dx + r * lddx + c, o);
      }
    }
  }
  float* out = partial + (int64_t)blockIdx.x * 2 * C;
#pragma unroll
  for (int k = 0; k < kLnK; ++k) {
    const int c = k * 256 + lane * 4;
    if (c < C) {
      *reinterpret_cast<float4*>(out + c) = make_float4(ag[k][0], ag[k][1], ag[k][2], ag[k][3]);
      *reinterpret_cast<float4*>(out + C + c) = make_float4(ab[k][0], ab[k][1], ab[k][2], ab[k][3]);
    }
  }
}

// dgamma/dbeta[j] += sum_g partial[g][j], j < 2C: 64 columns per block (coalesced rows), the
// block's 4 waves split the G partial rows and combine in LDS.
// blockIdx.y takes a slice of the G partial rows (kColsumSlices slices, fp32 atomics into the
// parameter gradients) so the reduction spreads over ~24 x 16 blocks instead of 24 serial ones.
constexpr int kColsumSlices = 16;

__global__ __launch_bounds__(256) void layernorm_colsum_kernel(const float* __restrict__ partial, int G, int C,
                                                               float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  const int per = (G + gridDim.y - 1) / gridDim.y;
  const int g0 = blockIdx.y * per, g1 = min(G, g0 + per);
  float s = 0.f;
  if (j < 2 * C)
    for (int g = g0 + w; g < g1; g += 4) s += partial[(int64_t)g * 2 * C + j];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && j < 2 * C) {
    const float t = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    if (gridDim.y == 1) {
      if (j < C)
        dgamma[j] += t;
      else
        dbeta[j - C] += t;
    } else {
      atomicAdd(j < C ? dgamma + j : dbeta + (j - C), t);
    }
  }
}

// 8 rows per wave: GPT-2 12.69-12.70 vs 12.74-12.75 ms/step (4 rows 12.86, 16 rows 13.2;
// profiles/r4/ab_gpt2_ln_bwd.txt). Its blocks are the partial rows.
static int ln_bwd_wave_blocks(int64_t M) {
  return (int)std::min<int64_t>(std::max<int64_t>((M + 7) / 8, 1), 4096);
}

// partial rows of layernorm_bwd (the scratch it needs: rows * 2 * C floats)
int layernorm_bwd_blocks(int64_t M) { return ln_bwd_wave_blocks(M); }

void layernorm_fwd(const bf16_t* x, int ldx, int64_t M, int C, const bf16_t* gamma, const bf16_t* beta, float eps,
                   bf16_t* y, int ldy, float* mean, float* rstd, hipStream_t s) {
  if (M <= 0) return;
  if (C > 1024 || C % 4) throw std::runtime_error("layernorm: C <= 1024 and C % 4 == 0");
  hipLaunchKernelGGL(layernorm_fwd_kernel, grid_for(M * 64, 256, 4096), 256, 0, s, x, ldx, M, C, gamma, beta, eps, y,
                     ldy, mean, rstd);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void layernorm_bwd(const bf16_t* x, int ldx, const bf16_t* dy, int lddy, int64_t M, int C, const bf16_t* gamma,
                   const float* mean, const float* rstd, bf16_t* dx, int lddx, float* dgamma, float* dbeta,
                   float* partial, bool accumulate_dx, hipStream_t s) {
  if (M <= 0) return;
  if (C > 1024 || C % 4) throw std::runtime_error("layernorm: C <= 1024 and C % 4 == 0");
  const int G = ln_bwd_wave_blocks(M);
  hipLaunchKernelGGL(layernorm_bwd_wave_kernel, G, 64, 0, s, x, ldx, dy, lddy, M, C, gamma, mean, rstd, dx, lddx,
                     partial, accumulate_dx);
  MINIPS_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(layernorm_colsum_kernel, dim3((2 * C + 63) / 64, G >= 64 ? kColsumSlices : 1), 256, 0, s,
                     partial, G, C, dgamma, dbeta);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------- softmax-xent
// logits are updated in place with the gradient ((softmax - onehot) * scale); columns [V, ld)
// inside the last 8-wide chunk are zeroed. One 1024-thread block per row; the row (up to
// 1024 * 8 * 7 = 57344 columns, GPT-2's 50304 included) stays in registers as PACKED 16-byte
// chunks (28 VGPRs), so HBM sees exactly one read and one write of the logits.
//   pass 1: per-thread online (max, sum of exp) over its chunks -> ONE block reduction of the
//           (max, sum) pairs (rescaled merge)
//   pass 2: g = exp(x - lse) * scale, packed stores
// An empty asm on the packed registers between the passes keeps the compiler from carrying the
// 56 unpacked floats of pass 1 into pass 2 (it did: 208 VGPRs, 2 waves/SIMD, one row per CU at a
// time -- 548 us for GPT-2's 8192 x 50304 logits, 3 TB/s).
constexpr int kXentThreads = 1024, kXentChunks = 7;

// Component q of a uint4 without taking its address (keeps the chunk array in registers).
__device__ __forceinline__ uint32_t u4get(const uint4& v, int q) { return q == 0 ? v.x : q == 1 ? v.y : q == 2
                                                                  ? v.z : v.w; }
__device__ __forceinline__ float u4elem(const uint4& v, int q) {
  const uint32_t w = u4get(v, q >> 1);
  return (q & 1) ? __uint_as_float(w & 0xffff0000u) : __uint_as_float(w << 16);
}

// (m, s) <- merge of two partial softmax denominators, in log2 units: s = sum 2^(x - m)
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  s = s * __builtin_amdgcn_exp2f(m - mn) + s2 * __builtin_amdgcn_exp2f(m2 - mn);
  m = mn;
}

__global__ __launch_bounds__(kXentThreads) void softmax_xent_kernel(bf16_t* __restrict__ logits, int ld, int64_t M,
                                                                    int V, const int64_t* __restrict__ labels,
                                                                    float scale, float* loss_sum, float* correct) {
  __shared__ float red_m[kXentThreads / 64], red_s[kXentThreads / 64], red_x[kXentThreads / 64];
  const int nfull = V >> 3;          // chunks with 8 valid columns
  const int tail = V & 7;            // valid columns of chunk nfull (0: none)
  const float L2E = 1.4426950408889634f;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // loss / hit sums accumulate in thread 0 over the block's rows: one atomic per block at the
  // end (one per row would serialise M same-address atomics at the memory side, ~12 ns each)
  float loss_acc = 0.f, hit_acc = 0.f;
  // the next row's chunks are loaded while this row is reduced and written (one block per CU:
  // the prefetch is what keeps HBM busy during the block's reductions)
  auto load_row = [&](int64_t r, uint4 (&dst)[kXentChunks]) {
    const bf16_t* row = logits + r * ld;
#pragma unroll
    for (int k = 0; k < kXentChunks; ++k) {
      const int ch = threadIdx.x + k * kXentThreads;
      dst[k] = (r < M && (ch < nfull || (ch == nfull && tail))) ? *reinterpret_cast<const uint4*>(row + ch * 8)
                                                               : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  uint4 vn[kXentChunks];
  load_row(blockIdx.x, vn);
  for (int64_t r = blockIdx.x; r < M; r += gridDim.x) {
    bf16_t* row = logits + r * ld;
    uint4 v[kXentChunks];
#pragma unroll
    for (int k = 0; k < kXentChunks; ++k) v[k] = vn[k];
    load_row(r + gridDim.x, vn);
    // pass 1 (log2 units): running max m and s = sum 2^(x*L2E - m) over this thread's values
    float m = -3.0e38f, sm = 0.f;
#pragma unroll
    for (int k = 0; k < kXentChunks; ++k) {
      const int ch = threadIdx.x + k * kXentThreads;
      const int nv = ch < nfull ? 8 : (ch == nfull ? tail : 0);
      if (nv == 0) continue;
      float x[8], cm = -3.0e38f;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        x[q] = q < nv ? u4elem(v[k], q) * L2E : -3.0e38f;
        cm = fmaxf(cm, x[q]);
      }
      float cs = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) cs += q < nv ? __builtin_amdgcn_exp2f(x[q] - cm) : 0.f;
      lse_merge(m, sm, cm, cs);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) lse_merge(m, sm, __shfl_xor(m, o, 64), __shfl_xor(sm, o, 64));
    const int64_t lab = labels[r];
    // the label's logit, read by its owner thread before any thread rewrites the row
    const bool has_lab = lab >= 0 && lab < V;
    const int lch = has_lab ? (int)(lab >> 3) : -1;
    float zl_part = 0.f;
#pragma unroll
    for (int k = 0; k < kXentChunks; ++k)
      if (threadIdx.x + k * kXentThreads == lch) zl_part = u4elem(v[k], (int)(lab & 7));
    const bool own = (lch >= 0) && ((lch % kXentThreads) == (int)threadIdx.x);
    zl_part = own ? zl_part : 0.f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) zl_part += __shfl_xor(zl_part, o, 64);
    __syncthreads();  // the previous row's readers of red_* are done
    if (lane == 0) {
      red_m[w] = m;
      red_s[w] = sm;
      red_x[w] = zl_part;
    }
    __syncthreads();
    float M2 = red_m[0], S2 = red_s[0], zl = red_x[0];
#pragma unroll
    for (int i = 1; i < kXentThreads / 64; ++i) {
      lse_merge(M2, S2, red_m[i], red_s[i]);
      zl += red_x[i];
    }
    const float lse2 = M2 + __log2f(S2);  // log2 of sum 2^(x*L2E)
    if (threadIdx.x == 0 && has_lab) {
      loss_acc += lse2 / L2E - zl;
      hit_acc += zl * L2E >= M2 ? 1.f : 0.f;
    }
    // pass 2: the packed registers only (asm: the unpacked pass-1 values are dead here)
#pragma unroll
    for (int k = 0; k < kXentChunks; ++k) asm volatile("" : "+v"(v[k].x), "+v"(v[k].y), "+v"(v[k].z), "+v"(v[k].w));
#pragma unroll
    for (int k = 0; k < kXentChunks; ++k) {
      const int ch = threadIdx.x + k * kXentThreads;
      const int nv = ch < nfull ? 8 : (ch == nfull ? tail : 0);
      if (nv == 0) continue;
      uint32_t o[4];
#pragma unroll
      for (int q2 = 0; q2 < 4; ++q2) {
        float g0 = __builtin_amdgcn_exp2f(u4elem(v[k], 2 * q2) * L2E - lse2) * scale;
        float g1 = __builtin_amdgcn_exp2f(u4elem(v[k], 2 * q2 + 1) * L2E - lse2) * scale;
        if (ch == lch) {  // the -onehot term, folded before rounding
          if ((int)(lab & 7) == 2 * q2) g0 -= scale;
          if ((int)(lab & 7) == 2 * q2 + 1) g1 -= scale;
        }
        o[q2] = pack_bf2(2 * q2 < nv ? g0 : 0.f, 2 * q2 + 1 < nv ? g1 : 0.f);
      }
      *reinterpret_cast<uint4*>(row + ch * 8) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
  if (threadIdx.x == 0) {
    atomicAdd(loss_sum, loss_acc);
    if (correct) atomicAdd(correct, hit_acc);
  }
}

// Few classes (V <= 64, the MLP's 10): one THREAD per row -- its <= 8 chunks stay in registers,
// neighbouring threads read neighbouring rows (coalesced), no block reductions per row. The
// block-per-row kernel above spends a 512-thread block and three barriers on each 10-wide row
// (143 us of the MLP's 340 us step at batch 8192).
constexpr int kXentSmallChunks = 8;
__global__ __launch_bounds__(256) void softmax_xent_small_kernel(bf16_t* __restrict__ logits, int ld, int64_t M,
                                                                 int V, const int64_t* __restrict__ labels,
                                                                 float scale, float* loss_sum, float* correct) {
  __shared__ float red[2][4];
  const float L2E = 1.4426950408889634f;
  const int nch = (V + 7) >> 3;
  float loss_acc = 0.f, hit_acc = 0.f;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < M; r += (int64_t)gridDim.x * blockDim.x) {
    bf16_t* row = logits + r * ld;
    uint4 v[kXentSmallChunks];
    float mx = -3.4e38f;
#pragma unroll
    for (int k = 0; k < kXentSmallChunks; ++k) {
      if (k < nch) {
        v[k] = *reinterpret_cast<const uint4*>(row + k * 8);
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (k * 8 + q < V) mx = fmaxf(mx, u4elem(v[k], q));
      }
    }
    const float ml2 = mx * L2E;
    float se = 0.f, zl = 0.f;
    const int64_t lab = labels[r];
#pragma unroll
    for (int k = 0; k < kXentSmallChunks; ++k) {
      if (k < nch) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float z = u4elem(v[k], q);
          if (k * 8 + q < V) se += __builtin_amdgcn_exp2f(z * L2E - ml2);
          if (k * 8 + q == lab) zl = z;
        }
      }
    }
    if (lab >= 0 && lab < V) {
      loss_acc += mx + __logf(se) - zl;
      hit_acc += zl >= mx ? 1.f : 0.f;
    }
    const float sinv = scale / se;
#pragma unroll
    for (int k = 0; k < kXentSmallChunks; ++k) {
      if (k < nch) {
        uint32_t o[4];
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) {
          float g[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int c = k * 8 + 2 * q2 + h;
            const float p = __builtin_amdgcn_exp2f(u4elem(v[k], 2 * q2 + h) * L2E - ml2) * sinv;
            g[h] = c < V ? p - (c == lab ? scale : 0.f) : 0.f;
          }
          o[q2] = pack_bf2(g[0], g[1]);
        }
        *reinterpret_cast<uint4*>(row + k * 8) = make_uint4(o[0], o[1], o[2], o[3]);
      }
    }
  }
  loss_acc = warp_sum(loss_acc);
  hit_acc = warp_sum(hit_acc);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][w] = loss_acc;
    red[1][w] = hit_acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(loss_sum, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    if (correct) atomicAdd(correct, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

void softmax_xent(bf16_t* logits, int ld, int64_t M, int V, const int64_t* labels, float scale, float* loss_sum,
                  float* correct, hipStream_t s) {
  if (M <= 0) return;
  if ((V + 7) / 8 > kXentThreads * kXentChunks || ld % 8 || ld < (V + 7) / 8 * 8)
    throw std::runtime_error("softmax_xent: V <= 53248 and ld % 8 == 0, ld >= align8(V)");
  if (V <= 8 * kXentSmallChunks) {
    hipLaunchKernelGGL(softmax_xent_small_kernel, (int)std::min<int64_t>((M + 255) / 256, 1024), 256, 0, s, logits,
                       ld, M, V, labels, scale, loss_sum, correct);
    MINIPS_HIP_CHECK(hipGetLastError());
    return;
  }
  // one 16-wave block per CU, each walking its rows with a one-row prefetch
  static const int ncu = [] {
    int dev = 0, n = 0;
    MINIPS_HIP_CHECK(hipGetDevice(&dev));
    MINIPS_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    return n > 0 ? n : 256;
  }();
  hipLaunchKernelGGL(softmax_xent_kernel, (int)std::min<int64_t>(M, ncu), kXentThreads, 0, s, logits, ld, M, V,
                     labels, scale, loss_sum, correct);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------- attention softmax
// S [Z][T][T] fp32 scores (already scaled) -> P bf16 with causal mask (col > row -> 0).
__global__ void causal_softmax_fwd_kernel(const float* __restrict__ S, int64_t rows, int T, bf16_t* __restrict__ P) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = wave; r < rows; r += nw) {
    const int i = (int)(r % T);
    const float* s = S + r * T;
    float mx = -3.4e38f;
    for (int c = lane; c <= i; c += 64) mx = fmaxf(mx, s[c]);
    mx = warp_max(mx);
    float se = 0.f;
    for (int c = lane; c <= i; c += 64) se += __expf(s[c] - mx);
    se = warp_sum(se);
    const float inv = 1.f / se;
    bf16_t* p = P + r * T;
    for (int c = lane; c < T; c += 64) p[c] = c <= i ? f2bf(__expf(s[c] - mx) * inv) : (bf16_t)0;
  }
}

// dS = P * (dP - rowsum(P * dP)) * scale  (dP fp32 [Z][T][T]) -> bf16
__global__ void causal_softmax_bwd_kernel(const bf16_t* __restrict__ P, const float* __restrict__ dP, int64_t rows,
                                          int T, float scale, bf16_t* __restrict__ dS) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = wave; r < rows; r += nw) {
    const int i = (int)(r % T);
    const bf16_t* p = P + r * T;
    const float* dp = dP + r * T;
    float dot = 0.f;
    for (int c = lane; c <= i; c += 64) dot += bf2f(p[c]) * dp[c];
    dot = warp_sum(dot);
    bf16_t* ds = dS + r * T;
    for (int c = lane; c < T; c += 64) ds[c] = c <= i ? f2bf(bf2f(p[c]) * (dp[c] - dot) * scale) : (bf16_t)0;
  }
}

void causal_softmax_fwd(const float* S, int64_t rows, int T, bf16_t* P, hipStream_t s) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(causal_softmax_fwd_kernel, grid_for(rows * 64, 256, 8192), 256, 0, s, S, rows, T, P);
  MINIPS_HIP_CHECK(hipGetLastError());
}
void causal_softmax_bwd(const bf16_t* P, const float* dP, int64_t rows, int T, float scale, bf16_t* dS,
                        hipStream_t s) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(causal_softmax_bwd_kernel, grid_for(rows * 64, 256, 8192), 256, 0, s, P, dP, rows, T, scale, dS);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------- elementwise
__device__ __forceinline__ float gelu_grad(float u) {
  const float k = 0.7978845608f, c = 0.044715f;
  const float t = tanhf(k * (u + c * u * u * u));
  return 0.5f * (1.f + t) + 0.5f * u * (1.f - t * t) * k * (1.f + 3.f * c * u * u);
}

__global__ void gelu_bwd_kernel(const bf16_t* __restrict__ dh, const bf16_t* __restrict__ u, int64_t n,
                                bf16_t* __restrict__ du) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    du[i] = f2bf(bf2f(dh[i]) * gelu_grad(bf2f(u[i])));
}
void gelu_bwd(const bf16_t* dh, const bf16_t* u, int64_t n, bf16_t* du, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gelu_bwd_kernel, grid_for(n, 256), 256, 0, s, dh, u, n, du);
  MINIPS_HIP_CHECK(hipGetLastError());
}

__global__ void add_bf16_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b, int64_t n,
                                bf16_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = f2bf(bf2f(a[i]) + bf2f(b[i]));
}
void add_bf16(const bf16_t* a, const bf16_t* b, int64_t n, bf16_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(add_bf16_kernel, grid_for(n, 256), 256, 0, s, a, b, n, out);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------- token + position embedding
// out[m, :C] = wte[tok[m], :C] + wpe[m % T, :C]; 8 bf16 (16 B) per thread, C % 8 == 0.
__global__ void embed_fwd_kernel(const bf16_t* __restrict__ wte, const bf16_t* __restrict__ wpe,
                                 const int64_t* __restrict__ tok, int64_t M, int T, int C, bf16_t* __restrict__ out,
                                 int ldo) {
  const int cv = C >> 3;
  const int64_t n = M * cv;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / cv;
    const int c = (int)(i - m * cv) << 3;
    const uint4 a = *(const uint4*)(wte + tok[m] * C + c);
    const uint4 b = *(const uint4*)(wpe + (m % T) * C + c);
    const uint32_t* pa = (const uint32_t*)&a;
    const uint32_t* pb = (const uint32_t*)&b;
    uint4 o;
    uint32_t* po = (uint32_t*)&o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float lo = __uint_as_float(pa[q] << 16) + __uint_as_float(pb[q] << 16);
      const float hi = __uint_as_float(pa[q] & 0xffff0000u) + __uint_as_float(pb[q] & 0xffff0000u);
      po[q] = pack_bf2(lo, hi);
    }
    *(uint4*)(out + m * ldo + c) = o;
  }
}
// dwte[tok[m]] += dx[m]; dwpe[m % T] += dx[m]   (fp32 atomics; token ids spread the wte rows)
__global__ void embed_bwd_kernel(const bf16_t* __restrict__ dx, int ldx, const int64_t* __restrict__ tok, int64_t M,
                                 int T, int C, float* __restrict__ dwte, float* __restrict__ dwpe) {
  const int cv = C >> 1;
  const int64_t n = M * cv;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / cv;
    const int c = (int)(i - m * cv) << 1;
    const uint32_t v = *(const uint32_t*)(dx + m * ldx + c);
    const float lo = __uint_as_float(v << 16), hi = __uint_as_float(v & 0xffff0000u);
    float* w = dwte + tok[m] * C + c;
    atomicAdd(w, lo);
    atomicAdd(w + 1, hi);
    float* p = dwpe + (m % T) * C + c;
    atomicAdd(p, lo);
    atomicAdd(p + 1, hi);
  }
}
void embed_fwd(const bf16_t* wte, const bf16_t* wpe, const int64_t* tok, int64_t M, int T, int C, bf16_t* out, int ldo,
               hipStream_t s) {
  if (M <= 0) return;
  hipLaunchKernelGGL(embed_fwd_kernel, grid_for(M * (C / 8), 256, 8192), 256, 0, s, wte, wpe, tok, M, T, C, out, ldo);
  MINIPS_HIP_CHECK(hipGetLastError());
}
void embed_bwd(const bf16_t* dx, int ldx, const int64_t* tok, int64_t M, int T, int C, float* dwte, float* dwpe,
               hipStream_t s) {
  if (M <= 0) return;
  hipLaunchKernelGGL(embed_bwd_kernel, grid_for(M * (C / 2), 256, 8192), 256, 0, s, dx, ldx, tok, M, T, C, dwte, dwpe);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------- DLRM interaction
// V [B][NV][D] bf16 -> out[b] = [V[b][dense_idx] (D) | V_i.V_j for i > j] at out + b*ldo.
// One block per sample (grid-stride); the sample's vectors are staged in LDS.
__device__ __forceinline__ void pair_of(int p, int* i, int* j) {
  int a = (int)((1.f + sqrtf(1.f + 8.f * p)) * 0.5f);
  while (a * (a - 1) / 2 > p) --a;
  while ((a + 1) * a / 2 <= p) ++a;
  *i = a;
  *j = p - a * (a - 1) / 2;
}

__global__ __launch_bounds__(256) void dlrm_interact_fwd_kernel(const bf16_t* __restrict__ V, int64_t B, int NV, int D,
                                                                int dense_idx, bf16_t* __restrict__ out, int ldo) {
  extern __shared__ float sv[];  // NV rows of D+1 floats (odd stride: lanes on different rows hit different banks)
  const int npairs = NV * (NV - 1) / 2;
  const int Dp = D + 1;
  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    const bf16_t* vb = V + b * NV * D;
    for (int e = threadIdx.x; e < NV * D; e += blockDim.x) sv[(e / D) * Dp + e % D] = bf2f(vb[e]);
    __syncthreads();
    bf16_t* ob = out + b * ldo;
    for (int d = threadIdx.x; d < D; d += blockDim.x) ob[d] = vb[dense_idx * D + d];
    for (int p = threadIdx.x; p < npairs; p += blockDim.x) {
      int i, j;
      pair_of(p, &i, &j);
      float acc = 0.f;
      for (int d = 0; d < D; ++d) acc += sv[i * Dp + d] * sv[j * Dp + d];
      ob[D + p] = f2bf(acc);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void dlrm_interact_bwd_kernel(const bf16_t* __restrict__ V, int64_t B, int NV, int D,
                                                                int dense_idx, const bf16_t* __restrict__ dout, int ldo,
                                                                float* __restrict__ dV, bf16_t* __restrict__ d_dense) {
  extern __shared__ float sm[];  // V: NV*D, dZ: NV*NV
  float* sv = sm;
  float* dz = sm + NV * D;
  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    const bf16_t* vb = V + b * NV * D;
    const bf16_t* ob = dout + b * ldo;
    for (int i = threadIdx.x; i < NV * D; i += blockDim.x) sv[i] = bf2f(vb[i]);
    for (int q = threadIdx.x; q < NV * NV; q += blockDim.x) {
      const int i = q / NV, j = q % NV;
      float g = 0.f;
      if (i != j) {
        const int hi = i > j ? i : j, lo = i > j ? j : i;
        g = bf2f(ob[D + hi * (hi - 1) / 2 + lo]);
      }
      dz[q] = g;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < NV * D; e += blockDim.x) {
      const int i = e / D, d = e % D;
      float acc = (i == dense_idx) ? bf2f(ob[d]) : 0.f;
      for (int j = 0; j < NV; ++j) acc += dz[i * NV + j] * sv[j * D + d];
      dV[b * NV * D + e] = acc;
      if (i == dense_idx) d_dense[b * D + d] = f2bf(sv[e] > 0.f ? acc : 0.f);
    }
    __syncthreads();
  }
}

// ---- MFMA interaction (NV <= 32, D in {16, 32, 64}): one wave per sample. The sample's NV x D
// matrix (padded to 32 rows, K padded to 32) is loaded straight into MFMA fragments (16 bytes per
// lane per fragment: row = lane & 15 of the tile, k = 8 * (lane >> 4)); Z = V V^T is three 16x16
// tiles of v_mfma_f32_16x16x32_bf16 (the lower triangle), written as the packed pairs.
typedef __bf16 v8bf_i __attribute__((ext_vector_type(8)));

__device__ __forceinline__ v8s load_frag(const bf16_t* vb, int NV, int D, int row, int k) {
  if (row < NV && k < D) return *reinterpret_cast<const v8s*>(vb + row * D + k);
  return v8s{0, 0, 0, 0, 0, 0, 0, 0};
}

template <int KS>  // K-steps of 32 (D = 16 -> 1 with zero padding, 32 -> 1, 64 -> 2)
__global__ __launch_bounds__(256) void dlrm_interact_fwd_mfma_kernel(const bf16_t* __restrict__ V, int64_t B, int NV,
                                                                     int D, int dense_idx, bf16_t* __restrict__ out,
                                                                     int ldo) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  if (b >= B) return;
  const bf16_t* vb = V + b * NV * D;
  v8s f[2][KS];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) f[t][ks] = load_frag(vb, NV, D, t * 16 + (lane & 15), ks * 32 + 8 * (lane >> 4));
  bf16_t* ob = out + b * ldo;
  if (lane * 8 < D)
    *reinterpret_cast<v8s*>(ob + lane * 8) = *reinterpret_cast<const v8s*>(vb + dense_idx * D + lane * 8);
#pragma unroll
  for (int tile = 0; tile < 3; ++tile) {  // (0,0), (1,0), (1,1)
    const int ti = tile == 0 ? 0 : 1, tj = tile == 2 ? 1 : 0;
    v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf_i, f[ti][ks]),
                                                    __builtin_bit_cast(v8bf_i, f[tj][ks]), acc, 0, 0, 0);
    const int col = tj * 16 + (lane & 15);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = ti * 16 + (lane >> 4) * 4 + e;
      if (row < NV && col < row) ob[D + row * (row - 1) / 2 + col] = f2bf(acc[e]);
    }
  }
}

// dV = dZ V with dZ the symmetric matrix of the packed pair gradients (+ the dense pass-through),
// one wave per sample: A = dZ fragments gathered from the packed dout (row = lane & 15 of the
// tile, 8 k's), B = V^T fragments read from the sample's V staged in LDS (column n = lane & 15,
// 8 consecutive vector indices), 2 x (D/16) output tiles of one v_mfma_f32_16x16x32_bf16 each.
template <int D, typename OutT>
__global__ __launch_bounds__(256) void dlrm_interact_bwd_mfma_kernel(const bf16_t* __restrict__ V, int64_t B, int NV,
                                                                     int dense_idx, const bf16_t* __restrict__ dout,
                                                                     int ldo, OutT* __restrict__ dV,
                                                                     bf16_t* __restrict__ d_dense) {
  __shared__ bf16_t sv[4][32 * D];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const bool valid = b < B;
  const bf16_t* vb = V + (valid ? b : 0) * NV * D;
  const bf16_t* ob = dout + (valid ? b : 0) * ldo;
  bf16_t* s = sv[w];
  for (int e = lane * 8; e < 32 * D; e += 64 * 8) {
    const int r = e / D;
    *reinterpret_cast<v8s*>(s + e) =
        (valid && r < NV) ? *reinterpret_cast<const v8s*>(vb + e) : v8s{0, 0, 0, 0, 0, 0, 0, 0};
  }
  __syncthreads();
  if (!valid) return;
  v8s a[2];
#pragma unroll
  for (int ti = 0; ti < 2; ++ti) {
    const int r = ti * 16 + (lane & 15);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = 8 * (lane >> 4) + q;
      bf16_t g = 0;
      if (r < NV && c < NV && r != c) {
        const int hi = r > c ? r : c, lo = r > c ? c : r;
        g = ob[D + hi * (hi - 1) / 2 + lo];
      }
      a[ti][q] = (short)g;
    }
  }
#pragma unroll
  for (int tn = 0; tn < D / 16; ++tn) {
    const int n = tn * 16 + (lane & 15);
    v8s bt;
#pragma unroll
    for (int q = 0; q < 8; ++q) bt[q] = (short)s[(8 * (lane >> 4) + q) * D + n];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti) {
      v4f acc = {0.f, 0.f, 0.f, 0.f};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf_i, a[ti]), __builtin_bit_cast(v8bf_i, bt),
                                                    acc, 0, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = ti * 16 + (lane >> 4) * 4 + e;
        if (row < NV) {
          float v = acc[e];
          if (row == dense_idx) {
            v += bf2f(ob[n]);
            d_dense[b * D + n] = f2bf(bf2f(s[row * D + n]) > 0.f ? v : 0.f);
          }
          if constexpr (sizeof(OutT) == 2)
            dV[(b * NV + row) * D + n] = f2bf(v);
          else
            dV[(b * NV + row) * D + n] = v;
        }
      }
    }
  }
}

void dlrm_interact_fwd(const bf16_t* V, int64_t B, int NV, int D, int dense_idx, bf16_t* out, int ldo, hipStream_t s) {
  if (B <= 0) return;
  if (NV <= 32 && (D == 16 || D == 32 || D == 64) && ldo % 8 == 0) {
    const unsigned grid = (unsigned)((B + 3) / 4);
    if (D == 64)
      hipLaunchKernelGGL(dlrm_interact_fwd_mfma_kernel<2>, grid, 256, 0, s, V, B, NV, D, dense_idx, out, ldo);
    else
      hipLaunchKernelGGL(dlrm_interact_fwd_mfma_kernel<1>, grid, 256, 0, s, V, B, NV, D, dense_idx, out, ldo);
    MINIPS_HIP_CHECK(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(dlrm_interact_fwd_kernel, (int)std::min<int64_t>(B, 8192), 256, NV * (D + 1)
                     * sizeof(float), s, V, B,
                     NV, D, dense_idx, out, ldo);
  MINIPS_HIP_CHECK(hipGetLastError());
}
template <typename OutT>
static void interact_bwd_mfma(const bf16_t* V, int64_t B, int NV, int D, int dense_idx, const bf16_t* dout, int ldo,
                              OutT* dV, bf16_t* d_dense, hipStream_t s) {
  const unsigned grid = (unsigned)((B + 3) / 4);
  if (D == 64)
    hipLaunchKernelGGL((dlrm_interact_bwd_mfma_kernel<64, OutT>), grid, 256, 0, s, V, B, NV, dense_idx, dout, ldo, dV,
                       d_dense);
  else if (D == 32)
    hipLaunchKernelGGL((dlrm_interact_bwd_mfma_kernel<32, OutT>), grid, 256, 0, s, V, B, NV, dense_idx, dout, ldo, dV,
                       d_dense);
  else
    hipLaunchKernelGGL((dlrm_interact_bwd_mfma_kernel<16, OutT>), grid, 256, 0, s, V, B, NV, dense_idx, dout, ldo, dV,
                       d_dense);
  MINIPS_HIP_CHECK(hipGetLastError());
}

bool dlrm_interact_mfma_ok(int NV, int D) { return NV <= 32 && (D == 16 || D == 32 || D == 64); }

void dlrm_interact_bwd_bf16(const bf16_t* V, int64_t B, int NV, int D, int dense_idx, const bf16_t* dout, int ldo,
                            bf16_t* dV, bf16_t* d_dense, hipStream_t s) {
  if (B <= 0) return;
  if (!dlrm_interact_mfma_ok(NV, D)) throw std::runtime_error("dlrm_interact_bwd: bf16 dV needs NV <= 32, D 16/32/64");
  interact_bwd_mfma(V, B, NV, D, dense_idx, dout, ldo, dV, d_dense, s);
}

void dlrm_interact_bwd(const bf16_t* V, int64_t B, int NV, int D, int dense_idx, const bf16_t* dout, int ldo,
                       float* dV, bf16_t* d_dense, hipStream_t s) {
  if (B <= 0) return;
  if (dlrm_interact_mfma_ok(NV, D)) {
    interact_bwd_mfma(V, B, NV, D, dense_idx, dout, ldo, dV, d_dense, s);
    return;
  }
  hipLaunchKernelGGL(dlrm_interact_bwd_kernel, (int)std::min<int64_t>(B, 8192), 256,
                     (NV * D + NV * NV) * sizeof(float), s, V, B, NV, D, dense_idx, dout, ldo, dV, d_dense);
  MINIPS_HIP_CHECK(hipGetLastError());
}

}  // namespace minips_k
