// bf16 embedding rows (SparseTable(value_dtype=torch.bfloat16)): half the HBM of fp32 rows, so the
// BASELINE's 10B-row x 64 DLRM table fits 8 x 288 GB (1.28 TB of rows + 40 GB of fp32 row-wise
// Adagrad state). The optimizer math runs in fp32; the new value goes back to bf16
// by STOCHASTIC rounding, so updates much smaller than a bf16 ulp are not lost on average
// (round-to-nearest would drop every update below half an ulp of the weight: a sparse row updated
// rarely with a small lr would never move).
//
//   rounding:  bits(x) + (16 random bits) then truncate to the top 16 bits -- rounds the magnitude
//              up with probability = the discarded fraction (unbiased: E[bf16(x)] = x)
//   random bits: a stateless hash of (row, column, apply counter, seed): reproducible runs,
//              independent across rows / columns / steps
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"

namespace minips_k {

namespace {

// 8 bf16 per lane (16-byte loads), D/8 lanes per row, rows grid-strided.
template <typename TO>
__global__ __launch_bounds__(256) void gather_bf16_rows_kernel(const bf16_t* __restrict__ table, int64_t ld,
                                                               const int64_t* __restrict__ keys, int64_t n,
                                                               int64_t base, int D, TO* __restrict__ out,
                                                               const int64_t* __restrict__ n_dev) {
  const int64_t nn = n_dev ? min(n, *n_dev) : n;
  const int nv = D / 8;
  const int64_t total = nn * nv;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = c / nv;
    const int j = (int)(c - i * nv);
    const uint4 v = reinterpret_cast<const uint4*>(table + (keys[i] - base) * ld)[j];
    if constexpr (sizeof(TO) == 2) {
      reinterpret_cast<uint4*>(out + i * D)[j] = v;
    } else {
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      float4 lo = make_float4(__uint_as_float(w[0] << 16), __uint_as_float(w[0] & 0xffff0000u),
                              __uint_as_float(w[1] << 16), __uint_as_float(w[1] & 0xffff0000u));
      float4 hi = make_float4(__uint_as_float(w[2] << 16), __uint_as_float(w[2] & 0xffff0000u),
                              __uint_as_float(w[3] << 16), __uint_as_float(w[3] & 0xffff0000u));
      reinterpret_cast<float4*>(out + i * D)[2 * j] = lo;
      reinterpret_cast<float4*>(out + i * D)[2 * j + 1] = hi;
    }
  }
}

// Row-wise Adagrad on bf16 rows (fp32 state): L = D/8 lanes per row, 8 values per lane.
//   s[row] += mean(g^2) (per column group [0, D1) / [D1, D));  w -= lr * g / (sqrt(s) + eps)
// opt 0: row-wise Adagrad; 1: w += scale * g (SGD / the reference add).
template <int OPT>
__global__ __launch_bounds__(256) void bf16_apply_kernel(bf16_t* __restrict__ table, int64_t ld,
                                                         float* __restrict__ state, float* __restrict__ state2, int D1,
                                                         const int64_t* __restrict__ keys, int64_t n, int64_t base,
                                                         int D, const float* __restrict__ grads, float lr, float eps,
                                                         float scale, uint32_t step, uint32_t seed,
                                                         const int64_t* __restrict__ n_dev) {
  const int64_t nn = n_dev ? min(n, *n_dev) : n;
  const int L = D / 8;  // 2, 4 or 8 lanes per row
  const int lane = threadIdx.x & 63, sub = lane / L, l = lane % L, per = 64 / L;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i0 = wave * per; i0 < nn; i0 += nw * per) {
    const int64_t i = i0 + sub;
    const bool ok = i < nn;
    const int64_t row = ok ? keys[i] - base : 0;
    float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    uint4 wv = make_uint4(0, 0, 0, 0);
    bf16_t* tr = table + row * ld + 8 * l;
    if (ok) {
      const float4 g0 = reinterpret_cast<const float4*>(grads + i * D)[2 * l];
      const float4 g1 = reinterpret_cast<const float4*>(grads + i * D)[2 * l + 1];
      g[0] = g0.x; g[1] = g0.y; g[2] = g0.z; g[3] = g0.w;
      g[4] = g1.x; g[5] = g1.y; g[6] = g1.z; g[7] = g1.w;
      wv = *reinterpret_cast<const uint4*>(tr);
    }
    float s1 = lr, s2 = lr;  // per-group step sizes (Adagrad), or the SGD scale
    if (OPT == 0) {
      float sq1 = 0.f, sq2 = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int c = 8 * l + q;
        if (c < D1) sq1 += g[q] * g[q];
        else sq2 += g[q] * g[q];
      }
      for (int o = 1; o < L; o <<= 1) {
        sq1 += __shfl_xor(sq1, o, 64);
        sq2 += __shfl_xor(sq2, o, 64);
      }
      const float st_old1 = ok ? state[row] : 0.f, st_old2 = (ok && D1 < D) ? state2[row] : 0.f;
      const float st1 = st_old1 + sq1 / (float)D1;
      const float st2 = D1 < D ? st_old2 + sq2 / (float)(D - D1) : 0.f;
      if (ok && l == 0) {
        state[row] = st1;
        if (D1 < D) state2[row] = st2;
      }
      s1 = -lr / (sqrtf(st1) + eps);
      s2 = -lr / (sqrtf(st2) + eps);
    } else {
      s1 = s2 = scale;
    }
    if (!ok) continue;
    const uint32_t w[4] = {wv.x, wv.y, wv.z, wv.w};
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c0 = 8 * l + 2 * e;
      const float a = __uint_as_float(w[e] << 16) + (c0 < D1 ? s1 : s2) * g[2 * e];
      const float b = __uint_as_float(w[e] & 0xffff0000u) + (c0 + 1 < D1 ? s1 : s2) * g[2 * e + 1];
      const uint32_t r = sr_hash((uint64_t)(row + base), (uint32_t)c0, step, seed);
      o[e] = (uint32_t)bf16_sr(a, r) | ((uint32_t)bf16_sr(b, r >> 16) << 16);
    }
    *reinterpret_cast<uint4*>(tr) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

void check_bf16_rows(int D, int64_t ld, const void* table) {
  if ((D != 16 && D != 32 && D != 64) || ld % 8 != 0 || reinterpret_cast<uintptr_t>(table) % 16 != 0)
    throw std::runtime_error("bf16 rows: D in {16, 32, 64}, 16-byte aligned rows");
}

}  // namespace

void gather_rows_bf16tab(const bf16_t* table, int64_t ld, const int64_t* keys, int64_t n, int64_t base, int D,
                         void* out, bool out_bf16, hipStream_t s, const int64_t* n_dev) {
  if (n <= 0) return;
  check_bf16_rows(D, ld, table);
  const int grid = grid_for(n * (D / 8), 256, 8192);
  if (out_bf16)
    hipLaunchKernelGGL(gather_bf16_rows_kernel<bf16_t>, grid, 256, 0, s, table, ld, keys, n, base, D,
                       static_cast<bf16_t*>(out), n_dev);
  else
    hipLaunchKernelGGL(gather_bf16_rows_kernel<float>, grid, 256, 0, s, table, ld, keys, n, base, D,
                       static_cast<float*>(out), n_dev);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void sparse_apply_bf16tab(int opt, bf16_t* table, int64_t ld, float* state, float* state2, int D1, const int64_t* keys,
                          int64_t n, int64_t base, int D, const float* grads, float lr, float eps, float scale,
                          uint32_t step, uint32_t seed, hipStream_t s, const int64_t* n_dev) {
  if (n <= 0) return;
  check_bf16_rows(D, ld, table);
  if (D1 <= 0 || D1 > D) D1 = D;
  if (opt == 0 && D1 < D && !state2) throw std::runtime_error("bf16 row-wise Adagrad: split rows need state2");
  if (reinterpret_cast<uintptr_t>(grads) % 16 != 0) throw std::runtime_error("bf16 apply: grads 16-byte aligned");
  const int rows_per_block = 4 * (64 / (D / 8));
  const int grid = (int)std::min<int64_t>((n + rows_per_block - 1) / rows_per_block, 16384);
  if (opt == 0)
    hipLaunchKernelGGL(bf16_apply_kernel<0>, grid, 256, 0, s, table, ld, state, state2, D1, keys, n, base, D, grads,
                       lr, eps, scale, step, seed, n_dev);
  else
    hipLaunchKernelGGL(bf16_apply_kernel<1>, grid, 256, 0, s, table, ld, state, state2, D1, keys, n, base, D, grads,
                       lr, eps, scale, step, seed, n_dev);
  MINIPS_HIP_CHECK(hipGetLastError());
}

}  // namespace minips_k
