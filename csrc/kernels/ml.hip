// Classic-ML worker kernels of the reference apps on the GPU data plane:
//   lr_sparse_step  (K7/K8) sparse logistic regression gradient over a CSR mini-batch,
//                   the math of apps/logistic_regression/lr_example.cpp:291-312
//   kmeans_assign   (K9)    nearest-centre assignment, apps/kmeans/kmeans_helper.hpp:45-66
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"

namespace minips_k {

template <typename T>
__device__ __forceinline__ T wave_sum_t(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// One wave per sample: lanes stride the sample's non-zeros. T = float (the performance path) or
// double (the reference's double tables, lr_example.cpp:182: parity runs).
template <typename T>
__global__ void lr_sparse_kernel(const int64_t* __restrict__ rowptr, const int64_t* __restrict__ cols,
                                 const float* __restrict__ vals, const float* __restrict__ labels, int64_t B,
                                 const T* __restrict__ w, T alpha, T* delta, float* correct) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  float hits = 0.f;
  for (int64_t i = wave; i < B; i += nwaves) {
    const int64_t s0 = rowptr[i], s1 = rowptr[i + 1];
    T dot = 0;
    for (int64_t j = s0 + lane; j < s1; j += 64) dot += w[cols[j]] * (T)vals[j];
    dot = wave_sum_t(dot);
    const T p = (T)1 / ((T)1 + exp(-dot));
    const T y = labels[i] < 0.f ? (T)0 : (T)labels[i];
    const T err = alpha * (y - p);
    if (delta)
      for (int64_t j = s0 + lane; j < s1; j += 64) atomicAdd(delta + cols[j], err * (T)vals[j]);
    if (lane == 0) hits += ((p > (T)0.5) == (y > (T)0.5)) ? 1.f : 0.f;
  }
  if (correct && lane == 0 && hits > 0.f) atomicAdd(correct, hits);
}

void lr_sparse_step(const int64_t* rowptr, const int64_t* cols, const float* vals, const float* labels, int64_t B,
                    const float* w, float alpha, float* delta, float* correct, hipStream_t s) {
  if (B <= 0) return;
  const int block = 256;
  hipLaunchKernelGGL(lr_sparse_kernel<float>, grid_for(B * 64, block, 4096), block, 0, s, rowptr, cols, vals, labels,
                     B, w, alpha, delta, correct);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void lr_sparse_step_f64(const int64_t* rowptr, const int64_t* cols, const float* vals, const float* labels, int64_t B,
                        const double* w, double alpha, double* delta, float* correct, hipStream_t s) {
  if (B <= 0) return;
  const int block = 256;
  hipLaunchKernelGGL(lr_sparse_kernel<double>, grid_for(B * 64, block, 4096), block, 0, s, rowptr, cols, vals,
                     labels, B, w, alpha, delta, correct);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// One wave per point, centres streamed k at a time; lanes split the dimension.
__global__ void kmeans_assign_kernel(const float* __restrict__ X, int64_t n, int d, const float* __restrict__ C, int k,
                                     int32_t* assign, float* dist) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave; i < n; i += nwaves) {
    const float* x = X + i * d;
    float best = 3.4e38f;
    int besti = 0;
    for (int c = 0; c < k; ++c) {
      const float* cc = C + (int64_t)c * d;
      float acc = 0.f;
      for (int j = lane; j < d; j += 64) {
        const float t = x[j] - cc[j];
        acc += t * t;
      }
      acc = warp_sum(acc);
      if (acc < best) {
        best = acc;
        besti = c;
      }
    }
    if (lane == 0) {
      assign[i] = besti;
      if (dist) dist[i] = best;
    }
  }
}

void kmeans_assign(const float* X, int64_t n, int d, const float* C, int k, int32_t* assign, float* dist,
                   hipStream_t s) {
  if (n <= 0) return;
  const int block = 256;
  hipLaunchKernelGGL(kmeans_assign_kernel, grid_for(n * 64, block, 4096), block, 0, s, X, n, d, C, k, assign, dist);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// MFMA form of the assignment: d(x, c) = |x|^2 + |c|^2 - 2 x.c with x.c from the bf16
// MFMA GEMM at ~fp32 accuracy via a hi/lo split: x = xh + xl (xh = bf16(x), xl = bf16(x - xh)),
// x.c ~= xh.ch + xh.cl + xl.ch, i.e. ONE GEMM over 3d-long rows A = [xh | xh | xl],
// B = [ch | cl | ch] (the dropped xl.cl term is ~2^-16 relative).
//   split3_kernel  fp32 [r, d] -> bf16 [r, ld] (ld >= 3d, zero pad) + row squared norms
//   argmin_kernel  one wave per row of S = A.B^T (fp32 [n, k]): argmin_c |c|^2 - 2 S[i, c]
__global__ void split3_kernel(const float* __restrict__ src, int64_t r, int d, bf16_t* __restrict__ out, int ld,
                              int order, float* __restrict__ norms) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave; i < r; i += nw) {
    const float* x = src + i * d;
    bf16_t* o = out + i * ld;
    float sq = 0.f;
    for (int j = lane; j < d; j += 64) {
      const float v = x[j];
      sq += v * v;
      const bf16_t h = f2bf(v);
      const bf16_t l = f2bf(v - bf2f(h));
      o[j] = h;                             // segment 0: hi
      o[d + j] = order == 0 ? h : l;        // A: [h | h | l]   B: [h | l | h]
      o[2 * d + j] = order == 0 ? l : h;
    }
    for (int j = 3 * d + lane; j < ld; j += 64) o[j] = f2bf(0.f);
    sq = warp_sum(sq);
    if (lane == 0) norms[i] = sq;
  }
}

__global__ void kmeans_argmin_kernel(const float* __restrict__ S, int64_t n, int k, const float* __restrict__ cn,
                                     const float* __restrict__ xn, int32_t* assign, float* dist) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave; i < n; i += nw) {
    const float* row = S + i * k;
    float best = 3.4e38f;
    int bi = 0x7fffffff;
    for (int c = lane; c < k; c += 64) {
      const float v = cn[c] - 2.f * row[c];
      if (v < best) {  // lanes walk c upward: the first minimum per lane wins
        best = v;
        bi = c;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ob < best || (ob == best && oi < bi)) {
        best = ob;
        bi = oi;
      }
    }
    if (lane == 0) {
      assign[i] = bi;
      if (dist) dist[i] = fmaxf(best + xn[i], 0.f);
    }
  }
}

void kmeans_split3(const float* src, int64_t r, int d, bf16_t* out, int ld, int order, float* norms, hipStream_t s) {
  if (r <= 0) return;
  if (ld < 3 * d) throw std::runtime_error("kmeans_split3: ld < 3d");
  hipLaunchKernelGGL(split3_kernel, grid_for(r * 64, 256, 8192), 256, 0, s, src, r, d, out, ld, order, norms);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void kmeans_argmin(const float* S, int64_t n, int k, const float* cn, const float* xn, int32_t* assign, float* dist,
                   hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(kmeans_argmin_kernel, grid_for(n * 64, 256, 8192), 256, 0, s, S, n, k, cn, xn, assign, dist);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- sparse (CSR) K-Means
// The reference K-Means clusters sparse libsvm points (webspam: 16.6M features) against dense
// centres: nearest centre over sparse x (kmeans_helper.hpp:45-66) and the centre update
// (kmeans.cpp:238-267). One wave per point, lanes over its non-zeros:
//   d_k = |x|^2 - 2 x.c_k + |c_k|^2   (|c_k|^2 precomputed per step: kmeans_cnorm)
__global__ void kmeans_cnorm_kernel(const float* __restrict__ C, int k, int64_t d, float* __restrict__ out) {
  // one block per centre
  const int c = blockIdx.x;
  float acc = 0.f;
  for (int64_t j = threadIdx.x; j < d; j += blockDim.x) {
    const float t = C[(int64_t)c * d + j];
    acc += t * t;
  }
  acc = warp_sum(acc);
  __shared__ float part[16];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) part[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += part[i];
    out[c] = t;
  }
}

__global__ void kmeans_assign_csr_kernel(const int64_t* __restrict__ rowptr, const int64_t* __restrict__ cols,
                                         const float* __restrict__ vals, int64_t n, const float* __restrict__ C,
                                         int k, int64_t d, const float* __restrict__ cnorm, int32_t* assign,
                                         float* dist) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave; i < n; i += nwaves) {
    const int64_t s0 = rowptr[i], s1 = rowptr[i + 1];
    float xn = 0.f;
    for (int64_t j = s0 + lane; j < s1; j += 64) xn += vals[j] * vals[j];
    xn = warp_sum(xn);
    float best = 3.4e38f;
    int besti = 0;
    for (int c = 0; c < k; ++c) {
      const float* cc = C + (int64_t)c * d;
      float dot = 0.f;
      for (int64_t j = s0 + lane; j < s1; j += 64) {
        const int64_t col = cols[j];
        if (col < d) dot += vals[j] * cc[col];
      }
      dot = warp_sum(dot);
      const float dd = xn - 2.f * dot + cnorm[c];
      if (dd < best) {
        best = dd;
        besti = c;
      }
    }
    if (lane == 0) {
      assign[i] = besti;
      if (dist) dist[i] = fmaxf(best, 0.f);
    }
  }
}

// sums[assign[i], col] += val over every non-zero of every point (the batch's centre sums)
__global__ void kmeans_csr_accum_kernel(const int64_t* __restrict__ rowptr, const int64_t* __restrict__ cols,
                                        const float* __restrict__ vals, int64_t n, const int32_t* __restrict__ assign,
                                        int64_t d, float* __restrict__ sums) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave; i < n; i += nwaves) {
    float* row = sums + (int64_t)assign[i] * d;
    for (int64_t j = rowptr[i] + lane; j < rowptr[i + 1]; j += 64) {
      const int64_t col = cols[j];
      if (col < d) atomicAdd(row + col, vals[j]);
    }
  }
}

void kmeans_assign_csr(const int64_t* rowptr, const int64_t* cols, const float* vals, int64_t n, const float* C,
                       int k, int64_t d, float* cnorm, int32_t* assign, float* dist, hipStream_t s) {
  if (n <= 0 || k <= 0) return;
  hipLaunchKernelGGL(kmeans_cnorm_kernel, k, 256, 0, s, C, k, d, cnorm);
  MINIPS_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(kmeans_assign_csr_kernel, grid_for(n * 64, 256, 4096), 256, 0, s, rowptr, cols, vals, n, C, k, d,
                     cnorm, assign, dist);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void kmeans_csr_accum(const int64_t* rowptr, const int64_t* cols, const float* vals, int64_t n, const int32_t* assign,
                      int64_t d, float* sums, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(kmeans_csr_accum_kernel, grid_for(n * 64, 256, 4096), 256, 0, s, rowptr, cols, vals, n, assign,
                     d, sums);
  MINIPS_HIP_CHECK(hipGetLastError());
}

}  // namespace minips_k
