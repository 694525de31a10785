// fp64 row kernels of the reference-precision tables (SparseTable(value_dtype=float64)): the
// reference LR runs CreateTable<double> (apps/logistic_regression/lr_example.cpp:182) and reads
// values as double (worker/kv_client_table.hpp:96-101); these keep parity runs exact.
//   gather_rows_f64    out[i] = table[keys[i] - base]                (VectorStorage::SubGet)
//   scatter_add_f64    acc[idx[i]] += src[i]                          (owner-side segment sum)
//   sparse_add_f64     table[keys[i] - base] += scale * grads[i]     (VectorStorage::SubAdd)
// A row is handled by 16 / 32 / 64 lanes (the smallest covering W); fp64 atomics are native.
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"

namespace minips_k {

__device__ __forceinline__ int lanes_for(int W) { return W <= 16 ? 16 : (W <= 32 ? 32 : 64); }

__global__ void gather_rows_f64_kernel(const double* __restrict__ table, int W, const int64_t* __restrict__ keys,
                                       int64_t base, int64_t n, const int64_t* __restrict__ n_dev,
                                       double* __restrict__ out) {
  const int64_t nn = n_dev ? min(n, *n_dev) : n;
  const int L = lanes_for(W), lane = threadIdx.x & 63, l = lane % L;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave * (64 / L) + lane / L; i < nn; i += nw * (64 / L)) {
    const double* row = table + (keys[i] - base) * (int64_t)W;
    for (int c = l; c < W; c += L) out[i * W + c] = row[c];
  }
}

__global__ void scatter_add_f64_kernel(const double* __restrict__ src, const int64_t* __restrict__ idx, int64_t n,
                                       int W, double* __restrict__ acc) {
  const int L = lanes_for(W), lane = threadIdx.x & 63, l = lane % L;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave * (64 / L) + lane / L; i < n; i += nw * (64 / L)) {
    double* row = acc + idx[i] * (int64_t)W;
    for (int c = l; c < W; c += L) atomicAdd(row + c, src[i * W + c]);
  }
}

__global__ void sparse_add_f64_kernel(double* __restrict__ table, int W, const int64_t* __restrict__ keys,
                                      int64_t base, const double* __restrict__ grads, int64_t n, double scale,
                                      const int64_t* __restrict__ n_dev) {
  const int64_t nn = n_dev ? min(n, *n_dev) : n;
  const int L = lanes_for(W), lane = threadIdx.x & 63, l = lane % L;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  // keys are unique per launch (owner-side dedupe): plain read-modify-write, no atomics
  for (int64_t i = wave * (64 / L) + lane / L; i < nn; i += nw * (64 / L)) {
    double* row = table + (keys[i] - base) * (int64_t)W;
    for (int c = l; c < W; c += L) row[c] += scale * grads[i * W + c];
  }
}

void gather_rows_f64(const double* table, int W, const int64_t* keys, int64_t base, int64_t n, const int64_t* n_dev,
                     double* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gather_rows_f64_kernel, grid_for(n * 64, 256, 4096), 256, 0, s, table, W, keys, base, n, n_dev,
                     out);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void scatter_add_rows_f64(const double* src, const int64_t* idx, int64_t n, int W, double* acc, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(scatter_add_f64_kernel, grid_for(n * 64, 256, 4096), 256, 0, s, src, idx, n, W, acc);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void sparse_add_f64(double* table, int W, const int64_t* keys, int64_t base, const double* grads, int64_t n,
                    double scale, const int64_t* n_dev, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(sparse_add_f64_kernel, grid_for(n * 64, 256, 4096), 256, 0, s, table, W, keys, base, grads, n,
                     scale, n_dev);
  MINIPS_HIP_CHECK(hipGetLastError());
}

}  // namespace minips_k
