// One-sided parameter-server data path over xGMI (SSP / ASP tables, minips_amd/ps/onesided.py).
//
// Every rank hipMallocs its shard and exports it with hipIpcGetMemHandle; every rank opens every
// peer's handle, so the whole row-partitioned table is addressable from any GPU through a small
// device-side table of base pointers (peer HBM is reached over xGMI, the own shard locally).
// A Get is then a direct gather of the requested rows from their owners' HBM and an Add an
// atomic scatter into them -- no collective, no owner-side participation, so a rank never waits
// for another rank's progress (the reference ASPModel replies and applies immediately,
// server/consistency/asp_model.cpp:18-26; SSP adds only the host-side staleness gate).
//
//   owner of key k   o = upper_bound(bounds, k) - 1   (bounds [P+1], equal key ranges)
//   row              k - bounds[o]  in the shard at bases[o]  ([rows_o, W] fp32, row-major)
//
// A row is handled by L = 16 / 32 / 64 lanes (the smallest that covers W, so narrow embedding
// rows pack 64 / L keys per wave); the scatter adds with global_atomic_add_f32, which executes
// at the memory side: adds from different GPUs to the same row never get lost
// (MI355X_MICROARCH.md 'Global float atomics').
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"

namespace minips_k {

__device__ __forceinline__ int owner_of(const int64_t* __restrict__ bounds, int P, int64_t k) {
  int lo = 0, hi = P;  // bounds[lo] <= k < bounds[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (bounds[mid] <= k) lo = mid;
    else hi = mid;
  }
  return lo;
}

template <typename TO>
__global__ __launch_bounds__(256) void remote_gather_kernel(const int64_t* __restrict__ bases,
                                                            const int64_t* __restrict__ bounds, int P,
                                                            const int64_t* __restrict__ keys, int64_t n,
                                                            const int64_t* __restrict__ n_dev, int W,
                                                            TO* __restrict__ out) {
  const int64_t nn = n_dev ? min(n, *n_dev) : n;
  const int L = W <= 16 ? 16 : (W <= 32 ? 32 : 64), per = 64 / L;
  const int lane = threadIdx.x & 63, l = lane % L;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave * per + lane / L; i < nn; i += nw * per) {
    const int64_t k = keys[i];
    if (k < bounds[0] || k >= bounds[P]) continue;  // never address outside the table
    const int o = owner_of(bounds, P, k);
    const float* row = reinterpret_cast<const float*>(bases[o]) + (k - bounds[o]) * (int64_t)W;
    for (int c = l; c < W; c += L) {
      const float v = row[c];
      if constexpr (sizeof(TO) == 2) {
        out[i * W + c] = (TO)(pack_bf2(v, 0.f) & 0xffffu);
      } else {
        out[i * W + c] = v;
      }
    }
  }
}

__global__ __launch_bounds__(256) void remote_scatter_add_kernel(const int64_t* __restrict__ bases,
                                                                 const int64_t* __restrict__ bounds, int P,
                                                                 const int64_t* __restrict__ keys, int64_t n,
                                                                 const int64_t* __restrict__ n_dev,
                                                                 const float* __restrict__ vals, int W, float scale) {
  if (n_dev) n = min(n, *n_dev);
  const int L = W <= 16 ? 16 : (W <= 32 ? 32 : 64), per = 64 / L;
  const int lane = threadIdx.x & 63, l = lane % L;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave * per + lane / L; i < n; i += nw * per) {
    const int64_t k = keys[i];
    if (k < bounds[0] || k >= bounds[P]) continue;  // never address outside the table
    const int o = owner_of(bounds, P, k);
    float* row = reinterpret_cast<float*>(bases[o]) + (k - bounds[o]) * (int64_t)W;
    for (int c = l; c < W; c += L) atomicAdd(row + c, scale * vals[i * W + c]);
  }
}

void remote_gather(const int64_t* bases, const int64_t* bounds, int P, const int64_t* keys, int64_t n,
                   const int64_t* n_dev, int W, void* out, bool out_bf16, hipStream_t s) {
  if (n <= 0) return;
  const int block = 256;
  const int grid = grid_for(n * 64, block, 8192);
  if (out_bf16)
    hipLaunchKernelGGL((remote_gather_kernel<bf16_t>), grid, block, 0, s, bases, bounds, P, keys, n, n_dev, W,
                       static_cast<bf16_t*>(out));
  else
    hipLaunchKernelGGL((remote_gather_kernel<float>), grid, block, 0, s, bases, bounds, P, keys, n, n_dev, W,
                       static_cast<float*>(out));
  MINIPS_HIP_CHECK(hipGetLastError());
}

void remote_scatter_add(const int64_t* bases, const int64_t* bounds, int P, const int64_t* keys, int64_t n,
                        const int64_t* n_dev, const float* vals, int W, float scale, hipStream_t s) {
  if (n <= 0) return;
  const int block = 256;
  hipLaunchKernelGGL(remote_scatter_add_kernel, grid_for(n * 64, block, 8192), block, 0, s, bases, bounds, P, keys,
                     n, n_dev, vals, W, scale);
  MINIPS_HIP_CHECK(hipGetLastError());
}

}  // namespace minips_k
