// Server-side fused dense optimizers on the fp32 master shard (after the reduce-scatter of
// gradients), optionally emitting the bf16 copy that the next all-gather (pull) ships.
// One pass over w/m/v/g: Adam(W) = 4 reads + 3 writes (+ 1 bf16 write) per element.
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"

namespace minips_k {

__global__ void adam_kernel(float* __restrict__ w, float* __restrict__ m, float* __restrict__ v,
                            float* __restrict__ g, int64_t n, float lr, float b1, float b2, float eps, float wd,
                            float bc1, float bc2, float gscale, bf16_t* __restrict__ wb,
                            const int* __restrict__ step_dev, bool zero_g, const int64_t* __restrict__ active) {
  if (active && *active == 0) return;  // an empty push (a Clock without an Add): nothing to apply
  if (step_dev) {  // device-side step (graph-replayable clocks): bias corrections from *step_dev
    const float t = (float)*step_dev;
    bc1 = 1.f - powf(b1, t);
    bc2 = 1.f - powf(b2, t);
  }
  const int64_t n4 = n >> 2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 W = reinterpret_cast<float4*>(w)[i], M = reinterpret_cast<float4*>(m)[i];
    float4 V = reinterpret_cast<float4*>(v)[i];
    const float4 G = reinterpret_cast<const float4*>(g)[i];
    float* Wp = &W.x;
    float* Mp = &M.x;
    float* Vp = &V.x;
    const float* Gp = &G.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gg = Gp[j] * gscale;
      Mp[j] = b1 * Mp[j] + (1.f - b1) * gg;
      Vp[j] = b2 * Vp[j] + (1.f - b2) * gg * gg;
      const float mh = Mp[j] / bc1, vh = Vp[j] / bc2;
      Wp[j] -= lr * (mh / (sqrtf(vh) + eps) + wd * Wp[j]);
    }
    reinterpret_cast<float4*>(w)[i] = W;
    reinterpret_cast<float4*>(m)[i] = M;
    reinterpret_cast<float4*>(v)[i] = V;
    if (wb) reinterpret_cast<uint2*>(wb)[i] = make_uint2(pack_bf2(W.x, W.y), pack_bf2(W.z, W.w));
    if (zero_g) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);  // next clock's accumulator
  }
  // tail
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float gg = g[i] * gscale;
    m[i] = b1 * m[i] + (1.f - b1) * gg;
    v[i] = b2 * v[i] + (1.f - b2) * gg * gg;
    w[i] -= lr * ((m[i] / bc1) / (sqrtf(v[i] / bc2) + eps) + wd * w[i]);
    if (wb) wb[i] = f2bf(w[i]);
    if (zero_g) g[i] = 0.f;
  }
}

static void check_align(const void* p, const char* what) {
  if (reinterpret_cast<uintptr_t>(p) & 15) throw std::runtime_error(std::string(what) + " must be 16-byte aligned");
}

void adam_apply(float* w, float* m, float* v, const float* g, int64_t n, float lr, float beta1, float beta2, float eps,
                float weight_decay, int step, float grad_scale, bf16_t* w_bf16, hipStream_t s, const int* step_dev,
                bool zero_g, const int64_t* active) {
  if (n <= 0) return;
  check_align(w, "adam w");
  check_align(m, "adam m");
  check_align(v, "adam v");
  check_align(g, "adam g");
  if (w_bf16 && (reinterpret_cast<uintptr_t>(w_bf16) & 7)) throw std::runtime_error("adam w_bf16 must be 8B aligned");
  const float bc1 = 1.f - powf(beta1, (float)step), bc2 = 1.f - powf(beta2, (float)step);
  const int block = 256;
  hipLaunchKernelGGL(adam_kernel, grid_for((n + 3) / 4, block), block, 0, s, w, m, v, const_cast<float*>(g),
                     n, lr, beta1, beta2, eps,
                     weight_decay, bc1, bc2, grad_scale, w_bf16, step_dev, zero_g, active);
  MINIPS_HIP_CHECK(hipGetLastError());
}

__global__ void sgd_kernel(float* __restrict__ w, const float* __restrict__ g, int64_t n, float lr, float gscale,
                           bf16_t* __restrict__ wb, const int64_t* __restrict__ active) {
  if (active && *active == 0) return;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float x = w[i] - lr * g[i] * gscale;
    w[i] = x;
    if (wb) wb[i] = f2bf(x);
  }
}

void sgd_apply(float* w, const float* g, int64_t n, float lr, float grad_scale, bf16_t* w_bf16, hipStream_t s,
               const int64_t* active) {
  if (n <= 0) return;
  const int block = 256;
  hipLaunchKernelGGL(sgd_kernel, grid_for(n, block), block, 0, s, w, g, n, lr, grad_scale, w_bf16, active);
  MINIPS_HIP_CHECK(hipGetLastError());
}

__global__ void adagrad_kernel(float* __restrict__ w, float* __restrict__ acc, const float* __restrict__ g, int64_t n,
                               float lr, float eps, float gscale, bf16_t* __restrict__ wb,
                               const int64_t* __restrict__ active) {
  if (active && *active == 0) return;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gg = g[i] * gscale;
    const float a = acc[i] + gg * gg;
    acc[i] = a;
    const float x = w[i] - lr * gg / (sqrtf(a) + eps);
    w[i] = x;
    if (wb) wb[i] = f2bf(x);
  }
}

void adagrad_apply(float* w, float* acc, const float* g, int64_t n, float lr, float eps, float grad_scale,
                   bf16_t* w_bf16, hipStream_t s, const int64_t* active) {
  if (n <= 0) return;
  const int block = 256;
  hipLaunchKernelGGL(adagrad_kernel, grid_for(n, block), block, 0, s, w, acc, g, n, lr, eps, grad_scale, w_bf16,
                     active);
  MINIPS_HIP_CHECK(hipGetLastError());
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}
__global__ void cast_bf16_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = bf2f(x[i]);
}

void cast_f32_bf16(const float* x, bf16_t* y, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, grid_for(n, 256), 256, 0, s, x, y, n);
  MINIPS_HIP_CHECK(hipGetLastError());
}
void cast_bf16_f32(const bf16_t* x, float* y, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(cast_bf16_f32_kernel, grid_for(n, 256), 256, 0, s, x, y, n);
  MINIPS_HIP_CHECK(hipGetLastError());
}

}  // namespace minips_k
