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
                            const int* __restrict__ step_dev, bool zero_g, const int64_t* __restrict__ active,
                            AdamSlabs sl) {
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
    float4 Gs = G;
    // split-K weight gradients left in their slab planes (adam_slabs): their sum lands here, the
    // one kernel that reads the gradient anyway (no separate reduce pass over the planes)
    for (int k = 0; k < sl.n; ++k) {
      const int64_t e = 4 * i - sl.off[k];
      if (e < 0 || e >= sl.len[k]) continue;
      const float* p = sl.p[k] + e;
      int z = 0;
      for (; z + 3 < sl.nsplit[k]; z += 4) {
        const float4 a0 = *reinterpret_cast<const float4*>(p + z * sl.plane[k]);
        const float4 a1 = *reinterpret_cast<const float4*>(p + (z + 1) * sl.plane[k]);
        const float4 a2 = *reinterpret_cast<const float4*>(p + (z + 2) * sl.plane[k]);
        const float4 a3 = *reinterpret_cast<const float4*>(p + (z + 3) * sl.plane[k]);
        Gs.x += (a0.x + a1.x) + (a2.x + a3.x);
        Gs.y += (a0.y + a1.y) + (a2.y + a3.y);
        Gs.z += (a0.z + a1.z) + (a2.z + a3.z);
        Gs.w += (a0.w + a1.w) + (a2.w + a3.w);
      }
      for (; z < sl.nsplit[k]; ++z) {
        const float4 a = *reinterpret_cast<const float4*>(p + z * sl.plane[k]);
        Gs.x += a.x;
        Gs.y += a.y;
        Gs.z += a.z;
        Gs.w += a.w;
      }
    }
    const float* Gp = &Gs.x;
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

// Several ranks: the reduce-scatter input of a dense clock. out = g + the split-K weight-gradient
// planes of its regions (the same fold as adam_kernel's), g cleared for the next clock -- one pass
// instead of a split-K reduce per weight gradient plus a clearing pass over the gradient.
__global__ void slab_pack_kernel(float* __restrict__ g, float* __restrict__ out, int64_t n4, AdamSlabs sl) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 G = reinterpret_cast<const float4*>(g)[i];
    for (int k = 0; k < sl.n; ++k) {
      const int64_t e = 4 * i - sl.off[k];
      if (e < 0 || e >= sl.len[k]) continue;
      const float* p = sl.p[k] + e;
      for (int z = 0; z < sl.nsplit[k]; ++z) {
        const float4 a = *reinterpret_cast<const float4*>(p + z * sl.plane[k]);
        G.x += a.x;
        G.y += a.y;
        G.z += a.z;
        G.w += a.w;
      }
    }
    reinterpret_cast<float4*>(out)[i] = G;
    reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

static void check_align(const void* p, const char* what) {
  if (reinterpret_cast<uintptr_t>(p) & 15) throw std::runtime_error(std::string(what) + " must be 16-byte aligned");
}

void slab_pack(float* g, float* out, int64_t n, const AdamSlabs* slabs, hipStream_t s) {
  AdamSlabs sl{};
  if (slabs) {
    sl = *slabs;
    for (int k = 0; k < sl.n; ++k)
      if ((sl.off[k] & 3) || (sl.len[k] & 3) || (sl.plane[k] & 3) || sl.off[k] < 0 || sl.off[k] + sl.len[k] > n ||
          (reinterpret_cast<uintptr_t>(sl.p[k]) & 15))
        throw std::runtime_error("slab_pack: 16-byte aligned planes and ranges inside the gradient");
  }
  if (n % 4 || (reinterpret_cast<uintptr_t>(g) & 15) || (reinterpret_cast<uintptr_t>(out) & 15))
    throw std::runtime_error("slab_pack: 16-byte aligned gradient of a multiple of 4 floats");
  if (n == 0) return;
  hipLaunchKernelGGL(slab_pack_kernel, grid_for(n / 4, 256, 4096), 256, 0, s, g, out, n / 4, sl);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void adam_apply(float* w, float* m, float* v, const float* g, int64_t n, float lr, float beta1, float beta2, float eps,
                float weight_decay, int step, float grad_scale, bf16_t* w_bf16, hipStream_t s, const int* step_dev,
                bool zero_g, const int64_t* active, const AdamSlabs* slabs) {
  AdamSlabs sl{};
  if (slabs) {
    sl = *slabs;
    for (int k = 0; k < sl.n; ++k)
      if ((sl.off[k] & 3) || (sl.len[k] & 3) || (sl.plane[k] & 3) || sl.off[k] < 0 || sl.off[k] + sl.len[k] > n ||
          (reinterpret_cast<uintptr_t>(sl.p[k]) & 15))
        throw std::runtime_error("adam slabs: 16-byte aligned planes and ranges inside the shard");
  }
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
                     weight_decay, bc1, bc2, grad_scale, w_bf16, step_dev, zero_g, active, sl);
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
