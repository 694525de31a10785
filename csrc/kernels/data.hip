// Fused on-device synthetic batch generator for the Criteo-shaped benchmarks (one launch per
// step instead of ~15 torch RNG/elementwise launches). Counter-based RNG (splitmix64 of
// seed, step, element), so batches are reproducible and independent of the launch shape.
//   dense  [B, n_dense] ~ N(0,1) (Box-Muller)
//   keys   [B, F]  id = floor((card+1)^u) - 1 (log-uniform / Zipf(1) head), scattered by a
//                  bijective multiplicative hash, plus the feature's row offset
//   labels [B]     Bernoulli(sigmoid(2 * (dense.w + 0.5*(#odd of the first 4 raw ids - 1))))
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"

namespace minips_k {

__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
  x += 0x9e3779b97f4a7c15ULL;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

__device__ __forceinline__ float u01f(uint64_t h) { return ((uint32_t)(h >> 40) + 0.5f) * (1.0f / 16777216.0f); }

__device__ __forceinline__ int64_t raw_id(uint64_t sb, int f, int64_t card) {
  const float u = u01f(splitmix(sb + 1000 + f));
  int64_t raw = (int64_t)floorf(__expf(u * __logf((float)card + 1.f)) - 1.f);
  return raw < 0 ? 0 : (raw >= card ? card - 1 : raw);
}

// Index space B*F (one key each) + B (dense features + label): no serial per-sample loop.
__global__ void criteo_synth_kernel(uint64_t seed, uint64_t step, const int64_t* __restrict__ step_dev,
                                    int64_t B, int F,
                                    const int64_t* __restrict__ cards,
                                    const int64_t* __restrict__ offsets, int n_dense, const float* __restrict__ w,
                                    float* __restrict__ dense, int64_t* __restrict__ keys, float* __restrict__ labels) {
  // step_dev: the step counter lives on the device (advanced by the caller's stream), so a step
  // captured in a HIP graph draws a new batch on every replay
  if (step_dev) step += (uint64_t)*step_dev;
  const uint64_t base = splitmix(seed * 0x632be59bd9b4e019ULL + step);
  const int64_t nk = B * F;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nk + B; e += (int64_t)gridDim.x * blockDim.x) {
    if (e < nk) {
      // 32-bit index math and a 64-bit modulo when the product fits (every Criteo card is < 2^32):
      // the 128-bit remainder is a long software routine, and it dominated this kernel
      const int64_t b = nk < (1LL << 31) ? (int64_t)((uint32_t)e / (uint32_t)F) : e / F;
      const int f = (int)(e - b * F);
      const uint64_t sb = splitmix(base ^ (uint64_t)b * 0xd1342543de82ef95ULL);
      const int64_t card = cards[f];
      const int64_t raw = raw_id(sb, f, card);
      uint64_t h;
      if (card < (1LL << 16)) {
        // raw < card < 2^16: (raw * (A mod card)) < 2^32 -- a 32-bit remainder, same value
        h = ((uint32_t)raw * (2654435761u % (uint32_t)card)) % (uint32_t)card;
      } else if (card < (1LL << 32)) {
        // product < 2^56: a double-precision quotient is off by at most one for card >= 2^16
        // (the 64-bit integer remainder is a long software routine); exact after the correction
        const uint64_t prod = (uint64_t)raw * 2654435761ULL;
        const int64_t q = (int64_t)((double)prod / (double)card);
        int64_t r = (int64_t)prod - q * card;
        if (r < 0) r += card;
        if (r >= card) r -= card;
        h = (uint64_t)r;
      } else {
        h = (uint64_t)(((unsigned __int128)raw * 2654435761ULL) % (unsigned __int128)card);
      }
      keys[e] = (int64_t)h + offsets[f];
    } else {
      const int64_t b = e - nk;
      const uint64_t sb = splitmix(base ^ (uint64_t)b * 0xd1342543de82ef95ULL);
      float logit = 0.f;
      for (int j = 0; j < n_dense; j += 2) {
        const float u1 = u01f(splitmix(sb + 2 * j + 1)), u2 = u01f(splitmix(sb + 2 * j + 2));
        const float r = sqrtf(-2.f * __logf(u1));
        float sn, cs;
        __sincosf(6.2831853f * u2, &sn, &cs);
        dense[b * n_dense + j] = r * cs;
        logit += r * cs * w[j];
        if (j + 1 < n_dense) {
          dense[b * n_dense + j + 1] = r * sn;
          logit += r * sn * w[j + 1];
        }
      }
      int odd = 0;
      for (int f = 0; f < 4 && f < F; ++f) odd += (int)(raw_id(sb, f, cards[f]) & 1);
      logit += 0.5f * ((float)odd - 1.f);
      const float noise = u01f(splitmix(sb + 5000));
      labels[b] = (1.f / (1.f + __expf(-2.f * logit)) > noise) ? 1.f : 0.f;
    }
  }
}

void criteo_synth(uint64_t seed, uint64_t step, const int64_t* step_dev, int64_t B, int F, const int64_t* cards,
                  const int64_t* offsets, int n_dense, const float* w, float* dense, int64_t* keys, float* labels,
                  hipStream_t s) {
  if (B <= 0) return;
  const int block = 256;
  hipLaunchKernelGGL(criteo_synth_kernel, grid_for(B * (F + 1), block, 4096), block, 0, s, seed, step,
                     step_dev, B, F, cards, offsets,
                     n_dense, w,
                     dense, keys, labels);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// DLRM-shaped batch (BASELINE config 5): keys uniform over the whole table (multiply-high of a
// 64-bit hash: unbiased enough, no 128-bit modulo even for 10B rows), dense N(0,1), label =
// dense[b][0] > 0 -- the same distribution as the torch.randint / randn generator it replaces,
// in one launch (torch's int64 randint took 228 us per DLRM batch).
__global__ void uniform_synth_kernel(uint64_t seed, uint64_t step, int64_t B, int F, uint64_t rows, int n_dense,
                                     float* __restrict__ dense, int64_t* __restrict__ keys,
                                     float* __restrict__ labels) {
  const uint64_t base = splitmix(seed * 0x632be59bd9b4e019ULL + step);
  const int64_t nk = B * F;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nk + B; e += (int64_t)gridDim.x * blockDim.x) {
    if (e < nk) {
      const uint64_t h = splitmix(base ^ ((uint64_t)e * 0xd1342543de82ef95ULL));
      keys[e] = (int64_t)__umul64hi(h, rows);
    } else {
      const int64_t b = e - nk;
      const uint64_t sb = splitmix(base ^ ((uint64_t)b * 0x9e3779b97f4a7c15ULL) ^ 0x5bd1e995ULL);
      for (int j = 0; j < n_dense; j += 2) {
        const float u1 = u01f(splitmix(sb + 2 * j + 1)), u2 = u01f(splitmix(sb + 2 * j + 2));
        const float r = sqrtf(-2.f * __logf(u1));
        float sn, cs;
        __sincosf(6.2831853f * u2, &sn, &cs);
        dense[b * n_dense + j] = r * cs;
        if (j == 0) labels[b] = r * cs > 0.f ? 1.f : 0.f;
        if (j + 1 < n_dense) dense[b * n_dense + j + 1] = r * sn;
      }
    }
  }
}

void uniform_synth(uint64_t seed, uint64_t step, int64_t B, int F, uint64_t rows, int n_dense, float* dense,
                   int64_t* keys, float* labels, hipStream_t s) {
  if (B <= 0) return;
  if (rows == 0 || n_dense < 1) throw std::runtime_error("uniform_synth: rows > 0 and n_dense >= 1");
  hipLaunchKernelGGL(uniform_synth_kernel, grid_for(B * (F + 1), 256, 4096), 256, 0, s, seed, step, B, F, rows,
                     n_dense, dense, keys, labels);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// ---- clock probe (diagnostics): one lane counts shader-clock cycles (s_memtime) against the
// constant 100 MHz real-time counter (s_memrealtime) over ~spin ticks, so the effective SCLK at that
// moment is cycles / ticks * 100 MHz. A one-wave launch on a side stream samples the clock while a
// workload runs (tools/step_probe.py curve, CLOCK_PROBE=1). Bounded spin.
__global__ __launch_bounds__(64) void clock_probe_kernel(int64_t* __restrict__ out, int spin) {
  if (threadIdx.x != 0) return;
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  uint64_t r1 = r0;
  for (int guard = 0; r1 - r0 < (uint64_t)spin && guard < (1 << 22); ++guard) r1 = __builtin_amdgcn_s_memrealtime();
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  r1 = __builtin_amdgcn_s_memrealtime();
  out[0] = (int64_t)(c1 - c0);
  out[1] = (int64_t)(r1 - r0);
}

// ---- modelled link time of an emulated collective (ps/comm.py LoopbackComm wire model): `blocks`
// one-wave workgroups -- the CUs an RCCL collective's channels occupy -- spin `ticks` of the 100 MHz
// real-time counter on the collective's stream. Bounded spin; writes nothing.
__global__ __launch_bounds__(64) void wire_spin_kernel(int spin) {
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  uint64_t r1 = r0;
  for (int guard = 0; r1 - r0 < (uint64_t)spin && guard < (1 << 22); ++guard) {
    __builtin_amdgcn_s_sleep(2);
    r1 = __builtin_amdgcn_s_memrealtime();
  }
}

void wire_spin(int spin_ticks, int blocks, hipStream_t s) {
  if (spin_ticks < 1 || spin_ticks > 1000000 || blocks < 1 || blocks > 256)
    throw std::runtime_error("wire_spin: 1 <= spin_ticks <= 1e6, 1 <= blocks <= 256");
  hipLaunchKernelGGL(wire_spin_kernel, blocks, 64, 0, s, spin_ticks);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// ---- loopback stand-ins of an emulated N-rank job (ps/comm.py LoopbackComm, ps/tables.py): the
// reduce-scatter's sum of the N equal slices (in slice order), and the re-base of this rank's own
// requests to owner s into its own range (key - s * step with s = min(key / step, P - 1), + base)
__global__ __launch_bounds__(256) void emu_sum_slices_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                             int64_t n4, int P) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 a = reinterpret_cast<const float4*>(in)[i];
    for (int r = 1; r < P; ++r) {
      const float4 b = reinterpret_cast<const float4*>(in)[r * n4 + i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    reinterpret_cast<float4*>(out)[i] = a;
  }
}

__global__ void emu_rebase_kernel(int64_t* __restrict__ keys, int64_t n, int64_t step, int P, int64_t base) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = keys[i];
    const int64_t s = min(k / step, (int64_t)(P - 1));
    keys[i] = k - s * step + base;
  }
}

void emu_sum_slices(const float* in, float* out, int64_t n, int P, hipStream_t s) {
  if (n % 4 || (reinterpret_cast<uintptr_t>(in) & 15) || (reinterpret_cast<uintptr_t>(out) & 15) || P < 1)
    throw std::runtime_error("emu_sum_slices: 16-byte aligned slices of a multiple of 4 floats");
  if (n == 0) return;
  hipLaunchKernelGGL(emu_sum_slices_kernel, grid_for(n / 4, 256, 4096), 256, 0, s, in, out, n / 4, P);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void emu_rebase(int64_t* keys, int64_t n, int64_t step, int P, int64_t base, hipStream_t s) {
  if (n <= 0) return;
  if (step <= 0) throw std::runtime_error("emu_rebase: step > 0");
  hipLaunchKernelGGL(emu_rebase_kernel, grid_for(n, 256, 4096), 256, 0, s, keys, n, step, P, base);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void clock_probe(int64_t* out, int spin_ticks, hipStream_t s) {
  if (spin_ticks < 1 || spin_ticks > 1000000) throw std::runtime_error("clock_probe: 1 <= spin_ticks <= 1e6");
  hipLaunchKernelGGL(clock_probe_kernel, 1, 64, 0, s, out, spin_ticks);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// ---- several device-to-device copies in ONE launch (a HIP-graph step's static input slots are
// refilled by 11 copies: as separate copy nodes each cost a dispatch gap, ~110 us in a row).
// 16-byte vectors over the 16-byte body of each pair, bytes over its tail.
__global__ __launch_bounds__(256) void multi_copy_kernel(MultiCopyArgs a) {
  const int64_t total = a.start[a.n];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int t = 0;
    while (t + 1 < a.n && a.start[t + 1] <= i) ++t;
    const int64_t j = i - a.start[t];
    if (j < a.n16[t]) {
      reinterpret_cast<uint4*>(a.dst[t])[j] = reinterpret_cast<const uint4*>(a.src[t])[j];
    } else {
      const int64_t b = a.n16[t] * 16 + (j - a.n16[t]);
      static_cast<char*>(a.dst[t])[b] = static_cast<const char*>(a.src[t])[b];
    }
  }
}

void multi_copy(const MultiCopyArgs& a, hipStream_t s) {
  if (a.n < 1 || a.n > kMultiCopyMax) throw std::runtime_error("multi_copy: 1..16 pairs");
  const int64_t total = a.start[a.n];
  if (total <= 0) return;
  hipLaunchKernelGGL(multi_copy_kernel, grid_for(total, 256, 2048), 256, 0, s, a);
  MINIPS_HIP_CHECK(hipGetLastError());
}

}  // namespace minips_k
