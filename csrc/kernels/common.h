// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
// Wave64 everywhere; bf16 handled as raw uint16 with round-to-nearest-even conversion.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define MINIPS_HIP_CHECK(expr)                                                      \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess) {                                                         \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + \
                               " at " __FILE__ ":" + std::to_string(__LINE__));     \
    }                                                                               \
  } while (0)

namespace minips_k {

constexpr int kWave = 64;

typedef uint16_t bf16_t;
typedef short v8s __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// fp32 -> bf16 round-to-nearest-even on the gfx950 converter (v_cvt_pk_bf16_f32: one VALU op for
// two values, NaN-preserving) instead of the integer rounding sequence.
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

__device__ __forceinline__ bf16_t f2bf(float f) { return (bf16_t)(pack_bf2(f, 0.f) & 0xffffu); }

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

// Stochastic rounding of bf16 rows (csrc/kernels/bf16rows.hip, the one-sided clock apply): a
// stateless hash of (row, column, apply counter, seed) gives the random bits, so runs reproduce.
__device__ __forceinline__ uint32_t sr_hash(uint64_t row, uint32_t col, uint32_t step, uint32_t seed) {
  uint64_t x = row * 0x9E3779B97F4A7C15ull ^ ((uint64_t)col << 32 | step) ^ ((uint64_t)seed * 0xD1B54A32D192ED03ull);
  x ^= x >> 31;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 29;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 32;
  return (uint32_t)x;
}

__device__ __forceinline__ bf16_t bf16_sr(float v, uint32_t rnd) {
  const uint32_t b = __float_as_uint(v);
  if ((b & 0x7f800000u) == 0x7f800000u) return (bf16_t)(b >> 16);  // inf / nan unchanged
  const uint32_t r = b + (rnd & 0xffffu);
  // a finite value never rounds up to inf: it saturates at the largest finite bf16 of its sign
  if ((r & 0x7f800000u) == 0x7f800000u) return (bf16_t)(((b >> 16) & 0x8000u) | 0x7f7fu);
  return (bf16_t)(r >> 16);
}

// Grid size for grid-stride memory-bound kernels: ~8 blocks/CU on 256 CUs.
inline int grid_for(int64_t work, int block, int cap = 2048) {
  int64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace minips_k
