// GPU hash-table shard (the MapStorage equivalent): open addressing with
// linear probing in HBM, 64-bit keys, one fp32 row of `W` values (+ optimizer state kept by the
// caller in slot order) per key.
//
//   hash_slots   lookup-or-insert: slot of every query key; a new key claims an EMPTY slot with
//                one 64-bit CAS and its row is initialised in the same kernel (zero, like
//                MapStorage's default-insert, or a deterministic per-key uniform [-a, a)), so a
//                Get of an unseen key returns the initial row and Adds accumulate into it
//   hash_rehash  moves every occupied slot (key, row, optional per-slot state) into a larger table
// Duplicates within one launch are safe: the CAS loser sees its own key and reuses the slot.
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace minips_k {

constexpr uint64_t kEmptyKey = ~0ull;

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__global__ void hash_slots_kernel(unsigned long long* __restrict__ tab_keys, int64_t cap, const int64_t* __restrict__ q,
                                  int64_t n, const int64_t* __restrict__ n_dev, int64_t* __restrict__ slots,
                                  float* __restrict__ vals, int W, float init_scale, uint64_t seed,
                                  int* __restrict__ counters) {
  const int64_t mask = cap - 1;
  // n_dev: the valid prefix of q is known only on the device (a dedupe's unique count): the
  // entries past it are left alone (slot -1) -- no host sync to trim q
  const int64_t n_valid = n_dev ? min(n, *n_dev) : n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long k = (unsigned long long)q[i];
    int64_t s = (int64_t)(mix64(k) & (uint64_t)mask);
    int64_t found = i < n_valid ? -1 : -2;
    bool inserted = false;
    for (int64_t probe = 0; found == -1 && probe < cap; ++probe) {
      const unsigned long long cur = tab_keys[s];
      if (cur == k) {
        found = s;
        break;
      }
      if (cur == kEmptyKey) {
        const unsigned long long prev = atomicCAS(tab_keys + s, kEmptyKey, k);
        if (prev == kEmptyKey) {  // inserted: initialise the row
          float* row = vals + s * W;
          for (int c = 0; c < W; ++c) {
            float v = 0.f;
            if (init_scale != 0.f) {
              const uint64_t h = mix64(k * 0x9e3779b97f4a7c15ull + seed + (uint64_t)c);
              v = init_scale * (2.f * (float)(h >> 40) * (1.f / 16777216.f) - 1.f);
            }
            row[c] = v;
          }
          inserted = true;
          found = s;
          break;
        }
        if (prev == k) {
          found = s;
          break;
        }
      }
      s = (s + 1) & mask;
    }
    // wave-aggregated counters: one atomic per wave, not one per inserted key (same-address
    // atomics serialise at the memory side)
    const unsigned long long ins = __ballot(inserted), full = __ballot(found == -1);
    const int leader = __ffsll((long long)__ballot(1)) - 1;
    if ((threadIdx.x & 63) == leader) {
      if (ins) atomicAdd(counters, __popcll(ins));
      if (full) atomicAdd(counters + 1, __popcll(full));  // table full
    }
    slots[i] = found < 0 ? -1 : found;
  }
}

__global__ void hash_rehash_kernel(const unsigned long long* __restrict__ old_keys, const float* __restrict__ old_vals,
                                   const float* __restrict__ old_state, int64_t old_cap,
                                   unsigned long long* __restrict__ new_keys, float* __restrict__ new_vals,
                                   float* __restrict__ new_state, int64_t new_cap, int W, int* __restrict__ counters) {
  const int64_t mask = new_cap - 1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < old_cap; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long k = old_keys[i];
    if (k == kEmptyKey) continue;
    int64_t s = (int64_t)(mix64(k) & (uint64_t)mask);
    for (int64_t probe = 0; probe < new_cap; ++probe) {
      if (atomicCAS(new_keys + s, kEmptyKey, k) == kEmptyKey) {
        for (int c = 0; c < W; ++c) new_vals[s * W + c] = old_vals[i * W + c];
        if (old_state) new_state[s] = old_state[i];
        atomicAdd(counters, 1);
        break;
      }
      s = (s + 1) & mask;
    }
  }
}

void hash_slots(unsigned long long* tab_keys, int64_t cap, const int64_t* q, int64_t n, int64_t* slots, float* vals,
                int W, float init_scale, uint64_t seed, int* counters, hipStream_t s, const int64_t* n_dev) {
  if (n <= 0) return;
  if (cap <= 0 || (cap & (cap - 1))) throw std::runtime_error("hash table capacity must be a power of two");
  hipLaunchKernelGGL(hash_slots_kernel, grid_for(n, 256, 4096), 256, 0, s, tab_keys, cap, q, n, n_dev, slots, vals,
                     W, init_scale, seed, counters);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void hash_rehash(const unsigned long long* old_keys, const float* old_vals, const float* old_state, int64_t old_cap,
                 unsigned long long* new_keys, float* new_vals, float* new_state, int64_t new_cap, int W, int* counters,
                 hipStream_t s) {
  if (new_cap <= 0 || (new_cap & (new_cap - 1))) throw std::runtime_error("hash table capacity must be a power of two");
  hipLaunchKernelGGL(hash_rehash_kernel, grid_for(old_cap, 256, 4096), 256, 0, s, old_keys, old_vals, old_state,
                     old_cap, new_keys, new_vals, new_state, new_cap, W, counters);
  MINIPS_HIP_CHECK(hipGetLastError());
}

}  // namespace minips_k
