// Bitmap key planning for range tables with a bounded key space (bucketize
// + unique + inverse): the batch's keys set bits in an N-bit map (one atomicOr each, the map is a
// few MB and stays in L2 / MALL), a popcount scan over the map ranks the set bits, and
//   uniq    = the set bits in key order (hence already grouped by owner: ranges are contiguous),
//   inverse = rank of each key = word prefix + popcount of the lower bits of its word,
//   counts  = rank(bounds[p+1]) - rank(bounds[p]), U = total set bits (device-side, no host sync).
// No hash probing and no per-unique-key atomics: for uniformly drawn ids (LR over 16.6M features,
// DLRM over 10^8 rows) the hash dedupe runs at a high load factor and is dominated by probe chains
// and random table writes; here the random traffic is one atomicOr per key into a small map.
// Deterministic: the unique order is the sorted key order.
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace minips_k {

constexpr int kBmThreads = 256;
constexpr int kBmWordsPerThread = 16;
constexpr int kBmWordsPerBlock = kBmThreads * kBmWordsPerThread;  // 4096 words = 131072 keys

__device__ __forceinline__ int64_t bm_route(int64_t key, uint64_t mult, uint64_t rn) {
  return mult ? (int64_t)(((uint64_t)key * mult) % rn) : key;
}

__global__ void bm_set_kernel(const int64_t* __restrict__ keys, int64_t n, uint64_t rmult, uint64_t rn,
                              int64_t space, uint32_t* __restrict__ bitmap, int64_t* __restrict__ oor) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = bm_route(keys[i], rmult, rn);
    if ((uint64_t)k >= (uint64_t)space) {  // outside the table: never written (no fault), but counted
      if (oor) atomicAdd(reinterpret_cast<unsigned long long*>(oor), 1ull);
      continue;
    }
    const uint32_t bit = 1u << (k & 31);
    uint32_t* w = bitmap + (k >> 5);
    if (!(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit)) atomicOr(w, bit);
  }
}

// popcount of each block's 4096 words -> block_sums[b]
__global__ __launch_bounds__(kBmThreads) void bm_count_kernel(const uint32_t* __restrict__ bitmap, int64_t nwords,
                                                              int64_t* __restrict__ block_sums) {
  __shared__ int red[kBmThreads / 64];
  const int64_t w0 = (int64_t)blockIdx.x * kBmWordsPerBlock + threadIdx.x;
  int c = 0;
#pragma unroll
  for (int j = 0; j < kBmWordsPerThread; ++j) {
    const int64_t w = w0 + (int64_t)j * kBmThreads;  // coalesced: consecutive threads, consecutive words
    if (w < nwords) c += __popc(bitmap[w]);
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) block_sums[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// exclusive scan of the block sums in place (one block; nb is small: N / 131072), total -> *U
__global__ __launch_bounds__(1024) void bm_scan_blocks_kernel(int64_t* __restrict__ block_sums, int nb,
                                                              int64_t* __restrict__ U) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int per = (nb + 1023) / 1024;
  int64_t s = 0;
  for (int j = 0; j < per; ++j) {
    const int b = t * per + j;
    if (b < nb) s += block_sums[b];
  }
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan of the 1024 partials
    const int64_t v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = t ? part[t - 1] : 0;
  for (int j = 0; j < per; ++j) {
    const int b = t * per + j;
    if (b < nb) {
      const int64_t v = block_sums[b];
      block_sums[b] = run;
      run += v;
    }
  }
  if (t == 1023) *U = part[1023];
}

// per-word rank bases + the unique keys: word w's set bits get ranks word_prefix[w] + 0, 1, ...
__global__ __launch_bounds__(kBmThreads) void bm_emit_kernel(const uint32_t* __restrict__ bitmap, int64_t nwords,
                                                             const int64_t* __restrict__ block_off,
                                                             int64_t* __restrict__ word_prefix,
                                                             int64_t* __restrict__ uniq) {
  __shared__ int tsum[kBmThreads];
  // thread t owns words [w0 + 16 t, +16) here (contiguous per thread, so its ranks are a run)
  const int64_t w0 = (int64_t)blockIdx.x * kBmWordsPerBlock + (int64_t)threadIdx.x * kBmWordsPerThread;
  uint32_t words[kBmWordsPerThread];
  int c = 0;
#pragma unroll
  for (int j = 0; j < kBmWordsPerThread; ++j) {
    words[j] = w0 + j < nwords ? bitmap[w0 + j] : 0u;
    c += __popc(words[j]);
  }
  tsum[threadIdx.x] = c;
  __syncthreads();
  for (int o = 1; o < kBmThreads; o <<= 1) {
    const int v = threadIdx.x >= o ? tsum[threadIdx.x - o] : 0;
    __syncthreads();
    tsum[threadIdx.x] += v;
    __syncthreads();
  }
  int64_t r = block_off[blockIdx.x] + (threadIdx.x ? tsum[threadIdx.x - 1] : 0);
#pragma unroll
  for (int j = 0; j < kBmWordsPerThread; ++j) {
    const int64_t w = w0 + j;
    if (w >= nwords) break;
    word_prefix[w] = r;
    uint32_t b = words[j];
    while (b) {
      const int bit = __ffs(b) - 1;
      uniq[r++] = (w << 5) + bit;
      b &= b - 1;
    }
  }
}

__device__ __forceinline__ int64_t bm_rank(const uint32_t* bitmap, const int64_t* word_prefix, int64_t nwords,
                                           int64_t U, int64_t k) {
  const int64_t w = k >> 5;
  if (w >= nwords) return U;
  const uint32_t lower = bitmap[w] & ((1u << (k & 31)) - 1u);
  return word_prefix[w] + __popc(lower);
}

__global__ void bm_inverse_kernel(const int64_t* __restrict__ keys, int64_t n, uint64_t rmult, uint64_t rn,
                                  int64_t space, const uint32_t* __restrict__ bitmap,
                                  const int64_t* __restrict__ word_prefix, int64_t nwords,
                                  const int64_t* __restrict__ U, int64_t* __restrict__ inverse) {
  const int64_t u = *U;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = bm_route(keys[i], rmult, rn);
    inverse[i] = (uint64_t)k < (uint64_t)space ? bm_rank(bitmap, word_prefix, nwords, u, k) : 0;
  }
}

// counts[p] = #unique keys in [bounds[p], bounds[p+1]); counts[P] = U
__global__ void bm_counts_kernel(const int64_t* __restrict__ bounds, int P, const uint32_t* __restrict__ bitmap,
                                 const int64_t* __restrict__ word_prefix, int64_t nwords, const int64_t* __restrict__ U,
                                 int64_t* __restrict__ counts) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t u = *U;
  if (p < P) {
    const int64_t lo = bm_rank(bitmap, word_prefix, nwords, u, bounds[p]);
    const int64_t hi = bm_rank(bitmap, word_prefix, nwords, u, bounds[p + 1]);
    counts[p] = hi - lo;
  }
  if (p == 0) counts[P] = u;
}

int64_t bitmap_plan_workspace_words(int64_t num_keys_space) {
  const int64_t nwords = (num_keys_space + 31) / 32;
  const int64_t nb = (nwords + kBmWordsPerBlock - 1) / kBmWordsPerBlock;
  // bitmap (uint32, rounded to int64 words) | word_prefix [nwords] | block sums [nb]
  return (nwords + 1) / 2 + nwords + nb;
}

void bitmap_plan(const int64_t* keys, int64_t n, int64_t num_keys_space, const int64_t* bounds, int P,
                 uint64_t rmult, uint64_t rn, int64_t* ws, int64_t* uniq, int64_t* inverse, int64_t* counts,
                 int64_t* U, hipStream_t s, int64_t* oor) {
  if (num_keys_space <= 0) throw std::runtime_error("bitmap_plan: empty key space");
  const int64_t nwords = (num_keys_space + 31) / 32;
  const int64_t nb = (nwords + kBmWordsPerBlock - 1) / kBmWordsPerBlock;
  if (nb > (1LL << 24)) throw std::runtime_error("bitmap_plan: key space too large");
  uint32_t* bitmap = reinterpret_cast<uint32_t*>(ws);
  int64_t* word_prefix = ws + (nwords + 1) / 2;
  int64_t* block_sums = word_prefix + nwords;
  MINIPS_HIP_CHECK(hipMemsetAsync(bitmap, 0, sizeof(uint32_t) * (size_t)nwords, s));
  if (n > 0)
    hipLaunchKernelGGL(bm_set_kernel, grid_for(n, 256, 8192), 256, 0, s, keys, n, rmult, rn, num_keys_space, bitmap,
                       oor);
  hipLaunchKernelGGL(bm_count_kernel, (unsigned)nb, kBmThreads, 0, s, bitmap, nwords, block_sums);
  hipLaunchKernelGGL(bm_scan_blocks_kernel, 1, 1024, 0, s, block_sums, (int)nb, U);
  hipLaunchKernelGGL(bm_emit_kernel, (unsigned)nb, kBmThreads, 0, s, bitmap, nwords, block_sums, word_prefix, uniq);
  if (n > 0)
    hipLaunchKernelGGL(bm_inverse_kernel, grid_for(n, 256, 8192), 256, 0, s, keys, n, rmult, rn, num_keys_space,
                       bitmap, word_prefix, nwords, U, inverse);
  hipLaunchKernelGGL(bm_counts_kernel, (P + 1 + 63) / 64, 64, 0, s, bounds, P, bitmap, word_prefix, nwords, U, counts);
  MINIPS_HIP_CHECK(hipGetLastError());
}

}  // namespace minips_k
