// Sparse-table kernels of the GPU parameter server:
//   K5/K4  unique_bucketize   hash dedupe of a batch's keys + grouping by owner shard
//   K2     gather_rows        server-side row gather (pull), fp32 -> fp32/bf16
//   K1     scatter_add_rows   worker-side gradient dedupe (segment sum via float atomics)
//   K1     sparse_rowwise_adagrad / sparse_sgd   server-side apply on the shard rows
//          embedding_bag_fwd/bwd                 pooled lookups (DLRM-style bags)
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"

namespace minips_k {

constexpr int64_t kEmpty = -1;

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ int owner_of(const int64_t* bounds, int P, int64_t key) {
  // upper_bound over P+1 sorted bounds (P <= a few dozen): linear scan is cheapest.
  int o = 0;
  for (int p = 1; p < P; ++p) o += (key >= bounds[p]) ? 1 : 0;
  return o;
}

// Wave-aggregated atomic add of 1 per active lane, grouped by `slot`: one atomic per
// distinct slot per wave instead of one per lane (a single shared counter otherwise
// serialises every unique key of the batch). Returns this lane's rank-ordered old value.
__device__ __forceinline__ unsigned long long wave_agg_inc(unsigned long long* ctr, int slot, bool active) {
  unsigned long long mine = 0;
  unsigned long long pending = __ballot(active);
  const int lane = threadIdx.x & 63;
  while (pending) {
    const int leader = __ffsll((long long)pending) - 1;
    const int s = __shfl(slot, leader);
    const unsigned long long grp = __ballot(active && slot == s) & pending;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(ctr + s, (unsigned long long)__popcll(grp));
    base = __shfl(base, leader);
    if ((grp >> lane) & 1ULL) mine = base + (unsigned long long)__popcll(grp & ((1ULL << lane) - 1ULL));
    pending &= ~grp;
  }
  return mine;
}

// Insert with block-local pre-dedupe: a block takes 256 keys of ONE feature (feature-major
// tile over a [B, F] batch, F = 1 for a flat key list), dedupes them in an LDS hash, and only
// the block-distinct keys probe the global table (read first, CAS only on an empty slot).
// Zipf-hot ids (a 3-value feature hit by every sample) otherwise hammer one global slot with
// thousands of CAS.
constexpr int kUbTile = 256;
constexpr int kUbLds = 512;

// element i of the feature-major order over a [rows_b, F] batch -> its index in the batch
__device__ __forceinline__ int64_t tile_phys(int64_t i, int64_t rows_b, int F) {
  if (rows_b * F < (1LL << 31)) {  // 32-bit division: the 64-bit one is a long software routine
    const uint32_t ui = (uint32_t)i, rb = (uint32_t)rows_b;
    const uint32_t f = ui / rb;
    return (int64_t)(ui - f * rb) * F + f;
  }
  return (i % rows_b) * F + i / rows_b;
}

// Optional key routing fused into the dedupe: key -> key * mult mod rn (a bijection of [0, rn) when
// mult is coprime to rn; the caller guarantees key * mult < 2^63). mult == 0: identity.
__device__ __forceinline__ int64_t route_key(int64_t key, uint64_t mult, uint64_t rn) {
  return mult ? (int64_t)(((uint64_t)key * mult) % rn) : key;
}

__global__ __launch_bounds__(kUbTile) void ub_insert_kernel(const int64_t* __restrict__ keys, int64_t n, int64_t rows_b,
                                                            int F, const int64_t* __restrict__ bounds, int P,
                                                            unsigned long long* table_keys, int64_t cap, int64_t* slot,
                                                            int32_t* flags, unsigned long long* sh_counts, int S,
                                                            uint64_t rmult, uint64_t rn, int* slot_cnt) {
  __shared__ unsigned long long lkey[kUbLds];
  __shared__ long long lgslot[kUbLds];
  __shared__ unsigned int lkcnt[kUbLds];  // occurrences of each block-distinct key (slot_cnt)
  __shared__ unsigned int lcount[256];  // per-owner claims of this block (P <= 256)
  const int t = threadIdx.x;
  for (int j = t; j < kUbLds; j += kUbTile) {
    lkey[j] = (unsigned long long)kEmpty;
    lkcnt[j] = 0;
  }
  for (int p = t; p < P; p += kUbTile) lcount[p] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kUbTile + t;
  const bool valid = i < n;
  int64_t phys = i;
  if (F > 1 && valid) phys = tile_phys(i, rows_b, F);  // feature-major tile
  const int64_t key = valid ? route_key(keys[phys], rmult, rn) : 0;
  int lslot = 0;
  bool lead = false;
  if (valid) {
    int h = (int)(mix64((uint64_t)key) & (kUbLds - 1));
    while (true) {
      unsigned long long prev = atomicCAS(lkey + h, (unsigned long long)kEmpty, (unsigned long long)key);
      if (prev == (unsigned long long)kEmpty) {
        lead = true;
        break;
      }
      if (prev == (unsigned long long)key) break;
      h = (h + 1) & (kUbLds - 1);
    }
    lslot = h;
    if (slot_cnt) atomicAdd(lkcnt + h, 1u);
  }
  __syncthreads();
  bool claimed = false;
  int owner = 0;
  if (lead) {
    const int64_t mask = cap - 1;
    int64_t h = (int64_t)(mix64((uint64_t)key * 0x9e3779b97f4a7c15ULL) & (uint64_t)mask);
    // global slots hold key + 1 (keys are < 2^63), so 0 marks an empty slot and the table is
    // cleared by the same zero memset as the per-owner counters (one memset per call)
    const unsigned long long tag = (unsigned long long)key + 1ULL;
    while (true) {
      unsigned long long cur = __hip_atomic_load(table_keys + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == tag) break;
      if (cur == 0ULL) {
        unsigned long long prev = atomicCAS(table_keys + h, 0ULL, tag);
        if (prev == 0ULL) {
          claimed = true;
          break;
        }
        if (prev == tag) break;
      }
      h = (h + 1) & mask;
    }
    lgslot[lslot] = h;
    // per-key lookup counts (the embedding-backward CSR's row sizes): one global atomic per
    // block-distinct key, not per lookup (Zipf-hot keys would serialise thousands)
    if (slot_cnt) atomicAdd(slot_cnt + h, (int)lkcnt[lslot]);
    if (claimed) {
      owner = owner_of(bounds, P, key);
      atomicAdd(lcount + owner, 1u);
    }
  }
  __syncthreads();
  // per-owner claim counts into counter shard blockIdx % S: every block adding to ONE counter
  // serialises ~n/256 memory-side atomics on one address (~12 ns each: tens of microseconds)
  unsigned long long* sh = sh_counts + (size_t)(blockIdx.x % S) * P;
  for (int p = t; p < P; p += kUbTile)
    if (lcount[p]) atomicAdd(sh + p, (unsigned long long)lcount[p]);
  if (valid) {  // tile order: ub_assign's block b sees exactly the elements of this block b
    slot[i] = lgslot[lslot];
    flags[i] = claimed ? 1 : 0;
  }
}

// Position assignment: one element per thread; ranks inside the block come from LDS
// counters and each block takes ONE global atomic per owner shard for its base, so the
// shared cursor sees (#blocks x P) atomics instead of one per unique key.
constexpr int kUbMaxP = 256;

__global__ __launch_bounds__(256) void ub_assign_kernel(const int64_t* __restrict__ keys, int64_t n, int64_t rows_b,
                                                        int F, const int64_t* __restrict__ bounds, int P,
                                                        const int64_t* __restrict__ slot,
                                                        const int32_t* __restrict__ flags,
                                                        const int64_t* __restrict__ sh_counts, int S,
                                                        unsigned long long* sh_cursor, int64_t* counts,
                                                        int64_t* table_pos, int64_t* out_keys, uint64_t rmult,
                                                        uint64_t rn, const int* __restrict__ slot_cnt,
                                                        int* __restrict__ csr_counts) {
  __shared__ int64_t offs[kUbMaxP];
  __shared__ int64_t tot[kUbMaxP];
  __shared__ unsigned int lcnt[kUbMaxP];
  __shared__ unsigned long long lbase[kUbMaxP];
  const int t = threadIdx.x;
  const int sh = (int)(blockIdx.x % S);
  // owner p's unique keys occupy [sum_{q<p} tot[q], +tot[p]); inside that range the shards follow
  // each other, so this block's shard starts pre[p] further (all from the insert's shard counts)
  // S * P <= 256 (ub_shards): one load per thread, all in flight at once (a per-owner loop over
  // the shards would chain S memory-side latencies -- the counters were just written by atomics)
  __shared__ int64_t shc[256];
  if (t < S * P) shc[t] = sh_counts[t];
  __syncthreads();
  for (int p = t; p < P; p += blockDim.x) {
    int64_t total = 0, pre = 0;
    for (int q = 0; q < S; ++q) {
      const int64_t c = shc[q * P + p];
      total += c;
      pre += q < sh ? c : 0;
    }
    tot[p] = total;
    offs[p] = pre;
    lcnt[p] = 0;
  }
  __syncthreads();
  if (t == 0) {
    int64_t acc = 0;
    for (int p = 0; p < P; ++p) {
      offs[p] += acc;
      acc += tot[p];
    }
    if (blockIdx.x == 0) counts[P] = acc;  // total unique: the device-side U (no host sync)
  }
  if (blockIdx.x == 0)
    for (int p = t; p < P; p += blockDim.x) counts[p] = tot[p];
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + t;
  const bool claimer = i < n && flags[i];
  int64_t key = 0;
  int o = 0;
  unsigned int r = 0;
  if (claimer) {
    key = route_key(keys[F > 1 ? tile_phys(i, rows_b, F) : i], rmult, rn);
    o = owner_of(bounds, P, key);
    r = atomicAdd(lcnt + o, 1u);
  }
  __syncthreads();
  unsigned long long* cur = sh_cursor + (size_t)sh * P;
  for (int p = t; p < P; p += blockDim.x) lbase[p] = lcnt[p] ? atomicAdd(cur + p, (unsigned long long)lcnt[p]) : 0ULL;
  __syncthreads();
  if (claimer) {
    const int64_t pos = offs[o] + (int64_t)lbase[o] + (int64_t)r;
    const int64_t sl = slot[i];
    table_pos[sl] = pos;
    out_keys[pos] = key;
    if (csr_counts) csr_counts[pos] = slot_cnt[sl];
  }
}

__global__ void ub_inverse_kernel(int64_t n, int64_t rows_b, int F, const int64_t* __restrict__ slot,
                                  const int64_t* __restrict__ table_pos, int64_t* inverse) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    inverse[F > 1 ? tile_phys(i, rows_b, F) : i] = table_pos[slot[i]];
}

int ub_shards(int P) { return std::max(1, std::min(32, 256 / std::max(P, 1))); }  // S * P <= 256

void unique_bucketize(const int64_t* keys, int64_t n, int F, const int64_t* bounds, int P, int64_t* table_keys,
                      int64_t* table_pos, int64_t cap, int64_t* slot, int32_t* flags, int64_t* counts,
                      int64_t* cursor, int64_t* out_keys, int64_t* inverse, hipStream_t s, uint64_t route_mult,
                      uint64_t route_n, int64_t extra_zero_bytes, int* csr_counts) {
  if (F < 1 || n % F) throw std::runtime_error("unique_bucketize: n must be a multiple of F");
  if (route_mult && !route_n) throw std::runtime_error("unique_bucketize: routing needs the row count");
  if (P < 1 || P > kUbMaxP) throw std::runtime_error("unique_bucketize: 1 <= P <= 256 owner shards");
  if (cap & (cap - 1)) throw std::runtime_error("unique_bucketize: capacity must be a power of two");
  if (n > 0 && cap <= n) throw std::runtime_error("unique_bucketize: capacity must exceed n");
  if (counts != table_keys + cap || cursor != counts + P + 1)
    throw std::runtime_error("unique_bucketize: expects one buffer table | counts | total | shard counters");
  // one buffer: table [cap] | counts [P] | total | shard counts [S*P] | shard cursors [S*P] |
  // (csr_counts: per-slot lookup counts, cap int32) | extra; `cursor` points at the shard counts
  // (the caller sizes it with ub_shards) -> one zero memset
  const int S = ub_shards(P);
  int64_t* sh_counts = cursor;
  int64_t* sh_cursor = cursor + (size_t)S * P;
  int* slot_cnt = csr_counts ? reinterpret_cast<int*>(sh_cursor + (size_t)S * P) : nullptr;
  if (csr_counts) extra_zero_bytes += cap * (int64_t)sizeof(int);
  MINIPS_HIP_CHECK(hipMemsetAsync(table_keys, 0, (cap + P + 1 + 2 * (int64_t)S * P) * sizeof(int64_t)
                                  + extra_zero_bytes, s));
  if (n == 0) return;
  const int block = 256;
  const int grid = grid_for(n, block, 4096);
  const int64_t tiles = (n + kUbTile - 1) / kUbTile;
  hipLaunchKernelGGL(ub_insert_kernel, dim3((unsigned)tiles), dim3(kUbTile), 0, s, keys, n, n / F, F, bounds, P,
                     (unsigned long long*)table_keys, cap, slot, flags, (unsigned long long*)sh_counts, S, route_mult,
                     route_n, slot_cnt);
  hipLaunchKernelGGL(ub_assign_kernel, dim3((unsigned)tiles), dim3(kUbTile), 0, s, keys, n, n / F, F, bounds, P, slot,
                     flags, sh_counts, S, (unsigned long long*)sh_cursor, counts, table_pos, out_keys, route_mult,
                     route_n, slot_cnt, csr_counts);
  hipLaunchKernelGGL(ub_inverse_kernel, grid, block, 0, s, n, n / F, F, slot, table_pos, inverse);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// --------------------------------------------------------------------------- gather
// n_dev (nullable): device-side row count (<= n, the grid's upper bound)
__device__ __forceinline__ int64_t dev_count(int64_t n, const int64_t* n_dev) { return n_dev ? min(n, *n_dev) : n; }

template <bool BF16>
__global__ void gather_rows_vec4(const float* __restrict__ table, int64_t ld, const int64_t* __restrict__ keys,
                                 int64_t n, int64_t base, int D4, void* out, const int64_t* n_dev) {
  const int64_t total = dev_count(n, n_dev) * D4;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = c / D4;
    const int d4 = (int)(c - i * D4);
    const float4 v = *reinterpret_cast<const float4*>(table + (keys[i] - base) * ld + d4 * 4);
    if (BF16) {
      uint2 o;
      o.x = pack_bf2(v.x, v.y);
      o.y = pack_bf2(v.z, v.w);
      reinterpret_cast<uint2*>(out)[c] = o;
    } else {
      reinterpret_cast<float4*>(out)[c] = v;
    }
  }
}

template <bool BF16>
__global__ void gather_rows_scalar(const float* __restrict__ table, int64_t ld, const int64_t* __restrict__ keys,
                                   int64_t n, int64_t base, int D, void* out, const int64_t* n_dev) {
  const int64_t total = dev_count(n, n_dev) * D;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = c / D;
    const int d = (int)(c - i * D);
    const float v = table[(keys[i] - base) * ld + d];
    if (BF16)
      reinterpret_cast<bf16_t*>(out)[c] = f2bf(v);
    else
      reinterpret_cast<float*>(out)[c] = v;
  }
}

void gather_rows(const float* table, int64_t ld, const int64_t* keys, int64_t n, int64_t base, int D, void* out,
                 bool out_bf16, hipStream_t s, const int64_t* n_dev) {
  if (n <= 0) return;
  const int block = 256;
  if (D % 4 == 0 && ld % 4 == 0) {
    const int grid = grid_for(n * (D / 4), block);
    if (out_bf16)
      hipLaunchKernelGGL(gather_rows_vec4<true>, grid, block, 0, s, table, ld, keys, n, base, D / 4, out, n_dev);
    else
      hipLaunchKernelGGL(gather_rows_vec4<false>, grid, block, 0, s, table, ld, keys, n, base, D / 4, out, n_dev);
  } else {
    const int grid = grid_for(n * D, block);
    if (out_bf16)
      hipLaunchKernelGGL(gather_rows_scalar<true>, grid, block, 0, s, table, ld, keys, n, base, D, out, n_dev);
    else
      hipLaunchKernelGGL(gather_rows_scalar<false>, grid, block, 0, s, table, ld, keys, n, base, D, out, n_dev);
  }
  MINIPS_HIP_CHECK(hipGetLastError());
}

// --------------------------------------------------------------------------- scatter-add
__device__ __forceinline__ float ld_f(const float* p) { return *p; }
__device__ __forceinline__ float ld_f(const bf16_t* p) { return bf2f(*p); }

template <typename T>
__global__ void scatter_add_rows_kernel(const T* __restrict__ src, int64_t n, int D, const int64_t* __restrict__ idx,
                                        float* acc) {
  const int64_t total = n * D;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = c / D;
    const int d = (int)(c - i * D);
    atomicAdd(acc + idx[i] * D + d, ld_f(src + c));
  }
}

void scatter_add_rows(const float* src, int64_t n, int D, const int64_t* idx, float* acc, hipStream_t s) {
  if (n <= 0) return;
  const int block = 256;
  hipLaunchKernelGGL(scatter_add_rows_kernel<float>, grid_for(n * D, block), block, 0, s, src, n, D, idx, acc);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// bf16 gradient rows (the compressed push payload) accumulated into fp32
void scatter_add_rows_bf16(const bf16_t* src, int64_t n, int D, const int64_t* idx, float* acc, hipStream_t s) {
  if (n <= 0) return;
  const int block = 256;
  hipLaunchKernelGGL(scatter_add_rows_kernel<bf16_t>, grid_for(n * D, block), block, 0, s, src, n, D, idx, acc);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// --------------------------------------------------------------------------- row-wise adagrad
// Half a wave per row (two rows per wave-instruction) for rows of <= 64 values: every lane holds
// its <= 2 gradient values in registers (one read), the two mean(g^2) reductions are xor
// shuffles inside the 32-lane half. Wider rows take a whole wave and stride.
// Columns [0, D1) share accumulator state[row]; columns [D1, D) share state2[row] (Wide&Deep
// keeps the deep embedding and the wide weight in one row, each with its own Adagrad state).
__global__ void sparse_rowwise_adagrad_half_kernel(float* table, int64_t ld, float* state, float* state2, int D1,
                                                   const int64_t* __restrict__ keys, int64_t n, int64_t base, int D,
                                                   const float* __restrict__ grads, float lr, float eps,
                                                   const int64_t* n_dev) {
  n = dev_count(n, n_dev);
  const int lane = threadIdx.x & 63, half = lane >> 5, l = lane & 31;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i0 = wave * 2; i0 < n; i0 += nwaves * 2) {
    const int64_t i = i0 + half;
    const bool ok = i < n;
    float g0 = 0.f, g1 = 0.f;
    int64_t row = 0;
    if (ok) {
      row = keys[i] - base;
      if (l < D) g0 = grads[i * D + l];
      if (l + 32 < D) g1 = grads[i * D + l + 32];
    }
    float sq1 = (l < D1 ? g0 * g0 : 0.f) + (l + 32 < D1 ? g1 * g1 : 0.f);
    float sq2 = (l >= D1 && l < D ? g0 * g0 : 0.f) + (l + 32 >= D1 && l + 32 < D ? g1 * g1 : 0.f);
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      sq1 += __shfl_xor(sq1, o, 64);
      sq2 += __shfl_xor(sq2, o, 64);
    }
    if (!ok) continue;
    const float st1 = state[row] + sq1 / (float)D1;
    const float st2 = D1 < D ? state2[row] + sq2 / (float)(D - D1) : 0.f;
    if (l == 0) {
      state[row] = st1;
      if (D1 < D) state2[row] = st2;
    }
    const float s1 = lr / (sqrtf(st1) + eps), s2 = lr / (sqrtf(st2) + eps);
    float* tr = table + row * ld;
    if (l < D) tr[l] -= (l < D1 ? s1 : s2) * g0;
    if (l + 32 < D) tr[l + 32] -= (l + 32 < D1 ? s1 : s2) * g1;
  }
}

// Rows of 16 < D <= 64 floats with D % 4 == 0 (16-byte rows): 8 lanes per row, one float4 per
// lane for columns [0, 32) and a second float4 for [32, D) on the first (D - 32) / 4 lanes, so a
// wave keeps 8 rows' loads in flight at once (the 32-lane variant above is latency-bound: key ->
// row -> read-modify-write, two rows per wave).
__global__ __launch_bounds__(256) void sparse_rowwise_adagrad_v4_kernel(float* table, int64_t ld, float* state,
                                                                        float* state2, int D1,
                                                                        const int64_t* __restrict__ keys, int64_t n,
                                                                        int64_t base, int D,
                                                                        const float* __restrict__ grads, float lr,
                                                                        float eps, const int64_t* n_dev,
                                                                        float* __restrict__ zero_g) {
  n = dev_count(n, n_dev);
  const int lane = threadIdx.x & 63, sub = lane >> 3, l = lane & 7;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int c0 = 4 * l, c1 = 32 + 4 * l;
  const bool has0 = c0 < D, has1 = c1 < D;  // D % 4 == 0: a float4 is all in or all out
  for (int64_t i0 = wave * 8; i0 < n; i0 += nwaves * 8) {
    const int64_t i = i0 + sub;
    const bool ok = i < n;
    const int64_t row = ok ? keys[i] - base : 0;
    float4 g0 = make_float4(0.f, 0.f, 0.f, 0.f), g1 = g0, t0 = g0, t1 = g0;
    float* tr = table + row * ld;
    if (ok && has0) {
      g0 = *reinterpret_cast<const float4*>(grads + i * D + c0);
      t0 = *reinterpret_cast<const float4*>(tr + c0);
      if (has1) {
        g1 = *reinterpret_cast<const float4*>(grads + i * D + c1);
        t1 = *reinterpret_cast<const float4*>(tr + c1);
      }
      if (zero_g) {  // (grads == zero_g) the next push's accumulator, cleared after the read
        *reinterpret_cast<float4*>(zero_g + i * D + c0) = make_float4(0.f, 0.f, 0.f, 0.f);
        if (has1) *reinterpret_cast<float4*>(zero_g + i * D + c1) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    const float st_old1 = ok ? state[row] : 0.f;
    const float st_old2 = ok && D1 < D ? state2[row] : 0.f;
    float sq1 = 0.f, sq2 = 0.f;
    const float a[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = (q < 4 ? c0 : c1) + (q & 3);
      const float sq = a[q] * a[q];
      if (c < D1) sq1 += sq;
      else sq2 += sq;  // zero beyond D: g1 stays 0 when !has1
    }
#pragma unroll
    for (int o = 4; o > 0; o >>= 1) {
      sq1 += __shfl_xor(sq1, o, 64);
      sq2 += __shfl_xor(sq2, o, 64);
    }
    if (!ok) continue;
    const float st1 = st_old1 + sq1 / (float)D1;
    const float st2 = D1 < D ? st_old2 + sq2 / (float)(D - D1) : 0.f;
    if (l == 0) {
      state[row] = st1;
      if (D1 < D) state2[row] = st2;
    }
    const float s1 = lr / (sqrtf(st1) + eps), s2 = lr / (sqrtf(st2) + eps);
    float o[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = (q < 4 ? c0 : c1) + (q & 3);
      o[q] -= (c < D1 ? s1 : s2) * a[q];
    }
    if (has0) *reinterpret_cast<float4*>(tr + c0) = make_float4(o[0], o[1], o[2], o[3]);
    if (has1) *reinterpret_cast<float4*>(tr + c1) = make_float4(o[4], o[5], o[6], o[7]);
  }
}

__global__ void sparse_rowwise_adagrad_kernel(float* table, int64_t ld, float* state, float* state2, int D1,
                                              const int64_t* __restrict__ keys, int64_t n, int64_t base, int D,
                                              const float* __restrict__ grads, float lr, float eps,
                                              const int64_t* n_dev) {
  n = dev_count(n, n_dev);
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave; i < n; i += nwaves) {
    const int64_t row = keys[i] - base;
    float sq1 = 0.f, sq2 = 0.f;
    for (int d = lane; d < D; d += 64) {
      float g = grads[i * D + d];
      if (d < D1) sq1 += g * g; else sq2 += g * g;
    }
    sq1 = warp_sum(sq1);
    const float st1 = state[row] + sq1 / (float)D1;
    float st2 = 0.f;
    if (D1 < D) {
      sq2 = warp_sum(sq2);
      st2 = state2[row] + sq2 / (float)(D - D1);
    }
    if (lane == 0) {
      state[row] = st1;
      if (D1 < D) state2[row] = st2;
    }
    const float s1 = lr / (sqrtf(st1) + eps);
    const float s2 = lr / (sqrtf(st2) + eps);
    for (int d = lane; d < D; d += 64) table[row * ld + d] -= (d < D1 ? s1 : s2) * grads[i * D + d];
  }
}

void sparse_rowwise_adagrad(float* table, int64_t ld, float* state, float* state2, int D1, const int64_t* keys,
                            int64_t n, int64_t base, int D, const float* grads, float lr, float eps, hipStream_t s,
                            const int64_t* n_dev, bool zero_g) {
  if (n <= 0) return;
  if (D1 <= 0 || D1 > D) D1 = D;
  if (D1 < D && !state2) throw std::runtime_error("sparse_rowwise_adagrad: split rows need state2");
  const int block = 256;
  const bool vec4 = D > 16 && D <= 64 && D % 4 == 0 && ld % 4 == 0 && reinterpret_cast<uintptr_t>(table) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(grads) % 16 == 0;
  if (vec4) {
    hipLaunchKernelGGL(sparse_rowwise_adagrad_v4_kernel, grid_for(n * 8, block, 16384), block, 0, s, table, ld, state,
                       state2, D1, keys, n, base, D, grads, lr, eps, n_dev,
                       zero_g ? const_cast<float*>(grads) : nullptr);
    zero_g = false;
  } else if (D <= 64) {
    hipLaunchKernelGGL(sparse_rowwise_adagrad_half_kernel, grid_for(n * 32, block, 8192), block, 0, s, table, ld,
                       state, state2, D1, keys, n, base, D, grads, lr, eps, n_dev);
  } else {
    hipLaunchKernelGGL(sparse_rowwise_adagrad_kernel, grid_for(n * 64, block, 4096), block, 0, s, table, ld, state,
                       state2, D1, keys, n, base, D, grads, lr, eps, n_dev);
  }
  // the other forms clear the gradient rows with a fill after the apply
  if (zero_g) MINIPS_HIP_CHECK(hipMemsetAsync(const_cast<float*>(grads), 0, sizeof(float) * (size_t)n * D, s));
  MINIPS_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------ owner side of a multi-rank push
// At N > 1 each owner receives one deduplicated gradient row per (requester, key) -- a key is
// pushed by at most P requesters -- and the owner-side dedupe (bitmap / hash planner) gives each
// received row its owned unique index own_inv[i]. owner_slots records, per owned unique row u,
// the received row of every requester s (slots[u * P + s], -1 = none); owner_rows_adagrad then
// sums each row's <= P contributions in requester order and applies the row-wise Adagrad in the
// same pass: no zeroed accumulator, no float atomics (the sum has one fixed order: deterministic),
// no second read of a gradient buffer. Rows are balanced by construction (<= P members each).
__global__ void owner_slots_kernel(const int64_t* __restrict__ own_inv, int64_t M, OwnerSegs segs, int P,
                                   int* __restrict__ slots) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
    int seg = 0;
    while (seg + 1 < P && i >= segs.off[seg + 1]) ++seg;
    slots[own_inv[i] * P + seg] = (int)i;
  }
}

void owner_slots(const int64_t* own_inv, int64_t M, const OwnerSegs& segs, int P, int* slots, int64_t cap,
                 hipStream_t s) {
  if (P < 1 || P > kOwnerMaxP) throw std::runtime_error("owner_slots: 1..16 requesters");
  MINIPS_HIP_CHECK(hipMemsetAsync(slots, 0xff, sizeof(int) * (size_t)cap * P, s));
  if (M <= 0) return;
  hipLaunchKernelGGL(owner_slots_kernel, grid_for(M, 256, 4096), 256, 0, s, own_inv, M, segs, P, slots);
  MINIPS_HIP_CHECK(hipGetLastError());
}

__device__ __forceinline__ float4 ld_row4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 ld_row4(const bf16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}

// 8 lanes per owned row (the v4 Adagrad layout: a float4 of columns [0, 32), a second of [32, D)
// on the first (D - 32) / 4 lanes); lane l holds slot l (and l + 8) of the row.
template <typename TG>
__global__ __launch_bounds__(256) void owner_rows_adagrad_kernel(float* table, int64_t ld, float* state,
                                                                 float* state2, int D1,
                                                                 const int64_t* __restrict__ keys, int64_t n,
                                                                 const int64_t* n_dev, int64_t base, int D,
                                                                 const TG* __restrict__ recv, int P,
                                                                 const int* __restrict__ slots, float lr, float eps) {
  n = dev_count(n, n_dev);
  const int lane = threadIdx.x & 63, sub = lane >> 3, l = lane & 7;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int c0 = 4 * l, c1 = 32 + 4 * l;
  const bool has0 = c0 < D, has1 = c1 < D;
  for (int64_t i0 = wave * 8; i0 < n; i0 += nwaves * 8) {
    const int64_t i = i0 + sub;
    const bool ok = i < n;
    const int64_t row = ok ? keys[i] - base : 0;
    const int sl0 = ok && l < P ? slots[i * P + l] : -1;
    const int sl1 = ok && l + 8 < P ? slots[i * P + l + 8] : -1;
    float* tr = table + row * ld;
    float4 t0 = make_float4(0.f, 0.f, 0.f, 0.f), t1 = t0, g0 = t0, g1 = t0;
    if (ok && has0) {
      t0 = *reinterpret_cast<const float4*>(tr + c0);
      if (has1) t1 = *reinterpret_cast<const float4*>(tr + c1);
    }
    const float st_old1 = ok ? state[row] : 0.f;
    const float st_old2 = ok && D1 < D ? state2[row] : 0.f;
#pragma unroll
    for (int s = 0; s < kOwnerMaxP; ++s) {
      if (s >= P) break;
      const int m = __shfl(s < 8 ? sl0 : sl1, (sub << 3) + (s & 7), 64);
      if (m >= 0 && has0) {
        const float4 v = ld_row4(recv + (int64_t)m * D + c0);
        g0.x += v.x; g0.y += v.y; g0.z += v.z; g0.w += v.w;
        if (has1) {
          const float4 w = ld_row4(recv + (int64_t)m * D + c1);
          g1.x += w.x; g1.y += w.y; g1.z += w.z; g1.w += w.w;
        }
      }
    }
    float sq1 = 0.f, sq2 = 0.f;
    const float a[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = (q < 4 ? c0 : c1) + (q & 3);
      const float sq = a[q] * a[q];
      if (c < D1) sq1 += sq;
      else sq2 += sq;
    }
#pragma unroll
    for (int o = 4; o > 0; o >>= 1) {
      sq1 += __shfl_xor(sq1, o, 64);
      sq2 += __shfl_xor(sq2, o, 64);
    }
    if (!ok) continue;
    const float st1 = st_old1 + sq1 / (float)D1;
    const float st2 = D1 < D ? st_old2 + sq2 / (float)(D - D1) : 0.f;
    if (l == 0) {
      state[row] = st1;
      if (D1 < D) state2[row] = st2;
    }
    const float s1 = lr / (sqrtf(st1) + eps), s2 = lr / (sqrtf(st2) + eps);
    float o[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = (q < 4 ? c0 : c1) + (q & 3);
      o[q] -= (c < D1 ? s1 : s2) * a[q];
    }
    if (has0) *reinterpret_cast<float4*>(tr + c0) = make_float4(o[0], o[1], o[2], o[3]);
    if (has1) *reinterpret_cast<float4*>(tr + c1) = make_float4(o[4], o[5], o[6], o[7]);
  }
}

void owner_rows_adagrad(float* table, int64_t ld, float* state, float* state2, int D1, const int64_t* keys, int64_t n,
                        const int64_t* n_dev, int64_t base, int D, const void* recv, bool recv_bf16, int P,
                        const int* slots, float lr, float eps, hipStream_t s) {
  if (n <= 0) return;
  if (D1 <= 0 || D1 > D) D1 = D;
  if (D1 < D && !state2) throw std::runtime_error("owner_rows_adagrad: split rows need state2");
  if (!(D > 16 && D <= 64 && D % 4 == 0 && ld % 4 == 0 && P >= 1 && P <= kOwnerMaxP))
    throw std::runtime_error("owner_rows_adagrad: rows of 16 < D <= 64 (D % 4 == 0), 1..16 requesters");
  const int block = 256;
  if (recv_bf16)
    hipLaunchKernelGGL(owner_rows_adagrad_kernel<bf16_t>, grid_for(n * 8, block, 16384), block, 0, s, table, ld, state,
                       state2, D1, keys, n, n_dev, base, D, static_cast<const bf16_t*>(recv), P, slots, lr, eps);
  else
    hipLaunchKernelGGL(owner_rows_adagrad_kernel<float>, grid_for(n * 8, block, 16384), block, 0, s, table, ld, state,
                       state2, D1, keys, n, n_dev, base, D, static_cast<const float*>(recv), P, slots, lr, eps);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// Direct-addressed owner apply (no owner-side dedupe): a persistent table rs[row * P + s] =
// {stamp, received row} per owned row and requester. owner_mark stamps the received keys of this
// push (each requester sends a key at most once: one writer per entry, no atomics); owner_apply
// takes 8 lanes per RECEIVED row, and the group whose requester is the lowest one that sent the
// row (the leader) sums the row's <= P contributions in requester order and applies the row-wise
// Adagrad -- the same arithmetic, in the same order, as owner_rows_adagrad over a deduplicated
// plan, without the bitmap planner, the slot scatter and their host calls. The stamp (the push
// number) retires the previous pushes' entries without clearing the table.
__device__ __forceinline__ int owner_seg(int64_t i, const OwnerSegs& segs, int P) {
  int seg = 0;
  while (seg + 1 < P && i >= segs.off[seg + 1]) ++seg;
  return seg;
}

__global__ void owner_mark_kernel(const int64_t* __restrict__ keys, int64_t M, int64_t base, OwnerSegs segs, int P,
                                  int2* __restrict__ rs, int stamp) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x)
    rs[(keys[i] - base) * P + owner_seg(i, segs, P)] = make_int2(stamp, (int)i);
}

template <typename TG>
__global__ __launch_bounds__(256) void owner_apply_kernel(float* table, int64_t ld, float* state, float* state2,
                                                          int D1, const int64_t* __restrict__ keys, int64_t M,
                                                          int64_t base, int D, const TG* __restrict__ recv,
                                                          OwnerSegs segs, int P, const int2* __restrict__ rs,
                                                          int stamp, float lr, float eps) {
  const int lane = threadIdx.x & 63, sub = lane >> 3, l = lane & 7;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int c0 = 4 * l, c1 = 32 + 4 * l;
  const bool has0 = c0 < D, has1 = c1 < D;
  for (int64_t i0 = wave * 8; i0 < M; i0 += nwaves * 8) {
    const int64_t i = i0 + sub;
    const bool in = i < M;
    const int me = in ? owner_seg(i, segs, P) : 0;
    const int64_t row = in ? keys[i] - base : 0;
    // everything that depends on the row alone is loaded together (one round trip after the key):
    // the stamp entries, the table row and its state -- the leader test then costs no extra trip
    const int2* e = rs + row * P;
    const int2 e0 = in && l < P ? e[l] : make_int2(-1, -1);
    const int2 e1 = in && l + 8 < P ? e[l + 8] : make_int2(-1, -1);
    float* tr = table + row * ld;
    float4 t0 = make_float4(0.f, 0.f, 0.f, 0.f), t1 = t0, g0 = t0, g1 = t0;
    if (in && has0) {
      t0 = *reinterpret_cast<const float4*>(tr + c0);
      if (has1) t1 = *reinterpret_cast<const float4*>(tr + c1);
    }
    const float st_old1 = in ? state[row] : 0.f;
    const float st_old2 = in && D1 < D ? state2[row] : 0.f;
    const int sl0 = e0.x == stamp ? e0.y : -1, sl1 = e1.x == stamp ? e1.y : -1;
    // the leader: no lower requester sent this row in this push
    const unsigned long long lower = __ballot(sl0 >= 0 && l < me) | __ballot(sl1 >= 0 && l + 8 < me);
    const bool ok = in && ((lower >> (sub << 3)) & 0xffull) == 0;
#pragma unroll
    for (int s = 0; s < kOwnerMaxP; ++s) {
      if (s >= P) break;
      const int m = __shfl(s < 8 ? sl0 : sl1, (sub << 3) + (s & 7), 64);
      if (ok && m >= 0 && has0) {
        const float4 v = ld_row4(recv + (int64_t)m * D + c0);
        g0.x += v.x; g0.y += v.y; g0.z += v.z; g0.w += v.w;
        if (has1) {
          const float4 w = ld_row4(recv + (int64_t)m * D + c1);
          g1.x += w.x; g1.y += w.y; g1.z += w.z; g1.w += w.w;
        }
      }
    }
    float sq1 = 0.f, sq2 = 0.f;
    const float a[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = (q < 4 ? c0 : c1) + (q & 3);
      const float sq = a[q] * a[q];
      if (c < D1) sq1 += sq;
      else sq2 += sq;
    }
#pragma unroll
    for (int o = 4; o > 0; o >>= 1) {
      sq1 += __shfl_xor(sq1, o, 64);
      sq2 += __shfl_xor(sq2, o, 64);
    }
    if (!ok) continue;
    const float st1 = st_old1 + sq1 / (float)D1;
    const float st2 = D1 < D ? st_old2 + sq2 / (float)(D - D1) : 0.f;
    if (l == 0) {
      state[row] = st1;
      if (D1 < D) state2[row] = st2;
    }
    const float s1 = lr / (sqrtf(st1) + eps), s2 = lr / (sqrtf(st2) + eps);
    float o[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = (q < 4 ? c0 : c1) + (q & 3);
      o[q] -= (c < D1 ? s1 : s2) * a[q];
    }
    if (has0) *reinterpret_cast<float4*>(tr + c0) = make_float4(o[0], o[1], o[2], o[3]);
    if (has1) *reinterpret_cast<float4*>(tr + c1) = make_float4(o[4], o[5], o[6], o[7]);
  }
}

void owner_push_adagrad(float* table, int64_t ld, float* state, float* state2, int D1, const int64_t* keys, int64_t M,
                        int64_t base, int64_t rows_local, int D, const void* recv, bool recv_bf16,
                        const OwnerSegs& segs, int P, void* rs, int stamp, float lr, float eps, hipStream_t s) {
  if (M <= 0) return;
  if (D1 <= 0 || D1 > D) D1 = D;
  if (D1 < D && !state2) throw std::runtime_error("owner_push_adagrad: split rows need state2");
  if (!(D > 16 && D <= 64 && D % 4 == 0 && ld % 4 == 0 && P >= 1 && P <= kOwnerMaxP && stamp >= 0))
    throw std::runtime_error("owner_push_adagrad: rows of 16 < D <= 64 (D % 4 == 0), 1..16 requesters");
  (void)rows_local;
  int2* e = static_cast<int2*>(rs);
  hipLaunchKernelGGL(owner_mark_kernel, grid_for(M, 256, 4096), 256, 0, s, keys, M, base, segs, P, e, stamp);
  MINIPS_HIP_CHECK(hipGetLastError());
  const int block = 256;
  if (recv_bf16)
    hipLaunchKernelGGL(owner_apply_kernel<bf16_t>, grid_for(M * 8, block, 16384), block, 0, s, table, ld, state,
                       state2, D1, keys, M, base, D, static_cast<const bf16_t*>(recv), segs, P, e, stamp, lr, eps);
  else
    hipLaunchKernelGGL(owner_apply_kernel<float>, grid_for(M * 8, block, 16384), block, 0, s, table, ld, state,
                       state2, D1, keys, M, base, D, static_cast<const float*>(recv), segs, P, e, stamp, lr, eps);
  MINIPS_HIP_CHECK(hipGetLastError());
}

__global__ void sparse_sgd_kernel(float* table, int64_t ld, const int64_t* __restrict__ keys, int64_t n, int64_t base,
                                  int D, const float* __restrict__ grads, float scale, const int64_t* n_dev) {
  const int64_t total = dev_count(n, n_dev) * D;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = c / D;
    const int d = (int)(c - i * D);
    table[(keys[i] - base) * ld + d] += scale * grads[c];
  }
}

void sparse_sgd(float* table, int64_t ld, const int64_t* keys, int64_t n, int64_t base, int D, const float* grads,
                float scale, hipStream_t s, const int64_t* n_dev) {
  if (n <= 0) return;
  const int block = 256;
  hipLaunchKernelGGL(sparse_sgd_kernel, grid_for(n * D, block), block, 0, s, table, ld, keys, n, base, D,
                     grads, scale, n_dev);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// --------------------------------------------------------------------------- embedding bag
__global__ void embedding_bag_fwd_kernel(const float* __restrict__ rows, const int64_t* __restrict__ idx,
                                         const int64_t* __restrict__ offsets, int64_t B, int D, bool mean,
                                         float* out) {
  const int64_t total = B * D;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = c / D;
    const int d = (int)(c - b * D);
    const int64_t s0 = offsets[b], s1 = offsets[b + 1];
    float acc = 0.f;
    for (int64_t j = s0; j < s1; ++j) acc += rows[idx[j] * D + d];
    if (mean && s1 > s0) acc /= (float)(s1 - s0);
    out[c] = acc;
  }
}

__global__ void embedding_bag_bwd_kernel(const float* __restrict__ grad_out, const int64_t* __restrict__ idx,
                                         const int64_t* __restrict__ offsets, int64_t B, int D, bool mean,
                                         float* grad_rows) {
  const int64_t total = B * D;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = c / D;
    const int d = (int)(c - b * D);
    const int64_t s0 = offsets[b], s1 = offsets[b + 1];
    float g = grad_out[c];
    if (mean && s1 > s0) g /= (float)(s1 - s0);
    for (int64_t j = s0; j < s1; ++j) atomicAdd(grad_rows + idx[j] * D + d, g);
  }
}

void embedding_bag_fwd(const float* rows, const int64_t* idx, const int64_t* offsets, int64_t B, int D, bool mean,
                       float* out, hipStream_t s) {
  if (B <= 0) return;
  const int block = 256;
  hipLaunchKernelGGL(embedding_bag_fwd_kernel, grid_for(B * D, block), block, 0, s, rows, idx, offsets, B, D, mean,
                     out);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void embedding_bag_bwd(const float* grad_out, const int64_t* idx, const int64_t* offsets, int64_t B, int D, bool mean,
                       float* grad_rows, hipStream_t s) {
  if (B <= 0) return;
  const int block = 256;
  hipLaunchKernelGGL(embedding_bag_bwd_kernel, grid_for(B * D, block), block, 0, s, grad_out, idx, offsets, B, D,
                     mean, grad_rows);
  MINIPS_HIP_CHECK(hipGetLastError());
}

}  // namespace minips_k

namespace minips_k {

// out[b, f*D : (f+1)*D] = rows[inv[b*F+f], 0:D] (bf16, 16-byte chunks; D % 8 == 0).
__global__ void lookup_rows_kernel(const bf16_t* __restrict__ rows, int row_stride, const int64_t* __restrict__ inv,
                                   int64_t B, int F, int D, bf16_t* __restrict__ out, int ldo) {
  const int chunks = D >> 3;
  const int64_t total = B * F * chunks;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t bf = c / chunks;
    const int ch = (int)(c - bf * chunks);
    const int64_t b = bf / F;
    const int f = (int)(bf - b * F);
    const bf16_t* src = rows + inv[bf] * row_stride + ch * 8;
    const uint2 lo = *reinterpret_cast<const uint2*>(src), hi = *reinterpret_cast<const uint2*>(src + 4);
    *reinterpret_cast<uint4*>(out + b * ldo + f * D + ch * 8) = make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
}

void lookup_rows(const bf16_t* rows, int row_stride, const int64_t* inv, int64_t B, int F, int D, bf16_t* out, int ldo,
                 hipStream_t s) {
  if (D % 8 || row_stride % 4 || ldo % 8) throw std::runtime_error("lookup_rows: D%8, row_stride%4, ldo%8 required");
  if (B <= 0) return;
  hipLaunchKernelGGL(lookup_rows_kernel, grid_for(B * F * (D / 8), 256, 8192), 256, 0, s, rows, row_stride, inv, B, F,
                     D, out, ldo);
  MINIPS_HIP_CHECK(hipGetLastError());
}

}  // namespace minips_k
