// Sort-based key planning of a [B, F] lookup batch whose F columns hold disjoint key ranges
// (Wide&Deep / DLRM: feature f's ids live in [base_f, base_f + card_f)).
//
// The hash dedupe (sparse.hip, unique_bucketize) resolves duplicates across workgroups with
// device-scope atomics (CAS probes, per-key counts, shard cursors). Those execute at the memory
// side on the multi-XCD part and slow every concurrently running kernel: the W&D step measured
// 0.450 ms with per-step planning vs 0.360 ms stepping through pre-planned batches
// (tools/step_probe.py ablation) even with the planning stream confined to 16 CUs. This planner uses
// no atomics at all:
//
//   plan_sort_col  one 1024-thread workgroup per column: the column's <= 16384 (key - base_f, b)
//                  pairs sit in registers (16 per thread) and are LSD radix-sorted in LDS, 4 bits
//                  per pass (ceil(col_bits[f] / 4) passes): per-thread packed 8-bit digit counters ->
//                  [digit][thread] LDS histogram -> block exclusive scan -> stable scatter ->
//                  reload. Run heads of the sorted keys give the column's unique keys in ascending
//                  order and each lookup's column-local unique index.
//   plan_emit      global unique index u = (sum of the unique counts of columns < f) + local:
//                  uniq[u] (routed key), inv[b*F + f] = u, and the embedding backward's CSR for
//                  free -- members (lookup ids grouped by u, ascending) and memrow (their u).
//
// Deterministic (no global atomics, stable sort); unique keys come out column-major, ascending
// inside a column. With several owners (P > 1, a multi-rank table) the sort key carries the
// owner shard of the routed key above the column-relative key (plan_transpose computes it), so
// each column's unique keys come out grouped by owner; plan_sort_col counts them per owner and
// plan_emit places unique (column c, owner p, k-th) at
//   (keys of owners < p) + (owner p's keys in columns < c) + k
// -- grouped by owner, column-major inside an owner -- with no separate regrouping pass.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace minips_k {

constexpr int kPsThreads = 1024, kPsItems = 16, kPsMax = kPsThreads * kPsItems;

// Exclusive scan of one value per thread over a 1024-thread block; *total = the sum. ws: >= 17
// uint32 of LDS; ends with a barrier (ws reusable).
__device__ __forceinline__ uint32_t ps_block_scan(uint32_t v, uint32_t* ws, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) ws[wave] = x;
  __syncthreads();
  if (wave == 0) {
    const uint32_t w = lane < 16 ? ws[lane] : 0u;
    uint32_t s = w;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const uint32_t y = __shfl_up(s, o, 64);
      if (lane >= o) s += y;
    }
    if (lane < 16) ws[lane] = s - w;
    if (lane == 15) ws[16] = s;
  }
  __syncthreads();
  const uint32_t res = ws[wave] + x - v;
  *total = ws[16];
  __syncthreads();
  return res;
}

__device__ __forceinline__ uint32_t ps_count(uint64_t lo, uint64_t hi, int d) {
  return (uint32_t)((d < 8 ? (lo >> (8 * d)) : (hi >> (8 * (d - 8)))) & 0xffu);
}

// [B, F] int64 keys -> column-major [F, B] uint32 (key - base_f) through a 64 x F LDS tile: the
// sort reads its column as contiguous 16-byte vectors instead of one 8-byte key per 208-byte row
// (that strided column gather pulled the whole batch through each sorting CU: ~70 us fixed cost).
// P > 1: the owner shard of the routed key goes above bit col_bits[f] (the sort then groups by it).
__device__ __forceinline__ int64_t ps_route(int64_t key, uint64_t mult, uint64_t rn);
__device__ __forceinline__ int ps_owner(const int64_t* bounds, int P, int64_t k);

__global__ __launch_bounds__(256) void plan_transpose_kernel(const int64_t* __restrict__ keys, int B, int F,
                                                             const int64_t* __restrict__ col_base,
                                                             const int32_t* __restrict__ col_bits,
                                                             const int64_t* __restrict__ bounds, int P,
                                                             uint64_t rmult, uint64_t rn,
                                                             uint32_t* __restrict__ krel) {
  __shared__ uint32_t tile[64][65];
  __shared__ int64_t basef[64];
  __shared__ int bitsf[64];
  __shared__ int64_t sb[17];
  const int t = threadIdx.x;
  if (t < F) {
    basef[t] = col_base[t];
    bitsf[t] = col_bits[t];
  }
  if (t <= P && P > 1) sb[t] = bounds[t];
  const int b0 = blockIdx.x * 64;
  __syncthreads();
  for (int e = t; e < 64 * F; e += 256) {  // coalesced row-major reads
    const int r = e / F, c = e - r * F;
    const int b = b0 + r;
    if (b < B) {
      const int64_t key = keys[(int64_t)b * F + c];
      uint32_t v = (uint32_t)(key - basef[c]);
      if (P > 1) v |= (uint32_t)ps_owner(sb, P, ps_route(key, rmult, rn)) << bitsf[c];
      tile[c][r] = v;
    }
  }
  __syncthreads();
  for (int e = t; e < 64 * F; e += 256) {  // coalesced column-major writes
    const int c = e >> 6, r = e & 63;
    const int b = b0 + r;
    if (b < B) krel[(int64_t)c * B + b] = tile[c][r];
  }
}

__global__ __launch_bounds__(kPsThreads) void plan_sort_col_kernel(const uint32_t* __restrict__ krel, int B,
                                                                   const int64_t* __restrict__ col_base,
                                                                   const int32_t* __restrict__ col_bits,
                                                                   int obits, int P,
                                                                   int32_t* __restrict__ sorted_b,
                                                                   int32_t* __restrict__ local_u,
                                                                   int64_t* __restrict__ ukey,
                                                                   int32_t* __restrict__ ucount,
                                                                   int32_t* __restrict__ ocnt) {
  __shared__ __attribute__((aligned(16))) uint16_t cnt[16 * kPsThreads];  // [digit][thread] counts -> offsets
  __shared__ __attribute__((aligned(16))) uint32_t skey[kPsMax];
  __shared__ __attribute__((aligned(16))) uint16_t sval[kPsMax];
  __shared__ uint32_t ws[20];
  __shared__ uint32_t lc[16];  // unique keys per owner (P > 1)
  const int t = threadIdx.x, f = blockIdx.x;
  const int64_t base = col_base[f];
  const int kbits = col_bits[f];
  const int nbits = kbits + obits;  // a small-cardinality column sorts in fewer passes
  const uint32_t kmask = kbits >= 32 ? 0xffffffffu : ((1u << kbits) - 1u);
  if (t < 16) lc[t] = 0;
  uint32_t k[kPsItems];
  uint32_t v[kPsItems];
  const uint32_t* col = krel + (int64_t)f * B;
  if ((B & 3) == 0 && (reinterpret_cast<uintptr_t>(krel) & 15) == 0 && t * kPsItems + kPsItems <= B) {
    // 4 x 16-byte loads of this thread's 16 keys
    const uint4* p = reinterpret_cast<const uint4*>(col + t * kPsItems);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint4 u = p[e];
      k[4 * e] = u.x;
      k[4 * e + 1] = u.y;
      k[4 * e + 2] = u.z;
      k[4 * e + 3] = u.w;
    }
  } else {
#pragma unroll
    for (int q = 0; q < kPsItems; ++q) {
      const int i = t * kPsItems + q;
      // padding items (i >= B) get the largest key: with the stable sort they land behind every
      // real item even when a real key ties with their truncated value
      k[q] = i < B ? col[i] : 0xffffffffu;
    }
  }
#pragma unroll
  for (int q = 0; q < kPsItems; ++q) v[q] = (uint32_t)(t * kPsItems + q);
  for (int shift = 0; shift < nbits; shift += 4) {
    uint64_t lo = 0, hi = 0;
#pragma unroll
    for (int q = 0; q < kPsItems; ++q) {
      const int d = (int)((k[q] >> shift) & 15u);
      if (d < 8) lo += 1ull << (8 * d);
      else hi += 1ull << (8 * (d - 8));
    }
#pragma unroll
    for (int d = 0; d < 16; ++d) cnt[d * kPsThreads + t] = (uint16_t)ps_count(lo, hi, d);
    __syncthreads();
    // exclusive scan in [digit][thread] order: thread t owns entries [16t, 16t + 16), read and
    // written as two 16-byte vectors (scalar 2-byte accesses at a 32-byte lane stride conflict)
    uint4* cv = reinterpret_cast<uint4*>(cnt) + 2 * t;
    const uint4 c0 = cv[0], c1 = cv[1];
    const uint32_t w[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    uint32_t o[8];
    uint32_t s = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint32_t a = w[e] & 0xffffu, b = w[e] >> 16;
      o[e] = s | ((s + a) << 16);
      s += a + b;
    }
    uint32_t tot;
    const uint32_t pre = ps_block_scan(s, ws, &tot);
    const uint32_t pre2 = pre | (pre << 16);  // offsets < 2^14 + 2^14: the halves never carry
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] += pre2;
    cv[0] = make_uint4(o[0], o[1], o[2], o[3]);
    cv[1] = make_uint4(o[4], o[5], o[6], o[7]);
    __syncthreads();
    uint64_t slo = 0, shi = 0;
#pragma unroll
    for (int q = 0; q < kPsItems; ++q) {
      const int d = (int)((k[q] >> shift) & 15u);
      const uint32_t r = ps_count(slo, shi, d);
      if (d < 8) slo += 1ull << (8 * d);
      else shi += 1ull << (8 * (d - 8));
      const uint32_t pos = (uint32_t)cnt[d * kPsThreads + t] + r;
      skey[pos] = k[q];
      sval[pos] = (uint16_t)v[q];
    }
    __syncthreads();
    {  // reload this thread's 16 consecutive items as 16-byte vectors (a scalar reload at a 64-byte
       // lane stride is a 16-way bank conflict per item)
      const uint4* kp = reinterpret_cast<const uint4*>(skey + t * kPsItems);
      const uint4* vp = reinterpret_cast<const uint4*>(sval + t * kPsItems);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint4 u = kp[e];
        k[4 * e] = u.x;
        k[4 * e + 1] = u.y;
        k[4 * e + 2] = u.z;
        k[4 * e + 3] = u.w;
      }
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const uint4 u = vp[e];
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          v[8 * e + 2 * h] = w[h] & 0xffffu;
          v[8 * e + 2 * h + 1] = w[h] >> 16;
        }
      }
    }
    __syncthreads();
  }
  // run heads of the sorted keys (skey still holds them: nbits >= 1 ran at least one pass)
  uint32_t heads = 0;
#pragma unroll
  for (int q = 0; q < kPsItems; ++q) {
    const int pos = t * kPsItems + q;
    const bool h = pos < B && (pos == 0 || k[q] != skey[pos - 1]);
    heads += h ? 1u : 0u;
  }
  uint32_t total;
  uint32_t run = ps_block_scan(heads, ws, &total);
  const int64_t col0 = (int64_t)f * B;
#pragma unroll
  for (int q = 0; q < kPsItems; ++q) {
    const int pos = t * kPsItems + q;
    if (pos >= B) break;
    const bool h = pos == 0 || k[q] != skey[pos - 1];
    if (h) ++run;
    const uint32_t lu = run - 1;
    sorted_b[col0 + pos] = (int32_t)v[q];
    local_u[col0 + pos] = (int32_t)lu;
    if (h) {
      ukey[col0 + lu] = base + (int64_t)(k[q] & kmask);
      if (P > 1) atomicAdd(&lc[k[q] >> kbits], 1u);  // (LDS: the owner bits above the key)
    }
  }
  if (t == 0) ucount[f] = (int32_t)total;
  if (P > 1) {
    __syncthreads();
    if (t < P) ocnt[f * P + t] = (int32_t)lc[t];
  }
}

// (key * mult) mod rn. The 64-bit integer remainder is a long software routine on the GPU; for the
// tables' sizes (product < 2^62, rn >= 2^20) a double-precision quotient is off by at most one
// (relative error <= 2^-52 of a quotient < 2^42), fixed by one correction step each way: exact.
__device__ __forceinline__ int64_t ps_route(int64_t key, uint64_t mult, uint64_t rn) {
  if (!mult) return key;
  const uint64_t prod = (uint64_t)key * mult;
  if (prod < (1ull << 62) && rn >= (1ull << 20)) {
    const int64_t q = (int64_t)((double)prod / (double)rn);
    int64_t r = (int64_t)prod - q * (int64_t)rn;
    if (r < 0) r += (int64_t)rn;
    if (r >= (int64_t)rn) r -= (int64_t)rn;
    return r;
  }
  return (int64_t)(prod % rn);
}

// column prefix of the unique counts (F <= 64), computed per block; returns U
__device__ __forceinline__ int64_t ps_col_prefix(const int32_t* __restrict__ ucount, int F, int64_t* basef,
                                                 int32_t* ucf) {
  const int t = threadIdx.x;
  if (t < F) ucf[t] = ucount[t];
  __syncthreads();
  if (t == 0) {
    int64_t acc = 0;
    for (int c = 0; c < F; ++c) {
      basef[c] = acc;
      acc += ucf[c];
    }
    basef[F] = acc;
  }
  __syncthreads();
  return basef[F];
}

__device__ __forceinline__ int ps_owner(const int64_t* bounds, int P, int64_t k) {
  int lo = 0, hi = P;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (bounds[mid] <= k) lo = mid;
    else hi = mid;
  }
  return lo;
}

// routed key of global unique index u (column-major: column c holds [basef[c], basef[c+1]))
__device__ __forceinline__ int64_t ps_ukey_routed(int64_t u, int F, int B, const int64_t* basef,
                                                  const int64_t* __restrict__ ukey, uint64_t rmult, uint64_t rn) {
  int lo = 0, hi = F;  // basef[lo] <= u < basef[hi] (binary search: F = 26 in W&D)
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (basef[mid] <= u) lo = mid;
    else hi = mid;
  }
  return ps_route(ukey[(int64_t)lo * B + (u - basef[lo])], rmult, rn);
}

constexpr int kPoMaxP = 16;

// P > 1: per block, from the per-column per-owner unique counts ocnt[F][P]: the owner offsets
// obase[p], the column prefixes colpre[c][p] (owner p's keys in columns < c) and the column-local
// starts cstart[c][p] (the column's keys of owners < p)
struct PoLayout {
  int64_t obase[kPoMaxP + 1];
  int32_t colpre[64][kPoMaxP];
  int32_t cstart[64][kPoMaxP + 1];
};

__device__ void po_layout(const int32_t* __restrict__ ocnt, int F, int P, PoLayout* L) {
  const int t = threadIdx.x;
  if (t < P) {  // one owner per thread: prefix over the columns
    int32_t acc = 0;
    for (int c = 0; c < F; ++c) {
      L->colpre[c][t] = acc;
      acc += ocnt[c * P + t];
    }
    L->obase[t + 1] = acc;  // (owner t's total, prefixed below)
  }
  if (t >= 64 && t < 64 + F) {  // one column per thread: prefix over the owners
    const int c = t - 64;
    int32_t acc = 0;
    for (int p = 0; p < P; ++p) {
      L->cstart[c][p] = acc;
      acc += ocnt[c * P + p];
    }
    L->cstart[c][P] = acc;
  }
  __syncthreads();
  if (t == 0) {
    L->obase[0] = 0;
    for (int p = 0; p < P; ++p) L->obase[p + 1] += L->obase[p];
  }
  __syncthreads();
}

// global position of column c's local unique index lu (P > 1)
__device__ __forceinline__ int64_t po_place(const PoLayout* L, int c, int P, int32_t lu) {
  int p = 0;
  while (p + 1 < P && L->cstart[c][p + 1] <= lu) ++p;
  return L->obase[p] + L->colpre[c][p] + (lu - L->cstart[c][p]);
}

__global__ __launch_bounds__(256) void plan_emit_kernel(int B, int F, const int32_t* __restrict__ sorted_b,
                                                        const int32_t* __restrict__ local_u,
                                                        const int64_t* __restrict__ ukey,
                                                        const int32_t* __restrict__ ucount, uint64_t rmult,
                                                        uint64_t rn, int P, const int32_t* __restrict__ ocnt,
                                                        int64_t* __restrict__ uniq, int64_t* __restrict__ inv,
                                                        int32_t* __restrict__ members, int32_t* __restrict__ memrow,
                                                        int64_t* __restrict__ counts, int32_t* __restrict__ pos_out,
                                                        int32_t* __restrict__ rowstart,
                                                        int32_t* __restrict__ rowidx) {
  __shared__ int64_t basef[65];
  __shared__ int32_t ucf[64];
  __shared__ PoLayout L;
  const int t = threadIdx.x;
  const int64_t U = ps_col_prefix(ucount, F, basef, ucf);
  if (P > 1) po_layout(ocnt, F, P, &L);
  if (blockIdx.x == 0 && t <= P) {
    if (P == 1) counts[t] = U;  // counts[0] = U, counts[1] = the device-side U
    else counts[t] = t < P ? L.obase[t + 1] - L.obase[t] : U;
  }
  const int64_t n = (int64_t)B * F;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + t; idx < n; idx += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(idx / B);
    const int pos = (int)(idx - (int64_t)c * B);
    const int32_t lu = local_u[idx];
    const int64_t u = P > 1 ? po_place(&L, c, P, lu) : basef[c] + lu;
    const int64_t j = (int64_t)sorted_b[idx] * F + c;
    inv[j] = u;
    members[idx] = (int32_t)j;
    memrow[idx] = (int32_t)u;
    if (pos_out) pos_out[j] = (int32_t)idx;  // the member-order row of lookup j (sorted dgrad rows)
    if (rowstart) {  // one owner: u's lookups are members [rowstart[u], rowstart[u + 1])
      if (pos == 0 || local_u[idx - 1] != lu) rowstart[u] = (int32_t)idx;
      if (idx == n - 1) rowstart[U] = (int32_t)n;
    }
    if (pos < ucf[c])  // column c's unique key number pos
      uniq[P > 1 ? po_place(&L, c, P, pos) : basef[c] + pos] = ps_route(ukey[idx], rmult, rn);
    // one owner: lookup j's table row (its routed key), so the input assembly reads the row
    // with one index load instead of the inv -> uniq chain
    if (rowidx) rowidx[j] = (int32_t)ps_route(ukey[(int64_t)c * B + lu], rmult, rn);
  }
}

int plan_owner_bits(int P) {
  int b = 0;
  while ((1 << b) < P) ++b;
  return b;
}

void plan_sorted(const int64_t* keys, int B, int F, const int64_t* col_base, const int32_t* col_bits,
                 uint64_t route_mult, uint64_t route_n, const int64_t* bounds, int P, int32_t* ws, int64_t* ukey,
                 int64_t* uniq, int64_t* inv, int32_t* members, int32_t* memrow, int64_t* counts, hipStream_t s,
                 int32_t* pos, int32_t* rowstart, int32_t* rowidx) {
  if (rowstart && P > 1) throw std::runtime_error("plan_sorted: row starts are for one owner");
  if (rowidx && (P > 1 || !route_mult || route_n > (uint64_t)INT32_MAX))
    throw std::runtime_error("plan_sorted: per-lookup rows need one owner and routed keys below 2^31");
  if (B < 1 || B > kPsMax) throw std::runtime_error("plan_sorted: 1 <= B <= 16384 rows per column");
  if (F < 1 || F > 64) throw std::runtime_error("plan_sorted: 1 <= F <= 64 columns");
  if (P < 1 || P > kPoMaxP) throw std::runtime_error("plan_sorted: 1 <= P <= 16 owners");
  if (route_mult && !route_n) throw std::runtime_error("plan_sorted: routing needs the row count");
  const int64_t n = (int64_t)B * F;
  // ws (plan_sorted_ws_ints): sorted_b [n] | local_u [n] | ucount [F] | (16-byte aligned)
  // column-major keys [n] | per-column owner counts [F * P]
  int32_t* sorted_b = ws;
  int32_t* local_u = ws + n;
  int32_t* ucount = ws + 2 * n;
  const int64_t kofs = (2 * n + F + 3) & ~int64_t(3);
  uint32_t* krel = reinterpret_cast<uint32_t*>(ws + kofs);  // 16-byte aligned
  int32_t* ocnt = ws + kofs + n;
  const int obits = P > 1 ? plan_owner_bits(P) : 0;
  hipLaunchKernelGGL(plan_transpose_kernel, (B + 63) / 64, 256, 0, s, keys, B, F, col_base, col_bits, bounds, P,
                     route_mult, route_n, krel);
  // one 1024-thread workgroup per column (round 4's chunked sort over F x 4 workgroups measured
  // slower in the W&D step -- 0.3708 vs 0.3657 ms, profiles/r4/ab_wd_knobs.txt -- and is gone)
  hipLaunchKernelGGL(plan_sort_col_kernel, F, kPsThreads, 0, s, krel, B, col_base, col_bits, obits, P, sorted_b,
                     local_u, ukey, ucount, ocnt);
  hipLaunchKernelGGL(plan_emit_kernel, grid_for(n, 256, 2048), 256, 0, s, B, F, sorted_b, local_u, ukey, ucount,
                     route_mult, route_n, P, ocnt, uniq, inv, members, memrow, counts, pos, rowstart, rowidx);
  MINIPS_HIP_CHECK(hipGetLastError());
}

int64_t plan_sorted_ws_ints(int64_t n, int F, int P) { return ((2 * n + F + 3) & ~int64_t(3)) + n + (int64_t)F * P; }

}  // namespace minips_k
