// Asynchronous parameter-server data path over xGMI (SSP / ASP tables, minips_amd/ps/onesided.py).
//
// Every rank hipMallocs its shard of each table and an inbox (one slot ring per requester), and
// exports both with hipIpcGetMemHandle; every rank maps every peer's buffers, so any GPU addresses
// every owner's rows and inboxes through small device tables of base pointers.
//
//   Get   ps_gather_rows: the requested rows straight from their owners' HBM (one-sided; 16-byte
//         loads per lane, every lane busy: the grid runs over (row, 16-byte chunk) pairs)
//   Add   ps_push_rows: the requester writes its clock's deduplicated (key, gradient row) batch,
//         grouped by owner, into slot (clock % depth) of its ring in each owner's inbox, with the
//         row count in the slot header -- no host round trip: the per-owner counts are read on
//         the device
//   apply HipApplier (the owner's AsyncServer thread, csrc/runtime/async_server.h): the owner
//         runs its optimizer (row-wise Adagrad / Adam / Adagrad / SGD / add) on the slot with ITS
//         OWN state, on its own high-priority stream, bounded by the header count
//
// Slot layouts (byte offsets inside the slot):
//   sparse  [0, 64) header: int64 row count | [64, 64 + 8 cap) int64 keys | then fp32 rows [cap, W]
//   dense   [0, 64) header: int64 1 (0 = a Clock without an Add) | [64, ...) fp32 gradient of the
//           owner's shard [n]
//
//   owner of key k   o = upper_bound(bounds, k) - 1   (bounds [P+1], equal key ranges)
//   row              k - bounds[o]  in the shard at bases[o]  ([rows_o, W] fp32 / bf16, row-major)
//
// Memory model (why a reader never sees a stale or a half-applied row):
//   * allocation (ipc_alloc, csrc/bindings/ops_py.cpp): inboxes are UNCACHED device memory
//     (hipDeviceMallocUncached: the owner's apply reads what the requester's xGMI writes put in
//     HBM, never an L2 copy of the slot from `depth` clocks ago); shards, pull copies and the
//     control lines are FINE-GRAINED (hipDeviceMallocFinegrained: coherent for peer access and
//     system-scope atomics);
//   * push: ps_push_rows is followed on its stream by a 64-workgroup system-scope release
//     (fence_l2: one write-back per XCD L2, after the push's stores drained at its kernel
//     boundary); the requester's publisher thread bumps `sent` only after both completed (an
//     event);
//   * apply: the owner's server thread brackets each table's applies of a batch with
//     ps_write_lock / ps_write_unlock on its apply stream. The lock word (one per table, in the
//     owner's fine-grained control line) has the writer bit 31 and a reader count. The writer
//     sets the bit (new readers wait), waits for the readers inside to leave, then the applies run;
//     ps_write_unlock runs 64 workgroups (every XCD) that each write back their XCD's L2 with a
//     system-scope release, and the last one to arrive clears the writer bit. `applied` is
//     published after that (an event again);
//   * read: ps_read_lock takes the read lock of every owner of the table (ascending owner order,
//     so readers and single-lock writers cannot deadlock), a 64-workgroup system-scope acquire
//     (fence_l2: every XCD's L2 drops peer-written lines; the next dispatch drops L1) precedes
//     the gather / pull kernel, and
//     ps_read_unlock leaves. A read therefore sees every owner's shard between two batches --
//     never half of one -- which is what the reference's single server thread guarantees
//     (server/server_thread.cpp:23-61: one Add or Get at a time per model);
//   * every spin is bounded (kSpinLimit of the 100 MHz real-time counter, ~2 s); a timeout sets a
//     bit of the rank's error word (host-mapped) and proceeds, and the host raises on it.
#include <algorithm>
#include <atomic>
#include <stdexcept>
#include <string>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "onesided.h"

namespace minips_k {

namespace {

constexpr int kFlushBlocks = 64;  // dealt round-robin over the 8 XCDs: every XCD's L2 is covered

// One system-scope fence per workgroup of a 64-workgroup launch -- once per XCD L2, not once per
// workgroup of the data kernel: a system-scope write-back / invalidate acts on the whole XCD L2,
// so 8192 gather / push workgroups each fencing flushed the L2 under every concurrently running
// GEMM (the round-4 one-sided trace: a 240 us push, wgrads at 2.3x their time). RELEASE: the
// preceding kernels' stores on this stream reach memory; acquire: later kernels on this stream
// re-read peer-written lines (the kernel boundary drains and the next dispatch drops L1).
template <bool RELEASE>
__global__ void ps_fence_kernel() {
  if (threadIdx.x != 0) return;
  if constexpr (RELEASE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// One-rank process (every owner is this device): the kernel boundaries of one stream and the
// owner's lock kernels order everything at agent scope, so the system-scope fences are skipped
// (ps_set_fences(false); each fence launch costs ~5 us of queue time).
static bool g_ps_fences = true;

void fence_l2(bool release, hipStream_t s) {
  if (!g_ps_fences) return;
  if (release) hipLaunchKernelGGL(ps_fence_kernel<true>, kFlushBlocks, 64, 0, s);
  else hipLaunchKernelGGL(ps_fence_kernel<false>, kFlushBlocks, 64, 0, s);
}

constexpr uint64_t kSpinLimit = 200000000ull;  // ticks of the 100 MHz real-time counter: ~2 s

__device__ __forceinline__ uint32_t ld_sys(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void flag_error(uint32_t* err, uint32_t bit) {
  if (err) __hip_atomic_fetch_or(err, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void ps_read_lock_kernel(const int64_t* __restrict__ locks, int P, uint32_t* held, uint32_t* err) {
  if (threadIdx.x != 0) return;
  uint32_t mask = 0;
  for (int o = 0; o < P; ++o) {
    uint32_t* w = reinterpret_cast<uint32_t*>(locks[o]);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      uint32_t v = ld_sys(w);
      if (!(v & kPsWriter) && __hip_atomic_compare_exchange_strong(w, &v, v + 1, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_SYSTEM)) {
        mask |= 1u << o;
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinLimit) {
        flag_error(err, kPsErrReadLock);
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
  }
  __hip_atomic_store(held, mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void ps_read_unlock_kernel(const int64_t* __restrict__ locks, int P, uint32_t* held) {
  if (threadIdx.x != 0) return;
  const uint32_t mask = __hip_atomic_load(held, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int o = 0; o < P; ++o)
    if (mask & (1u << o))
      __hip_atomic_fetch_sub(reinterpret_cast<uint32_t*>(locks[o]), 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void ps_write_lock_kernel(uint32_t* lock, uint32_t* err) {
  if (threadIdx.x != 0) return;
  __hip_atomic_fetch_or(lock, kPsWriter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (ld_sys(lock) & ~kPsWriter) {  // readers inside
    if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinLimit) {
      flag_error(err, kPsErrWriteLock);
      break;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

__global__ void ps_write_unlock_kernel(uint32_t* lock, uint32_t* count) {
  if (threadIdx.x != 0) return;
  __threadfence_system();  // this XCD's dirty lines (the applies of the batch) reach memory
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (__hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM) == kFlushBlocks - 1) {
    __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_fetch_and(lock, ~kPsWriter, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// one-rank form: every reader is on this device, so an agent-scope release suffices
__global__ void ps_write_unlock_local_kernel(uint32_t* lock) {
  if (threadIdx.x != 0) return;
  __hip_atomic_fetch_and(lock, ~kPsWriter, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int upper_owner(const int64_t* __restrict__ b, int P, int64_t k) {
  int lo = 0, hi = P;  // b[lo] <= k < b[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (b[mid] <= k) lo = mid;
    else hi = mid;
  }
  return lo;
}

// chunk = 4 floats (VEC) or 1 float
template <bool VEC>
__global__ __launch_bounds__(256) void ps_push_rows_kernel(const int64_t* __restrict__ uniq,
                                                           const int64_t* __restrict__ counts,
                                                           const int64_t* __restrict__ U_dev, int64_t n,
                                                           const float* __restrict__ g, int W,
                                                           const int64_t* __restrict__ inbox, int P,
                                                           int64_t slot_off, int64_t cap) {
  __shared__ int64_t start[kPsMaxWorld + 1];
  if (threadIdx.x == 0) {
    int64_t s = 0;
    for (int o = 0; o < P; ++o) {
      start[o] = s;
      s += counts[o];
    }
    start[P] = s;
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)P) {  // every owner's header, empty segments too
    *reinterpret_cast<int64_t*>(reinterpret_cast<char*>(inbox[threadIdx.x]) + slot_off) = counts[threadIdx.x];
  }
  const int64_t U = U_dev ? min(n, *U_dev) : n;
  const int nv = VEC ? W / 4 : W;
  const int64_t total = U * nv;
  const int64_t rows_off = kPsSlotHeader + 8 * cap;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = c / nv;
    const int j = (int)(c - i * nv);
    const int o = upper_owner(start, P, i);
    const int64_t pos = i - start[o];
    char* slot = reinterpret_cast<char*>(inbox[o]) + slot_off;
    if (j == 0) reinterpret_cast<int64_t*>(slot + kPsSlotHeader)[pos] = uniq[i];
    float* dst = reinterpret_cast<float*>(slot + rows_off) + pos * W;
    if constexpr (VEC) {
      reinterpret_cast<float4*>(dst)[j] = reinterpret_cast<const float4*>(g + i * W)[j];
    } else {
      dst[j] = g[i * W + j];
    }
  }
}

__global__ void ps_set_headers_kernel(const int64_t* __restrict__ inbox, int P, int64_t slot_off, int64_t value) {
  if (threadIdx.x < (unsigned)P)
    *reinterpret_cast<int64_t*>(reinterpret_cast<char*>(inbox[threadIdx.x]) + slot_off) = value;
}

template <bool VEC, typename TO>
__global__ __launch_bounds__(256) void ps_gather_rows_kernel(const int64_t* __restrict__ bases,
                                                             const int64_t* __restrict__ bounds, int P,
                                                             const int64_t* __restrict__ keys, int64_t n,
                                                             const int64_t* __restrict__ n_dev, int W,
                                                             TO* __restrict__ out) {
  __shared__ int64_t b[kPsMaxWorld + 1];
  __shared__ int64_t base_ptr[kPsMaxWorld];
  if (threadIdx.x <= (unsigned)P) b[threadIdx.x] = bounds[threadIdx.x];
  if (threadIdx.x < (unsigned)P) base_ptr[threadIdx.x] = bases[threadIdx.x];
  __syncthreads();
  const int64_t nn = n_dev ? min(n, *n_dev) : n;
  const int nv = VEC ? W / 4 : W;
  const int64_t total = nn * nv;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = c / nv;
    const int j = (int)(c - i * nv);
    const int64_t k = keys[i];
    if (k < b[0] || k >= b[P]) {  // never address outside the table: a zero row
      if constexpr (VEC) {
        if constexpr (sizeof(TO) == 2) reinterpret_cast<uint2*>(out + i * W)[j] = make_uint2(0u, 0u);
        else reinterpret_cast<float4*>(out + i * W)[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        out[i * W + j] = (TO)0;
      }
      continue;
    }
    const int o = upper_owner(b, P, k);
    const float* row = reinterpret_cast<const float*>(base_ptr[o]) + (k - b[o]) * (int64_t)W;
    if constexpr (VEC) {
      const float4 v = reinterpret_cast<const float4*>(row)[j];
      if constexpr (sizeof(TO) == 2) {
        reinterpret_cast<uint2*>(out + i * W)[j] = make_uint2(pack_bf2(v.x, v.y), pack_bf2(v.z, v.w));
      } else {
        reinterpret_cast<float4*>(out + i * W)[j] = v;
      }
    } else {
      const float v = row[j];
      if constexpr (sizeof(TO) == 2) {
        out[i * W + j] = f2bf(v);
      } else {
        out[i * W + j] = v;
      }
    }
  }
}

// bf16 shards: 8 values per 16-byte load, W / 8 lanes per row
template <typename TO>
__global__ __launch_bounds__(256) void ps_gather_bf16_kernel(const int64_t* __restrict__ bases,
                                                             const int64_t* __restrict__ bounds, int P,
                                                             const int64_t* __restrict__ keys, int64_t n,
                                                             const int64_t* __restrict__ n_dev, int W,
                                                             TO* __restrict__ out) {
  __shared__ int64_t b[kPsMaxWorld + 1];
  __shared__ int64_t base_ptr[kPsMaxWorld];
  if (threadIdx.x <= (unsigned)P) b[threadIdx.x] = bounds[threadIdx.x];
  if (threadIdx.x < (unsigned)P) base_ptr[threadIdx.x] = bases[threadIdx.x];
  __syncthreads();
  const int64_t nn = n_dev ? min(n, *n_dev) : n;
  const int nv = W / 8;
  const int64_t total = nn * nv;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = c / nv;
    const int j = (int)(c - i * nv);
    const int64_t k = keys[i];
    uint4 v = make_uint4(0, 0, 0, 0);
    if (k >= b[0] && k < b[P]) {
      const int o = upper_owner(b, P, k);
      v = reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(base_ptr[o]) + (k - b[o]) * (int64_t)W)[j];
    }
    if constexpr (sizeof(TO) == 2) {
      reinterpret_cast<uint4*>(out + i * W)[j] = v;
    } else {
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      float4* d = reinterpret_cast<float4*>(out + i * W) + 2 * j;
      d[0] = make_float4(__uint_as_float(w[0] << 16), __uint_as_float(w[0] & 0xffff0000u), __uint_as_float(w[1] << 16),
                         __uint_as_float(w[1] & 0xffff0000u));
      d[1] = make_float4(__uint_as_float(w[2] << 16), __uint_as_float(w[2] & 0xffff0000u), __uint_as_float(w[3] << 16),
                         __uint_as_float(w[3] & 0xffff0000u));
    }
  }
}

// ---- Map storage (open addressing, linear probing; keys are the mixed 63-bit keys, ~0 = empty)
constexpr unsigned long long kPsEmpty = ~0ull;

__device__ __forceinline__ uint64_t ps_mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// slot of key k in (hk, cap), -1 if absent (a reader: never inserts)
__device__ __forceinline__ int64_t ps_hash_find(const unsigned long long* hk, int64_t cap, unsigned long long k) {
  int64_t s = (int64_t)(ps_mix(k) & (uint64_t)(cap - 1));
  for (int64_t probe = 0; probe < cap; ++probe) {
    const unsigned long long cur = hk[s];
    if (cur == k) return s;
    if (cur == kPsEmpty) return -1;
    s = (s + 1) & (cap - 1);
  }
  return -1;
}

template <typename TO>
__global__ __launch_bounds__(256) void ps_hash_gather_kernel(const int64_t* __restrict__ hkeys,
                                                             const int64_t* __restrict__ hvals,
                                                             const int64_t* __restrict__ bounds, int P, int64_t cap,
                                                             const int64_t* __restrict__ keys, int64_t n,
                                                             const int64_t* __restrict__ n_dev, int W,
                                                             TO* __restrict__ out) {
  __shared__ int64_t b[kPsMaxWorld + 1];
  if (threadIdx.x <= (unsigned)P) b[threadIdx.x] = bounds[threadIdx.x];
  __syncthreads();
  const int64_t nn = n_dev ? min(n, *n_dev) : n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nn; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = keys[i];
    int64_t s = -1;
    int o = 0;
    if (k >= b[0] && k < b[P]) {
      o = upper_owner(b, P, k);
      s = ps_hash_find(reinterpret_cast<const unsigned long long*>(hkeys[o]), cap, (unsigned long long)k);
    }
    const float* row = s >= 0 ? reinterpret_cast<const float*>(hvals[o]) + s * (int64_t)W : nullptr;
    for (int c = 0; c < W; ++c) {
      const float v = row ? row[c] : 0.f;
      if constexpr (sizeof(TO) == 2) out[i * W + c] = f2bf(v);
      else out[i * W + c] = v;
    }
  }
}

// Owner-side apply of one inbox slot into the Map storage: one wave per row; lane 0 finds or
// inserts the key (the owner is the only inserter; distinct keys race only on empty slots: CAS),
// then the row is updated (OPT 0: w += scale g; 2: row-wise Adagrad with per-slot state).
template <int OPT>
__global__ __launch_bounds__(256) void ps_hash_apply_kernel(unsigned long long* __restrict__ hk, int64_t cap,
                                                            float* __restrict__ vals, float* __restrict__ state,
                                                            int W, const int64_t* __restrict__ keys,
                                                            const float* __restrict__ g,
                                                            const int64_t* __restrict__ cnt,
                                                            int64_t n_max, float lr, float eps, float scale,
                                                            uint32_t* err) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t n = min(n_max, *cnt);
  for (int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; i < n; i += nw) {
    int64_t slot = -1;
    if (lane == 0) {
      const unsigned long long k = (unsigned long long)keys[i];
      int64_t s = (int64_t)(ps_mix(k) & (uint64_t)(cap - 1));
      for (int64_t probe = 0; probe < cap; ++probe) {
        unsigned long long cur = hk[s];
        if (cur == kPsEmpty) cur = atomicCAS(hk + s, kPsEmpty, k);
        if (cur == kPsEmpty || cur == k) {  // claimed (the row is zero: MapStorage's default-insert) or found
          slot = s;
          break;
        }
        s = (s + 1) & (cap - 1);
      }
      if (slot < 0) flag_error(err, kPsErrHashFull);
    }
    slot = __shfl(slot, 0, 64);
    if (slot < 0) continue;
    float* row = vals + slot * (int64_t)W;
    const float* gr = g + i * (int64_t)W;
    float step = scale;
    if (OPT == 2) {
      float sq = 0.f;
      for (int c = lane; c < W; c += 64) sq += gr[c] * gr[c];
      sq = warp_sum(sq);
      const float st = state[slot] + sq / (float)W;
      if (lane == 0) state[slot] = st;
      step = -lr / (sqrtf(st) + eps);
    }
    for (int c = lane; c < W; c += 64) row[c] += step * gr[c];
  }
}

// Pull copies: 16-byte chunks of the selected owners' buffers (owner ids packed 4 bits each)
__global__ __launch_bounds__(256) void ps_pull_kernel(const int64_t* __restrict__ srcs, uint64_t owners,
                                                      int64_t chunks, char* __restrict__ dst, int64_t shard_bytes,
                                                      int count) {
  const int64_t total = chunks * count;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total; c += (int64_t)gridDim.x * blockDim.x) {
    const int sel = (int)(c / chunks);
    const int64_t j = c - (int64_t)sel * chunks;
    const int o = (int)((owners >> (4 * sel)) & 15);
    const uint4 v = reinterpret_cast<const uint4*>(srcs[o])[j];
    reinterpret_cast<uint4*>(dst + o * shard_bytes)[j] = v;
  }
}

}  // namespace

void ps_set_fences(bool on) { g_ps_fences = on; }

void ps_read_lock(const int64_t* locks, int P, uint32_t* held, uint32_t* err, hipStream_t s) {
  if (P < 1 || P > kPsMaxWorld) throw std::runtime_error("ps_read_lock: P out of range");
  hipLaunchKernelGGL(ps_read_lock_kernel, 1, 64, 0, s, locks, P, held, err);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void ps_read_unlock(const int64_t* locks, int P, uint32_t* held, hipStream_t s) {
  hipLaunchKernelGGL(ps_read_unlock_kernel, 1, 64, 0, s, locks, P, held);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void ps_write_lock(uint32_t* lock, uint32_t* err, hipStream_t s) {
  hipLaunchKernelGGL(ps_write_lock_kernel, 1, 64, 0, s, lock, err);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void ps_write_unlock(uint32_t* lock, uint32_t* flush_count, hipStream_t s) {
  if (!g_ps_fences) {
    hipLaunchKernelGGL(ps_write_unlock_local_kernel, 1, 64, 0, s, lock);
    MINIPS_HIP_CHECK(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(ps_write_unlock_kernel, kFlushBlocks, 64, 0, s, lock, flush_count);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void ps_gather_rows_bf16tab(const int64_t* bases, const int64_t* bounds, int P, const int64_t* keys, int64_t n,
                            const int64_t* n_dev, int W, void* out, bool out_bf16, hipStream_t s) {
  if (n <= 0) return;
  if (P < 1 || P > kPsMaxWorld) throw std::runtime_error("ps_gather_rows_bf16tab: P out of range");
  if (W % 8 || reinterpret_cast<uintptr_t>(out) % 16) throw std::runtime_error("bf16 gather: W % 8, aligned out");
  const int grid = grid_for(n * (W / 8), 256, 8192);
  fence_l2(false, s);
  if (out_bf16)
    hipLaunchKernelGGL(ps_gather_bf16_kernel<bf16_t>, grid, 256, 0, s, bases, bounds, P, keys, n, n_dev, W,
                       static_cast<bf16_t*>(out));
  else
    hipLaunchKernelGGL(ps_gather_bf16_kernel<float>, grid, 256, 0, s, bases, bounds, P, keys, n, n_dev, W,
                       static_cast<float*>(out));
  MINIPS_HIP_CHECK(hipGetLastError());
}

void ps_hash_gather(const int64_t* hkeys, const int64_t* hvals, const int64_t* bounds, int P, int64_t cap,
                    const int64_t* keys, int64_t n, const int64_t* n_dev, int W, void* out, bool out_bf16,
                    hipStream_t s) {
  if (n <= 0) return;
  if (P < 1 || P > kPsMaxWorld) throw std::runtime_error("ps_hash_gather: P out of range");
  if (cap <= 0 || (cap & (cap - 1))) throw std::runtime_error("ps_hash_gather: capacity must be a power of two");
  const int grid = grid_for(n, 256, 4096);
  fence_l2(false, s);
  if (out_bf16)
    hipLaunchKernelGGL(ps_hash_gather_kernel<bf16_t>, grid, 256, 0, s, hkeys, hvals, bounds, P, cap, keys, n, n_dev,
                       W, static_cast<bf16_t*>(out));
  else
    hipLaunchKernelGGL(ps_hash_gather_kernel<float>, grid, 256, 0, s, hkeys, hvals, bounds, P, cap, keys, n, n_dev,
                       W, static_cast<float*>(out));
  MINIPS_HIP_CHECK(hipGetLastError());
}

void ps_pull(const int64_t* srcs, uint64_t owners, int count, int64_t shard_bytes, void* dst, hipStream_t s) {
  if (count <= 0) return;
  if (count > kPsMaxWorld || shard_bytes % 16 || reinterpret_cast<uintptr_t>(dst) % 16)
    throw std::runtime_error("ps_pull: <= 16 owners, 16-byte aligned shards");
  const int64_t chunks = shard_bytes / 16;
  fence_l2(false, s);
  hipLaunchKernelGGL(ps_pull_kernel, grid_for(chunks * count, 256, 8192), 256, 0, s, srcs, owners, chunks,
                     static_cast<char*>(dst), shard_bytes, count);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void ps_push_rows(const int64_t* uniq, const int64_t* counts, const int64_t* U_dev, int64_t n, const float* g, int W,
                  const int64_t* inbox, int P, int64_t slot_off, int64_t cap, hipStream_t s) {
  if (P < 1 || P > kPsMaxWorld) throw std::runtime_error("ps_push_rows: P out of range");
  if (n > cap) throw std::runtime_error("ps_push_rows: more rows than an inbox slot holds");
  const int block = 256;
  const bool vec = W % 4 == 0 && reinterpret_cast<uintptr_t>(g) % 16 == 0 && slot_off % 16 == 0 && cap % 2 == 0;
  const int64_t work = std::max<int64_t>(1, n * (vec ? W / 4 : W));
  const int grid = grid_for(work, block, 8192);
  if (vec)
    hipLaunchKernelGGL(ps_push_rows_kernel<true>, grid, block, 0, s, uniq, counts, U_dev, n, g, W, inbox, P,
                       slot_off, cap);
  else
    hipLaunchKernelGGL(ps_push_rows_kernel<false>, grid, block, 0, s, uniq, counts, U_dev, n, g, W, inbox, P,
                       slot_off, cap);
  fence_l2(true, s);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// The dense push of one clock: owner o's slice grad[o * S, (o + 1) * S) into the data area of slot
// `slot_off` of its inbox, and grad cleared for the next clock -- one pass (read once, write the
// slot and the zero) instead of P copies and a fill. `sl`: split-K weight-gradient planes whose
// sums are added on the way (the regions' offsets in grad; no reduce kernels before the push).
__global__ __launch_bounds__(256) void ps_push_dense_kernel(float* __restrict__ grad, const int64_t* __restrict__ inbox,
                                                            int P, int64_t data_off, int64_t S4, AdamSlabs sl) {
  const int64_t total = (int64_t)P * S4;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(e / S4);
    const int64_t k = e - (int64_t)o * S4;
    float4 v = reinterpret_cast<const float4*>(grad)[e];
    for (int r = 0; r < sl.n; ++r) {
      const int64_t x = 4 * e - sl.off[r];
      if (x < 0 || x >= sl.len[r]) continue;
      const float* p = sl.p[r] + x;
      for (int z = 0; z < sl.nsplit[r]; ++z) {
        const float4 a = *reinterpret_cast<const float4*>(p + z * sl.plane[r]);
        v.x += a.x;
        v.y += a.y;
        v.z += a.z;
        v.w += a.w;
      }
    }
    reinterpret_cast<float4*>(reinterpret_cast<char*>(inbox[o]) + data_off)[k] = v;
    reinterpret_cast<float4*>(grad)[e] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

void ps_push_dense(float* grad, const int64_t* inbox, int P, int64_t data_off, int64_t S, hipStream_t s,
                   const AdamSlabs* slabs) {
  if (P < 1 || P > kPsMaxWorld) throw std::runtime_error("ps_push_dense: P out of range");
  if (S % 4 || data_off % 16 || reinterpret_cast<uintptr_t>(grad) % 16)
    throw std::runtime_error("ps_push_dense: 16-byte aligned shards");
  AdamSlabs sl;
  if (slabs) {
    sl = *slabs;
    for (int r = 0; r < sl.n; ++r)
      if (sl.off[r] % 4 || sl.len[r] % 4 || sl.plane[r] % 4 || reinterpret_cast<uintptr_t>(sl.p[r]) % 16)
        throw std::runtime_error("ps_push_dense: slab regions must be 16-byte aligned");
  }
  hipLaunchKernelGGL(ps_push_dense_kernel, grid_for((int64_t)P * (S / 4), 256, 8192), 256, 0, s, grad, inbox, P,
                     data_off, S / 4, sl);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void ps_set_headers(const int64_t* inbox, int P, int64_t slot_off, int64_t value, hipStream_t s) {
  if (P < 1 || P > kPsMaxWorld) throw std::runtime_error("ps_set_headers: P out of range");
  hipLaunchKernelGGL(ps_set_headers_kernel, 1, 64, 0, s, inbox, P, slot_off, value);
  fence_l2(true, s);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void ps_gather_rows(const int64_t* bases, const int64_t* bounds, int P, const int64_t* keys, int64_t n,
                    const int64_t* n_dev, int W, void* out, bool out_bf16, hipStream_t s) {
  if (n <= 0) return;
  if (P < 1 || P > kPsMaxWorld) throw std::runtime_error("ps_gather_rows: P out of range");
  const int block = 256;
  const bool vec = W % 4 == 0 && reinterpret_cast<uintptr_t>(out) % (out_bf16 ? 8 : 16) == 0;
  const int grid = grid_for(n * (vec ? W / 4 : W), block, 8192);
  fence_l2(false, s);
#define MINIPS_PS_GATHER(V, T)                                                                                \
  hipLaunchKernelGGL((ps_gather_rows_kernel<V, T>), grid, block, 0, s, bases, bounds, P, keys, n, n_dev, W, \
                     static_cast<T*>(out))
  if (vec && out_bf16) MINIPS_PS_GATHER(true, bf16_t);
  else if (vec) MINIPS_PS_GATHER(true, float);
  else if (out_bf16) MINIPS_PS_GATHER(false, bf16_t);
  else MINIPS_PS_GATHER(false, float);
#undef MINIPS_PS_GATHER
  MINIPS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- clock-coalesced owner applies
// SSP tables with a stateful optimizer (AsyncServer::SetCoalesce): clock c's slots of the P
// requesters are applied as ONE optimizer step, with the gradient rows of a key summed in
// requester order -- the BSP update of that clock (tables.py owner_push_adagrad: same per-row
// arithmetic). Slot r of clock c: inbox + r * stride_r + slot_off.
//
// Sparse: a persistent direct-addressed table rs[row * P + r] = {stamp, index in r's slot}
// (ps_clock_mark: each requester's slot holds a key at most once -- one writer per entry); the
// apply takes 8 lanes per received row and the group of the LOWEST requester that sent the row
// sums the <= P contributions and applies the row-wise Adagrad (fp32 rows, or bf16 rows with
// stochastic rounding). The stamp (an apply counter of the owner, never rewound) retires older
// entries without clearing the table.
__global__ void ps_clock_mark_kernel(const char* __restrict__ inbox, int64_t stride_r, int64_t slot_off, int64_t base,
                                     int P, int2* __restrict__ rs, int stamp) {
  const int r = blockIdx.y;
  const char* slot = inbox + r * stride_r + slot_off;
  const int64_t n = *reinterpret_cast<const int64_t*>(slot);
  const int64_t* keys = reinterpret_cast<const int64_t*>(slot + kPsSlotHeader);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    rs[(keys[i] - base) * P + r] = make_int2(stamp, (int)i);
}

template <bool BF16>
__global__ __launch_bounds__(256) void ps_clock_adagrad_kernel(void* table, int64_t ld, float* state, float* state2,
                                                               int D1, const char* __restrict__ inbox, int64_t stride_r,
                                                               int64_t slot_off, int64_t cap, int64_t base, int D,
                                                               int P, const int2* __restrict__ rs, int stamp, float lr,
                                                               float eps, uint32_t step, uint32_t seed) {
  const int me = blockIdx.y;  // the requester whose slot this block walks (wave-uniform)
  const char* slot = inbox + me * stride_r + slot_off;
  const int64_t n = *reinterpret_cast<const int64_t*>(slot);
  const int64_t* keys = reinterpret_cast<const int64_t*>(slot + kPsSlotHeader);
  const int64_t rows_off = kPsSlotHeader + 8 * cap;
  const int lane = threadIdx.x & 63, sub = lane >> 3, l = lane & 7;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int c0 = 4 * l, c1 = 32 + 4 * l;
  const bool has0 = c0 < D, has1 = c1 < D;
  for (int64_t i0 = wave * 8; i0 < n; i0 += nwaves * 8) {
    const int64_t i = i0 + sub;
    const bool in = i < n;
    const int64_t row = in ? keys[i] - base : 0;
    const int2* e = rs + row * P;
    const int2 e0 = in && l < P ? e[l] : make_int2(-1, -1);
    const int2 e1 = in && l + 8 < P ? e[l + 8] : make_int2(-1, -1);
    float t[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (in && has0) {
      if constexpr (BF16) {
        const bf16_t* tr = static_cast<const bf16_t*>(table) + row * ld;
        const uint2 a = *reinterpret_cast<const uint2*>(tr + c0);
        t[0] = __uint_as_float(a.x << 16); t[1] = __uint_as_float(a.x & 0xffff0000u);
        t[2] = __uint_as_float(a.y << 16); t[3] = __uint_as_float(a.y & 0xffff0000u);
        if (has1) {
          const uint2 b = *reinterpret_cast<const uint2*>(tr + c1);
          t[4] = __uint_as_float(b.x << 16); t[5] = __uint_as_float(b.x & 0xffff0000u);
          t[6] = __uint_as_float(b.y << 16); t[7] = __uint_as_float(b.y & 0xffff0000u);
        }
      } else {
        const float* tr = static_cast<const float*>(table) + row * ld;
        const float4 a = *reinterpret_cast<const float4*>(tr + c0);
        t[0] = a.x; t[1] = a.y; t[2] = a.z; t[3] = a.w;
        if (has1) {
          const float4 b = *reinterpret_cast<const float4*>(tr + c1);
          t[4] = b.x; t[5] = b.y; t[6] = b.z; t[7] = b.w;
        }
      }
    }
    const float st_old1 = in ? state[row] : 0.f;
    const float st_old2 = in && D1 < D ? state2[row] : 0.f;
    const int sl0 = e0.x == stamp ? e0.y : -1, sl1 = e1.x == stamp ? e1.y : -1;
    // the leader: no lower requester sent this row in this clock
    const unsigned long long lower = __ballot(sl0 >= 0 && l < me) | __ballot(sl1 >= 0 && l + 8 < me);
    const bool ok = in && ((lower >> (sub << 3)) & 0xffull) == 0;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < P; ++s) {
      const int m = __shfl(s < 8 ? sl0 : sl1, (sub << 3) + (s & 7), 64);
      if (ok && m >= 0 && has0) {
        const float* g = reinterpret_cast<const float*>(inbox + s * stride_r + slot_off + rows_off) + (int64_t)m * D;
        const float4 v = *reinterpret_cast<const float4*>(g + c0);
        a[0] += v.x; a[1] += v.y; a[2] += v.z; a[3] += v.w;
        if (has1) {
          const float4 w = *reinterpret_cast<const float4*>(g + c1);
          a[4] += w.x; a[5] += w.y; a[6] += w.z; a[7] += w.w;
        }
      }
    }
    float sq1 = 0.f, sq2 = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = (q < 4 ? c0 : c1) + (q & 3);
      if (c < D1) sq1 += a[q] * a[q];
      else if (c < D) sq2 += a[q] * a[q];
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
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = (q < 4 ? c0 : c1) + (q & 3);
      t[q] -= (c < D1 ? s1 : s2) * a[q];
    }
    if constexpr (BF16) {
      bf16_t* tr = static_cast<bf16_t*>(table) + row * ld;
      uint32_t o[4];
#pragma unroll
      for (int e2 = 0; e2 < 4; ++e2) {
        const int c = (e2 < 2 ? c0 : c1) + 2 * (e2 & 1);
        const uint32_t rnd = sr_hash((uint64_t)(row + base), (uint32_t)c, step, seed);
        o[e2] = (uint32_t)bf16_sr(t[2 * e2], rnd) | ((uint32_t)bf16_sr(t[2 * e2 + 1], rnd >> 16) << 16);
      }
      if (has0) *reinterpret_cast<uint2*>(tr + c0) = make_uint2(o[0], o[1]);
      if (has1) *reinterpret_cast<uint2*>(tr + c1) = make_uint2(o[2], o[3]);
    } else {
      float* tr = static_cast<float*>(table) + row * ld;
      if (has0) *reinterpret_cast<float4*>(tr + c0) = make_float4(t[0], t[1], t[2], t[3]);
      if (has1) *reinterpret_cast<float4*>(tr + c1) = make_float4(t[4], t[5], t[6], t[7]);
    }
  }
}

// Dense: out = sum over requesters (in order) of the active slots' gradients; *active_out = the
// number of active pushes (the optimizer kernel skips a clock nobody added to).
__global__ __launch_bounds__(256) void ps_clock_sum_dense_kernel(const char* __restrict__ inbox, int64_t stride_r,
                                                                 int64_t slot_off, int P, int64_t n4,
                                                                 float* __restrict__ out,
                                                                 int64_t* __restrict__ active_out) {
  uint32_t act = 0;  // requesters whose slot holds a push (bit r)
  for (int r = 0; r < P; ++r)
    if (*reinterpret_cast<const int64_t*>(inbox + r * stride_r + slot_off) != 0) act |= 1u << r;
  if (blockIdx.x == 0 && threadIdx.x == 0) *active_out = __popc(act);
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n4; j += (int64_t)gridDim.x * blockDim.x) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = 0; r < P; ++r) {
      if (!(act >> r & 1u)) continue;
      const float4 v =
          reinterpret_cast<const float4*>(inbox + r * stride_r + slot_off + kPsSlotHeader)[j];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    reinterpret_cast<float4*>(out)[j] = acc;
  }
}

// ------------------------------------------------------------------------------ owner-side apply
HipApplier::HipApplier(int device, int tables) : dev_(device), descs_(tables) {
  for (auto& d : descs_) d.kind = -1;
}

HipApplier::~HipApplier() {
  for (auto& e : events_)
    if (e) (void)hipEventDestroy(e);
  if (stream_) (void)hipStreamDestroy(stream_);
}

void HipApplier::SetSparse(int t, const PsSparseDesc& d) {
  descs_.at(t).sp = d;
  descs_.at(t).kind = 0;
}

void HipApplier::SetDense(int t, const PsDenseDesc& d) {
  descs_.at(t).dn = d;
  descs_.at(t).kind = 1;
  descs_.at(t).step.store(d.step);
}

void HipApplier::ThreadInit() {
  MINIPS_HIP_CHECK(hipSetDevice(dev_));
  int lo = 0, hi = 0;
  MINIPS_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  // the owner's applies are short and on every requester's critical path (SSP gates on them):
  // the highest priority lets them start beside a running step
  MINIPS_HIP_CHECK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi));
  for (auto& e : events_) MINIPS_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
}

void HipApplier::BeginTable(int t) {
  const Desc& d = descs_.at(t);
  uint32_t* lock = d.kind == 0 ? d.sp.lock : d.dn.lock;
  if (lock) ps_write_lock(lock, err_, stream_);
}

void HipApplier::EndTable(int t) {
  const Desc& d = descs_.at(t);
  uint32_t* lock = d.kind == 0 ? d.sp.lock : d.dn.lock;
  uint32_t* flush = d.kind == 0 ? d.sp.flush : d.dn.flush;
  if (lock) ps_write_unlock(lock, flush, stream_);
}

uint64_t HipApplier::Submit() {
  const uint64_t ticket = submitted_++;
  MINIPS_HIP_CHECK(hipEventRecord(events_[ticket % kEvents], stream_));
  return ticket;
}

// (the server keeps at most 2 batches in flight, so an event is never re-recorded before its wait)
void HipApplier::Wait(uint64_t ticket) { MINIPS_HIP_CHECK(hipEventSynchronize(events_[ticket % kEvents])); }

void HipApplier::Apply(int t, int r, int64_t c) {
  Desc& d = descs_.at(t);
  if (d.kind == 0) {
    const PsSparseDesc& p = d.sp;
    char* slot = p.inbox + ((int64_t)r * p.depth + c % p.depth) * p.slot_bytes;
    const int64_t* cnt = reinterpret_cast<const int64_t*>(slot);
    const int64_t* keys = reinterpret_cast<const int64_t*>(slot + kPsSlotHeader);
    const float* g = reinterpret_cast<const float*>(slot + kPsSlotHeader + 8 * p.cap);
    if (p.hash_cap > 0) {  // Map storage
      const int grid = (int)std::min<int64_t>((p.cap + 3) / 4, 4096);
      const float scale = p.opt == kPsAdd ? 1.f : -p.lr;
      if (p.opt == kPsRowwiseAdagrad)
        hipLaunchKernelGGL(ps_hash_apply_kernel<2>, grid, 256, 0, stream_, p.hkeys, p.hash_cap, p.table, p.state, p.W,
                           keys, g, cnt, p.cap, p.lr, p.eps, scale, err_);
      else
        hipLaunchKernelGGL(ps_hash_apply_kernel<0>, grid, 256, 0, stream_, p.hkeys, p.hash_cap, p.table, p.state, p.W,
                           keys, g, cnt, p.cap, p.lr, p.eps, scale, err_);
      MINIPS_HIP_CHECK(hipGetLastError());
      return;
    }
    if (p.bf16) {  // bf16 rows: fp32 math and state, stochastic rounding keyed by the apply count
      const uint32_t step = (uint32_t)d.step.fetch_add(1);
      bf16_t* tab = reinterpret_cast<bf16_t*>(p.table);
      const int code = p.opt == kPsRowwiseAdagrad ? 0 : 1;
      const float scale = p.opt == kPsAdd ? 1.f : -p.lr;
      sparse_apply_bf16tab(code, tab, p.ld, p.state, p.state2, p.D1, keys, p.cap, p.base, p.W, g, p.lr, p.eps, scale,
                           step, p.seed, stream_, cnt);
      return;
    }
    switch (p.opt) {
      case kPsAdd: sparse_sgd(p.table, p.ld, keys, p.cap, p.base, p.W, g, 1.f, stream_, cnt); break;
      case kPsSgd: sparse_sgd(p.table, p.ld, keys, p.cap, p.base, p.W, g, -p.lr, stream_, cnt); break;
      case kPsRowwiseAdagrad:
        sparse_rowwise_adagrad(p.table, p.ld, p.state, p.state2, p.D1, keys, p.cap, p.base, p.W, g, p.lr, p.eps,
                               stream_, cnt);
        break;
      default: throw std::runtime_error("async server: sparse optimizer " + std::to_string(p.opt));
    }
  } else if (d.kind == 1) {
    const PsDenseDesc& p = d.dn;
    const char* slot = p.inbox + ((int64_t)r * p.depth + c % p.depth) * p.slot_bytes;
    const int64_t* active = reinterpret_cast<const int64_t*>(slot);  // header: 0 = a Clock without an Add
    const float* g = reinterpret_cast<const float*>(slot + kPsSlotHeader);
    switch (p.opt) {
      case kPsAdd: sgd_apply(p.w, g, p.n, -1.f, 1.f, p.wb, stream_, active); break;
      case kPsSgd: sgd_apply(p.w, g, p.n, p.lr, 1.f, p.wb, stream_, active); break;
      case kPsAdagrad: adagrad_apply(p.w, p.m, g, p.n, p.lr, p.eps, 1.f, p.wb, stream_, active); break;
      case kPsAdam: {
        // one optimizer step per push (an empty push still counts one: its header is on the device)
        const int64_t step = d.step.fetch_add(1) + 1;
        adam_apply(p.w, p.m, p.v, g, p.n, p.lr, p.b1, p.b2, p.eps, p.wd, (int)step, 1.f, p.wb, stream_, nullptr,
                   false, active);
        break;
      }
      default: throw std::runtime_error("async server: dense optimizer " + std::to_string(p.opt));
    }
  } else {
    throw std::runtime_error("async server: table " + std::to_string(t) + " has no descriptor");
  }
}

void HipApplier::ApplyClock(int t, int64_t c, int world) {
  Desc& d = descs_.at(t);
  if (d.kind == 0 && d.sp.rs && d.sp.opt == kPsRowwiseAdagrad && d.sp.hash_cap == 0) {
    const PsSparseDesc& p = d.sp;
    const int64_t stride = (int64_t)p.depth * p.slot_bytes, off = (c % p.depth) * p.slot_bytes;
    const int stamp = (int)(++d.stamp);
    const uint32_t step = p.bf16 ? (uint32_t)d.step.fetch_add(1) : 0u;
    const int D1 = p.D1 <= 0 || p.D1 > p.W ? p.W : p.D1;
    dim3 gm((unsigned)std::max<int64_t>(1, std::min<int64_t>((p.cap + 255) / 256, 2048 / world)), (unsigned)world);
    hipLaunchKernelGGL(ps_clock_mark_kernel, gm, 256, 0, stream_, p.inbox, stride, off, p.base, world,
                       reinterpret_cast<int2*>(p.rs), stamp);
    dim3 ga((unsigned)std::max<int64_t>(1, std::min<int64_t>((p.cap * 8 + 255) / 256, 8192 / world)), (unsigned)world);
    if (p.bf16)
      hipLaunchKernelGGL(ps_clock_adagrad_kernel<true>, ga, 256, 0, stream_, (void*)p.table, p.ld, p.state, p.state2,
                         D1, p.inbox, stride, off, p.cap, p.base, p.W, world, reinterpret_cast<const int2*>(p.rs),
                         stamp, p.lr, p.eps, step, p.seed);
    else
      hipLaunchKernelGGL(ps_clock_adagrad_kernel<false>, ga, 256, 0, stream_, (void*)p.table, p.ld, p.state, p.state2,
                         D1, p.inbox, stride, off, p.cap, p.base, p.W, world, reinterpret_cast<const int2*>(p.rs),
                         stamp, p.lr, p.eps, step, p.seed);
    MINIPS_HIP_CHECK(hipGetLastError());
    return;
  }
  if (d.kind == 1 && d.dn.sum && (d.dn.opt == kPsAdam || d.dn.opt == kPsAdagrad)) {
    const PsDenseDesc& p = d.dn;
    const int64_t stride = (int64_t)p.depth * p.slot_bytes, off = (c % p.depth) * p.slot_bytes;
    hipLaunchKernelGGL(ps_clock_sum_dense_kernel, grid_for(p.n / 4, 256, 4096), 256, 0, stream_, p.inbox, stride, off,
                       world, p.n / 4, p.sum, p.sum_active);
    MINIPS_HIP_CHECK(hipGetLastError());
    if (p.opt == kPsAdam) {
      // one optimizer step per clock (BSP's count), whatever the number of pushes
      const int64_t step = d.step.fetch_add(1) + 1;
      adam_apply(p.w, p.m, p.v, p.sum, p.n, p.lr, p.b1, p.b2, p.eps, p.wd, (int)step, 1.f, p.wb, stream_, nullptr,
                 false, p.sum_active);
    } else {
      adagrad_apply(p.w, p.m, p.sum, p.n, p.lr, p.eps, 1.f, p.wb, stream_, p.sum_active);
    }
    return;
  }
  Applier::ApplyClock(t, c, world);  // linear rules (add / SGD), Map storage: push by push
}

void HipApplier::Flush() { MINIPS_HIP_CHECK(hipStreamSynchronize(stream_)); }

}  // namespace minips_k
