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
//   row              k - bounds[o]  in the shard at bases[o]  ([rows_o, W] fp32, row-major)
#include <atomic>
#include <stdexcept>
#include <string>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "onesided.h"

namespace minips_k {

namespace {

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

}  // namespace

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
  MINIPS_HIP_CHECK(hipGetLastError());
}

void ps_set_headers(const int64_t* inbox, int P, int64_t slot_off, int64_t value, hipStream_t s) {
  if (P < 1 || P > kPsMaxWorld) throw std::runtime_error("ps_set_headers: P out of range");
  hipLaunchKernelGGL(ps_set_headers_kernel, 1, 64, 0, s, inbox, P, slot_off, value);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void ps_gather_rows(const int64_t* bases, const int64_t* bounds, int P, const int64_t* keys, int64_t n,
                    const int64_t* n_dev, int W, void* out, bool out_bf16, hipStream_t s) {
  if (n <= 0) return;
  if (P < 1 || P > kPsMaxWorld) throw std::runtime_error("ps_gather_rows: P out of range");
  const int block = 256;
  const bool vec = W % 4 == 0 && reinterpret_cast<uintptr_t>(out) % (out_bf16 ? 8 : 16) == 0;
  const int grid = grid_for(n * (vec ? W / 4 : W), block, 8192);
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

// ------------------------------------------------------------------------------ owner-side apply
HipApplier::HipApplier(int device, int tables) : dev_(device), descs_(tables) {
  for (auto& d : descs_) d.kind = -1;
}

HipApplier::~HipApplier() {
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
}

void HipApplier::Apply(int t, int r, int64_t c) {
  Desc& d = descs_.at(t);
  if (d.kind == 0) {
    const PsSparseDesc& p = d.sp;
    char* slot = p.inbox + ((int64_t)r * p.depth + c % p.depth) * p.slot_bytes;
    const int64_t* cnt = reinterpret_cast<const int64_t*>(slot);
    const int64_t* keys = reinterpret_cast<const int64_t*>(slot + kPsSlotHeader);
    const float* g = reinterpret_cast<const float*>(slot + kPsSlotHeader + 8 * p.cap);
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

void HipApplier::Flush() { MINIPS_HIP_CHECK(hipStreamSynchronize(stream_)); }

}  // namespace minips_k
