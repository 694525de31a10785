// Wide&Deep worker kernels: input assembly (embedding lookup + dense concat + wide sum),
// the fused output head (Linear Hd->1 + BCE-with-logits forward+backward), and the
// embedding-gradient scatter into the per-unique-key gradient rows that are pushed to the
// owning server shards.
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "common.h"
#include "kernels.h"

namespace minips_k {

// One thread per (sample, 8-column chunk): a 16-byte store of 8 bf16; threads past the
// chunks compute the per-sample wide sums (one thread per sample) so no thread serialises.
__global__ void wd_assemble_kernel(const float* __restrict__ dense, int n_dense, const bf16_t* __restrict__ rows,
                                   int row_stride, const int64_t* __restrict__ inv, int64_t B, int F, int D,
                                   bf16_t* __restrict__ X, int ldx, float* __restrict__ wide_logit, int ones_col,
                                   float* __restrict__ zero_out) {
  if (zero_out && blockIdx.x == 0 && threadIdx.x == 0) *zero_out = 0.f;
  const int chunks = ldx >> 3;
  const int emb_cols = F * D;
  const int64_t total = B * chunks;
  // items [0, total): 8-column chunks of X; items [total, total + 32B): (sample, feature lane)
  // pairs of the wide sum -- 32 lanes per sample load their features' wide weights in parallel
  // and reduce with shuffles (a serial per-sample loop is 26 dependent loads). total is rounded
  // up to a multiple of 64 so a wave never mixes the two kinds of items.
  const int64_t total_r = (total + 63) & ~63ll;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total_r + 32 * B;
       c += (int64_t)gridDim.x * blockDim.x) {
    if (c >= total_r) {
      const int64_t k = c - total_r, b = k >> 5;
      const int f = (int)(k & 31);
      float w = f < F ? bf2f(rows[inv[b * F + f] * row_stride + D]) : 0.f;
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) w += __shfl_xor(w, o, 64);
      if (f == 0) wide_logit[b] = w;
      continue;
    }
    if (c >= total) continue;
    const int64_t b = c / chunks;
    const int col0 = (int)(c - b * chunks) * 8;
    uint32_t packed[4];
    if (col0 + 8 <= emb_cols && (D & 7) == 0) {
      // whole chunk inside one embedding: two 8-byte loads of the pulled bf16 row
      const int f = col0 / D, d = col0 - f * D;
      const bf16_t* src = rows + inv[b * F + f] * row_stride + d;
      const uint2 lo = *reinterpret_cast<const uint2*>(src);
      const uint2 hi = *reinterpret_cast<const uint2*>(src + 4);
      packed[0] = lo.x;
      packed[1] = lo.y;
      packed[2] = hi.x;
      packed[3] = hi.y;
    } else {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = col0 + j;
        if (col < emb_cols) {
          const int f = col / D, d = col - f * D;
          v[j] = bf2f(rows[inv[b * F + f] * row_stride + d]);
        } else if (col < emb_cols + n_dense) {
          v[j] = dense[b * n_dense + (col - emb_cols)];
        } else {
          v[j] = col == ones_col ? 1.f : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) packed[j] = pack_bf2(v[2 * j], v[2 * j + 1]);
    }
    *reinterpret_cast<uint4*>(X + b * ldx + col0) = make_uint4(packed[0], packed[1], packed[2], packed[3]);
  }
}

void wd_assemble(const float* dense, int n_dense, const bf16_t* rows, int row_stride, const int64_t* inv, int64_t B,
                 int F, int D, bf16_t* X, int ldx, float* wide_logit, int ones_col, hipStream_t s, float* zero_out) {
  if (ldx % 8) throw std::runtime_error("wd_assemble: ldx must be a multiple of 8");
  if (F * D + n_dense > ldx) throw std::runtime_error("wd_assemble: ldx too small");
  if (ones_col >= ldx) throw std::runtime_error("wd_assemble: ones_col out of range");
  if (row_stride % 4) throw std::runtime_error("wd_assemble: row_stride must be a multiple of 4");
  if (B <= 0) return;
  const int block = 256;
  if (F > 32) throw std::runtime_error("wd_assemble: at most 32 features");
  // every thread must take the same number of grid-stride steps through the wide-sum items (their
  // shuffles need all 32 lanes of a sample): size the grid so the loop runs exactly once
  const int64_t items = ((B * (ldx / 8) + 63) & ~63ll) + 32 * B;
  hipLaunchKernelGGL(wd_assemble_kernel, (int)((items + block - 1) / block), block, 0, s, dense, n_dense, rows,
                     row_stride, inv, B, F, D, X, ldx, wide_logit, ones_col, zero_out);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// wd_assemble straight from the fp32 table shard (one rank: the Get's row gather folded in): the
// row of lookup (b, f) is tab[uniq[inv[b*F + f]] - base], converted to bf16 exactly as the gather
// kernel does (pack_bf2), so X is bit-identical to gather_rows + wd_assemble. Saves the gathered
// [U, W] bf16 rows' write + re-read and one launch; repeated hot rows hit in L2 / MALL.
__global__ void wd_assemble_tab_kernel(const float* __restrict__ dense, int n_dense, const float* __restrict__ tab,
                                       int64_t tab_ld, const int64_t* __restrict__ uniq, int64_t base,
                                       const int64_t* __restrict__ inv, int64_t B, int F, int D,
                                       bf16_t* __restrict__ X, int ldx, float* __restrict__ wide_logit, int ones_col,
                                       float* __restrict__ zero_out, const int32_t* __restrict__ rowidx) {
  if (zero_out && blockIdx.x == 0 && threadIdx.x == 0) *zero_out = 0.f;
  const int chunks = ldx >> 3;
  const int emb_cols = F * D;
  const int64_t total = B * chunks;
  const int64_t total_r = (total + 63) & ~63ll;
  // the planner's per-lookup row (one coalesced index load) or the inv -> uniq chain
  auto row_of = [&](int64_t b, int f) {
    const int64_t r = rowidx ? (int64_t)rowidx[b * F + f] : uniq[inv[b * F + f]];
    return tab + (r - base) * tab_ld;
  };
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total_r + 32 * B;
       c += (int64_t)gridDim.x * blockDim.x) {
    if (c >= total_r) {
      const int64_t k = c - total_r, b = k >> 5;
      const int f = (int)(k & 31);
      // the wide weight goes through bf16 as in the gathered path
      float w = f < F ? __uint_as_float(pack_bf2(row_of(b, f)[D], 0.f) << 16) : 0.f;
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) w += __shfl_xor(w, o, 64);
      if (f == 0) wide_logit[b] = w;
      continue;
    }
    if (c >= total) continue;
    const int64_t b = c / chunks;
    const int col0 = (int)(c - b * chunks) * 8;
    uint32_t packed[4];
    if (col0 + 8 <= emb_cols && (D & 7) == 0) {
      const int f = col0 / D, d = col0 - f * D;
      const float* src = row_of(b, f) + d;
      const float4 lo = *reinterpret_cast<const float4*>(src);
      const float4 hi = *reinterpret_cast<const float4*>(src + 4);
      packed[0] = pack_bf2(lo.x, lo.y);
      packed[1] = pack_bf2(lo.z, lo.w);
      packed[2] = pack_bf2(hi.x, hi.y);
      packed[3] = pack_bf2(hi.z, hi.w);
    } else {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = col0 + j;
        if (col < emb_cols) {
          const int f = col / D, d = col - f * D;
          v[j] = __uint_as_float(pack_bf2(row_of(b, f)[d], 0.f) << 16);
        } else if (col < emb_cols + n_dense) {
          v[j] = dense[b * n_dense + (col - emb_cols)];
        } else {
          v[j] = col == ones_col ? 1.f : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) packed[j] = pack_bf2(v[2 * j], v[2 * j + 1]);
    }
    *reinterpret_cast<uint4*>(X + b * ldx + col0) = make_uint4(packed[0], packed[1], packed[2], packed[3]);
  }
}

void wd_assemble_tab(const float* dense, int n_dense, const float* tab, int64_t tab_ld, const int64_t* uniq,
                     int64_t base, const int64_t* inv, int64_t B, int F, int D, bf16_t* X, int ldx,
                     float* wide_logit, int ones_col, hipStream_t s, float* zero_out, const int32_t* rowidx) {
  if (ldx % 8) throw std::runtime_error("wd_assemble_tab: ldx must be a multiple of 8");
  if (F * D + n_dense > ldx) throw std::runtime_error("wd_assemble_tab: ldx too small");
  if (ones_col >= ldx) throw std::runtime_error("wd_assemble_tab: ones_col out of range");
  if (tab_ld % 4 || (D & 7) || tab_ld < D + 1) throw std::runtime_error("wd_assemble_tab: 16-byte rows, D % 8 == 0");
  if (F > 32) throw std::runtime_error("wd_assemble_tab: at most 32 features");
  if (B <= 0) return;
  const int block = 256;
  // (measured: a lane-per-lookup form -- 9 x 16-byte loads of one 144-byte row per lane, a half-wave
  // per sample -- ran the W&D step 15 us slower: 26 rows per wave-instruction vs 8 here)
  const int64_t items = ((B * (ldx / 8) + 63) & ~63ll) + 32 * B;
  hipLaunchKernelGGL(wd_assemble_tab_kernel, (int)((items + block - 1) / block), block, 0, s, dense, n_dense, tab,
                     tab_ld, uniq, base, inv, B, F, D, X, ldx, wide_logit, ones_col, zero_out, rowidx);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// One wave per sample (grid-stride); each lane owns Hd/64 columns and keeps its dw / colsum
// partials in registers across all samples it visits: one atomic per lane per column at the end.
constexpr int kHeadWaves = 16;  // 1024-thread blocks: 4x the waves in flight, same atomic count
constexpr int kHeadGroup = 16, kHeadMaxGroups = 16;  // two-level fold: <= 256 blocks

// PER_LANE consecutive bf16 of a row as one vector access (8 B for 4, 16 B for 8): the
// element-wise 2-byte loads / stores cost 4-8 memory instructions per lane instead of one
template <int PER_LANE>
__device__ __forceinline__ void head_load(const bf16_t* p, float (&h)[PER_LANE]) {
  if constexpr (PER_LANE == 4) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    h[0] = __uint_as_float(u.x << 16);
    h[1] = __uint_as_float(u.x & 0xffff0000u);
    h[2] = __uint_as_float(u.y << 16);
    h[3] = __uint_as_float(u.y & 0xffff0000u);
  } else if constexpr (PER_LANE == 8) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      h[2 * q] = __uint_as_float(w[q] << 16);
      h[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
    }
  } else {
#pragma unroll
    for (int j = 0; j < PER_LANE; ++j) h[j] = bf2f(p[j]);
  }
}

// v holds bf16-exact values (already rounded): their top 16 bits are the bf16 encoding
template <int PER_LANE>
__device__ __forceinline__ void head_store(bf16_t* p, const float (&v)[PER_LANE]) {
  auto pk = [](float lo, float hi) { return (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xffff0000u); };
  if constexpr (PER_LANE == 4) {
    *reinterpret_cast<uint2*>(p) = make_uint2(pk(v[0], v[1]), pk(v[2], v[3]));
  } else if constexpr (PER_LANE == 8) {
    *reinterpret_cast<uint4*>(p) = make_uint4(pk(v[0], v[1]), pk(v[2], v[3]), pk(v[4], v[5]), pk(v[6], v[7]));
  } else {
#pragma unroll
    for (int j = 0; j < PER_LANE; ++j) p[j] = f2bf(v[j]);
  }
}

template <int PER_LANE>
__global__ __launch_bounds__(64 * kHeadWaves) void wd_head_kernel(const bf16_t* __restrict__ H, int64_t B, int Hd,
                                                      const bf16_t* __restrict__ w, const bf16_t* __restrict__ b0,
                                                      const float* __restrict__ wide, const float* __restrict__ y,
                                                      bf16_t* __restrict__ dH, float* dw, float* db, float* dwide,
                                                      float* loss_sum, float* colsum, float scale,
                                                      float* __restrict__ slab, unsigned* ticket) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  float wl[PER_LANE], dwl[PER_LANE], csl[PER_LANE];
#pragma unroll
  for (int j = 0; j < PER_LANE; ++j) {
    wl[j] = bf2f(w[lane * PER_LANE + j]);
    dwl[j] = 0.f;
    csl[j] = 0.f;
  }
  const float bias = bf2f(b0[0]);
  float dbl = 0.f, lossl = 0.f;
  // S samples per iteration: their loads and wave reductions are independent (ILP), so a wave
  // pays one L2 round trip per S samples instead of per sample.
  constexpr int S = 4;
  for (int64_t b0s = wave * S; b0s < B; b0s += nwaves * S) {
    float h[S][PER_LANE];
    float z[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int64_t b = b0s + s;
#pragma unroll
      for (int j = 0; j < PER_LANE; ++j) h[s][j] = 0.f;
      if (b < B) head_load<PER_LANE>(H + b * Hd + lane * PER_LANE, h[s]);
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < PER_LANE; ++j) acc += h[s][j] * wl[j];
      z[s] = acc;
    }
#pragma unroll
    for (int s = 0; s < S; ++s) z[s] = warp_sum(z[s]);
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int64_t b = b0s + s;
      if (b >= B) break;
      const float zz = z[s] + bias + wide[b];
      const float label = y[b] > 0.5f ? 1.f : 0.f;
      const float p = sigmoidf_(zz);
      const float dz = (p - label) * scale;
      if (lane == 0) {
        dwide[b] = dz;
        dbl += dz;
        lossl += fmaxf(zz, 0.f) - zz * label + log1pf(__expf(-fabsf(zz)));
      }
      float gv[PER_LANE];
#pragma unroll
      for (int j = 0; j < PER_LANE; ++j) {
        dwl[j] += dz * h[s][j];
        gv[j] = bf2f(f2bf(h[s][j] > 0.f ? dz * wl[j] : 0.f));
        csl[j] += gv[j];
      }
      head_store<PER_LANE>(dH + b * Hd + lane * PER_LANE, gv);
    }
  }
  // reduce the waves of the block in LDS into the block's partial row of the slab; the LAST block
  // to finish folds every partial row and adds the totals into dw / colsum / db / loss -- one
  // writer per output instead of (blocks) same-address fp32 atomics per column, which serialise
  // at the memory side (the head kernel took 24 us in the W&D step that way)
  constexpr int NC = 64 * PER_LANE, NP = 2 * NC + 2;  // a partial row: dw | colsum | db | loss
  __shared__ float red[2][kHeadWaves][NC];
  __shared__ float red_s[2][kHeadWaves];
  __shared__ int last;
  const int wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < PER_LANE; ++j) {
    red[0][wv][lane * PER_LANE + j] = dwl[j];
    red[1][wv][lane * PER_LANE + j] = csl[j];
  }
  if (lane == 0) {
    red_s[0][wv] = dbl;
    red_s[1][wv] = lossl;
  }
  __syncthreads();
  // Two-level fold of the blocks' partial rows (slab [blocks + groups][NP]), every hand-off in the
  // write-through form of cdna_hip_programming.md Guideline 16 (R1: sc1 stores, drain, relaxed
  // ticket; the reader acquires once): the last block of each group of kHeadGroup folds its
  // group's rows (kHeadGroup independent loads per column, one round trip), the last group folder
  // folds the group rows into dw / colsum / db / loss. (One last block folding all 128 rows --
  // 32 dependent round trips per column -- was most of the kernel's 27-36 us.)
  const int nb = (int)gridDim.x, ngroups = (nb + kHeadGroup - 1) / kHeadGroup;
  const int grp = blockIdx.x / kHeadGroup;
  const int g0 = grp * kHeadGroup, gn = min(kHeadGroup, nb - g0);
  float* row = slab + (int64_t)blockIdx.x * NP;
  for (int c = threadIdx.x; c < NC; c += blockDim.x) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < kHeadWaves; ++w) {
      a += red[0][w][c];
      b += red[1][w][c];
    }
    __hip_atomic_store(row + c, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(row + NC + c, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < kHeadWaves; ++w) {
      a += red_s[0][w];
      b += red_s[1][w];
    }
    __hip_atomic_store(row + 2 * NC, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(row + 2 * NC + 1, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ticket + 1 + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == (unsigned)gn - 1;
    if (last) {
      __hip_atomic_store(ticket + 1 + grp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next call
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  float* grow = slab + (int64_t)(nb + grp) * NP;  // this group's folded row
  for (int c = threadIdx.x; c < NP; c += blockDim.x) {
    float v[kHeadGroup];
#pragma unroll
    for (int k = 0; k < kHeadGroup; ++k) v[k] = k < gn ? slab[(int64_t)(g0 + k) * NP + c] : 0.f;
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < kHeadGroup; ++k) tot += v[k];
    __hip_atomic_store(grow + c, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == (unsigned)ngroups - 1;
    if (last) {
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  for (int c = threadIdx.x; c < NP; c += blockDim.x) {
    if (c >= NC && c < 2 * NC && !colsum) continue;
    float v[kHeadMaxGroups];
#pragma unroll
    for (int k = 0; k < kHeadMaxGroups; ++k) v[k] = k < ngroups ? slab[(int64_t)(nb + k) * NP + c] : 0.f;
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < kHeadMaxGroups; ++k) tot += v[k];
    if (c < NC) dw[c] += tot;
    else if (c < 2 * NC) colsum[c - NC] += tot;
    else if (c == 2 * NC) *db += tot;
    else *loss_sum += tot;
  }
}

void wd_head(const bf16_t* H, int64_t B, int Hd, const bf16_t* w, const bf16_t* b0, const float* wide_logit,
             const float* labels, bf16_t* dH, float* dw, float* db, float* dwide, float* loss_sum, float* dH_colsum,
             float grad_scale, hipStream_t s) {
  if (B <= 0) return;
  const int block = 64 * kHeadWaves;
  // per-block LDS reduction, partial rows, the last block folds them (one block per CU at most)
  // 256 blocks (every CU, one sample iteration per wave): W&D 0.3632-0.3637 vs 0.3672-0.3678 ms at
  // 128 (profiles/r4/ab_wd_knobs.txt); the two-level fold takes at most 256
  static const int max_blocks = [] {
    const char* e = std::getenv("MINIPS_HEAD_BLOCKS");
    return e ? std::atoi(e) : 256;
  }();
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(max_blocks, (B + 63) / 64));
  // the partial slab + ticket of this device: allocated once (zero ticket), before any capture
  static thread_local std::vector<std::pair<int, void*>> ws_cache;
  int dev = 0;
  MINIPS_HIP_CHECK(hipGetDevice(&dev));
  void* ws = nullptr;
  for (auto& e : ws_cache)
    if (e.first == dev) ws = e.second;
  const size_t slab_bytes = sizeof(float) * (256 + kHeadMaxGroups) * (2 * 512 + 2);
  if (!ws) {
    MINIPS_HIP_CHECK(hipMalloc(&ws, slab_bytes + 256));
    MINIPS_HIP_CHECK(hipMemset(ws, 0, slab_bytes + 256));
    ws_cache.push_back({dev, ws});
  }
  float* slab = static_cast<float*>(ws);
  unsigned* ticket = reinterpret_cast<unsigned*>(static_cast<char*>(ws) + slab_bytes);
  if (grid > 256) throw std::runtime_error("wd_head: at most 256 blocks");
  switch (Hd) {
    case 64 * 1: hipLaunchKernelGGL(wd_head_kernel<1>, grid, block, 0, s, H, B, Hd, w, b0, wide_logit, labels,
                                    dH, dw, db, dwide, loss_sum, dH_colsum, grad_scale, slab, ticket); break;
    case 64 * 2: hipLaunchKernelGGL(wd_head_kernel<2>, grid, block, 0, s, H, B, Hd, w, b0, wide_logit, labels,
                                    dH, dw, db, dwide, loss_sum, dH_colsum, grad_scale, slab, ticket); break;
    case 64 * 4: hipLaunchKernelGGL(wd_head_kernel<4>, grid, block, 0, s, H, B, Hd, w, b0, wide_logit, labels,
                                    dH, dw, db, dwide, loss_sum, dH_colsum, grad_scale, slab, ticket); break;
    case 64 * 8: hipLaunchKernelGGL(wd_head_kernel<8>, grid, block, 0, s, H, B, Hd, w, b0, wide_logit, labels,
                                    dH, dw, db, dwide, loss_sum, dH_colsum, grad_scale, slab, ticket); break;
    default: throw std::runtime_error("wd_head: Hd must be 64, 128, 256 or 512, got " + std::to_string(Hd));
  }
  MINIPS_HIP_CHECK(hipGetLastError());
}

// out[c] += sum_r x[r, c] (x bf16 [M, N] row-major, ld; N % 8 == 0): the bias gradient of a
// Linear from its output gradient. A block owns a 64-column strip and a chunk of rows; each
// thread sums 8 columns (one 16-byte load per row) over every 32nd row of the chunk, the
// block folds its 32 row-lanes in LDS and issues one atomic per column. Chunks are sized for
// ~2 blocks per CU, so a column takes only M / rows_per_block same-address atomics (fp32
// atomics from every XCD meet at the memory side: a per-wave atomic in a GEMM epilogue --
// 256 per column -- cost the W&D dgrad 44 us).
__global__ __launch_bounds__(256) void colsum_bf16_kernel(const bf16_t* __restrict__ x, int64_t M, int N, int ld,
                                                          int rows_per_block, float* __restrict__ out) {
  __shared__ float red[32][65];
  const int t = threadIdx.x, c8 = (t & 7) * 8, rl = t >> 3;
  const int col0 = blockIdx.x * 64 + c8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col0 < N) {
    for (int64_t r = r0 + rl; r < r1; r += 32) {
      const uint4 u = *reinterpret_cast<const uint4*>(x + r * ld + col0);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[2 * q] += __uint_as_float(w[q] << 16);
        acc[2 * q + 1] += __uint_as_float(w[q] & 0xffff0000u);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl][c8 + e] = acc[e];
  __syncthreads();
  if (t < 64) {
    float v = 0.f;
#pragma unroll 8
    for (int i = 0; i < 32; ++i) v += red[i][t];
    const int col = blockIdx.x * 64 + t;
    if (col < N) atomicAdd(out + col, v);
  }
}

void colsum_bf16(const bf16_t* x, int64_t M, int N, int ld, float* out, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  if (N % 8 || ld % 8) throw std::runtime_error("colsum_bf16: N and ld must be multiples of 8");
  const int strips = (N + 63) / 64;
  const int64_t chunks = std::max<int64_t>(1, std::min<int64_t>(512 / strips, (M + 255) / 256));
  const int rpb = (int)((M + chunks - 1) / chunks);
  hipLaunchKernelGGL(colsum_bf16_kernel, dim3(strips, (unsigned)chunks), 256, 0, s, x, M, N, ld, rpb, out);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// Embedding backward with block-local dedupe: a block owns TB consecutive samples of ONE
// feature, dedupes their unique-row ids in an LDS hash (compact ids by an LDS counter), sums
// the gradient vectors of duplicates with LDS float atomics, and issues ONE global atomic per
// distinct row per tile. Zipf-hot rows (e.g. a 3-value feature hit by every sample) would
// otherwise serialise thousands of same-address global atomics. Work is linearised over
// (lookup, column) so every wave-instruction touches contiguous row segments.
constexpr int kEmbTB = 256;
constexpr int kEmbHash = 512;

__device__ __forceinline__ float ld_grad(const float* p) { return *p; }
__device__ __forceinline__ float ld_grad(const bf16_t* p) { return bf2f(*p); }

template <typename TX>
__global__ __launch_bounds__(kEmbTB) void wd_emb_backward_kernel(const TX* __restrict__ dX, int ldx,
                                                                 const float* __restrict__ dwide,
                                                                 const int64_t* __restrict__ inv, int64_t B, int F,
                                                                 int D, float* __restrict__ grad_rows,
                                                                 int row_stride) {
  __shared__ int hkey[kEmbHash];
  __shared__ int hidx[kEmbHash];
  __shared__ int cidx[kEmbTB];
  __shared__ int rowof[kEmbTB];
  __shared__ int nd;
  extern __shared__ float acc[];  // [distinct][W]
  const int t = threadIdx.x;
  const int f = blockIdx.y;
  const int64_t b0 = (int64_t)blockIdx.x * kEmbTB;
  const int W = dwide ? D + 1 : D;
  const int nb = (int)min((int64_t)kEmbTB, B - b0);
  for (int j = t; j < kEmbHash; j += kEmbTB) hkey[j] = -1;
  if (t == 0) nd = 0;
  __syncthreads();
  int myslot = -1;
  bool lead = false;
  int r = -1;
  if (t < nb) {
    r = (int)inv[(b0 + t) * F + f];
    int h = (int)((uint32_t)r * 2654435761u >> 23) & (kEmbHash - 1);
    while (true) {
      const int prev = atomicCAS(hkey + h, -1, r);
      if (prev == -1) {
        lead = true;
        break;
      }
      if (prev == r) break;
      h = (h + 1) & (kEmbHash - 1);
    }
    myslot = h;
  }
  __syncthreads();
  if (lead) {
    const int id = atomicAdd(&nd, 1);
    hidx[myslot] = id;
    rowof[id] = r;
  }
  __syncthreads();
  if (t < nb) cidx[t] = hidx[myslot];
  const int ndist = nd;
  for (int i = t; i < ndist * W; i += kEmbTB) acc[i] = 0.f;
  __syncthreads();
  // deep part: element e = (lookup k, column d)
  for (int e = t; e < nb * D; e += kEmbTB) {
    const int k = e / D, d = e - k * D;
    atomicAdd(acc + cidx[k] * W + d, ld_grad(dX + (b0 + k) * ldx + (int64_t)f * D + d));
  }
  if (dwide && t < nb) atomicAdd(acc + cidx[t] * W + D, dwide[b0 + t]);
  __syncthreads();
  for (int e = t; e < ndist * W; e += kEmbTB) {
    const int k = e / W, d = e - k * W;
    atomicAdd(grad_rows + (int64_t)rowof[k] * row_stride + d, acc[e]);
  }
}

template <typename TX>
static void emb_backward(const TX* dX, int ldx, const float* dwide, const int64_t* inv, int64_t B, int F, int D,
                         float* grad_rows, int row_stride, hipStream_t s) {
  if (B <= 0) return;
  if (row_stride < D + (dwide ? 1 : 0)) throw std::runtime_error("wd_emb_backward: row_stride too small");
  const size_t lds = (size_t)kEmbTB * (D + 1) * sizeof(float);
  if (lds > 96 * 1024) throw std::runtime_error("wd_emb_backward: D too large");
  dim3 grid((unsigned)((B + kEmbTB - 1) / kEmbTB), (unsigned)F);
  hipLaunchKernelGGL(wd_emb_backward_kernel<TX>, grid, dim3(kEmbTB), lds, s, dX, ldx, dwide, inv, B, F, D, grad_rows,
                     row_stride);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void wd_emb_backward(const float* dX, int ldx, const float* dwide, const int64_t* inv, int64_t B, int F, int D,
                     float* grad_rows, int row_stride, hipStream_t s) {
  emb_backward(dX, ldx, dwide, inv, B, F, D, grad_rows, row_stride, s);
}
void wd_emb_backward_bf16(const bf16_t* dX, int ldx, const float* dwide, const int64_t* inv, int64_t B, int F, int D,
                          float* grad_rows, int row_stride, hipStream_t s) {
  emb_backward(dX, ldx, dwide, inv, B, F, D, grad_rows, row_stride, s);
}

// ---------------------------------------------------------------------------------------------
// Segment-sum embedding backward (no float atomics): the lookups are grouped by unique row in a
// CSR built from `inv`, then every unique row sums its members in registers and is written once.
//   seg_count  per (feature, 256-sample tile): LDS-hash dedupe of the tile's rows, one integer
//              atomic per distinct row per tile (hot rows see <= B/256 atomics, not B)
//   scan       exclusive prefix sum of the U counts (three coalesced passes)
//   seg_fill   same traversal; a tile reserves a contiguous range per distinct row with one
//              atomic on its cursor and drops its lookups in by their LDS rank
//   seg_sum    fixed-size pieces of the row-sorted lookups per wave (below): loads are batched so
//              a Zipf-hot row with thousands of lookups is spread over many waves instead of
//              serialising one, and only rows cut by a piece boundary need an fp32 atomic

struct TileDedupe {
  int hkey[kEmbHash];
  int hidx[kEmbHash];
  int cnt[kEmbTB];
  int rowof[kEmbTB];
  int base[kEmbTB];
  int nd;
};

// Fills the LDS dedupe of the tile; returns (via refs) this thread's row and its distinct index.
__device__ __forceinline__ void tile_dedupe(TileDedupe& T, const int64_t* __restrict__ inv, int64_t b0, int nb, int F,
                                            int f, int t, int& r, int& di, int& rank) {
  for (int j = t; j < kEmbHash; j += kEmbTB) T.hkey[j] = -1;
  if (t < kEmbTB) T.cnt[t] = 0;
  if (t == 0) T.nd = 0;
  __syncthreads();
  int slot = -1;
  bool lead = false;
  r = -1;
  if (t < nb) {
    r = (int)inv[(b0 + t) * F + f];
    int h = (int)((uint32_t)r * 2654435761u >> 23) & (kEmbHash - 1);
    while (true) {
      const int prev = atomicCAS(T.hkey + h, -1, r);
      if (prev == -1) {
        lead = true;
        break;
      }
      if (prev == r) break;
      h = (h + 1) & (kEmbHash - 1);
    }
    slot = h;
  }
  __syncthreads();
  if (lead) {
    const int id = atomicAdd(&T.nd, 1);
    T.hidx[slot] = id;
    T.rowof[id] = r;
  }
  __syncthreads();
  di = -1;
  rank = 0;
  if (t < nb) {
    di = T.hidx[slot];
    rank = atomicAdd(T.cnt + di, 1);
  }
  __syncthreads();
}

__global__ __launch_bounds__(kEmbTB) void emb_seg_count_kernel(const int64_t* __restrict__ inv, int64_t B, int F,
                                                               int* __restrict__ counts) {
  __shared__ TileDedupe T;
  const int t = threadIdx.x, f = blockIdx.y;
  const int64_t b0 = (int64_t)blockIdx.x * kEmbTB;
  const int nb = (int)min((int64_t)kEmbTB, B - b0);
  int r, di, rank;
  tile_dedupe(T, inv, b0, nb, F, f, t, r, di, rank);
  if (t < T.nd) atomicAdd(counts + T.rowof[t], T.cnt[t]);
}

// Exclusive prefix sum offsets[i] = sum(counts[0..i)), offsets[U] = total, in three coalesced
// passes over 1024-element tiles (tile sums -> scan of the tile sums -> per-tile scan + prefix).
constexpr int kScanTile = 1024;

__device__ __forceinline__ int block_excl_scan256(int v, int* sh, int* total) {
  // 256 threads: wave-level inclusive scan with shuffles, then the 4 wave totals
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  int base = 0;
  for (int i = 0; i < w; ++i) base += sh[i];
  *total = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return base + x - v;
}

__global__ __launch_bounds__(256) void emb_scan_reduce_kernel(const int* __restrict__ counts, int U,
                                                              int* __restrict__ tile_sums) {
  __shared__ int sh[4];
  const int i0 = blockIdx.x * kScanTile + threadIdx.x * 4;
  int v = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) v += (i0 + q < U) ? counts[i0 + q] : 0;
  int tot;
  block_excl_scan256(v, sh, &tot);
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void emb_scan_top_kernel(int* __restrict__ tile_sums, int ntiles) {
  __shared__ int sh[4];
  int carry = 0;
  for (int base = 0; base < ntiles; base += 256) {
    const int i = base + threadIdx.x;
    const int v = i < ntiles ? tile_sums[i] : 0;
    int tot;
    const int ex = block_excl_scan256(v, sh, &tot);
    if (i < ntiles) tile_sums[i] = carry + ex;
    carry += tot;
  }
}

__global__ __launch_bounds__(256) void emb_scan_final_kernel(const int* __restrict__ counts, int U,
                                                             const int* __restrict__ tile_prefix,
                                                             int* __restrict__ offsets) {
  __shared__ int sh[4];
  const int i0 = blockIdx.x * kScanTile + threadIdx.x * 4;
  int c[4], v = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    c[q] = (i0 + q < U) ? counts[i0 + q] : 0;
    v += c[q];
  }
  int tot;
  int run = tile_prefix[blockIdx.x] + block_excl_scan256(v, sh, &tot);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (i0 + q < U) offsets[i0 + q] = run;
    run += c[q];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 255) offsets[U] = tile_prefix[blockIdx.x] + tot;
}

__global__ __launch_bounds__(kEmbTB) void emb_seg_fill_kernel(const int64_t* __restrict__ inv, int64_t B, int F,
                                                              const int* __restrict__ offsets,
                                                              int* __restrict__ cursor, int* __restrict__ members,
                                                              int* __restrict__ memrow) {
  __shared__ TileDedupe T;
  const int t = threadIdx.x, f = blockIdx.y;
  const int64_t b0 = (int64_t)blockIdx.x * kEmbTB;
  const int nb = (int)min((int64_t)kEmbTB, B - b0);
  int r, di, rank;
  tile_dedupe(T, inv, b0, nb, F, f, t, r, di, rank);
  if (t < T.nd) T.base[t] = offsets[T.rowof[t]] + atomicAdd(cursor + T.rowof[t], T.cnt[t]);
  __syncthreads();
  if (t < nb) {
    const int pos = T.base[di] + rank;
    members[pos] = (int)((b0 + t) * F + f);  // lookup id j = b*F + f
    memrow[pos] = r;
  }
}

// Piecewise segmented sum over the row-sorted lookups: a wave owns a piece of 64/D x kSegG
// consecutive members, each D-lane group a contiguous kSegG of them, read kSegBatch at a time
// (independent loads in flight). A group flushes its running sum at every row change: a plain
// store when the row lies entirely inside the group's range, an fp32 atomic otherwise (only
// rows cut by a range boundary -- grad_rows is zero-filled first).
constexpr int kSegG = 16, kSegBatch = 8;  // defaults; MINIPS_SEG_CFG picks other (G, batch) pairs

// 4 consecutive gradient values of one lookup row segment.
__device__ __forceinline__ float4 ld_grad4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 ld_grad4(const bf16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}

template <int D>
__device__ __forceinline__ void seg_flush(float* __restrict__ grad_rows, int row_stride, int row, float4 acc,
                                          float accw, bool wide, int prev_row, int next_row, int l) {
  float* out = grad_rows + (int64_t)row * row_stride + 4 * l;
  if (row != prev_row && row != next_row) {  // the whole row lies inside this group's range
    if ((row_stride & 3) == 0)
      *reinterpret_cast<float4*>(out) = acc;  // 16-byte rows: one vector store
    else {
      out[0] = acc.x;
      out[1] = acc.y;
      out[2] = acc.z;
      out[3] = acc.w;
    }
    if (wide && l == 0) out[D] = accw;
  } else {
    atomicAdd(out + 0, acc.x);
    atomicAdd(out + 1, acc.y);
    atomicAdd(out + 2, acc.z);
    atomicAdd(out + 3, acc.w);
    if (wide && l == 0) atomicAdd(out + D, accw);
  }
}

// Piecewise segmented sum over the row-sorted lookups. A group of D/VW lanes reads one lookup's
// D values as VW-wide vectors (VW = 8: one 16-byte load of 8 bf16 per lane, 64/(D/8) lookups per
// wave-instruction; VW = 4: 8-byte loads); each group owns kSegG consecutive lookups, loaded
// kSegBatch at a time (independent loads in flight), and flushes its running sum at every row
// change: a plain store when the row lies entirely inside the group's range, fp32 atomics when
// the row continues across the range boundary (grad_rows is zero-filled first).
// SORTED: dX holds the lookups' gradient rows in member order ([total, D], row m = lookup
// members[m]): the loads become one contiguous stream and members is read only for dwide.
template <int VW>
__device__ __forceinline__ void ld_gradv(const bf16_t* p, float (&v)[VW]) {
  if constexpr (VW == 8) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[2 * e] = __uint_as_float(w[e] << 16);
      v[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
    }
  } else {
    const float4 f = ld_grad4(p);
    v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
  }
}
template <int VW>
__device__ __forceinline__ void ld_gradv(const float* p, float (&v)[VW]) {
#pragma unroll
  for (int h = 0; h < VW / 4; ++h) {
    const float4 f = *reinterpret_cast<const float4*>(p + 4 * h);
    v[4 * h] = f.x; v[4 * h + 1] = f.y; v[4 * h + 2] = f.z; v[4 * h + 3] = f.w;
  }
}

template <int D, int VW>
__device__ __forceinline__ void seg_flushv(float* __restrict__ grad_rows, int row_stride, int row,
                                           const float (&acc)[VW], float accw, bool wide, int prev_row, int next_row,
                                           int l) {
#pragma unroll
  for (int h = 0; h < VW / 4; ++h)  // the wide weight goes out with chunk 0 only
    seg_flush<D>(grad_rows, row_stride, row, make_float4(acc[4 * h], acc[4 * h + 1], acc[4 * h + 2], acc[4 * h + 3]),
                 accw, wide && h == 0, prev_row, next_row, (VW / 4) * l + h);
}

template <typename TX, int D, int kSegG, int kSegBatch, bool SORTED, int VW>
__global__ __launch_bounds__(256) void emb_seg_sum_kernel(const TX* __restrict__ dX, int ldx,
                                                          const float* __restrict__ dwide, int F,
                                                          const int* __restrict__ members,
                                                          const int* __restrict__ memrow, int total,
                                                          float* __restrict__ grad_rows, int row_stride,
                                                          int diag) {
  constexpr int L = D / VW, PER = 64 / L;
  const int lane = threadIdx.x & 63, sub = lane / L, l = lane % L;
  const bool wide = dwide != nullptr;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t piece = wave; piece * (PER * kSegG) < total; piece += nw) {
    const int a = (int)(piece * (PER * kSegG)) + sub * kSegG;
    const int b = min(total, a + kSegG);
    // diag (MINIPS_SEG_DIAG=1, timing only, wrong sums): every flush is a plain store
    const int prev_row = diag ? -2 : ((a > 0 && a <= total) ? memrow[a - 1] : -1);
    const int next_row = diag ? -2 : (b < total ? memrow[b] : -1);
    int cur = -1;
    float acc[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) acc[e] = 0.f;
    float accw = 0.f;
    for (int m0 = a; m0 < b; m0 += kSegBatch) {
      int u[kSegBatch], bb[kSegBatch];
      float v[kSegBatch][VW];
      float vw[kSegBatch];
#pragma unroll
      for (int q = 0; q < kSegBatch; ++q) {
        const int m = m0 + q;
        u[q] = m < b ? memrow[m] : -1;
        const TX* src;
        if (SORTED) {
          src = dX + (int64_t)(m < b ? m : a) * D + VW * l;
          bb[q] = (wide && l == 0 && m < b) ? members[m] / F : 0;
        } else {
          const int j = m < b ? members[m] : 0;
          bb[q] = j / F;
          const int ff = j - bb[q] * F;
          src = dX + (int64_t)bb[q] * ldx + ff * D + VW * l;
        }
        ld_gradv<VW>(src, v[q]);
        vw[q] = (wide && l == 0 && m < b) ? dwide[bb[q]] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < kSegBatch; ++q) {
        if (u[q] < 0) break;
        if (u[q] != cur) {
          if (cur >= 0) seg_flushv<D, VW>(grad_rows, row_stride, cur, acc, accw, wide, prev_row, next_row, l);
          cur = u[q];
#pragma unroll
          for (int e = 0; e < VW; ++e) acc[e] = 0.f;
          accw = 0.f;
        }
#pragma unroll
        for (int e = 0; e < VW; ++e) acc[e] += v[q][e];
        accw += vw[q];
      }
    }
    // A Zipf-hot row covers whole waves: combine the groups' partials in registers first, so a
    // hot row takes one atomic per wave instead of one per group (same-address atomics serialise
    // at the memory side).
    const int c0 = __shfl(cur, 0, 64);
    if (!diag && __all(cur == c0) && c0 >= 0) {
#pragma unroll
      for (int o = L; o < 64; o <<= 1) {
#pragma unroll
        for (int e = 0; e < VW; ++e) acc[e] += __shfl_xor(acc[e], o, 64);
        accw += __shfl_xor(accw, o, 64);
      }
      const int p0 = __shfl(prev_row, 0, 64), n1 = __shfl(next_row, 63, 64);
      if (sub == 0) seg_flushv<D, VW>(grad_rows, row_stride, c0, acc, accw, wide, p0, n1, l);
    } else if (cur >= 0) {
      seg_flushv<D, VW>(grad_rows, row_stride, cur, acc, accw, wide, prev_row, next_row, l);
    }
  }
}

// Zero rows [0, min(U, *U_dev)) of an fp32 [*, stride] matrix (float4 stores; stride % 4 == 0).
__global__ void zero_rows_dev_kernel(float* __restrict__ rows, int stride, int64_t U,
                                     const int64_t* __restrict__ U_dev) {
  const int64_t n = min(U, *U_dev) * (stride >> 2);
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x)
    reinterpret_cast<float4*>(rows)[c] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// CSR of the lookups grouped by unique row (depends on `inv` only, so the PS builds it at
// planning time, off the critical path). ws: counts[U] | cursor[U] | offsets[U+1] | tiles;
// members/memrow: [B*F] lookup ids and their rows, sorted by row.
void emb_build_csr(const int64_t* inv, int64_t B, int F, int U, int* ws, int* members, int* memrow, hipStream_t s,
                   int* zeroed_cc, bool counts_ready) {
  if (B <= 0 || U <= 0) return;
  // counts | cursor: 2U ints that must start at zero -- a caller-provided, already-zeroed block
  // (cleared by the dedupe's memset) or the head of ws
  int* counts = zeroed_cc ? zeroed_cc : ws;
  int* cursor = counts + U;
  int* offsets = zeroed_cc ? ws : cursor + U;
  int* tiles = offsets + U + 1;
  const int ntiles = (U + kScanTile - 1) / kScanTile;
  if (!zeroed_cc) MINIPS_HIP_CHECK(hipMemsetAsync(counts, 0, sizeof(int) * 2 * (size_t)U, s));
  dim3 grid((unsigned)((B + kEmbTB - 1) / kEmbTB), (unsigned)F);
  // counts_ready: the dedupe already wrote the per-row lookup counts into zeroed_cc[0, U)
  if (!(counts_ready && zeroed_cc)) hipLaunchKernelGGL(emb_seg_count_kernel, grid, dim3(kEmbTB), 0, s, inv, B,
                                                       F, counts);
  hipLaunchKernelGGL(emb_scan_reduce_kernel, ntiles, 256, 0, s, counts, U, tiles);
  hipLaunchKernelGGL(emb_scan_top_kernel, 1, 256, 0, s, tiles, ntiles);
  hipLaunchKernelGGL(emb_scan_final_kernel, ntiles, 256, 0, s, counts, U, tiles, offsets);
  hipLaunchKernelGGL(emb_seg_fill_kernel, grid, dim3(kEmbTB), 0, s, inv, B, F, offsets, cursor, members, memrow);
  MINIPS_HIP_CHECK(hipGetLastError());
}

template <typename TX>
static void emb_seg_sum(const TX* dX, int ldx, const float* dwide, int64_t B, int F, int D, const int* members,
                        const int* memrow, float* grad_rows, int row_stride, int U, hipStream_t s,
                        const int64_t* U_dev, bool sorted_rows = false, bool zeroed = false) {
  const int total = (int)(B * F);
  if (zeroed) {
    // the buffer's rows are zero already (the previous apply cleared them after reading)
  } else if (U_dev && row_stride % 4 == 0)
    hipLaunchKernelGGL(zero_rows_dev_kernel, grid_for((int64_t)U * (row_stride / 4), 256, 4096), 256, 0, s, grad_rows,
                       row_stride, (int64_t)U, U_dev);
  else
    MINIPS_HIP_CHECK(hipMemsetAsync(grad_rows, 0, sizeof(float) * (size_t)U * row_stride, s));
  static const int cfg = [] {
    const char* e = std::getenv("MINIPS_SEG_CFG");
    return e ? std::atoi(e) : 0;
  }();
  static const int diag = [] {
    const char* e = std::getenv("MINIPS_SEG_DIAG");
    return e ? std::atoi(e) : 0;
  }();
  // cfg 0: G=16 lookups per group loaded 8 at a time; 1: G=16 in one batch of 16; 2: G=8 x 8;
  // 3: G=32 x 16
  const int G = cfg == 2 ? 8 : cfg == 3 ? 32 : 16;
  // MINIPS_SEG_VEC=8: 16-byte gradient loads (8 values per lane; 16-byte aligned rows only).
  // Measured slower in the W&D step (0.436 vs 0.417 ms, profiles/r3/ab_seg_vec.txt): fewer lanes
  // per row halves the waves in flight on the latency-bound segment walk, so 8-byte loads stay
  // the default.
  static const int vec_env = [] {
    const char* e = std::getenv("MINIPS_SEG_VEC");
    return e ? std::atoi(e) : 4;
  }();
  const bool vec8 = vec_env == 8 && (sorted_rows ? true : (ldx % 8 == 0)) &&
                    reinterpret_cast<uintptr_t>(dX) % 16 == 0;
  const int VWn = vec8 ? 8 : 4;
  const int per_wave = (64 / (D / VWn)) * G;  // lookups per wave piece
  const int pieces = (total + per_wave - 1) / per_wave;
  const int blocks = std::max(1, std::min((pieces + 3) / 4, 65535));
#define MINIPS_SEG_LAUNCH3(DD, GG, BB, VV)                                                                           \
  if (sorted_rows)                                                                                                  \
    hipLaunchKernelGGL((emb_seg_sum_kernel<TX, DD, GG, BB, true, VV>), blocks, 256, 0, s, dX, ldx, dwide, F,        \
                       members, memrow, total, grad_rows, row_stride, diag);                                        \
  else                                                                                                              \
    hipLaunchKernelGGL((emb_seg_sum_kernel<TX, DD, GG, BB, false, VV>), blocks, 256, 0, s, dX, ldx, dwide, F,       \
                       members, memrow, total, grad_rows, row_stride, diag);
#define MINIPS_SEG_LAUNCH2(DD, GG, BB)       \
  if (vec8) {                               \
    MINIPS_SEG_LAUNCH3(DD, GG, BB, 8)       \
  } else {                                  \
    MINIPS_SEG_LAUNCH3(DD, GG, BB, 4)       \
  }
#define MINIPS_SEG_LAUNCH(DD)                  \
  if (cfg == 1) {                              \
    MINIPS_SEG_LAUNCH2(DD, 16, 16)             \
  } else if (cfg == 2) {                       \
    MINIPS_SEG_LAUNCH2(DD, 8, 8)               \
  } else if (cfg == 3) {                       \
    MINIPS_SEG_LAUNCH2(DD, 32, 16)             \
  } else {                                     \
    MINIPS_SEG_LAUNCH2(DD, kSegG, kSegBatch)   \
  }
  switch (D) {
    case 16:
      MINIPS_SEG_LAUNCH(16)
      break;
    case 32:
      MINIPS_SEG_LAUNCH(32)
      break;
    case 64:
      MINIPS_SEG_LAUNCH(64)
      break;
    default:
      throw std::runtime_error("emb_backward_seg: D must be 16, 32 or 64");
  }
#undef MINIPS_SEG_LAUNCH3
#undef MINIPS_SEG_LAUNCH2
#undef MINIPS_SEG_LAUNCH
  MINIPS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- fused backward + row-wise Adagrad
// One rank (the PS shard is local): the segmented sum above feeds the row-wise Adagrad apply
// directly instead of writing grad_rows [U, W] fp32 and reading it back in a second kernel
// (sparse_rowwise_adagrad), and no zero-fill of grad_rows. Same piecewise traversal (a D/4-lane
// group owns G consecutive row-sorted lookups); when a group reaches a row's first lookup it
// also loads that row's table values and Adagrad state in the same batch as the gradient loads
// (no dependent load at the flush). A row that lies entirely inside one group's range is
// updated in place at its flush; a row cut by a group boundary (Zipf-hot rows, range edges)
// is accumulated with fp32 atomics into a persistent zeroed scratch [U, scr_ld], and a second
// kernel applies it -- one thread group per group boundary that is the row's FIRST cut -- and
// clears the scratch row again. Semantics of ops.sparse_rowwise_adagrad with state2 for
// columns [D1, W): sq1 = mean over [0, D1), sq2 = mean over [D1, W) (zero pad columns count).
struct SegAdagradArgs {
  const int64_t* uniq;  // [U] unique keys (table row = key - base)
  int64_t base;
  float* table;         // [rows, ld] fp32
  int ld, W, D1;
  float* state;         // [rows]
  float* state2;        // [rows] or null (D1 == W)
  float lr, eps;
  float* scr;           // [U, scr_ld] fp32, zero outside a call
  int scr_ld;
};

// sum over the L lanes of one row group (xor partners stay inside the group: all active)
template <int L>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = 1; o < L; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Row-wise Adagrad of one row held by the L lanes of a group: acc = emb gradient columns
// [4l, 4l+4), accw = wide gradient at column D (lane 0). t/tw = the row's current values,
// st1_old/st2_old its Adagrad state (on every lane of the group).
template <int D>
__device__ __forceinline__ void seg_adagrad_apply(const SegAdagradArgs& a, int64_t row, float4 acc, float accw,
                                                  bool wide, float4 t, float tw, float st1_old, float st2_old, int l) {
  constexpr int L = D / 4;
  const float sq_e = group_sum<L>(acc.x * acc.x + acc.y * acc.y + acc.z * acc.z + acc.w * acc.w);
  const float sq_w = group_sum<L>(l == 0 ? accw * accw : 0.f);
  const bool split = a.D1 < a.W;  // D1 == D: the wide column (and the pad) has its own state
  const float st1 = st1_old + (split ? sq_e : sq_e + sq_w) / (float)a.D1;
  const float st2 = split ? st2_old + sq_w / (float)(a.W - a.D1) : 0.f;
  const float s1 = a.lr / (sqrtf(st1) + a.eps), s2 = split ? a.lr / (sqrtf(st2) + a.eps) : s1;
  float* tr = a.table + row * (int64_t)a.ld;
  *reinterpret_cast<float4*>(tr + 4 * l) =
      make_float4(t.x - s1 * acc.x, t.y - s1 * acc.y, t.z - s1 * acc.z, t.w - s1 * acc.w);
  if (l == 0) {
    if (wide) tr[D] = tw - s2 * accw;
    a.state[row] = st1;
    if (split) a.state2[row] = st2;
  }
}

template <typename TX, int D, int G, int NB>
__global__ __launch_bounds__(256) void emb_seg_adagrad_kernel(const TX* __restrict__ dX, int ldx,
                                                              const float* __restrict__ dwide, int F,
                                                              const int* __restrict__ members,
                                                              const int* __restrict__ memrow, int total,
                                                              SegAdagradArgs a) {
  constexpr int L = D / 4, PER = 64 / L;
  const int lane = threadIdx.x & 63, sub = lane / L, l = lane % L;
  const bool wide = dwide != nullptr;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t piece = wave; piece * (PER * G) < total; piece += nw) {
    const int ga = (int)(piece * (PER * G)) + sub * G;
    const int gb = min(total, ga + G);
    const int prev_row = (ga > 0 && ga <= total) ? memrow[ga - 1] : -1;
    const int next_row = gb < total ? memrow[gb] : -1;
    int cur = -1, last = prev_row;
    bool cur_has = false;
    int64_t cur_trow = 0;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f), ct = acc;
    float accw = 0.f, ctw = 0.f, cs1 = 0.f, cs2 = 0.f;
    auto flush = [&]() {
      if (cur != prev_row && cur != next_row) {  // whole row inside this group: apply now
        if (cur_has) seg_adagrad_apply<D>(a, cur_trow, acc, accw, wide, ct, ctw, cs1, cs2, l);
      } else {
        float* out = a.scr + (int64_t)cur * a.scr_ld + 4 * l;
        atomicAdd(out + 0, acc.x);
        atomicAdd(out + 1, acc.y);
        atomicAdd(out + 2, acc.z);
        atomicAdd(out + 3, acc.w);
        if (wide && l == 0) atomicAdd(a.scr + (int64_t)cur * a.scr_ld + D, accw);
      }
    };
    for (int m0 = ga; m0 < gb; m0 += NB) {
      int u[NB];
      bool st[NB];
      int64_t trow[NB];
      float4 v[NB], t[NB];
      float vw[NB], tw[NB], s1[NB], s2[NB];
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const int m = m0 + q;
        const bool ok = m < gb;
        u[q] = ok ? memrow[m] : -1;
        const int j = ok ? members[m] : 0;
        const int bb = j / F, ff = j - bb * F;
        v[q] = ok ? ld_grad4(dX + (int64_t)bb * ldx + ff * D + 4 * l) : make_float4(0.f, 0.f, 0.f, 0.f);
        vw[q] = (wide && l == 0 && ok) ? dwide[bb] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < NB; ++q) {  // the first lookup of a row in this range: its table row too
        st[q] = u[q] >= 0 && u[q] != (q == 0 ? last : u[q - 1]);
        trow[q] = st[q] ? a.uniq[u[q]] - a.base : 0;
      }
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        t[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        tw[q] = s1[q] = s2[q] = 0.f;
        if (st[q]) {
          const float* tr = a.table + trow[q] * (int64_t)a.ld;
          t[q] = *reinterpret_cast<const float4*>(tr + 4 * l);
          if (wide && l == 0) tw[q] = tr[D];
          s1[q] = a.state[trow[q]];  // every lane: each scales its own columns
          if (a.state2) s2[q] = a.state2[trow[q]];
        }
      }
      last = u[NB - 1] >= 0 ? u[NB - 1] : last;
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        if (u[q] < 0) break;
        if (u[q] != cur) {
          if (cur >= 0) flush();
          cur = u[q];
          cur_has = st[q];
          cur_trow = trow[q];
          ct = t[q];
          ctw = tw[q];
          cs1 = s1[q];
          cs2 = s2[q];
          acc = make_float4(0.f, 0.f, 0.f, 0.f);
          accw = 0.f;
        }
        acc.x += v[q].x;
        acc.y += v[q].y;
        acc.z += v[q].z;
        acc.w += v[q].w;
        accw += vw[q];
      }
    }
    // A Zipf-hot row spanning the whole wave: combine the groups' partials in registers first
    // (one atomic per wave instead of one per group: same-address atomics serialise at the
    // memory side). Such a row is cut by group boundaries, so the cut-row kernel applies it.
    const int c0 = __shfl(cur, 0, 64);
    if (__all(cur == c0) && c0 >= 0) {
#pragma unroll
      for (int o = L; o < 64; o <<= 1) {
        acc.x += __shfl_xor(acc.x, o, 64);
        acc.y += __shfl_xor(acc.y, o, 64);
        acc.z += __shfl_xor(acc.z, o, 64);
        acc.w += __shfl_xor(acc.w, o, 64);
        accw += __shfl_xor(accw, o, 64);
      }
      if (sub == 0) {
        float* out = a.scr + (int64_t)c0 * a.scr_ld + 4 * l;
        atomicAdd(out + 0, acc.x);
        atomicAdd(out + 1, acc.y);
        atomicAdd(out + 2, acc.z);
        atomicAdd(out + 3, acc.w);
        if (wide && l == 0) atomicAdd(a.scr + (int64_t)c0 * a.scr_ld + D, accw);
      }
    } else if (cur >= 0) {
      flush();
    }
  }
}

// Rows cut by a group boundary: boundary b = k*G handles the row iff the row continues across
// b and b is its first cut (the previous boundary does not cut the same row).
template <int D>
__global__ __launch_bounds__(256) void emb_cut_adagrad_kernel(const int* __restrict__ memrow, int total, int G,
                                                              bool wide, SegAdagradArgs a) {
  constexpr int L = D / 4, PER = 64 / L;
  const int lane = threadIdx.x & 63, l = lane % L;
  const int64_t nb = (total - 1) / G;  // boundaries 1..nb
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t k = 1 + wave * PER + lane / L; k <= nb; k += nw * PER) {
    const int b = (int)(k * G);
    const int u = memrow[b];
    if (memrow[b - 1] != u) continue;
    if (b - G > 0 && memrow[b - G - 1] == u) continue;
    float* sr = a.scr + (int64_t)u * a.scr_ld;
    const float4 g = *reinterpret_cast<const float4*>(sr + 4 * l);
    const float gw = (wide && l == 0) ? sr[D] : 0.f;
    *reinterpret_cast<float4*>(sr + 4 * l) = make_float4(0.f, 0.f, 0.f, 0.f);  // scratch clean for the next call
    if (wide && l == 0) sr[D] = 0.f;
    const int64_t row = a.uniq[u] - a.base;
    const float* tr = a.table + row * (int64_t)a.ld;
    const float4 t = *reinterpret_cast<const float4*>(tr + 4 * l);
    const float tw = (wide && l == 0) ? tr[D] : 0.f;
    const float s1 = a.state[row];
    const float s2 = a.state2 ? a.state2[row] : 0.f;
    seg_adagrad_apply<D>(a, row, g, gw, wide, t, tw, s1, s2, l);
  }
}

// ---------------------------------------------------------------- row-parallel backward + Adagrad
// One rank, row-sorted gradient rows (the dgrad GEMM's permuted-rows epilogue writes dX[m] = the
// gradient of lookup members[m], rows grouped by unique row u): row u's lookups are the contiguous
// rows [rowstart[u], rowstart[u + 1]) of dX. Instead of cutting the lookup stream into fixed pieces
// (emb_seg_sum / emb_seg_adagrad: a data-dependent flush per row change and fp32 atomics on every
// row cut by a piece boundary -- 0.9 TB/s, plus a zero-filled grad_rows buffer read back by the
// Adagrad kernel), each ROW is one unit of work:
//   cold rows (<= hot lookups, nearly all of them): a group of D/8 lanes sums the row's lookups
//     with 16-byte bf16 loads (4 lookups in flight per lane), its table row and Adagrad state are
//     loaded before the sum (independent of it), and the update is written in place -- no
//     intermediate buffer, no atomics, each row touched once;
//   hot rows (Zipf heads: up to thousands of lookups) are appended to a list (one atomic per hot
//   row) and summed by a whole workgroup each (64 lane groups + an LDS reduction), so no wave
//   waits on a row thousands of lookups long.
// Semantics of ops.sparse_rowwise_adagrad with state2 for columns [D1, W) (the wide weight + pad).
struct RowsAdagradArgs {
  const int64_t* uniq;
  int64_t base;
  float* table;
  int ld, W, D1;
  float* state;
  float* state2;
  float lr, eps;
};

__device__ __forceinline__ void acc_bf16x8(float (&acc)[8], uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    acc[2 * e] += __uint_as_float(w[e] << 16);
    acc[2 * e + 1] += __uint_as_float(w[e] & 0xffff0000u);
  }
}

// new values of this lane's 8 deep columns (t0, t1) and of the wide column (lane 0 of the group)
template <int L>
__device__ __forceinline__ void rows_apply(const RowsAdagradArgs& a, int64_t trow, const float (&g)[8], float gw,
                                           bool wide, float4 t0, float4 t1, float tw, float st1_old, float st2_old,
                                           int l, int D) {
  float sq = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) sq += g[e] * g[e];
  sq = group_sum<L>(sq);
  const float sqw = group_sum<L>(l == 0 ? gw * gw : 0.f);
  const bool split = a.D1 < a.W;
  const float st1 = st1_old + (split ? sq : sq + sqw) / (float)a.D1;
  const float st2 = split ? st2_old + sqw / (float)(a.W - a.D1) : 0.f;
  const float s1 = a.lr / (sqrtf(st1) + a.eps), s2 = split ? a.lr / (sqrtf(st2) + a.eps) : s1;
  float* tr = a.table + trow * (int64_t)a.ld + 8 * l;
  reinterpret_cast<float4*>(tr)[0] =
      make_float4(t0.x - s1 * g[0], t0.y - s1 * g[1], t0.z - s1 * g[2], t0.w - s1 * g[3]);
  reinterpret_cast<float4*>(tr)[1] =
      make_float4(t1.x - s1 * g[4], t1.y - s1 * g[5], t1.z - s1 * g[6], t1.w - s1 * g[7]);
  if (l == 0) {
    if (wide) a.table[trow * (int64_t)a.ld + D] = tw - s2 * gw;
    a.state[trow] = st1;
    if (split) a.state2[trow] = st2;
  }
}

// the gradient row of member m (lookup j = members[m]): row-sorted (ldx == 0) or lookup order
template <int D>
__device__ __forceinline__ const bf16_t* grad_row(const bf16_t* dX, int ldx, int F, int m, int j) {
  if (ldx == 0) return dX + (int64_t)m * D;
  const int b = j / F;
  return dX + (int64_t)b * ldx + (j - b * F) * D;
}

template <int D>
__global__ __launch_bounds__(256) void emb_rows_adagrad_kernel(const bf16_t* __restrict__ dX, int ldx,
                                                               const float* __restrict__ dwide, int F,
                                                               const int* __restrict__ members,
                                                               const int* __restrict__ rowstart,
                                                               const int64_t* __restrict__ U_dev, int64_t U_max,
                                                               RowsAdagradArgs a, int* __restrict__ ws,
                                                               int hmax, int hot) {
  constexpr int L = D / 8, PER = 64 / L, CHW = 8 * (256 / L);
  int* cnt = ws;  // {hot rows, chunks, hot-kernel block ticket}
  int* hot_row = ws + 4;
  int* hot_need = hot_row + hmax;
  int2* chunk = reinterpret_cast<int2*>(hot_need + hmax + (hmax & 1));
  const int lane = threadIdx.x & 63, sub = lane / L, l = lane % L;
  const bool wide = dwide != nullptr;
  const int64_t U = min(U_max, *U_dev);
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t u0 = wave * PER; u0 < U; u0 += nw * PER) {
    const int64_t u = u0 + sub;
    const bool ok = u < U;
    const int s = ok ? rowstart[u] : 0, e = ok ? rowstart[u + 1] : 0;
    const bool cold = ok && e - s <= hot;
    if (ok && !cold && l == 0) {  // a hot row: its chunks go to emb_hot_adagrad_kernel
      const int h = atomicAdd(cnt, 1), nc = (e - s + CHW - 1) / CHW;
      const int c0 = atomicAdd(cnt + 1, nc);
      hot_row[h] = (int)u;
      hot_need[h] = nc;
      for (int k = 0; k < nc; ++k) chunk[c0 + k] = make_int2(h, k);
    }
    // the row's current values and state: independent of the sum, loaded ahead of it
    const int64_t trow = cold ? a.uniq[u] - a.base : 0;
    float4 t0 = make_float4(0.f, 0.f, 0.f, 0.f), t1 = t0;
    float tw = 0.f, st1 = 0.f, st2 = 0.f;
    if (cold) {
      const float* tr = a.table + trow * (int64_t)a.ld + 8 * l;
      t0 = reinterpret_cast<const float4*>(tr)[0];
      t1 = reinterpret_cast<const float4*>(tr)[1];
      if (wide && l == 0) tw = a.table[trow * (int64_t)a.ld + D];
      st1 = a.state[trow];
      if (a.state2) st2 = a.state2[trow];
    }
    float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float gw = 0.f;
    const int end = cold ? e : s;
    if (ldx != 0 && hot <= 32) {
      // lookup order: the group's lanes fetch the row's member list cooperatively (one round
      // trip), then every lookup's j comes by a lane shuffle and its gradient slice loads 8 at a
      // time -- 2 + cnt / 8 dependent round trips instead of 2 per 4 lookups
      constexpr int MK = (32 + L - 1) / L;
      const int cnt = end - s, gbase = lane - l;
      int mj[MK];
#pragma unroll
      for (int k = 0; k < MK; ++k) {
        const int q = l + L * k;
        mj[k] = q < cnt ? members[s + q] : 0;
      }
#pragma unroll
      for (int q0 = 0; q0 < 32; q0 += 8) {
        uint4 v[8];
        float w[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int q = q0 + i;
          const int j = __shfl(mj[q / L], gbase + q % L, 64);
          const bool in = q < cnt;
          const int b = j / F;
          v[i] = in ? *reinterpret_cast<const uint4*>(dX + (int64_t)b * ldx + (j - b * F) * D + 8 * l)
                    : make_uint4(0, 0, 0, 0);
          w[i] = (wide && l == 0 && in) ? dwide[b] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          acc_bf16x8(g, v[i]);
          gw += w[i];
        }
      }
    } else {
      for (int m = s; m < end; m += 4) {
        uint4 v[4];
        float w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int mm = m + q;
          const bool in = mm < end;
          const int j = (in && (ldx || wide)) ? members[mm] : 0;
          v[q] = in ? *reinterpret_cast<const uint4*>(grad_row<D>(dX, ldx, F, mm, j) + 8 * l) : make_uint4(0, 0, 0, 0);
          w[q] = (wide && l == 0 && in) ? dwide[j / F] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc_bf16x8(g, v[q]);
          gw += w[q];
        }
      }
    }
    if (cold) rows_apply<L>(a, trow, g, gw, wide, t0, t1, tw, st1, st2, l, D);
  }
}

// Hot rows in workgroup chunks of G * 8 lookups (G = 256 / L lane groups, 8 loads in flight per
// lane): a chunk folds in LDS; a row of one chunk is applied by that workgroup, a longer row's
// chunks add their partial rows into hot_acc (memory-side fp32 atomics, one per column per chunk:
// a row thousands of lookups long costs ~10 atomics per address, not thousands) and draw a ticket;
// the row's last chunk applies (agent-scope acquire, then the sums) and re-zeroes hot_acc / the
// ticket for the next call. The cold kernel wrote the chunk list: ws = {hot rows, chunks, block
// ticket, pad, hot_row [Hmax], hot_need [Hmax], chunk (hot index, chunk index) [Cmax]}; the hot
// kernel's last block re-zeroes the counters.
template <int D>
__device__ __forceinline__ void hot_apply(const RowsAdagradArgs& a, int64_t trow, int t, float v, float vw,
                                          bool wide) {
  const float sq = warp_sum(t < D ? v * v : 0.f);
  const float sqw = wide ? vw * vw : 0.f;
  const bool split = a.D1 < a.W;
  const float st1 = a.state[trow] + (split ? sq : sq + sqw) / (float)a.D1;
  const float st2 = split ? a.state2[trow] + sqw / (float)(a.W - a.D1) : 0.f;
  const float s1 = a.lr / (sqrtf(st1) + a.eps), s2 = split ? a.lr / (sqrtf(st2) + a.eps) : s1;
  float* tr = a.table + trow * (int64_t)a.ld;
  if (t < D) tr[t] -= s1 * v;
  if (t == 0 && wide) tr[D] -= s2 * vw;
  if (t == 0) {
    a.state[trow] = st1;
    if (split) a.state2[trow] = st2;
  }
}

template <int D>
__global__ __launch_bounds__(256) void emb_hot_adagrad_kernel(const bf16_t* __restrict__ dX, int ldx,
                                                              const float* __restrict__ dwide, int F,
                                                              const int* __restrict__ members,
                                                              const int* __restrict__ rowstart, RowsAdagradArgs a,
                                                              int* __restrict__ ws, int hmax,
                                                              float* __restrict__ hot_acc,
                                                              unsigned* __restrict__ hot_tick) {
  constexpr int L = D / 8, G = 256 / L, CHW = 8 * G;
  __shared__ float red[G][D + 1];
  const int t = threadIdx.x, g = t / L, l = t % L;
  const bool wide = dwide != nullptr;
  const int* hot_row = ws + 4;
  const int* hot_need = hot_row + hmax;
  const int2* chunk = reinterpret_cast<const int2*>(hot_need + hmax);
  const int nch = ws[1];
  for (int c = blockIdx.x; c < nch; c += gridDim.x) {
    const int2 hk = chunk[c];
    const int u = hot_row[hk.x], need = hot_need[hk.x];
    const int s = rowstart[u] + hk.y * CHW, e = min(rowstart[u + 1], s + CHW);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float accw = 0.f;
    int jj[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int m = s + g + q * G;
      jj[q] = (m < e && (ldx || wide)) ? members[m] : 0;
    }
    uint4 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int m = s + g + q * G;
      v[q] = m < e ? *reinterpret_cast<const uint4*>(grad_row<D>(dX, ldx, F, m, jj[q]) + 8 * l)
                   : make_uint4(0, 0, 0, 0);
      if (wide && l == 0 && m < e) accw += dwide[jj[q] / F];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) acc_bf16x8(acc, v[q]);
#pragma unroll
    for (int q = 0; q < 8; ++q) red[g][8 * l + q] = acc[q];
    if (l == 0) red[g][D] = accw;
    __syncthreads();
    if (t < 64) {  // wave 0: lane c < D folds column c, lane 0 also the wide column
      float vv = 0.f, vw = 0.f;
      if (t < D)
        for (int k = 0; k < G; ++k) vv += red[k][t];
      if (t == 0 && wide)
        for (int k = 0; k < G; ++k) vw += red[k][D];
      const int64_t trow = a.uniq[u] - a.base;
      if (need == 1) {
        hot_apply<D>(a, trow, t, vv, __shfl(vw, 0, 64), wide);
      } else {
        float* ha = hot_acc + (int64_t)hk.x * (D + 1);
        if (t < D) atomicAdd(ha + t, vv);
        if (t == 0 && wide) atomicAdd(ha + D, vw);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's adds performed before its ticket
        unsigned last = 0;
        if (t == 0) {
          last = __hip_atomic_fetch_add(hot_tick + hk.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                 (unsigned)need - 1;
          if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
        }
        last = __shfl(last, 0, 64);
        if (last) {  // every chunk of the row has added: its sum is complete
          const float sv = t < D ? __hip_atomic_load(ha + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
          const float sw = wide ? __hip_atomic_load(ha + D, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
          hot_apply<D>(a, trow, t, sv, sw, wide);
          if (t < D) __hip_atomic_store(ha + t, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (t == 0) {
            if (wide) __hip_atomic_store(ha + D, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(hot_tick + hk.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
    }
    __syncthreads();  // red is reused by the next chunk
  }
  // the last block to finish zeroes the counters for the next call (every block read them at its
  // start): no memset node in front of every call (7 us of queue time per W&D step), graph-safe
  if (t == 0 && atomicAdd(ws + 2, 1) == (int)gridDim.x - 1) {
    ws[0] = 0;
    ws[1] = 0;
    ws[2] = 0;
  }
}

// hot-row capacities of emb_rows_adagrad for n lookups and threshold hot: rows with more than
// `hot` lookups (Hmax) and their chunks (Cmax)
static inline void rows_hot_caps(int64_t n, int hot, int D, int64_t& hmax, int64_t& cmax) {
  const int chw = 8 * (256 / (D / 8));
  hmax = n / (hot + 1) + 1;
  cmax = hmax + n / chw + 1;
}

int64_t emb_rows_ws_ints(int64_t n, int hot, int D) {
  int64_t hmax, cmax;
  rows_hot_caps(n, hot, D, hmax, cmax);
  return 4 + 2 * hmax + 2 * cmax;
}

int64_t emb_rows_hot_rows(int64_t n, int hot, int D) {
  int64_t hmax, cmax;
  rows_hot_caps(n, hot, D, hmax, cmax);
  return hmax;
}

void emb_rows_adagrad(const bf16_t* dX, int ldx, const float* dwide, int F, int D, const int* members,
                      const int* rowstart, const int64_t* U_dev, int64_t U_max, const int64_t* uniq, int64_t base,
                      float* table, int ld, int W, float* state, float* state2, int D1, float lr, float eps,
                      int* ws, float* hot_acc, unsigned* hot_tick, int hot, hipStream_t s) {
  if (U_max <= 0) return;
  if (ld % 4 || reinterpret_cast<uintptr_t>(table) % 16 || reinterpret_cast<uintptr_t>(dX) % 16 || ldx % 8)
    throw std::runtime_error("emb_rows_adagrad: 16-byte aligned rows");
  if (D1 <= 0 || D1 > W) D1 = W;
  if (D1 < W && !state2) throw std::runtime_error("emb_rows_adagrad: split rows need state2");
  if (D != 16 && D != 32 && D != 64) throw std::runtime_error("emb_rows_adagrad: D must be 16, 32 or 64");
  int64_t hmax, cmax;
  rows_hot_caps(U_max, hot, D, hmax, cmax);  // U_max = the lookups (rowstart has n + 1 entries)
  const RowsAdagradArgs a{uniq, base, table, ld, W, D1, state, state2, lr, eps};
  const int per_block = 4 * (64 / (D / 8));
  const int grid = (int)std::min<int64_t>((U_max + per_block - 1) / per_block, 8192);
  const int hgrid = (int)std::min<int64_t>(cmax, 2048);
#define MINIPS_ROWS_ADA(DD)                                                                                      \
  hipLaunchKernelGGL((emb_rows_adagrad_kernel<DD>), grid, 256, 0, s, dX, ldx, dwide, F, members, rowstart,     \
                     U_dev, U_max, a, ws, (int)hmax, hot);                                                        \
  hipLaunchKernelGGL((emb_hot_adagrad_kernel<DD>), hgrid, 256, 0, s, dX, ldx, dwide, F, members, rowstart, a, ws, \
                     (int)hmax, hot_acc, hot_tick);
  switch (D) {
    case 16:
      MINIPS_ROWS_ADA(16)
      break;
    case 32:
      MINIPS_ROWS_ADA(32)
      break;
    default:
      MINIPS_ROWS_ADA(64)
      break;
  }
#undef MINIPS_ROWS_ADA
  MINIPS_HIP_CHECK(hipGetLastError());
}

void emb_seg_adagrad(const void* dX, bool bf16, int ldx, const float* dwide, int64_t B, int F, int D,
                     const int* members, const int* memrow, const int64_t* uniq, int64_t base, float* table, int ld,
                     int W, float* state, float* state2, int D1, float lr, float eps, float* scr, int scr_ld,
                     hipStream_t s) {
  const int total = (int)(B * F);
  if (total <= 0) return;
  const SegAdagradArgs a{uniq, base, table, ld, W, D1, state, state2, lr, eps, scr, scr_ld};
  static const int nb_cfg = [] {
    const char* e = std::getenv("MINIPS_SEGADA_NB");
    return e ? std::atoi(e) : 4;  // W&D step: NB 4 0.473, 8 0.487, 16 0.515 ms (unfused 0.465)
  }();
  constexpr int G = 16;
  const int pieces = (total + (256 / D) * G - 1) / ((256 / D) * G);
  const int blocks = std::max(1, std::min((pieces + 3) / 4, 65535));
  const int64_t nbound = (total - 1) / G;
  const int cut_blocks = (int)std::max<int64_t>(1, std::min<int64_t>((nbound * (D / 4) + 255) / 256, 65535));
#define MINIPS_SEGADA(DD)                                                                                       \
  if (bf16 && nb_cfg == 16)                                                                                     \
    hipLaunchKernelGGL((emb_seg_adagrad_kernel<bf16_t, DD, G, 16>), blocks, 256, 0, s,                          \
                       static_cast<const bf16_t*>(dX), ldx, dwide, F, members, memrow, total, a);              \
  else if (bf16 && nb_cfg == 4)                                                                                 \
    hipLaunchKernelGGL((emb_seg_adagrad_kernel<bf16_t, DD, G, 4>), blocks, 256, 0, s,                           \
                       static_cast<const bf16_t*>(dX), ldx, dwide, F, members, memrow, total, a);              \
  else if (bf16)                                                                                                \
    hipLaunchKernelGGL((emb_seg_adagrad_kernel<bf16_t, DD, G, 8>), blocks, 256, 0, s,                           \
                       static_cast<const bf16_t*>(dX), ldx, dwide, F, members, memrow, total, a);              \
  else                                                                                                          \
    hipLaunchKernelGGL((emb_seg_adagrad_kernel<float, DD, G, 8>), blocks, 256, 0, s,                           \
                       static_cast<const float*>(dX), ldx, dwide, F, members, memrow, total, a);               \
  if (nbound > 0)                                                                                               \
    hipLaunchKernelGGL((emb_cut_adagrad_kernel<DD>), cut_blocks, 256, 0, s, memrow, total, G, dwide != nullptr, a);
  switch (D) {
    case 16:
      MINIPS_SEGADA(16)
      break;
    case 32:
      MINIPS_SEGADA(32)
      break;
    case 64:
      MINIPS_SEGADA(64)
      break;
    default:
      throw std::runtime_error("emb_seg_adagrad: D must be 16, 32 or 64");
  }
#undef MINIPS_SEGADA
  MINIPS_HIP_CHECK(hipGetLastError());
}

void emb_backward_csr(const void* dX, bool bf16, int ldx, const float* dwide, int64_t B, int F, int D,
                      const int* members, const int* memrow, float* grad_rows, int row_stride, int U, hipStream_t s,
                      const int64_t* U_dev, bool sorted_rows, bool zeroed) {
  if (B <= 0 || U <= 0) return;
  if (row_stride < D + (dwide ? 1 : 0)) throw std::runtime_error("emb_backward_csr: row_stride too small");
  if (bf16)
    emb_seg_sum(static_cast<const bf16_t*>(dX), ldx, dwide, B, F, D, members, memrow, grad_rows, row_stride, U, s,
                U_dev, sorted_rows, zeroed);
  else
    emb_seg_sum(static_cast<const float*>(dX), ldx, dwide, B, F, D, members, memrow, grad_rows, row_stride, U, s,
                U_dev, sorted_rows, zeroed);
}

__global__ void emb_csr_positions_kernel(const int* __restrict__ members, int64_t n, int* __restrict__ pos) {
  for (int64_t m = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; m < n; m += (int64_t)gridDim.x * blockDim.x)
    pos[members[m]] = (int)m;
}

void emb_csr_positions(const int* members, int64_t n, int* pos, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(emb_csr_positions_kernel, grid_for(n, 256, 4096), 256, 0, s, members, n, pos);
  MINIPS_HIP_CHECK(hipGetLastError());
}

void emb_backward_segment(const void* dX, bool bf16, int ldx, const float* dwide, const int64_t* inv, int64_t B, int F,
                          int D, float* grad_rows, int row_stride, int U, int* ws, hipStream_t s,
                          const int64_t* U_dev) {
  if (B <= 0 || U <= 0) return;
  // ws: counts[U] | cursor[U] | offsets[U+1] | tiles[U/1024+1] | members[B*F] | memrow[B*F]
  int* members = ws + 3 * U + 1 + (U / 1024 + 1);
  int* memrow = members + B * F;
  emb_build_csr(inv, B, F, U, ws, members, memrow, s);
  emb_backward_csr(dX, bf16, ldx, dwide, B, F, D, members, memrow, grad_rows, row_stride, U, s, U_dev);
}

}  // namespace minips_k
