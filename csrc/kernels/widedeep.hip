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
                                                      float* __restrict__ slab, unsigned* ticket, int defer) {
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
    float z[S], wv[S], yv[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int64_t b = b0s + s;
      // the wide logit and label load with the row (not after the wave reduction: one round trip)
      wv[s] = b < B ? wide[b] : 0.f;
      yv[s] = b < B ? y[b] : 0.f;
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
      const float zz = z[s] + bias + wv[s];
      const float label = yv[s] > 0.5f ? 1.f : 0.f;
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
  if (defer) {  // wd_head_fold (a later kernel, off the dgrad chain) folds the partial rows
    for (int c = threadIdx.x; c < NC; c += blockDim.x) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w = 0; w < kHeadWaves; ++w) {
        a += red[0][w][c];
        b += red[1][w][c];
      }
      row[c] = a;
      row[NC + c] = b;
    }
    if (threadIdx.x == 0) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w = 0; w < kHeadWaves; ++w) {
        a += red_s[0][w];
        b += red_s[1][w];
      }
      row[2 * NC] = a;
      row[2 * NC + 1] = b;
    }
    return;
  }
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

// The deferred fold of wd_head's per-block partial rows (slab [nb][2*NC + 2]) into dw / colsum /
// db / loss: a block owns 32 columns, its 16 row chunks each sum their rows in order, then chunk
// order in LDS -- one fixed summation order (deterministic). Issued on the weight-gradient stream
// right behind the head, it takes the two ticketed fold levels (~8 us of the head's ~17, the last
// blocks waiting on each other's write-through round trips) off the dgrad chain.
constexpr int kFoldCols = 32, kFoldChunks = 16;
__global__ __launch_bounds__(kFoldCols * kFoldChunks) void wd_head_fold_kernel(const float* __restrict__ slab,
                                                                               int nb, int NC, float* dw,
                                                                               float* colsum, float* db,
                                                                               float* loss_sum) {
  __shared__ float red[kFoldChunks][kFoldCols + 1];
  const int NP = 2 * NC + 2;
  const int cl = threadIdx.x % kFoldCols, ch = threadIdx.x / kFoldCols;
  const int c = blockIdx.x * kFoldCols + cl;
  const int per = (nb + kFoldChunks - 1) / kFoldChunks;
  const int r0 = ch * per, r1 = min(nb, r0 + per);
  float acc = 0.f;
  if (c < NP) {
    for (int r = r0; r < r1; r += 8) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = r + k < r1 ? slab[(int64_t)(r + k) * NP + c] : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += v[k];
    }
  }
  red[ch][cl] = acc;
  __syncthreads();
  if (ch != 0 || c >= NP) return;
  float tot = 0.f;
#pragma unroll
  for (int k = 0; k < kFoldChunks; ++k) tot += red[k][cl];
  if (c < NC) dw[c] += tot;
  else if (c < 2 * NC) {
    if (colsum) colsum[c - NC] += tot;
  } else if (c == 2 * NC) *db += tot;
  else *loss_sum += tot;
}

namespace {
// 256 blocks (every CU, one sample iteration per wave): W&D 0.3632-0.3637 vs 0.3672-0.3678 ms at
// 128 (profiles/r4/ab_wd_knobs.txt); the two-level fold takes at most 256
int head_grid(int64_t B) { return (int)std::max<int64_t>(1, std::min<int64_t>(256, (B + 63) / 64)); }

// the partial slab + ticket of this device: allocated once (zero ticket), before any capture
void head_ws(float** slab, unsigned** ticket) {
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
  *slab = static_cast<float*>(ws);
  *ticket = reinterpret_cast<unsigned*>(static_cast<char*>(ws) + slab_bytes);
}
}  // namespace

void wd_head(const bf16_t* H, int64_t B, int Hd, const bf16_t* w, const bf16_t* b0, const float* wide_logit,
             const float* labels, bf16_t* dH, float* dw, float* db, float* dwide, float* loss_sum, float* dH_colsum,
             float grad_scale, hipStream_t s, bool defer_fold) {
  if (B <= 0) return;
  const int block = 64 * kHeadWaves;
  // per-block LDS reduction, partial rows; the last block folds them (one block per CU at most),
  // or wd_head_fold does (defer_fold)
  const int grid = head_grid(B), defer = defer_fold ? 1 : 0;
  float* slab = nullptr;
  unsigned* ticket = nullptr;
  head_ws(&slab, &ticket);
  switch (Hd) {
    case 64 * 1: hipLaunchKernelGGL(wd_head_kernel<1>, grid, block, 0, s, H, B, Hd, w, b0, wide_logit, labels,
                                    dH, dw, db, dwide, loss_sum, dH_colsum, grad_scale, slab, ticket, defer); break;
    case 64 * 2: hipLaunchKernelGGL(wd_head_kernel<2>, grid, block, 0, s, H, B, Hd, w, b0, wide_logit, labels,
                                    dH, dw, db, dwide, loss_sum, dH_colsum, grad_scale, slab, ticket, defer); break;
    case 64 * 4: hipLaunchKernelGGL(wd_head_kernel<4>, grid, block, 0, s, H, B, Hd, w, b0, wide_logit, labels,
                                    dH, dw, db, dwide, loss_sum, dH_colsum, grad_scale, slab, ticket, defer); break;
    case 64 * 8: hipLaunchKernelGGL(wd_head_kernel<8>, grid, block, 0, s, H, B, Hd, w, b0, wide_logit, labels,
                                    dH, dw, db, dwide, loss_sum, dH_colsum, grad_scale, slab, ticket, defer); break;
    default: throw std::runtime_error("wd_head: Hd must be 64, 128, 256 or 512, got " + std::to_string(Hd));
  }
  MINIPS_HIP_CHECK(hipGetLastError());
}

void wd_head_fold(int64_t B, int Hd, float* dw, float* db, float* loss_sum, float* dH_colsum, hipStream_t s) {
  if (B <= 0) return;
  if (Hd != 64 && Hd != 128 && Hd != 256 && Hd != 512)
    throw std::runtime_error("wd_head_fold: Hd must be 64, 128, 256 or 512, got " + std::to_string(Hd));
  float* slab = nullptr;
  unsigned* ticket = nullptr;
  head_ws(&slab, &ticket);
  const int NP = 2 * Hd + 2;
  hipLaunchKernelGGL(wd_head_fold_kernel, (NP + kFoldCols - 1) / kFoldCols, kFoldCols * kFoldChunks, 0, s, slab,
                     head_grid(B), Hd, dw, dH_colsum, db, loss_sum);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// out[c] += sum_r x[r, c] (x bf16 [M, N] row-major, ld; N % 8 == 0): the bias gradient of a
// Linear from its output gradient. Two kernels, one fixed summation order (deterministic, unlike
// one same-address fp32 atomic per block and column): a block owns a 64-column strip and a chunk
// of rows -- each thread sums 8 columns (one 16-byte load per row) over every 32nd row of the
// chunk, the block folds its 32 row-lanes in LDS and writes its partial row; then one small block
// per strip adds the strip's partial rows in chunk order into out. (A last-arriver fold inside the
// first kernel kept every block alive for a ticket round trip: 16 vs 9 us beside the W&D dgrad.)
__global__ __launch_bounds__(256) void colsum_bf16_kernel(const bf16_t* __restrict__ x, int64_t M, int N, int ld,
                                                          int rows_per_block, float* __restrict__ slab) {
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
    slab[((int64_t)blockIdx.x * gridDim.y + blockIdx.y) * 64 + t] = v;
  }
}

// strip s (a 256-thread block): thread (q, c) sums chunks q, q + 4, ... of column c (8 loads in
// flight), the 4 quarter sums meet in LDS in quarter order
__global__ __launch_bounds__(256) void colsum_fold_kernel(const float* __restrict__ slab, int nchunk, int N,
                                                          float* __restrict__ out) {
  __shared__ float red[4][64];
  const int t = threadIdx.x, c = t & 63, qtr = t >> 6;
  const float* strip = slab + (int64_t)blockIdx.x * nchunk * 64;
  float tot = 0.f;
  for (int i0 = qtr; i0 < nchunk; i0 += 32) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = i0 + 4 * k < nchunk ? strip[(int64_t)(i0 + 4 * k) * 64 + c] : 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) tot += v[k];
  }
  red[qtr][c] = tot;
  __syncthreads();
  const int col = blockIdx.x * 64 + t;
  if (t < 64 && col < N) out[col] += (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
}

void colsum_bf16(const bf16_t* x, int64_t M, int N, int ld, float* out, float* slab, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  if (N % 8 || ld % 8) throw std::runtime_error("colsum_bf16: N and ld must be multiples of 8");
  const int strips = (N + 63) / 64;
  const int64_t chunks = colsum_chunks(M, N);
  const int rpb = (int)((M + chunks - 1) / chunks);
  hipLaunchKernelGGL(colsum_bf16_kernel, dim3(strips, (unsigned)chunks), 256, 0, s, x, M, N, ld, rpb, slab);
  hipLaunchKernelGGL(colsum_fold_kernel, strips, 256, 0, s, slab, (int)chunks, N, out);
  MINIPS_HIP_CHECK(hipGetLastError());
}

int64_t colsum_chunks(int64_t M, int N) {
  const int strips = (N + 63) / 64;
  return std::max<int64_t>(1, std::min<int64_t>(std::max(1, 512 / strips), (M + 255) / 256));
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

// 4 consecutive gradient values of one lookup row segment.
__device__ __forceinline__ float4 ld_grad4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 ld_grad4(const bf16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}

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

// Deterministic piecewise segmented sum over the row-sorted lookups (no atomics: two identical
// runs produce bit-identical rows -- the reference BSP applies each superstep's buffered Adds in
// one fixed order, server/consistency/bsp_model.cpp:14-32). A group of L = D/VW lanes reads one
// lookup's D values as VW-wide vectors; each group owns G consecutive lookups (loaded BATCH at a
// time, independent loads in flight) and a wave the PER = 64/L consecutive groups of a "piece".
//   * a row entirely inside one group is summed in registers and stored once;
//   * a row cut by group boundaries inside the piece is completed by an in-wave carry chain: the
//     groups hand their boundary partials to the next group in group order (shuffles), and the
//     group where the row ends stores it;
//   * a row cut by a piece boundary leaves its piece partials in `part` (HEAD: the piece's part of
//     a row that started in an earlier piece, TAIL: the part of the row the piece ends inside), and
//     emb_seg_fix_kernel sums them in piece order -- a Zipf-hot row spanning many pieces costs one
//     partial per piece, not one per lookup.
// Every row [0, U) is written exactly once, wide column and the pad columns [D+1, row_stride) too:
// no zero-fill pass. Output fp32 (the local apply) or bf16 (the push payload at N > 1).
// SORTED: dX holds the lookups' gradient rows in member order ([total, D], row m = lookup members[m]).
template <int VW>
__device__ __forceinline__ void st_row_vals(float* p, const float (&v)[VW]) {
#pragma unroll
  for (int h = 0; h < VW / 4; ++h)
    reinterpret_cast<float4*>(p)[h] = make_float4(v[4 * h], v[4 * h + 1], v[4 * h + 2], v[4 * h + 3]);
}
template <int VW>
__device__ __forceinline__ void st_row_vals(bf16_t* p, const float (&v)[VW]) {
#pragma unroll
  for (int h = 0; h < VW / 4; ++h)
    reinterpret_cast<uint2*>(p)[h] = make_uint2(pack_bf2(v[4 * h], v[4 * h + 1]), pack_bf2(v[4 * h + 2], v[4 * h + 3]));
}
__device__ __forceinline__ void st_scalar(float* p, float v) { *p = v; }
__device__ __forceinline__ void st_scalar(bf16_t* p, float v) { *p = f2bf(v); }

// lane l of a row's group stores its VW values; lane 0 also the wide column D and zero pads
template <typename TO, int D, int VW>
__device__ __forceinline__ void seg_store_row(TO* __restrict__ out, int row_stride, int row, const float (&acc)[VW],
                                              float accw, bool wide, int l) {
  TO* o = out + (int64_t)row * row_stride;
  if ((row_stride & 3) == 0) {
    st_row_vals<VW>(o + VW * l, acc);
  } else {  // (rows not 16-byte aligned: scalar stores)
#pragma unroll
    for (int e = 0; e < VW; ++e) st_scalar(o + VW * l + e, acc[e]);
  }
  if (l == 0)
    for (int c = D; c < row_stride; ++c) st_scalar(o + c, (c == D && wide) ? accw : 0.f);
}

constexpr int seg_part_stride(int D) { return D + 4; }

template <int D, int VW>
__device__ __forceinline__ void seg_store_part(float* __restrict__ part, int64_t slot, const float (&acc)[VW],
                                               float accw, int l) {
  float* o = part + slot * seg_part_stride(D);
  st_row_vals<VW>(o + VW * l, acc);
  if (l == 0) o[D] = accw;
}

template <typename TX, typename TO, int D, int G, int BATCH, bool SORTED, int VW>
__global__ __launch_bounds__(256) void emb_seg_det_kernel(const TX* __restrict__ dX, int ldx,
                                                          const float* __restrict__ dwide, int F,
                                                          const int* __restrict__ members,
                                                          const int* __restrict__ memrow, int total,
                                                          TO* __restrict__ out, int row_stride,
                                                          float* __restrict__ part) {
  constexpr int L = D / VW, PER = 64 / L, PW = PER * G;
  const int lane = threadIdx.x & 63, sub = lane / L, l = lane % L;
  const bool wide = dwide != nullptr;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t piece = wave; piece * PW < total; piece += nw) {
    const int wbase = (int)(piece * PW);
    const int a = wbase + sub * G, b = min(total, a + G);
    const bool has = a < b;
    const int prev_row = (has && a > 0) ? memrow[a - 1] : -1;
    const int next_row = (has && b < total) ? memrow[b] : -1;
    const int wave_prev = wbase > 0 ? memrow[wbase - 1] : -1;
    int cur = -1, rf = -1, rl = -1;
    bool first = true, hasF = false, interior = false, hasL = false;
    float acc[VW], fv[VW], lv[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) acc[e] = fv[e] = lv[e] = 0.f;
    float accw = 0.f, fw = 0.f, lw = 0.f;
    for (int m0 = a; m0 < b; m0 += BATCH) {
      int u[BATCH], bb[BATCH];
      float v[BATCH][VW];
      float vw[BATCH];
#pragma unroll
      for (int q = 0; q < BATCH; ++q) {
        const int m = m0 + q;
        u[q] = m < b ? memrow[m] : -1;
        const TX* src;
        if (SORTED) {
          src = dX + (int64_t)(m < b ? m : a) * D + VW * l;
          bb[q] = (wide && l == 0 && m < b) ? members[m] / F : 0;
        } else {
          const int j = m < b ? members[m] : members[a];
          bb[q] = j / F;
          const int ff = j - bb[q] * F;
          src = dX + (int64_t)bb[q] * ldx + ff * D + VW * l;
        }
        ld_gradv<VW>(src, v[q]);
        vw[q] = (wide && l == 0 && m < b) ? dwide[bb[q]] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < BATCH; ++q) {
        if (u[q] < 0) break;
        if (u[q] != cur) {
          if (cur >= 0) {  // a finished row that is not the group's last
            if (first && cur == prev_row) {  // it came from the previous group
#pragma unroll
              for (int e = 0; e < VW; ++e) fv[e] = acc[e];
              fw = accw;
              hasF = true;
              rf = cur;
            } else {
              seg_store_row<TO, D, VW>(out, row_stride, cur, acc, accw, wide, l);
            }
            first = false;
          }
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
    if (cur >= 0) {  // the group's last row
      if (first && cur == prev_row) {
#pragma unroll
        for (int e = 0; e < VW; ++e) fv[e] = acc[e];
        fw = accw;
        hasF = true;
        rf = cur;
        interior = cur == next_row;  // the whole group is one row that also continues
      } else if (cur == next_row) {
#pragma unroll
        for (int e = 0; e < VW; ++e) lv[e] = acc[e];
        lw = accw;
        hasL = true;
        rl = cur;
      } else {
        seg_store_row<TO, D, VW>(out, row_stride, cur, acc, accw, wide, l);
      }
    }
    // in-wave carry chain, in group order: group s receives group s-1's carry (the partial of the
    // row that continues into s) and completes or extends it
    float cv[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) cv[e] = 0.f;
    float cw = 0.f;
    int crow = -1;
    const int src = (lane - L) & 63;
#pragma unroll
    for (int s = 0; s < PER; ++s) {
      float iv[VW];
#pragma unroll
      for (int e = 0; e < VW; ++e) iv[e] = __shfl(cv[e], src, 64);
      const float iw = __shfl(cw, src, 64);
      const int irow = __shfl(crow, src, 64);
      if (sub == s) {
        const bool carried = s > 0 && irow >= 0 && irow == rf;
        if (hasF) {
          float tv[VW];
#pragma unroll
          for (int e = 0; e < VW; ++e) tv[e] = carried ? iv[e] + fv[e] : fv[e];
          const float tw = carried ? iw + fw : fw;
          if (interior) {
#pragma unroll
            for (int e = 0; e < VW; ++e) cv[e] = tv[e];
            cw = tw;
            crow = rf;
          } else {
            if (wbase > 0 && rf == wave_prev) seg_store_part<D, VW>(part, 2 * piece, tv, tw, l);  // HEAD
            else seg_store_row<TO, D, VW>(out, row_stride, rf, tv, tw, wide, l);
#pragma unroll
            for (int e = 0; e < VW; ++e) cv[e] = lv[e];
            cw = lw;
            crow = hasL ? rl : -1;
          }
        } else {
#pragma unroll
          for (int e = 0; e < VW; ++e) cv[e] = lv[e];
          cw = lw;
          crow = hasL ? rl : -1;
        }
      }
    }
    if (sub == PER - 1 && crow >= 0) seg_store_part<D, VW>(part, 2 * piece + 1, cv, cw, l);  // TAIL
  }
}

// Rows cut by piece boundaries: one WAVE per piece whose last row r starts inside it and
// continues. Its PER lane groups walk the following pieces in windows of PER (group g takes
// pieces p + g, p + g + PER, ...; every load of a window is independent -- a Zipf-hot row spans
// dozens of pieces, and a serial walk of dependent loads took 37 us): a piece contributes TAIL
// when r covers it whole, HEAD where r ends; then the groups' sums meet in a fixed shuffle tree.
// The summation order is fixed by the row's span: deterministic.
template <typename TO, int D, int VW, int PW>
__global__ __launch_bounds__(256) void emb_seg_fix_kernel(const int* __restrict__ memrow, int total,
                                                          const float* __restrict__ part, TO* __restrict__ out,
                                                          int row_stride, bool wide) {
  constexpr int L = D / VW, PER = 64 / L, SP = seg_part_stride(D);
  const int lane = threadIdx.x & 63, sub = lane / L, l = lane % L;
  const int64_t npieces = ((int64_t)total + PW - 1) / PW;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t p = wave; p < npieces; p += nw) {
    const int bw = (int)(p * PW), ew = (int)min((int64_t)total, (p + 1) * PW);
    const int r = memrow[ew - 1];
    if (!(ew < total && memrow[ew] == r)) continue;              // ends inside this piece: done there
    if (bw > 0 && memrow[bw] == r && memrow[bw - 1] == r) continue;  // started in an earlier piece
    float s[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) s[e] = 0.f;
    float sw = 0.f;
    constexpr int QPG = 4;  // pieces per group per window: PER * QPG pieces per memory round trip
    for (int64_t w0 = p;; w0 += PER * QPG) {
      bool end = false;
#pragma unroll
      for (int k = 0; k < QPG; ++k) {
      const int64_t q = w0 + k * PER + sub;
      const bool valid = q < npieces;
      const int64_t qc = valid ? q : p;  // (out-of-range groups load piece p's slots, unused)
      // every load of the window is issued before any is used: both boundary keys of piece q and
      // both of its partial slots (HEAD, TAIL) -- one memory round trip per window
      const int mb = memrow[qc * PW];
      const int64_t eq = min((int64_t)total, (qc + 1) * PW);
      const int me = eq < total ? memrow[eq] : -1;
      const float* ph = part + (2 * qc) * SP;
      const float* pt = ph + SP;
      float vh[VW], vt[VW];
      ld_gradv<VW>(ph + VW * l, vh);
      ld_gradv<VW>(pt + VW * l, vt);
      const float wh = ph[D], wt = pt[D];
      // piece q's part of r: TAIL of p itself, TAIL of a piece r covers whole, HEAD where r ends
      const bool in = valid && (q == p || mb == r);
      const bool through = in && me == r;
      const bool tail = q == p || through;
      if (in) {
#pragma unroll
        for (int e = 0; e < VW; ++e) s[e] += tail ? vt[e] : vh[e];
        sw += tail ? wt : wh;
      }
      end = end || !through;
      }
      // the window ends the walk when some piece of it is not a through piece of r
      if (__any(end)) break;
    }
    // fixed-order tree over the groups (xor partners at distance L, 2L, ...)
#pragma unroll
    for (int o = L; o < 64; o <<= 1) {
#pragma unroll
      for (int e = 0; e < VW; ++e) s[e] += __shfl_xor(s[e], o, 64);
      sw += __shfl_xor(sw, o, 64);
    }
    if (sub == 0) seg_store_row<TO, D, VW>(out, row_stride, r, s, sw, wide, l);
  }
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

constexpr int kSegG = 16, kSegBatch = 8, kSegVW = 4;

constexpr int seg_per_piece(int D) { return (64 / (D / kSegVW)) * kSegG; }

int64_t emb_seg_part_floats(int64_t total, int D) {
  const int64_t pw = seg_per_piece(D);
  return 2 * ((total + pw - 1) / pw) * seg_part_stride(D);
}

template <typename TX, typename TO>
static void emb_seg_det(const TX* dX, int ldx, const float* dwide, int64_t B, int F, int D, const int* members,
                        const int* memrow, TO* out, int row_stride, float* part, hipStream_t s, bool sorted_rows) {
  const int total = (int)(B * F);
  const int64_t pw = seg_per_piece(D);
  const int64_t pieces = (total + pw - 1) / pw;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((pieces + 3) / 4, 65535));
  const int fix_blocks = (int)std::max<int64_t>(1, std::min<int64_t>((pieces + 3) / 4, 4096));  // a wave per piece
#define MINIPS_SEG_DET(DD)                                                                                         \
  if (sorted_rows)                                                                                                \
    hipLaunchKernelGGL((emb_seg_det_kernel<TX, TO, DD, kSegG, kSegBatch, true, kSegVW>), blocks, 256, 0, s, dX,    \
                       ldx, dwide, F, members, memrow, total, out, row_stride, part);                             \
  else                                                                                                            \
    hipLaunchKernelGGL((emb_seg_det_kernel<TX, TO, DD, kSegG, kSegBatch, false, kSegVW>), blocks, 256, 0, s, dX,   \
                       ldx, dwide, F, members, memrow, total, out, row_stride, part);                             \
  if (pieces > 1)                                                                                                 \
    hipLaunchKernelGGL((emb_seg_fix_kernel<TO, DD, kSegVW, seg_per_piece(DD)>), fix_blocks, 256, 0, s, memrow,     \
                       total, part, out, row_stride, dwide != nullptr);
  switch (D) {
    case 16:
      MINIPS_SEG_DET(16)
      break;
    case 32:
      MINIPS_SEG_DET(32)
      break;
    case 64:
      MINIPS_SEG_DET(64)
      break;
    default:
      throw std::runtime_error("emb_backward_seg: D must be 16, 32 or 64");
  }
#undef MINIPS_SEG_DET
  MINIPS_HIP_CHECK(hipGetLastError());
}

void emb_backward_csr(const void* dX, bool bf16, int ldx, const float* dwide, int64_t B, int F, int D,
                      const int* members, const int* memrow, void* out, bool out_bf16, int row_stride, float* part,
                      hipStream_t s, bool sorted_rows) {
  if (B <= 0) return;
  if (row_stride < D + (dwide ? 1 : 0)) throw std::runtime_error("emb_backward_csr: row_stride too small");
  if (bf16 && out_bf16)
    emb_seg_det(static_cast<const bf16_t*>(dX), ldx, dwide, B, F, D, members, memrow, static_cast<bf16_t*>(out),
                row_stride, part, s, sorted_rows);
  else if (bf16)
    emb_seg_det(static_cast<const bf16_t*>(dX), ldx, dwide, B, F, D, members, memrow, static_cast<float*>(out),
                row_stride, part, s, sorted_rows);
  else if (out_bf16)
    emb_seg_det(static_cast<const float*>(dX), ldx, dwide, B, F, D, members, memrow, static_cast<bf16_t*>(out),
                row_stride, part, s, sorted_rows);
  else
    emb_seg_det(static_cast<const float*>(dX), ldx, dwide, B, F, D, members, memrow, static_cast<float*>(out),
                row_stride, part, s, sorted_rows);
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
                          int D, void* out, bool out_bf16, int row_stride, int U, int* ws, float* part, hipStream_t s) {
  if (B <= 0 || U <= 0) return;
  // ws: counts[U] | cursor[U] | offsets[U+1] | tiles[U/1024+1] | members[B*F] | memrow[B*F]
  int* members = ws + 3 * U + 1 + (U / 1024 + 1);
  int* memrow = members + B * F;
  emb_build_csr(inv, B, F, U, ws, members, memrow, s);
  emb_backward_csr(dX, bf16, ldx, dwide, B, F, D, members, memrow, out, out_bf16, row_stride, part, s, false);
}

}  // namespace minips_k
