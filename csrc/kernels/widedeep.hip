// Wide&Deep worker kernels: input assembly (embedding lookup + dense concat + wide sum),
// the fused output head (Linear Hd->1 + BCE-with-logits forward+backward), and the
// embedding-gradient scatter into the per-unique-key gradient rows that are pushed to the
// owning server shards.
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"

namespace minips_k {

// One thread per (sample, 8-column chunk): a 16-byte store of 8 bf16; threads past the
// chunks compute the per-sample wide sums (one thread per sample) so no thread serialises.
__global__ void wd_assemble_kernel(const float* __restrict__ dense, int n_dense, const bf16_t* __restrict__ rows,
                                   int row_stride, const int64_t* __restrict__ inv, int64_t B, int F, int D,
                                   bf16_t* __restrict__ X, int ldx, float* __restrict__ wide_logit, int ones_col) {
  const int chunks = ldx >> 3;
  const int emb_cols = F * D;
  const int64_t total = B * chunks;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total + B;
       c += (int64_t)gridDim.x * blockDim.x) {
    if (c >= total) {
      const int64_t b = c - total;
      float w = 0.f;
      const int64_t* iv = inv + b * F;
      for (int f = 0; f < F; ++f) w += bf2f(rows[iv[f] * row_stride + D]);
      wide_logit[b] = w;
      continue;
    }
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
                 int F, int D, bf16_t* X, int ldx, float* wide_logit, int ones_col, hipStream_t s) {
  if (ldx % 8) throw std::runtime_error("wd_assemble: ldx must be a multiple of 8");
  if (F * D + n_dense > ldx) throw std::runtime_error("wd_assemble: ldx too small");
  if (ones_col >= ldx) throw std::runtime_error("wd_assemble: ones_col out of range");
  if (row_stride % 4) throw std::runtime_error("wd_assemble: row_stride must be a multiple of 4");
  if (B <= 0) return;
  const int block = 256;
  hipLaunchKernelGGL(wd_assemble_kernel, grid_for(B * (ldx / 8 + 1), block, 8192), block, 0, s, dense, n_dense, rows,
                     row_stride, inv, B, F, D, X, ldx, wide_logit, ones_col);
  MINIPS_HIP_CHECK(hipGetLastError());
}

// One wave per sample (grid-stride); each lane owns Hd/64 columns and keeps its dw / colsum
// partials in registers across all samples it visits: one atomic per lane per column at the end.
template <int PER_LANE>
__global__ __launch_bounds__(256) void wd_head_kernel(const bf16_t* __restrict__ H, int64_t B, int Hd,
                                                      const bf16_t* __restrict__ w, const bf16_t* __restrict__ b0,
                                                      const float* __restrict__ wide, const float* __restrict__ y,
                                                      bf16_t* __restrict__ dH, float* dw, float* db, float* dwide,
                                                      float* loss_sum, float* colsum, float scale) {
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
      if (b < B) {
        const bf16_t* hp = H + b * Hd + lane * PER_LANE;
#pragma unroll
        for (int j = 0; j < PER_LANE; ++j) h[s][j] = bf2f(hp[j]);
      }
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
      bf16_t* dp = dH + b * Hd + lane * PER_LANE;
#pragma unroll
      for (int j = 0; j < PER_LANE; ++j) {
        dwl[j] += dz * h[s][j];
        const bf16_t g = f2bf(h[s][j] > 0.f ? dz * wl[j] : 0.f);
        dp[j] = g;
        csl[j] += bf2f(g);
      }
    }
  }
  // reduce the 4 waves of the block in LDS, then one global atomic per column per block
  __shared__ float red[2][4][64 * PER_LANE];
  __shared__ float red_s[2][4];
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
  for (int c = threadIdx.x; c < 64 * PER_LANE; c += blockDim.x) {
    atomicAdd(dw + c, red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c]);
    if (colsum) atomicAdd(colsum + c, red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c]);
  }
  if (threadIdx.x == 0) {
    atomicAdd(db, red_s[0][0] + red_s[0][1] + red_s[0][2] + red_s[0][3]);
    atomicAdd(loss_sum, red_s[1][0] + red_s[1][1] + red_s[1][2] + red_s[1][3]);
  }
}

void wd_head(const bf16_t* H, int64_t B, int Hd, const bf16_t* w, const bf16_t* b0, const float* wide_logit,
             const float* labels, bf16_t* dH, float* dw, float* db, float* dwide, float* loss_sum, float* dH_colsum,
             float grad_scale, hipStream_t s) {
  if (B <= 0) return;
  const int block = 256;
  const int grid = (int)std::min<int64_t>(128, (B + 15) / 16);  // per-block LDS reduction, then atomics
  switch (Hd) {
    case 64 * 1: hipLaunchKernelGGL(wd_head_kernel<1>, grid, block, 0, s, H, B, Hd, w, b0, wide_logit, labels, dH, dw, db, dwide, loss_sum, dH_colsum, grad_scale); break;
    case 64 * 2: hipLaunchKernelGGL(wd_head_kernel<2>, grid, block, 0, s, H, B, Hd, w, b0, wide_logit, labels, dH, dw, db, dwide, loss_sum, dH_colsum, grad_scale); break;
    case 64 * 4: hipLaunchKernelGGL(wd_head_kernel<4>, grid, block, 0, s, H, B, Hd, w, b0, wide_logit, labels, dH, dw, db, dwide, loss_sum, dH_colsum, grad_scale); break;
    case 64 * 8: hipLaunchKernelGGL(wd_head_kernel<8>, grid, block, 0, s, H, B, Hd, w, b0, wide_logit, labels, dH, dw, db, dwide, loss_sum, dH_colsum, grad_scale); break;
    default: throw std::runtime_error("wd_head: Hd must be 64, 128, 256 or 512, got " + std::to_string(Hd));
  }
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

}  // namespace minips_k
