// bf16 MFMA GEMM entry points (kernels.h): argument checks, split-K slabs and their reduction, and
// the per-layout dispatch into the kernel templates of gemm_kernels.h (instantiated in gemm_l*.hip).
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>
#include <algorithm>

#include "gemm_kernels.h"

namespace minips_k {

static int dispatch_layout(bool a_km, bool b_kn, int epi, const bf16_t* A, const bf16_t* B, int M, int N, int K,
                           int lda, int ldb, int split_k, const EpiArgs& ep, int batch, hipStream_t s) {
  if (!a_km && !b_kn) return gemm_dispatch<false, false>(epi, A, B, M, N, K, lda, ldb, split_k, ep, batch, s);
  if (!a_km && b_kn) return gemm_dispatch<false, true>(epi, A, B, M, N, K, lda, ldb, split_k, ep, batch, s);
  if (a_km && b_kn) return gemm_dispatch<true, true>(epi, A, B, M, N, K, lda, ldb, split_k, ep, batch, s);
  return gemm_dispatch<true, false>(epi, A, B, M, N, K, lda, ldb, split_k, ep, batch, s);
}

// out[r][c] (ldc) += sum_s slab[s][r][c]   (slab [nsplit][M][N] fp32, float4 over columns)
// (Tried instead: an in-kernel "last split of a tile reduces" fixup with per-tile arrival
// counters. Correct, but the agent-scope release it needs is an L2 writeback per workgroup on
// the multi-XCD part: W&D step 0.52 -> 0.79 ms. The separate streaming reduce stays.)
__global__ void splitk_reduce_kernel(const float* __restrict__ slab, int nsplit, int M, int N, float* __restrict__ out,
                                     int ldc) {
  const int n4 = N >> 2;
  const int64_t total = (int64_t)M * n4, plane = (int64_t)M * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / n4;
    const int c = (int)(i - r * n4) * 4;
    const float* p = slab + r * N + c;
    float4 a = *reinterpret_cast<const float4*>(p);
    int z = 1;
    for (; z + 3 < nsplit; z += 4) {  // 4 independent plane loads in flight per thread
      const float4 b0 = *reinterpret_cast<const float4*>(p + z * plane);
      const float4 b1 = *reinterpret_cast<const float4*>(p + (z + 1) * plane);
      const float4 b2 = *reinterpret_cast<const float4*>(p + (z + 2) * plane);
      const float4 b3 = *reinterpret_cast<const float4*>(p + (z + 3) * plane);
      a.x += (b0.x + b1.x) + (b2.x + b3.x);
      a.y += (b0.y + b1.y) + (b2.y + b3.y);
      a.z += (b0.z + b1.z) + (b2.z + b3.z);
      a.w += (b0.w + b1.w) + (b2.w + b3.w);
    }
    for (; z < nsplit; ++z) {
      const float4 b = *reinterpret_cast<const float4*>(p + z * plane);
      a.x += b.x;
      a.y += b.y;
      a.z += b.z;
      a.w += b.w;
    }
    float* o = out + r * ldc + c;
    o[0] += a.x;
    o[1] += a.y;
    o[2] += a.z;
    o[3] += a.w;
  }
}

// out_bf16[r][c] (ldc) = sum_s slab[s][r][c]: the split-K form of a plain bf16-output GEMM (a long-K
// dgrad such as GPT-2's LM head, dh = dlogits wte with K = 50304 and only 8192 x 768 outputs)
__global__ void splitk_reduce_bf16_kernel(const float* __restrict__ slab, int nsplit, int M, int N,
                                          bf16_t* __restrict__ out, int ldc) {
  const int n4 = N >> 2;
  const int64_t total = (int64_t)M * n4, plane = (int64_t)M * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / n4;
    const int c = (int)(i - r * n4) * 4;
    const float* p = slab + r * N + c;
    float4 a = *reinterpret_cast<const float4*>(p);
    for (int z = 1; z < nsplit; ++z) {
      const float4 b = *reinterpret_cast<const float4*>(p + z * plane);
      a.x += b.x;
      a.y += b.y;
      a.z += b.z;
      a.w += b.w;
    }
    *reinterpret_cast<uint2*>(out + r * ldc + c) = make_uint2(pack_bf2(a.x, a.y), pack_bf2(a.z, a.w));
  }
}

void gemm_bf16_batched(const bf16_t* A, const bf16_t* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                       bool a_km, bool b_kn, int epi, const bf16_t* bias, const bf16_t* mask, int ldmask,
                       float* colsum, float alpha, int split_k, int batch, int inner, int64_t sa_o, int64_t sa_i,
                       int64_t sb_o, int64_t sb_i, int64_t sc_o, int64_t sc_i, hipStream_t s, float* slab,
                       const int* perm, int seg, int colsum_ld, int tile) {
  if (M <= 0 || N <= 0 || K <= 0 || batch <= 0) return;
  if (epi == kEpiPermRowsBf16 && (!perm || seg <= 0 || seg % 8 || N % seg || batch != 1 || split_k > 1))
    throw std::runtime_error("gemm: the permuted-rows epilogue needs perm, seg % 8 == 0, N % seg == 0, no batch");
  if (split_k < 1) split_k = 1;
  if (split_k > 1 && epi != kEpiAtomicF32 && !(epi == kEpiStoreBf16 && slab))
    throw std::runtime_error("gemm: split_k needs the atomic epilogue (or a plain bf16 store with a slab)");
  if (batch > 1 && (mask || colsum)) throw std::runtime_error("gemm: batched mode has no mask/colsum epilogue");
  if (inner < 1) inner = 1;
  int nsplit = 1;
  if (slab && split_k > 1 && batch == 1 && N % 4 == 0) {
    const bool bf16_out = epi == kEpiStoreBf16;
    // split-K without atomics: every K slice stores its partial tile into its own slab plane,
    // one streaming kernel adds the planes into C (measured faster than fp32 atomics)
    EpiArgs sp{slab, N, nullptr, nullptr, 0, nullptr, alpha, 1, 0, 0, 0, 0, 0, 0, (int64_t)M * N, nullptr, 0};
    sp.tile = tile;
    nsplit = dispatch_layout(a_km, b_kn, kEpiStoreF32, A, B, M, N, K, lda, ldb, split_k, sp, batch, s);
    MINIPS_HIP_CHECK(hipGetLastError());
    if (bf16_out)
      hipLaunchKernelGGL(splitk_reduce_bf16_kernel, grid_for((int64_t)M * (N / 4), 256, 4096), 256, 0, s, slab, nsplit,
                         M, N, (bf16_t*)C, ldc);
    else
      hipLaunchKernelGGL(splitk_reduce_kernel, grid_for((int64_t)M * (N / 4), 256, 4096), 256, 0, s, slab, nsplit, M,
                         N, (float*)C, ldc);
    MINIPS_HIP_CHECK(hipGetLastError());
    return;
  }
  EpiArgs ep{C, ldc, bias, mask, ldmask, colsum, alpha, inner, sa_o, sa_i, sb_o, sb_i, sc_o, sc_i, 0, perm, seg};
  ep.colsum_ld = colsum_ld > 0 ? colsum_ld : 1;
  ep.tile = tile;
  // an accumulating GEMM with one K slice has one writer per output element: read-add-write
  // instead of memory-side fp32 atomics
  if (epi == kEpiAtomicF32 && split_k == 1) epi = kEpiAccumF32;
  nsplit = dispatch_layout(a_km, b_kn, epi, A, B, M, N, K, lda, ldb, split_k, ep, batch, s);
  (void)nsplit;
  MINIPS_HIP_CHECK(hipGetLastError());
}

int gemm_slab(const bf16_t* A, const bf16_t* B, float* slab, int M, int N, int K, int lda, int ldb, bool a_km,
              bool b_kn, int split_k, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (N % 4) throw std::runtime_error("gemm_slab: N % 4 == 0");
  EpiArgs sp{slab, N, nullptr, nullptr, 0, nullptr, 1.f, 1, 0, 0, 0, 0, 0, 0, (int64_t)M * N, nullptr, 0};
  const int nsplit = dispatch_layout(a_km, b_kn, kEpiStoreF32, A, B, M, N, K, lda, ldb, std::max(1, split_k), sp, 1, s);
  MINIPS_HIP_CHECK(hipGetLastError());
  return nsplit;
}

void gemm_bf16(const bf16_t* A, const bf16_t* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
               bool a_km, bool b_kn, int epi, const bf16_t* bias, const bf16_t* mask, int ldmask, float* colsum,
               float alpha, int split_k, hipStream_t s) {
  gemm_bf16_batched(A, B, C, M, N, K, lda, ldb, ldc, a_km, b_kn, epi, bias, mask, ldmask, colsum, alpha, split_k, 1,
                    1, 0, 0, 0, 0, 0, 0, s, nullptr);
}

}  // namespace minips_k
