// GEMM kernels of one operand layout, tn (wgrad: A [K][M], B [K][N]): the epilogue dispatch of gemm_kernels.h
// instantiated in its own translation unit (the four layouts compile in parallel).
#include <stdexcept>
#include <string>

#include "gemm_kernels.h"

namespace minips_k {

template <>
int gemm_dispatch<true, true>(int epi, const bf16_t* A, const bf16_t* B, int M, int N, int K, int lda, int ldb,
                            int split_k, const EpiArgs& ep, int batch, hipStream_t s) {
  int nsplit = 1;
  MINIPS_GEMM_EPI_DISPATCH(true, true)
  return nsplit;
}

}  // namespace minips_k
