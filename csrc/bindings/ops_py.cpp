// Torch-facing bindings of the gfx950 kernels (module minips_amd._kernels).
// Every op validates device/dtype/shape/contiguity on the host BEFORE launching, so a bad
// shape raises a Python exception instead of faulting the GPU, and launches on the current
// HIP stream of the tensor's device (graph-capture safe: no allocation or sync in here).
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/extension.h>

#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <tuple>

#include "../comm/rccl_comm.h"
#include "../kernels/kernels.h"
#include "../kernels/onesided.h"

namespace {

using minips_k::bf16_t;

hipStream_t stream_of(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

// Several outputs carved out of ONE caching-allocator block (256-byte aligned views): a planner
// call hands back ~10 tensors, and one allocation + views costs a fraction of ten allocations on
// the step's host path. The block lives while any of its views does.
std::vector<at::Tensor> carve(const at::TensorOptions& o,
                              const std::vector<std::pair<int64_t, at::ScalarType>>& parts) {
  std::vector<int64_t> offs;
  int64_t total = 0;
  for (const auto& p : parts) {
    offs.push_back(total);
    total += (p.first * (int64_t)c10::elementSize(p.second) + 255) & ~int64_t(255);
  }
  at::Tensor buf = at::empty({std::max<int64_t>(total, 256)}, o.dtype(at::kByte));
  std::vector<at::Tensor> out;
  out.reserve(parts.size());
  for (size_t i = 0; i < parts.size(); ++i)
    out.push_back(buf.narrow(0, offs[i], parts[i].first * (int64_t)c10::elementSize(parts[i].second))
                      .view(parts[i].second));
  return out;
}

void check_gpu(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_dtype(const at::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
}
template <typename T>
T* ptr(const at::Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}
template <typename T>
T* opt_ptr(const c10::optional<at::Tensor>& t, at::ScalarType dt, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_gpu(*t, name);
  check_dtype(*t, dt, name);
  return reinterpret_cast<T*>(t->data_ptr());
}

// fp32 1-D vector that may be a strided view (e.g. one column of a weight-gradient matrix)
float* strided_vec_ptr(const c10::optional<at::Tensor>& t, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->dim() == 1 && t->stride(0) >= 1, name,
              ": a 1-D fp32 GPU tensor (any positive stride)");
  return t->data_ptr<float>();
}

// C = A . B with layout flags; see gemm.hip. Returns nothing (C preallocated).
// Batched mode (batch > 1): operands are flat buffers addressed with 2-level strides; every
// batch's extent is bounds-checked against the tensor sizes before launch.
// One validated GEMM launch: every pointer, dimension and epilogue argument of gemm_bf16_batched,
// so that a LaunchList can replay it without re-validating (the checks ran when it was prepared).
struct GemmLaunch {
  const bf16_t *A, *B;
  void* C;
  int M, N, K, lda, ldb, ldc;
  bool a_km, b_kn;
  int epi;
  const bf16_t *bias, *mask;
  int ldmask;
  float* colsum;
  float alpha;
  int split_k, batch, inner;
  int64_t st[6];
  float* slab;
  const int* perm;
  int seg, colsum_ld;
  int tile = 0;
  void launch(hipStream_t s) const {
    minips_k::gemm_bf16_batched(A, B, C, M, N, K, lda, ldb, ldc, a_km, b_kn, epi, bias, mask, ldmask, colsum, alpha,
                                split_k, batch, inner, st[0], st[1], st[2], st[3], st[4], st[5], s, slab, perm, seg,
                                colsum_ld, tile);
  }
};

// a GEMM tile hint: 0 (the launcher's choice), 128 (128x128), 200 (256x128) or 256 (256x256)
int check_tile(int64_t tile) {
  TORCH_CHECK(tile == 0 || tile == 128 || tile == 200 || tile == 256, "gemm tile hint: 0, 128, 200 or 256");
  return (int)tile;
}

// Validates a gemm() call and returns its launch; ``slab`` receives the split-K planes it needs
// (a caching-allocator block), if any.
GemmLaunch prepare_gemm(const at::Tensor& A, const at::Tensor& B, at::Tensor& C, int64_t M, int64_t N, int64_t K,
                        bool a_km, bool b_kn, int64_t epi, const c10::optional<at::Tensor>& bias,
                        const c10::optional<at::Tensor>& mask, const c10::optional<at::Tensor>& colsum, double alpha,
                        int64_t split_k, int64_t batch, int64_t inner, int64_t lda_, int64_t ldb_, int64_t ldc_,
                        const std::vector<int64_t>& strides, const c10::optional<at::Tensor>& perm, int64_t seg,
                        at::Tensor& slab) {
  // 2-D operands may be column-sliced views: rows contiguous (stride(1) == 1), ld = stride(0).
  auto check_mat = [](const at::Tensor& t, const char* n) {
    TORCH_CHECK(t.is_cuda(), n, " must be a GPU tensor");
    TORCH_CHECK(t.dim() == 2 ? t.stride(1) == 1 : t.is_contiguous(), n, " rows must be contiguous");
  };
  check_mat(A, "A");
  check_mat(B, "B");
  check_mat(C, "C");
  check_dtype(A, at::kBFloat16, "A");
  check_dtype(B, at::kBFloat16, "B");
  const bool f32_out = epi == minips_k::kEpiStoreF32 || epi == minips_k::kEpiAtomicF32;
  check_dtype(C, f32_out ? at::kFloat : at::kBFloat16, "C");
  const bool permuted = epi == minips_k::kEpiPermRowsBf16;
  const int* perm_p = opt_ptr<int>(perm, at::kInt, "perm");
  if (permuted) {
    // C is [M * N / seg, seg] rows in the permuted order; perm lists M * N / seg distinct rows of it
    TORCH_CHECK(perm_p && seg > 0 && seg % 8 == 0 && N % seg == 0 && batch <= 1 && split_k <= 1,
                "permuted rows: perm, seg % 8 == 0, N % seg == 0, no batch / split-K");
    TORCH_CHECK(perm->numel() >= M * (N / seg) && C.is_contiguous() && C.numel() >= M * N,
                "permuted rows: perm [M*N/seg] and a contiguous C of >= M*N values");
  }
  TORCH_CHECK(K % 8 == 0, "K must be a multiple of 8");
  if (a_km) TORCH_CHECK(M % 8 == 0, "KM layout needs M % 8 == 0");
  if (b_kn) TORCH_CHECK(N % 8 == 0, "KN layout needs N % 8 == 0");
  const int64_t a_rows = a_km ? K : M, a_cols = a_km ? M : K;
  const int64_t b_rows = b_kn ? K : N, b_cols = b_kn ? N : K;
  int64_t lda, ldb, ldc;
  std::vector<int64_t> st(6, 0);
  if (batch <= 1) {
    TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "gemm operands must be 2-D");
    TORCH_CHECK(A.size(0) >= a_rows && A.size(1) >= a_cols, "A shape ", A.sizes(), " vs M,N,K=", M, ",", N, ",", K);
    TORCH_CHECK(B.size(0) >= b_rows && B.size(1) >= b_cols, "B shape ", B.sizes(), " vs M,N,K=", M, ",", N, ",", K);
    TORCH_CHECK(permuted || (C.size(0) >= M && C.size(1) >= N), "C shape ", C.sizes(), " vs M,N=", M, ",", N);
    lda = A.stride(0);
    ldb = B.stride(0);
    ldc = C.stride(0);
    batch = 1;
    inner = 1;
  } else {
    TORCH_CHECK(strides.size() == 6, "batched gemm needs 6 strides");
    st = strides;
    lda = lda_;
    ldb = ldb_;
    ldc = ldc_;
    TORCH_CHECK(inner >= 1 && batch % inner == 0, "batch must be a multiple of inner");
    auto extent = [&](int64_t rows, int64_t cols, int64_t ld, int64_t so, int64_t si) {
      return (batch / inner - 1) * so + (inner - 1) * si + (rows - 1) * ld + cols;
    };
    TORCH_CHECK(extent(a_rows, a_cols, lda, st[0], st[1]) <= A.numel(), "batched A out of bounds");
    TORCH_CHECK(extent(b_rows, b_cols, ldb, st[2], st[3]) <= B.numel(), "batched B out of bounds");
    TORCH_CHECK(extent(M, N, ldc, st[4], st[5]) <= C.numel(), "batched C out of bounds");
    TORCH_CHECK(!mask.has_value() && !colsum.has_value(), "batched gemm has no mask/colsum");
  }
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0, "leading dims must be multiples of 8 (16-byte rows)");
  for (int i = 0; i < 4; ++i) TORCH_CHECK(st[i] % 8 == 0, "operand batch strides must be multiples of 8");
  const bf16_t* bias_p = opt_ptr<bf16_t>(bias, at::kBFloat16, "bias");
  if (bias_p) TORCH_CHECK(bias->numel() >= N, "bias too short");
  const bf16_t* mask_p = nullptr;
  int ldmask = 0;
  if (mask.has_value() && mask->defined()) {
    check_mat(*mask, "mask");
    check_dtype(*mask, at::kBFloat16, "mask");
    mask_p = ptr<bf16_t>(*mask);
    TORCH_CHECK(mask->dim() == 2 && mask->size(0) == M && mask->size(1) >= N, "mask shape ", mask->sizes());
    ldmask = (int)mask->stride(0);
  }
  const bool needs_mask = epi == minips_k::kEpiReluMaskBf16 || epi == minips_k::kEpiBiasGeluAuxBf16 ||
                          epi == minips_k::kEpiGeluGradBf16 || epi == minips_k::kEpiBiasGeluDAuxBf16 ||
                          epi == minips_k::kEpiMulAuxBf16;
  if (needs_mask) TORCH_CHECK(mask_p, "this epilogue needs mask/aux");
  float* colsum_p = strided_vec_ptr(colsum, "colsum");
  if (colsum_p) {
    // a 1-D view may be strided (a column of a weight-gradient matrix: the folded-bias column)
    TORCH_CHECK(colsum->dim() == 1 && colsum->numel() >= N && colsum->stride(0) >= 1, "colsum: 1-D, >= N values");
  }
  const int colsum_ld = colsum_p ? (int)colsum->stride(0) : 1;
  if (epi == minips_k::kEpiStoreBf16 && split_k > 1)
    TORCH_CHECK(batch <= 1 && N % 4 == 0 && ldc % 4 == 0, "split-K bf16 store: no batch, N % 4 == 0, ldc % 4 == 0");
  // split-K slices land in fp32 slab planes and one reduce kernel adds them (deterministic, no atomics)
  if (split_k > 1 && batch <= 1 &&
      (epi == minips_k::kEpiAtomicF32 || epi == minips_k::kEpiStoreBf16) && N % 4 == 0)
    slab = at::empty({split_k * M * N}, A.options().dtype(at::kFloat));  // caching allocator, stream-ordered
  GemmLaunch g{ptr<bf16_t>(A), ptr<bf16_t>(B), C.data_ptr(), (int)M, (int)N, (int)K, (int)lda, (int)ldb, (int)ldc,
               a_km, b_kn, (int)epi, bias_p, mask_p, ldmask, colsum_p, (float)alpha, (int)split_k, (int)batch,
               (int)inner, {st[0], st[1], st[2], st[3], st[4], st[5]}, slab.defined() ? ptr<float>(slab) : nullptr,
               perm_p, (int)seg, colsum_ld};
  return g;
}

void gemm(const at::Tensor& A, const at::Tensor& B, at::Tensor& C, int64_t M, int64_t N, int64_t K, bool a_km,
          bool b_kn, int64_t epi, const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& mask,
          const c10::optional<at::Tensor>& colsum, double alpha, int64_t split_k, int64_t batch, int64_t inner,
          int64_t lda_, int64_t ldb_, int64_t ldc_, std::vector<int64_t> strides,
          const c10::optional<at::Tensor>& perm, int64_t seg, int64_t tile) {
  c10::hip::HIPGuardMasqueradingAsCUDA gd(A.device());
  at::Tensor slab;
  GemmLaunch g = prepare_gemm(A, B, C, M, N, K, a_km, b_kn, epi, bias, mask, colsum, alpha, split_k, batch, inner,
                              lda_, ldb_, ldc_, strides, perm, seg, slab);
  g.tile = check_tile(tile);
  g.launch(stream_of(A));
}

// Bitmap planner of a bounded key space (keys, after the optional routing k * mult mod rn, in
// [0, num_rows)): same outputs as unique_bucketize -- (sorted unique keys [n] (first U valid),
// inverse [n], counts [P], U [1]) -- with no hash table.
std::vector<at::Tensor> bitmap_plan(const at::Tensor& keys, const at::Tensor& bounds, int64_t num_rows,
                                    int64_t route_mult, int64_t route_n, const c10::optional<at::Tensor>& oor) {
  check_gpu(keys, "keys");
  check_gpu(bounds, "bounds");
  check_dtype(keys, at::kLong, "keys");
  check_dtype(bounds, at::kLong, "bounds");
  TORCH_CHECK(keys.is_contiguous() && bounds.dim() == 1 && bounds.numel() >= 2, "bitmap_plan args");
  TORCH_CHECK(num_rows > 0 && num_rows <= (1LL << 36), "bitmap_plan: 0 < num_rows <= 2^36");
  TORCH_CHECK(!route_mult || route_n == num_rows, "bitmap_plan: routing must map into [0, num_rows)");
  const int64_t n = keys.numel();
  const int P = (int)bounds.numel() - 1;
  auto opts = keys.options();
  auto ws = at::empty({minips_k::bitmap_plan_workspace_words(num_rows)}, opts);
  auto uniq = at::empty({std::max<int64_t>(n, 1)}, opts), inverse = at::empty({n}, opts);
  auto counts = at::empty({P + 1}, opts), U = at::empty({1}, opts);
  c10::hip::HIPGuardMasqueradingAsCUDA g(keys.device());
  minips_k::bitmap_plan(ptr<int64_t>(keys), n, num_rows, ptr<int64_t>(bounds), P, (uint64_t)route_mult,
                        (uint64_t)route_n, ptr<int64_t>(ws), ptr<int64_t>(uniq), ptr<int64_t>(inverse),
                        ptr<int64_t>(counts), ptr<int64_t>(U), stream_of(keys),
                        opt_ptr<int64_t>(oor, at::kLong, "oor"));
  return {uniq, inverse, counts.narrow(0, 0, P), U};
}

// Returns (unique keys grouped by owner [n] (first U valid), inverse [n], counts [P], U [1]).
std::vector<at::Tensor> unique_bucketize(const at::Tensor& keys, const at::Tensor& bounds, int64_t F,
                                         int64_t route_mult, int64_t route_n, int64_t extra_zero_ints,
                                         bool csr_counts) {
  check_gpu(keys, "keys");
  check_gpu(bounds, "bounds");
  check_dtype(keys, at::kLong, "keys");
  check_dtype(bounds, at::kLong, "bounds");
  TORCH_CHECK(bounds.dim() == 1 && bounds.numel() >= 2, "bounds must be [P+1]");
  const int64_t n = keys.numel();
  const int P = (int)bounds.numel() - 1;
  // capacity: the smallest power of two >= 1.6 n (every key fits: U <= n < cap), so even a batch
  // of all-distinct keys (DLRM / LR ids drawn uniformly from 10^8 rows: U ~ n) probes at load
  // <= 0.63 -- at next_pow2(n) such a batch ran at load ~0.8 and its linear-probing inserts took
  // 141 us for 426K keys (profiles/r2/dlrm_1gpu_kernels_before.txt). Criteo-shaped batches (U ~ n/5)
  // use the sort planner (plan.hip) instead.
  int64_t cap = 1024;
  while (cap * 5 < n * 8) cap <<= 1;
  if (cap <= n) cap <<= 1;
  auto opts = keys.options();
  // table_keys | counts[P] | total | shard counters [2*S*P] in one allocation: one zero memset
  const int64_t extra64 = (std::max<int64_t>(extra_zero_ints, 0) + 1) / 2;  // int32 count -> int64 words
  const int64_t shw = 2 * (int64_t)minips_k::ub_shards(P) * P;
  // csr_counts: the first n ints of the extra block receive the per-unique-key lookup counts (the
  // embedding-backward CSR's row sizes), from per-slot counters (cap int32) cleared by the memset
  TORCH_CHECK(!csr_counts || extra_zero_ints >= n, "csr_counts needs extra_zero_ints >= n");
  const int64_t scw = csr_counts ? cap / 2 : 0;
  auto zbuf = at::empty({cap + P + 1 + shw + scw + extra64}, opts);
  auto table_keys = zbuf.narrow(0, 0, cap), table_pos = at::empty({cap}, opts);
  auto slot = at::empty({n}, opts), flags = at::empty({n}, opts.dtype(at::kInt));
  auto counts = zbuf.narrow(0, cap, P + 1), cursor = zbuf.narrow(0, cap + P + 1, shw);
  auto out_keys = at::empty({n}, opts), inverse = at::empty({n}, opts);
  c10::hip::HIPGuardMasqueradingAsCUDA g(keys.device());
  TORCH_CHECK(F >= 1 && n % F == 0, "unique_bucketize: numel must be a multiple of F");
  minips_k::unique_bucketize(ptr<int64_t>(keys), n, (int)F, ptr<int64_t>(bounds), P, ptr<int64_t>(table_keys),
                             ptr<int64_t>(table_pos), cap, ptr<int64_t>(slot), ptr<int32_t>(flags),
                             ptr<int64_t>(counts), ptr<int64_t>(cursor), ptr<int64_t>(out_keys), ptr<int64_t>(inverse),
                             stream_of(keys), (uint64_t)route_mult, (uint64_t)route_n, extra64 * 8,
                             csr_counts ? reinterpret_cast<int*>(zbuf.data_ptr<int64_t>() + cap + P + 1 + shw + scw)
                                        : nullptr);
  std::vector<at::Tensor> out{out_keys, inverse, counts.narrow(0, 0, P), counts.narrow(0, P, 1)};
  if (extra64) out.push_back(zbuf.narrow(0, cap + P + 1 + shw + scw, extra64).view(at::kInt));  // zeroed workspace
  return out;
}

static const int64_t* count_ptr(const c10::optional<at::Tensor>& n_dev) {
  if (!n_dev.has_value() || !n_dev->defined()) return nullptr;
  TORCH_CHECK(n_dev->is_cuda() && n_dev->scalar_type() == at::kLong && n_dev->numel() >= 1, "n_dev: int64 GPU scalar");
  return n_dev->data_ptr<int64_t>();
}

void gather_rows(const at::Tensor& table, const at::Tensor& keys, int64_t base, at::Tensor& out,
                 const c10::optional<at::Tensor>& n_dev) {
  check_gpu(keys, "keys");
  check_gpu(out, "out");
  TORCH_CHECK(table.is_cuda() && table.dim() == 2 && table.stride(1) == 1, "table must be a row-major GPU matrix");
  check_dtype(keys, at::kLong, "keys");
  const int64_t n = keys.numel();
  TORCH_CHECK(out.dim() == 2 && out.size(0) >= n, "out shape ", out.sizes());
  const int D = (int)out.size(1);
  TORCH_CHECK(D <= table.size(1), "out row wider than table row");
  if (table.scalar_type() == at::kDouble) {  // reference-precision tables (f64.hip)
    check_dtype(out, at::kDouble, "out");
    TORCH_CHECK(D == table.size(1) && table.is_contiguous() && out.is_contiguous(), "fp64 gather: whole rows");
    c10::hip::HIPGuardMasqueradingAsCUDA g(keys.device());
    minips_k::gather_rows_f64(ptr<double>(table), D, ptr<int64_t>(keys), base, n, count_ptr(n_dev), ptr<double>(out),
                              stream_of(keys));
    return;
  }
  TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16, "out must be fp32 or bf16");
  if (table.scalar_type() == at::kBFloat16) {  // bf16 rows (bf16rows.hip)
    TORCH_CHECK(D == table.size(1) && out.is_contiguous(), "bf16 table gather: whole rows");
    c10::hip::HIPGuardMasqueradingAsCUDA g(keys.device());
    minips_k::gather_rows_bf16tab(ptr<bf16_t>(table), table.stride(0), ptr<int64_t>(keys), n, base, D, out.data_ptr(),
                                  out.scalar_type() == at::kBFloat16, stream_of(keys), count_ptr(n_dev));
    return;
  }
  check_dtype(table, at::kFloat, "table");
  c10::hip::HIPGuardMasqueradingAsCUDA g(keys.device());
  minips_k::gather_rows(ptr<float>(table), table.stride(0), ptr<int64_t>(keys), n, base, D, out.data_ptr(),
                        out.scalar_type() == at::kBFloat16, stream_of(keys), count_ptr(n_dev));
}

// fp32 gradient rows into bf16 table rows (stochastic rounding): opt 0 row-wise Adagrad, 1 w += scale*g
void sparse_apply_bf16(int64_t opt, at::Tensor& table, const c10::optional<at::Tensor>& state,
                       const c10::optional<at::Tensor>& state2, int64_t D1, const at::Tensor& keys, int64_t base,
                       const at::Tensor& grads, double lr, double eps, double scale, int64_t step, int64_t seed,
                       const c10::optional<at::Tensor>& n_dev) {
  TORCH_CHECK(table.is_cuda() && table.dim() == 2 && table.stride(1) == 1, "table: row-major GPU matrix");
  check_dtype(table, at::kBFloat16, "table");
  check_gpu(keys, "keys");
  check_dtype(keys, at::kLong, "keys");
  check_gpu(grads, "grads");
  check_dtype(grads, at::kFloat, "grads");
  const int64_t n = keys.numel();
  const int D = (int)table.size(1);
  TORCH_CHECK(grads.dim() == 2 && grads.size(0) >= n && grads.size(1) == D, "grads [>= n, D]");
  float* st = opt_ptr<float>(state, at::kFloat, "state");
  float* st2 = opt_ptr<float>(state2, at::kFloat, "state2");
  TORCH_CHECK(opt != 0 || (st && state->numel() >= table.size(0)), "row-wise Adagrad needs its state");
  c10::hip::HIPGuardMasqueradingAsCUDA g(keys.device());
  minips_k::sparse_apply_bf16tab((int)opt, ptr<bf16_t>(table), table.stride(0), st, st2, (int)D1, ptr<int64_t>(keys),
                                 n, base, D, ptr<float>(grads), (float)lr, (float)eps, (float)scale, (uint32_t)step,
                                 (uint32_t)seed, stream_of(keys), count_ptr(n_dev));
}

void lookup_rows(const at::Tensor& rows, const at::Tensor& inv, int64_t F, int64_t D, at::Tensor& out) {
  check_gpu(rows, "rows");
  check_gpu(inv, "inv");
  TORCH_CHECK(out.is_cuda() && out.dim() == 2 && out.stride(1) == 1, "out must be a row-major GPU matrix");
  check_dtype(rows, at::kBFloat16, "rows");
  check_dtype(out, at::kBFloat16, "out");
  const int64_t B = out.size(0);
  TORCH_CHECK(inv.numel() == B * F && rows.size(1) >= D && out.size(1) >= F * D, "lookup_rows shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(rows.device());
  minips_k::lookup_rows(ptr<bf16_t>(rows), (int)rows.size(1), ptr<int64_t>(inv), B, (int)F, (int)D, ptr<bf16_t>(out),
                        (int)out.stride(0), stream_of(rows));
}

void scatter_add_rows(const at::Tensor& src, const at::Tensor& idx, at::Tensor& acc) {
  check_gpu(src, "src");
  check_gpu(idx, "idx");
  check_gpu(acc, "acc");
  check_dtype(idx, at::kLong, "idx");
  TORCH_CHECK(src.dim() == 2 && acc.dim() == 2 && src.size(1) == acc.size(1) && src.is_contiguous(),
              "row widths differ");
  TORCH_CHECK(idx.numel() == src.size(0), "idx/src length mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA g(src.device());
  if (src.scalar_type() == at::kDouble) {
    check_dtype(acc, at::kDouble, "acc");
    minips_k::scatter_add_rows_f64(ptr<double>(src), ptr<int64_t>(idx), src.size(0), (int)src.size(1),
                                   ptr<double>(acc), stream_of(src));
    return;
  }
  TORCH_CHECK(src.scalar_type() == at::kFloat || src.scalar_type() == at::kBFloat16, "src must be fp32 or bf16");
  check_dtype(acc, at::kFloat, "acc");
  if (src.scalar_type() == at::kFloat)
    minips_k::scatter_add_rows(ptr<float>(src), src.size(0), (int)src.size(1), ptr<int64_t>(idx), ptr<float>(acc),
                               stream_of(src));
  else
    minips_k::scatter_add_rows_bf16(ptr<bf16_t>(src), src.size(0), (int)src.size(1), ptr<int64_t>(idx),
                                    ptr<float>(acc), stream_of(src));
}

// slots [cap * P] int32 of the owned unique rows (see kernels.h owner_slots)
at::Tensor owner_slots(const at::Tensor& own_inv, std::vector<int64_t> splits, int64_t cap) {
  check_gpu(own_inv, "own_inv");
  check_dtype(own_inv, at::kLong, "own_inv");
  const int P = (int)splits.size();
  TORCH_CHECK(P >= 1 && P <= minips_k::kOwnerMaxP, "owner_slots: 1..16 requesters");
  minips_k::OwnerSegs segs{};
  int64_t off = 0;
  for (int p = 0; p < P; ++p) {
    segs.off[p] = off;
    off += splits[p];
  }
  segs.off[P] = off;
  TORCH_CHECK(off == own_inv.numel(), "owner_slots: splits must sum to the received rows");
  at::Tensor slots = at::empty({std::max<int64_t>(cap, 1) * P}, own_inv.options().dtype(at::kInt));
  c10::hip::HIPGuardMasqueradingAsCUDA g(own_inv.device());
  minips_k::owner_slots(ptr<int64_t>(own_inv), own_inv.numel(), segs, P, slots.data_ptr<int>(),
                        std::max<int64_t>(cap, 1), stream_of(own_inv));
  return slots;
}

void owner_rows_adagrad(at::Tensor& table, at::Tensor& state, const c10::optional<at::Tensor>& state2, int64_t D1,
                        const at::Tensor& keys, int64_t n, const c10::optional<at::Tensor>& n_dev, int64_t base,
                        const at::Tensor& recv, int64_t P, const at::Tensor& slots, double lr, double eps) {
  TORCH_CHECK(table.is_cuda() && table.dim() == 2 && table.stride(1) == 1, "table must be a row-major GPU matrix");
  check_dtype(table, at::kFloat, "table");
  check_gpu(state, "state");
  check_gpu(keys, "keys");
  check_gpu(recv, "recv");
  check_gpu(slots, "slots");
  check_dtype(slots, at::kInt, "slots");
  TORCH_CHECK(recv.scalar_type() == at::kFloat || recv.scalar_type() == at::kBFloat16, "recv: fp32 or bf16 rows");
  TORCH_CHECK(recv.dim() == 2 && recv.is_contiguous() && recv.size(1) <= table.size(1), "recv [M, D] contiguous");
  TORCH_CHECK(keys.numel() >= n && slots.numel() >= n * P, "keys / slots shorter than n");
  float* s2 = opt_ptr<float>(state2, at::kFloat, "state2");
  c10::hip::HIPGuardMasqueradingAsCUDA g(table.device());
  minips_k::owner_rows_adagrad(ptr<float>(table), table.stride(0), ptr<float>(state), s2, (int)D1, ptr<int64_t>(keys),
                               n, count_ptr(n_dev), base, (int)recv.size(1), recv.data_ptr(),
                               recv.scalar_type() == at::kBFloat16, (int)P, slots.data_ptr<int>(), (float)lr,
                               (float)eps, stream_of(table));
}

// direct-addressed owner apply of one push (kernels.h owner_push_adagrad); rs: int32 [rows_local * P * 2]
void owner_push_adagrad(at::Tensor& table, at::Tensor& state, const c10::optional<at::Tensor>& state2, int64_t D1,
                        const at::Tensor& keys, int64_t base, const at::Tensor& recv, std::vector<int64_t> splits,
                        at::Tensor& rs, int64_t stamp, double lr, double eps) {
  TORCH_CHECK(table.is_cuda() && table.dim() == 2 && table.stride(1) == 1, "table must be a row-major GPU matrix");
  check_dtype(table, at::kFloat, "table");
  check_gpu(state, "state");
  check_gpu(keys, "keys");
  check_dtype(keys, at::kLong, "keys");
  check_gpu(recv, "recv");
  check_gpu(rs, "rs");
  check_dtype(rs, at::kInt, "rs");
  TORCH_CHECK(recv.scalar_type() == at::kFloat || recv.scalar_type() == at::kBFloat16, "recv: fp32 or bf16 rows");
  TORCH_CHECK(recv.dim() == 2 && recv.is_contiguous() && recv.size(1) <= table.size(1), "recv [M, D] contiguous");
  const int P = (int)splits.size();
  TORCH_CHECK(P >= 1 && P <= minips_k::kOwnerMaxP, "owner_push_adagrad: 1..16 requesters");
  minips_k::OwnerSegs segs{};
  int64_t off = 0;
  for (int p = 0; p < P; ++p) {
    segs.off[p] = off;
    off += splits[p];
  }
  segs.off[P] = off;
  TORCH_CHECK(off == keys.numel() && off <= recv.size(0), "owner_push_adagrad: splits must sum to the received keys");
  TORCH_CHECK(rs.is_contiguous() && rs.numel() >= table.size(0) * P * 2, "owner_push_adagrad: rs [rows * P] int2");
  TORCH_CHECK(off < (int64_t)INT32_MAX, "owner_push_adagrad: < 2^31 received rows");
  float* s2 = opt_ptr<float>(state2, at::kFloat, "state2");
  c10::hip::HIPGuardMasqueradingAsCUDA g(table.device());
  minips_k::owner_push_adagrad(ptr<float>(table), table.stride(0), ptr<float>(state), s2, (int)D1, ptr<int64_t>(keys),
                               off, base, table.size(0), (int)recv.size(1), recv.data_ptr(),
                               recv.scalar_type() == at::kBFloat16, segs, P, rs.data_ptr(), (int)stamp, (float)lr,
                               (float)eps, stream_of(table));
}

void sparse_rowwise_adagrad(at::Tensor& table, at::Tensor& state, const c10::optional<at::Tensor>& state2, int64_t D1,
                            const at::Tensor& keys, int64_t base, const at::Tensor& grads, double lr, double eps,
                            const c10::optional<at::Tensor>& n_dev, bool zero_g) {
  TORCH_CHECK(table.is_cuda() && table.dim() == 2 && table.stride(1) == 1, "table must be a row-major GPU matrix");
  check_gpu(state, "state");
  check_gpu(keys, "keys");
  check_gpu(grads, "grads");
  check_dtype(table, at::kFloat, "table");
  check_dtype(grads, at::kFloat, "grads");
  TORCH_CHECK(grads.dim() == 2 && grads.size(0) == keys.numel() && grads.size(1) <= table.size(1), "grads shape");
  float* s2 = opt_ptr<float>(state2, at::kFloat, "state2");
  c10::hip::HIPGuardMasqueradingAsCUDA g(table.device());
  minips_k::sparse_rowwise_adagrad(ptr<float>(table), table.stride(0), ptr<float>(state), s2, (int)D1,
                                   ptr<int64_t>(keys), keys.numel(), base, (int)grads.size(1), ptr<float>(grads),
                                   (float)lr, (float)eps, stream_of(table), count_ptr(n_dev), zero_g);
}

void sparse_sgd(at::Tensor& table, const at::Tensor& keys, int64_t base, const at::Tensor& grads, double scale,
                const c10::optional<at::Tensor>& n_dev) {
  TORCH_CHECK(table.is_cuda() && table.dim() == 2 && table.stride(1) == 1, "table must be a row-major GPU matrix");
  check_gpu(keys, "keys");
  check_gpu(grads, "grads");
  TORCH_CHECK(grads.dim() == 2 && grads.size(0) == keys.numel() && grads.size(1) <= table.size(1), "grads shape");
  check_dtype(keys, at::kLong, "keys");
  c10::hip::HIPGuardMasqueradingAsCUDA g(table.device());
  if (table.scalar_type() == at::kDouble) {
    check_dtype(grads, at::kDouble, "grads");
    TORCH_CHECK(grads.size(1) == table.size(1) && table.is_contiguous(), "fp64 apply: whole rows");
    minips_k::sparse_add_f64(ptr<double>(table), (int)table.size(1), ptr<int64_t>(keys), base, ptr<double>(grads),
                             keys.numel(), scale, count_ptr(n_dev), stream_of(table));
    return;
  }
  check_dtype(table, at::kFloat, "table");
  check_dtype(grads, at::kFloat, "grads");
  minips_k::sparse_sgd(ptr<float>(table), table.stride(0), ptr<int64_t>(keys), keys.numel(), base,
                       (int)grads.size(1), ptr<float>(grads), (float)scale, stream_of(table), count_ptr(n_dev));
}

void embedding_bag_fwd(const at::Tensor& rows, const at::Tensor& idx, const at::Tensor& offsets, bool mean,
                       at::Tensor& out) {
  check_gpu(rows, "rows");
  check_gpu(idx, "idx");
  check_gpu(offsets, "offsets");
  check_gpu(out, "out");
  TORCH_CHECK(out.size(0) == offsets.numel() - 1 && out.size(1) == rows.size(1), "out shape");
  c10::hip::HIPGuardMasqueradingAsCUDA g(rows.device());
  minips_k::embedding_bag_fwd(ptr<float>(rows), ptr<int64_t>(idx), ptr<int64_t>(offsets), out.size(0),
                              (int)rows.size(1), mean, ptr<float>(out), stream_of(rows));
}

void embedding_bag_bwd(const at::Tensor& grad_out, const at::Tensor& idx, const at::Tensor& offsets, bool mean,
                       at::Tensor& grad_rows) {
  check_gpu(grad_out, "grad_out");
  check_gpu(grad_rows, "grad_rows");
  TORCH_CHECK(grad_out.size(1) == grad_rows.size(1), "width mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA g(grad_out.device());
  minips_k::embedding_bag_bwd(ptr<float>(grad_out), ptr<int64_t>(idx), ptr<int64_t>(offsets), grad_out.size(0),
                              (int)grad_out.size(1), mean, ptr<float>(grad_rows), stream_of(grad_out));
}

void wd_assemble(const at::Tensor& dense, const at::Tensor& rows, const at::Tensor& inv, int64_t F, int64_t D,
                 at::Tensor& X, at::Tensor& wide_logit, int64_t ones_col, const c10::optional<at::Tensor>& zero) {
  float* z = opt_ptr<float>(zero, at::kFloat, "zero");
  if (z) TORCH_CHECK(zero->numel() >= 1, "zero: at least one element");
  check_gpu(dense, "dense");
  check_gpu(rows, "rows");
  check_gpu(inv, "inv");
  check_gpu(X, "X");
  check_gpu(wide_logit, "wide_logit");
  check_dtype(rows, at::kBFloat16, "rows");
  check_dtype(X, at::kBFloat16, "X");
  check_dtype(dense, at::kFloat, "dense");
  const int64_t B = X.size(0);
  TORCH_CHECK(inv.numel() == B * F, "inv must be [B*F]");
  TORCH_CHECK(dense.size(0) == B, "dense rows");
  TORCH_CHECK(rows.size(1) > D, "rows must hold D deep values + the wide weight");
  c10::hip::HIPGuardMasqueradingAsCUDA g(X.device());
  minips_k::wd_assemble(ptr<float>(dense), (int)dense.size(1), ptr<bf16_t>(rows), (int)rows.size(1),
                        ptr<int64_t>(inv), B, (int)F, (int)D, ptr<bf16_t>(X), (int)X.size(1), ptr<float>(wide_logit),
                        (int)ones_col, stream_of(X), z);
}

// wd_assemble reading the fp32 table shard directly: row of lookup (b, f) = tab[uniq[inv] - base]
void wd_assemble_tab(const at::Tensor& dense, const at::Tensor& tab, const at::Tensor& uniq, int64_t base,
                     const at::Tensor& inv, int64_t F, int64_t D, at::Tensor& X, at::Tensor& wide_logit,
                     int64_t ones_col, const c10::optional<at::Tensor>& zero,
                     const c10::optional<at::Tensor>& rowidx) {
  float* z = opt_ptr<float>(zero, at::kFloat, "zero");
  if (z) TORCH_CHECK(zero->numel() >= 1, "zero: at least one element");
  for (const at::Tensor* t : {&dense, &tab, &uniq, &inv, (const at::Tensor*)&X, (const at::Tensor*)&wide_logit})
    check_gpu(*t, "wd_assemble_tab");
  check_dtype(tab, at::kFloat, "tab");
  check_dtype(uniq, at::kLong, "uniq");
  check_dtype(inv, at::kLong, "inv");
  check_dtype(X, at::kBFloat16, "X");
  check_dtype(dense, at::kFloat, "dense");
  TORCH_CHECK(tab.dim() == 2 && tab.stride(1) == 1, "tab must be a row-major [rows, W] matrix");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(tab.data_ptr()) % 16 == 0, "tab must be 16-byte aligned");
  const int64_t B = X.size(0);
  TORCH_CHECK(inv.numel() == B * F, "inv must be [B*F]");
  TORCH_CHECK(dense.size(0) == B, "dense rows");
  TORCH_CHECK(tab.size(1) > D, "tab rows must hold D deep values + the wide weight");
  const int32_t* ri = nullptr;
  if (rowidx && rowidx->defined()) {
    check_gpu(*rowidx, "rowidx");
    check_dtype(*rowidx, at::kInt, "rowidx");
    TORCH_CHECK(rowidx->numel() == B * F, "rowidx must be [B*F]");
    ri = rowidx->data_ptr<int32_t>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(X.device());
  minips_k::wd_assemble_tab(ptr<float>(dense), (int)dense.size(1), ptr<float>(tab), tab.stride(0),
                            ptr<int64_t>(uniq), base, ptr<int64_t>(inv), B, (int)F, (int)D, ptr<bf16_t>(X),
                            (int)X.size(1), ptr<float>(wide_logit), (int)ones_col, stream_of(X), z, ri);
}

void wd_head(const at::Tensor& H, const at::Tensor& w, const at::Tensor& b0, const at::Tensor& wide_logit,
             const at::Tensor& labels, at::Tensor& dH, at::Tensor& dw, at::Tensor& db, at::Tensor& dwide,
             at::Tensor& loss_sum, const c10::optional<at::Tensor>& dH_colsum, double grad_scale, bool defer_fold) {
  for (auto* t : {&H, &w, &b0, &wide_logit, &labels}) check_gpu(*t, "wd_head input");
  check_dtype(H, at::kBFloat16, "H");
  check_dtype(w, at::kBFloat16, "w");
  check_dtype(b0, at::kBFloat16, "b0");
  check_dtype(dH, at::kBFloat16, "dH");
  TORCH_CHECK(dH.sizes() == H.sizes(), "dH shape");
  TORCH_CHECK(w.numel() == H.size(1) && dw.numel() == H.size(1), "w/dw length");
  float* cs = opt_ptr<float>(dH_colsum, at::kFloat, "dH_colsum");
  c10::hip::HIPGuardMasqueradingAsCUDA g(H.device());
  minips_k::wd_head(ptr<bf16_t>(H), H.size(0), (int)H.size(1), ptr<bf16_t>(w), ptr<bf16_t>(b0),
                    ptr<float>(wide_logit), ptr<float>(labels), ptr<bf16_t>(dH), ptr<float>(dw), ptr<float>(db),
                    ptr<float>(dwide), ptr<float>(loss_sum), cs, (float)grad_scale, stream_of(H), defer_fold);
}

struct HeadFoldLaunch {
  int64_t B;
  int Hd;
  float *dw, *db, *loss, *colsum;
  void launch(hipStream_t s) const { minips_k::wd_head_fold(B, Hd, dw, db, loss, colsum, s); }
};

HeadFoldLaunch prepare_head_fold(int64_t B, int64_t Hd, at::Tensor& dw, at::Tensor& db, at::Tensor& loss_sum,
                                 const c10::optional<at::Tensor>& dH_colsum) {
  for (auto* t : {&dw, &db, &loss_sum}) {
    check_gpu(*t, "wd_head_fold output");
    check_dtype(*t, at::kFloat, "wd_head_fold output");
  }
  TORCH_CHECK(dw.numel() == Hd && db.numel() >= 1 && loss_sum.numel() >= 1, "wd_head_fold: dw [Hd], db, loss");
  float* cs = opt_ptr<float>(dH_colsum, at::kFloat, "dH_colsum");
  TORCH_CHECK(!cs || dH_colsum->numel() >= Hd, "wd_head_fold: dH_colsum >= Hd floats");
  return HeadFoldLaunch{B, (int)Hd, ptr<float>(dw), ptr<float>(db), ptr<float>(loss_sum), cs};
}

// the totals of the last wd_head(defer_fold=True) of this device (same B, Hd), on dw's stream
void wd_head_fold(int64_t B, int64_t Hd, at::Tensor& dw, at::Tensor& db, at::Tensor& loss_sum,
                  const c10::optional<at::Tensor>& dH_colsum) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(dw.device());
  prepare_head_fold(B, Hd, dw, db, loss_sum, dH_colsum).launch(stream_of(dw));
}

// Lookup CSR grouped by unique row (members/memrow int32 [B*F]) for U (upper-bound) rows.
std::vector<at::Tensor> emb_build_csr(const at::Tensor& inv, int64_t F, int64_t U,
                                      const c10::optional<at::Tensor>& zeroed, bool counts_ready) {
  check_gpu(inv, "inv");
  check_dtype(inv, at::kLong, "inv");
  const int64_t n = inv.numel();
  TORCH_CHECK(F >= 1 && n % F == 0 && U >= 1 && U < (1ll << 31) && n < (1ll << 31), "emb_build_csr shapes");
  auto io = inv.options().dtype(at::kInt);
  int* zc = nullptr;
  if (zeroed.has_value() && zeroed->defined()) {
    TORCH_CHECK(zeroed->is_cuda() && zeroed->scalar_type() == at::kInt && zeroed->numel() >= 2 * U,
                "zeroed: int32 GPU block of >= 2U (already zero)");
    zc = zeroed->data_ptr<int>();
  }
  at::Tensor ws = at::empty({(zc ? 0 : 2 * U) + U + 1 + U / 1024 + 1}, io);
  at::Tensor members = at::empty({n}, io), memrow = at::empty({n}, io);
  c10::hip::HIPGuardMasqueradingAsCUDA g(inv.device());
  minips_k::emb_build_csr(ptr<int64_t>(inv), n / F, (int)F, (int)U, ws.data_ptr<int>(), members.data_ptr<int>(),
                          memrow.data_ptr<int>(), stream_of(inv), zc, counts_ready && zc);
  return {members, memrow};
}

void wd_emb_backward(const at::Tensor& dX, const c10::optional<at::Tensor>& dwide, const at::Tensor& inv, int64_t F,
                     int64_t D, at::Tensor& grad_rows, int64_t x_off, const c10::optional<at::Tensor>& members,
                     const c10::optional<at::Tensor>& memrow, bool sorted_rows) {
  check_gpu(dX, "dX");
  const float* dw = opt_ptr<float>(dwide, at::kFloat, "dwide");
  check_gpu(inv, "inv");
  check_gpu(grad_rows, "grad_rows");
  TORCH_CHECK(dX.scalar_type() == at::kFloat || dX.scalar_type() == at::kBFloat16, "dX must be fp32 or bf16");
  const bool out_bf = grad_rows.scalar_type() == at::kBFloat16;
  TORCH_CHECK(out_bf || grad_rows.scalar_type() == at::kFloat, "grad_rows must be fp32 or bf16");
  TORCH_CHECK(dX.dim() == 2 && dX.stride(1) == 1, "dX must be a row-major matrix");
  if (sorted_rows) {  // dX [B*F, D] in the CSR's member order (kEpiPermRowsBf16 dgrad output)
    TORCH_CHECK(members.has_value() && members->defined() && x_off == 0 && dX.size(1) == D && dX.is_contiguous() &&
                    dX.size(0) == inv.numel() && inv.numel() % F == 0, "sorted rows: dX [B*F, D] + the CSR");
  }
  const int64_t B = sorted_rows ? inv.numel() / F : dX.size(0);
  TORCH_CHECK(inv.numel() == B * F && (sorted_rows || dX.size(1) >= x_off + F * D) &&
                  grad_rows.size(1) >= D + (dw ? 1 : 0), "shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(dX.device());
  if ((D == 16 || D == 32 || D == 64) && grad_rows.size(0) < (1ll << 31) && B * F < (1ll << 31) && x_off % 4 == 0 &&
      dX.stride(0) % 4 == 0) {
    // segment-sum path: writes rows [0, U) of grad_rows exactly once (deterministic)
    const int64_t U = grad_rows.size(0);
    TORCH_CHECK(grad_rows.stride(1) == 1, "grad_rows must be row-major");
    const bool bf0 = dX.scalar_type() == at::kBFloat16;
    const void* base0 = bf0 ? (const void*)(ptr<bf16_t>(dX) + x_off) : (const void*)(ptr<float>(dX) + x_off);
    at::Tensor part = at::empty({minips_k::emb_seg_part_floats(B * F, D)}, dX.options().dtype(at::kFloat));
    if (members.has_value() && members->defined()) {  // CSR prebuilt at planning time
      TORCH_CHECK(memrow.has_value() && members->numel() == B * F && memrow->numel() == B * F &&
                      members->scalar_type() == at::kInt && memrow->scalar_type() == at::kInt,
                  "members/memrow: int32 [B*F]");
      minips_k::emb_backward_csr(base0, bf0, (int)dX.stride(0), dw, B, (int)F, (int)D, members->data_ptr<int>(),
                                 memrow->data_ptr<int>(), grad_rows.data_ptr(), out_bf, (int)grad_rows.stride(0),
                                 part.data_ptr<float>(), stream_of(dX), sorted_rows);
      return;
    }
    at::Tensor ws = at::empty({3 * U + 1 + 2 * B * F + U / 1024 + 1}, inv.options().dtype(at::kInt));
    minips_k::emb_backward_segment(base0, bf0, (int)dX.stride(0), dw, ptr<int64_t>(inv), B, (int)F, (int)D,
                                   grad_rows.data_ptr(), out_bf, (int)grad_rows.stride(0), (int)U, ws.data_ptr<int>(),
                                   part.data_ptr<float>(), stream_of(dX));
    return;
  }
  TORCH_CHECK(!out_bf, "bf16 gradient rows need the segment-sum path (D 16 / 32 / 64, 4-aligned strides)");
  if (dX.scalar_type() == at::kFloat)
    minips_k::wd_emb_backward(ptr<float>(dX) + x_off, (int)dX.stride(0), dw, ptr<int64_t>(inv), B, (int)F, (int)D,
                              ptr<float>(grad_rows), (int)grad_rows.size(1), stream_of(dX));
  else
    minips_k::wd_emb_backward_bf16(ptr<bf16_t>(dX) + x_off, (int)dX.stride(0), dw, ptr<int64_t>(inv), B, (int)F,
                                   (int)D, ptr<float>(grad_rows), (int)grad_rows.size(1), stream_of(dX));
}

// Sort-based planning of a [B, F] batch with disjoint column key ranges (see kernels.h).
// Returns (uniq, inv, counts [1], U_dev [1], members, memrow).
std::vector<at::Tensor> plan_sorted(const at::Tensor& keys, const at::Tensor& col_base, const at::Tensor& col_bits,
                                    std::vector<int64_t> col_bits_host, int64_t route_mult, int64_t route_n,
                                    const at::Tensor& bounds, bool with_positions) {
  check_gpu(bounds, "bounds");
  check_dtype(bounds, at::kLong, "bounds");
  const int64_t P = bounds.numel() - 1;
  TORCH_CHECK(P >= 1 && P <= 16, "plan_sorted: 1..16 owners");
  check_gpu(keys, "keys");
  check_dtype(keys, at::kLong, "keys");
  check_gpu(col_base, "col_base");
  check_dtype(col_base, at::kLong, "col_base");
  check_gpu(col_bits, "col_bits");
  check_dtype(col_bits, at::kInt, "col_bits");
  TORCH_CHECK(keys.dim() == 2, "keys: [B, F]");
  const int64_t B = keys.size(0), F = keys.size(1);
  TORCH_CHECK(B >= 1 && B <= 16384 && F >= 1 && F <= 64, "plan_sorted: 1 <= B <= 16384, 1 <= F <= 64");
  TORCH_CHECK(col_base.numel() == F && col_bits.numel() == F && (int64_t)col_bits_host.size() == F,
              "one base / bit count per column");
  // the host copy of the device bit counts is what is validated (the kernel trusts the device one)
  const int obits = P > 1 ? minips_k::plan_owner_bits((int)P) : 0;
  for (int64_t b : col_bits_host)
    TORCH_CHECK(b >= 1 && b + obits <= 32, "col_bits: 1..32, owner bits included (plan_sorted_ok)");
  const int64_t n = B * F;
  // one owner: each row's lookup range in member order (the row-parallel embedding backward);
  // one owner, routed keys below 2^31: each lookup's table row (the input assembly's index)
  const bool want_rs = P == 1, want_ri = P == 1 && route_mult && route_n > 0 && route_n <= INT32_MAX;
  auto parts = carve(keys.options(), {{minips_k::plan_sorted_ws_ints(n, (int)F, (int)P), at::kInt},
                                      {n, at::kLong}, {n, at::kLong}, {n, at::kLong}, {n, at::kInt}, {n, at::kInt},
                                      {P + 1, at::kLong}, {with_positions ? n : 0, at::kInt},
                                      {want_rs ? n + 1 : 0, at::kInt}, {want_ri ? n : 0, at::kInt}});
  auto &ws = parts[0], &ukey = parts[1], &uniq = parts[2], &inv = parts[3], &members = parts[4], &memrow = parts[5],
       &counts = parts[6];
  at::Tensor pos = with_positions ? parts[7] : at::Tensor();
  at::Tensor rowstart = want_rs ? parts[8] : at::Tensor();
  at::Tensor rowidx = want_ri ? parts[9] : at::Tensor();
  c10::hip::HIPGuardMasqueradingAsCUDA g(keys.device());
  minips_k::plan_sorted(ptr<int64_t>(keys), (int)B, (int)F, ptr<int64_t>(col_base), col_bits.data_ptr<int32_t>(),
                        (uint64_t)route_mult, (uint64_t)route_n, ptr<int64_t>(bounds), (int)P, ws.data_ptr<int32_t>(),
                        ptr<int64_t>(ukey),
                        ptr<int64_t>(uniq), ptr<int64_t>(inv), members.data_ptr<int32_t>(), memrow.data_ptr<int32_t>(),
                        ptr<int64_t>(counts), stream_of(keys), with_positions ? pos.data_ptr<int32_t>() : nullptr,
                        rowstart.defined() ? rowstart.data_ptr<int32_t>() : nullptr,
                        rowidx.defined() ? rowidx.data_ptr<int32_t>() : nullptr);
  // (members, memrow, positions or None, rowstart, rowidx or None) with one owner
  if (rowstart.defined())
    return {uniq, inv, counts.narrow(0, 0, P), counts.narrow(0, P, 1), members, memrow, pos, rowstart, rowidx};
  if (with_positions) return {uniq, inv, counts.narrow(0, 0, P), counts.narrow(0, P, 1), members, memrow, pos};
  return {uniq, inv, counts.narrow(0, 0, P), counts.narrow(0, P, 1), members, memrow};
}

// A dedicated HIP stream (hipStreamCreateWithPriority), returned as an integer handle for
// torch.cuda.ExternalStream. torch.cuda.Stream() hands out streams round-robin from a pool of 32 per
// priority, so past 32 of them two "independent" streams silently alias (and a table's clock work
// serialises behind another's planning); tables and the planning stream take their own instead
// (never destroyed: the Python side reuses a dead owner's stream, see ps/comm.py).
int64_t new_stream(int64_t device, int64_t priority) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  hipStream_t st = nullptr;
  const hipError_t e = hipStreamCreateWithPriority(&st, hipStreamNonBlocking, (int)priority);
  TORCH_CHECK(e == hipSuccess, "hipStreamCreateWithPriority: ", hipGetErrorString(e));
  return reinterpret_cast<int64_t>(st);
}

struct ColsumLaunch {
  const bf16_t* x;
  int64_t M;
  int N, ld;
  float *out, *slab;
  void launch(hipStream_t s) const { minips_k::colsum_bf16(x, M, N, ld, out, slab, s); }
};

ColsumLaunch prepare_colsum(const at::Tensor& x, at::Tensor& out, at::Tensor& slab) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "x: row-major GPU matrix");
  check_dtype(x, at::kBFloat16, "x");
  check_gpu(out, "out");
  check_dtype(out, at::kFloat, "out");
  TORCH_CHECK(out.numel() >= x.size(1) && x.size(1) % 8 == 0 && x.stride(0) % 8 == 0,
              "colsum: out >= N floats, N and the row stride multiples of 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "colsum: x must be 16-byte aligned");
  // the blocks' partial rows: a caching-allocator block on the stream (reused, no fill)
  const int64_t strips = (x.size(1) + 63) / 64;
  slab = at::empty({minips_k::colsum_chunks(x.size(0), (int)x.size(1)) * strips * 64}, out.options().dtype(at::kFloat));
  return ColsumLaunch{ptr<bf16_t>(x), x.size(0), (int)x.size(1), (int)x.stride(0), ptr<float>(out),
                      slab.data_ptr<float>()};
}

void colsum_bf16(const at::Tensor& x, at::Tensor& out) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor slab;
  prepare_colsum(x, out, slab).launch(stream_of(x));
}

void adam_apply(at::Tensor& w, at::Tensor& m, at::Tensor& v, const at::Tensor& g, double lr, double beta1,
                double beta2, double eps, double weight_decay, int64_t step, double grad_scale,
                const c10::optional<at::Tensor>& w_bf16, const c10::optional<at::Tensor>& step_dev, bool zero_g,
                const std::vector<std::tuple<at::Tensor, int64_t, int64_t, int64_t>>& slabs) {
  for (auto* t : {&w, &m, &v}) {
    check_gpu(*t, "adam state");
    check_dtype(*t, at::kFloat, "adam state");
  }
  check_gpu(g, "g");
  check_dtype(g, at::kFloat, "g");
  TORCH_CHECK(w.numel() == m.numel() && w.numel() == v.numel() && w.numel() == g.numel(), "adam sizes differ");
  bf16_t* wb = opt_ptr<bf16_t>(w_bf16, at::kBFloat16, "w_bf16");
  if (wb) TORCH_CHECK(w_bf16->numel() == w.numel(), "w_bf16 size");
  // (slab [nsplit * plane] fp32, nsplit, plane, offset of its region in g): the region's length is the plane
  minips_k::AdamSlabs sl;
  TORCH_CHECK(slabs.size() <= 4, "adam: at most 4 slab regions");
  for (const auto& t : slabs) {
    const at::Tensor& p = std::get<0>(t);
    const int64_t ns = std::get<1>(t), plane = std::get<2>(t), off = std::get<3>(t);
    check_gpu(p, "slab");
    check_dtype(p, at::kFloat, "slab");
    TORCH_CHECK(ns >= 1 && p.numel() >= ns * plane && off >= 0 && off + plane <= g.numel(), "adam slab bounds");
    sl.p[sl.n] = ptr<float>(p);
    sl.nsplit[sl.n] = (int)ns;
    sl.plane[sl.n] = plane;
    sl.len[sl.n] = plane;
    sl.off[sl.n] = off;
    ++sl.n;
  }
  c10::hip::HIPGuardMasqueradingAsCUDA gd(w.device());
  minips_k::adam_apply(ptr<float>(w), ptr<float>(m), ptr<float>(v), ptr<float>(g), w.numel(), (float)lr, (float)beta1,
                       (float)beta2, (float)eps, (float)weight_decay, (int)step, (float)grad_scale, wb, stream_of(w),
                       step_dev.has_value() && step_dev->defined() ? step_dev->data_ptr<int>() : nullptr, zero_g,
                       nullptr, sl.n ? &sl : nullptr);
}

// several ranks: the dense clock's reduce-scatter input = g + its split-K slab planes, g cleared
void slab_pack(at::Tensor& g, at::Tensor& out,
               const std::vector<std::tuple<at::Tensor, int64_t, int64_t, int64_t>>& slabs) {
  check_gpu(g, "g");
  check_gpu(out, "out");
  check_dtype(g, at::kFloat, "g");
  check_dtype(out, at::kFloat, "out");
  TORCH_CHECK(out.numel() == g.numel(), "slab_pack: out and g sizes differ");
  minips_k::AdamSlabs sl;
  TORCH_CHECK(slabs.size() <= 4, "slab_pack: at most 4 slab regions");
  for (const auto& t : slabs) {
    const at::Tensor& p = std::get<0>(t);
    const int64_t ns = std::get<1>(t), plane = std::get<2>(t), off = std::get<3>(t);
    check_gpu(p, "slab");
    check_dtype(p, at::kFloat, "slab");
    TORCH_CHECK(ns >= 1 && p.numel() >= ns * plane && off >= 0 && off + plane <= g.numel(), "slab_pack slab bounds");
    sl.p[sl.n] = ptr<float>(p);
    sl.nsplit[sl.n] = (int)ns;
    sl.plane[sl.n] = plane;
    sl.len[sl.n] = plane;
    sl.off[sl.n] = off;
    ++sl.n;
  }
  minips_k::slab_pack(ptr<float>(g), ptr<float>(out), g.numel(), sl.n ? &sl : nullptr, stream_of(g));
}

void emu_sum_slices(const at::Tensor& in, at::Tensor& out, int64_t P) {
  check_gpu(in, "in");
  check_gpu(out, "out");
  check_dtype(in, at::kFloat, "in");
  check_dtype(out, at::kFloat, "out");
  TORCH_CHECK(in.numel() == out.numel() * P, "emu_sum_slices: in = P x out");
  minips_k::emu_sum_slices(ptr<float>(in), ptr<float>(out), out.numel(), (int)P, stream_of(in));
}

void emu_rebase(at::Tensor& keys, int64_t step, int64_t P, int64_t base) {
  check_gpu(keys, "keys");
  check_dtype(keys, at::kLong, "keys");
  minips_k::emu_rebase(ptr<int64_t>(keys), keys.numel(), step, (int)P, base, stream_of(keys));
}

// split-K GEMM into slab planes without their reduction (the Adam kernel folds them): returns nsplit
int64_t gemm_slab(const at::Tensor& A, const at::Tensor& B, at::Tensor& slab, int64_t M, int64_t N, int64_t K,
                  bool a_km, bool b_kn, int64_t split_k) {
  check_gpu(A, "A");
  check_gpu(B, "B");
  check_gpu(slab, "slab");
  check_dtype(A, at::kBFloat16, "A");
  check_dtype(B, at::kBFloat16, "B");
  check_dtype(slab, at::kFloat, "slab");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2, "2-D operands");
  TORCH_CHECK(slab.numel() >= split_k * M * N, "slab: >= split_k * M * N floats");
  const int64_t lda = A.stride(0), ldb = B.stride(0);
  c10::hip::HIPGuardMasqueradingAsCUDA gd(A.device());
  return minips_k::gemm_slab(ptr<bf16_t>(A), ptr<bf16_t>(B), ptr<float>(slab), (int)M, (int)N, (int)K, (int)lda,
                             (int)ldb, a_km, b_kn, (int)split_k, stream_of(A));
}

void sgd_apply(at::Tensor& w, const at::Tensor& g, double lr, double grad_scale,
               const c10::optional<at::Tensor>& w_bf16) {
  check_gpu(w, "w");
  check_gpu(g, "g");
  TORCH_CHECK(w.numel() == g.numel(), "sizes differ");
  bf16_t* wb = opt_ptr<bf16_t>(w_bf16, at::kBFloat16, "w_bf16");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(w.device());
  minips_k::sgd_apply(ptr<float>(w), ptr<float>(g), w.numel(), (float)lr, (float)grad_scale, wb, stream_of(w));
}

void adagrad_apply(at::Tensor& w, at::Tensor& acc, const at::Tensor& g, double lr, double eps, double grad_scale,
                   const c10::optional<at::Tensor>& w_bf16) {
  check_gpu(w, "w");
  check_gpu(acc, "acc");
  check_gpu(g, "g");
  TORCH_CHECK(w.numel() == g.numel() && w.numel() == acc.numel(), "sizes differ");
  bf16_t* wb = opt_ptr<bf16_t>(w_bf16, at::kBFloat16, "w_bf16");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(w.device());
  minips_k::adagrad_apply(ptr<float>(w), ptr<float>(acc), ptr<float>(g), w.numel(), (float)lr, (float)eps,
                          (float)grad_scale, wb, stream_of(w));
}

void cast_f32_bf16(const at::Tensor& x, at::Tensor& y) {
  check_gpu(x, "x");
  check_gpu(y, "y");
  check_dtype(x, at::kFloat, "x");
  check_dtype(y, at::kBFloat16, "y");
  TORCH_CHECK(x.numel() == y.numel(), "sizes differ");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(x.device());
  minips_k::cast_f32_bf16(ptr<float>(x), ptr<bf16_t>(y), x.numel(), stream_of(x));
}

void lr_sparse_step(const at::Tensor& rowptr, const at::Tensor& cols, const at::Tensor& vals,
                    const at::Tensor& labels, const at::Tensor& w, double alpha,
                    const c10::optional<at::Tensor>& delta, const c10::optional<at::Tensor>& correct) {
  for (auto* t : {&rowptr, &cols, &vals, &labels, &w}) check_gpu(*t, "lr input");
  check_dtype(vals, at::kFloat, "vals");
  TORCH_CHECK(rowptr.numel() == labels.numel() + 1, "rowptr must be [B+1]");
  if (w.scalar_type() == at::kDouble) {  // reference-precision LR (double tables)
    double* d = opt_ptr<double>(delta, at::kDouble, "delta");
    if (d) TORCH_CHECK(delta->numel() == w.numel(), "delta must match w");
    float* c = opt_ptr<float>(correct, at::kFloat, "correct");
    c10::hip::HIPGuardMasqueradingAsCUDA gd(w.device());
    minips_k::lr_sparse_step_f64(ptr<int64_t>(rowptr), ptr<int64_t>(cols), ptr<float>(vals), ptr<float>(labels),
                                 labels.numel(), ptr<double>(w), alpha, d, c, stream_of(w));
    return;
  }
  check_dtype(w, at::kFloat, "w");
  float* d = opt_ptr<float>(delta, at::kFloat, "delta");
  if (d) TORCH_CHECK(delta->numel() == w.numel(), "delta must match w");
  float* c = opt_ptr<float>(correct, at::kFloat, "correct");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(w.device());
  minips_k::lr_sparse_step(ptr<int64_t>(rowptr), ptr<int64_t>(cols), ptr<float>(vals), ptr<float>(labels),
                           labels.numel(), ptr<float>(w), (float)alpha, d, c, stream_of(w));
}

void kmeans_assign(const at::Tensor& X, const at::Tensor& C, at::Tensor& assign,
                   const c10::optional<at::Tensor>& dist) {
  check_gpu(X, "X");
  check_gpu(C, "C");
  check_gpu(assign, "assign");
  check_dtype(X, at::kFloat, "X");
  check_dtype(C, at::kFloat, "C");
  check_dtype(assign, at::kInt, "assign");
  TORCH_CHECK(X.size(1) == C.size(1) && assign.numel() == X.size(0), "kmeans shapes");
  float* dp = opt_ptr<float>(dist, at::kFloat, "dist");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(X.device());
  minips_k::kmeans_assign(ptr<float>(X), X.size(0), (int)X.size(1), ptr<float>(C), (int)C.size(0),
                          ptr<int32_t>(assign), dp, stream_of(X));
}

void kmeans_split3(const at::Tensor& src, at::Tensor& out, int64_t order, at::Tensor& norms) {
  check_gpu(src, "src");
  check_gpu(out, "out");
  check_gpu(norms, "norms");
  check_dtype(src, at::kFloat, "src");
  check_dtype(out, at::kBFloat16, "out");
  check_dtype(norms, at::kFloat, "norms");
  TORCH_CHECK(src.is_contiguous() && out.is_contiguous() && out.size(0) == src.size(0) &&
                  out.size(1) >= 3 * src.size(1) && norms.numel() >= src.size(0), "kmeans_split3 shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(src.device());
  minips_k::kmeans_split3(ptr<float>(src), src.size(0), (int)src.size(1), ptr<bf16_t>(out), (int)out.size(1),
                          (int)order, ptr<float>(norms), stream_of(src));
}

void kmeans_argmin(const at::Tensor& S, const at::Tensor& cn, const at::Tensor& xn, at::Tensor& assign,
                   const c10::optional<at::Tensor>& dist) {
  for (const at::Tensor* t : {&S, &cn, &xn}) {
    check_gpu(*t, "kmeans_argmin arg");
    check_dtype(*t, at::kFloat, "kmeans_argmin arg");
  }
  check_dtype(assign, at::kInt, "assign");
  TORCH_CHECK(S.dim() == 2 && S.is_contiguous() && cn.numel() >= S.size(1) && xn.numel() >= S.size(0) &&
                  assign.numel() >= S.size(0), "kmeans_argmin shapes");
  float* dp = opt_ptr<float>(dist, at::kFloat, "dist");
  c10::hip::HIPGuardMasqueradingAsCUDA g(S.device());
  minips_k::kmeans_argmin(ptr<float>(S), S.size(0), (int)S.size(1), ptr<float>(cn), ptr<float>(xn),
                          ptr<int32_t>(assign), dp, stream_of(S));
}

void criteo_synth(int64_t seed, int64_t step, const c10::optional<at::Tensor>& step_dev, const at::Tensor& cards,
                  const at::Tensor& offsets, const at::Tensor& w, at::Tensor& dense, at::Tensor& keys,
                  at::Tensor& labels) {
  for (const at::Tensor* t : {&cards, &offsets, &w, (const at::Tensor*)&dense, (const at::Tensor*)&keys,
                              (const at::Tensor*)&labels}) check_gpu(*t, "criteo_synth arg");
  check_dtype(keys, at::kLong, "keys");
  check_dtype(cards, at::kLong, "cards");
  const int64_t B = labels.numel();
  const int F = (int)cards.numel();
  TORCH_CHECK(keys.numel() == B * F && dense.size(0) == B && w.numel() == dense.size(1), "criteo_synth shapes");
  const int64_t* sd = nullptr;
  if (step_dev && step_dev->defined()) {
    check_gpu(*step_dev, "step_dev");
    check_dtype(*step_dev, at::kLong, "step_dev");
    sd = ptr<int64_t>(*step_dev);
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(keys.device());
  minips_k::criteo_synth((uint64_t)seed, (uint64_t)step, sd, B, F, ptr<int64_t>(cards), ptr<int64_t>(offsets),
                         (int)dense.size(1), ptr<float>(w), ptr<float>(dense), ptr<int64_t>(keys), ptr<float>(labels),
                         stream_of(keys));
}

// dst[i].copy_(src[i]) for every pair, in one launch on dst[0]'s current stream (same byte sizes,
// contiguous, one device; at most 16 pairs per launch)
void multi_copy(const std::vector<at::Tensor>& dst, const std::vector<at::Tensor>& src) {
  TORCH_CHECK(dst.size() == src.size() && !dst.empty(), "multi_copy: matching non-empty lists");
  for (size_t base = 0; base < dst.size(); base += minips_k::kMultiCopyMax) {
    minips_k::MultiCopyArgs a{};
    a.n = (int)std::min<size_t>(minips_k::kMultiCopyMax, dst.size() - base);
    a.start[0] = 0;
    for (int t = 0; t < a.n; ++t) {
      const at::Tensor& d = dst[base + t];
      const at::Tensor& s = src[base + t];
      TORCH_CHECK(d.is_cuda() && s.is_cuda() && d.get_device() == s.get_device(), "multi_copy: one GPU");
      TORCH_CHECK(d.is_contiguous() && s.is_contiguous(), "multi_copy: contiguous tensors");
      const int64_t nb = d.numel() * d.element_size();
      TORCH_CHECK(nb == s.numel() * s.element_size(), "multi_copy: byte sizes differ");
      a.dst[t] = d.data_ptr();
      a.src[t] = s.data_ptr();
      const bool al = (reinterpret_cast<uintptr_t>(a.dst[t]) & 15) == 0 &&
                      (reinterpret_cast<uintptr_t>(a.src[t]) & 15) == 0;
      a.n16[t] = al ? nb / 16 : 0;
      a.tail[t] = nb - a.n16[t] * 16;
      a.start[t + 1] = a.start[t] + a.n16[t] + a.tail[t];
    }
    minips_k::multi_copy(a, stream_of(dst[base]));
  }
}

// out: int64 [2] on the GPU; launched on `stream` (a torch stream handle; 0 = out's current stream)
void clock_probe(at::Tensor& out, int64_t spin_ticks, int64_t stream) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kLong && out.numel() >= 2 && out.is_contiguous(),
              "clock_probe: out must be a contiguous int64 CUDA tensor of >= 2 elements");
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : stream_of(out);
  minips_k::clock_probe(ptr<int64_t>(out), (int)spin_ticks, s);
}

void uniform_synth(int64_t seed, int64_t step, int64_t rows, at::Tensor& dense, at::Tensor& keys, at::Tensor& labels) {
  for (const at::Tensor* t : {(const at::Tensor*)&dense, (const at::Tensor*)&keys, (const at::Tensor*)&labels})
    check_gpu(*t, "uniform_synth arg");
  check_dtype(keys, at::kLong, "keys");
  check_dtype(dense, at::kFloat, "dense");
  check_dtype(labels, at::kFloat, "labels");
  TORCH_CHECK(keys.dim() == 2 && dense.dim() == 2 && keys.is_contiguous() && dense.is_contiguous() &&
                  labels.is_contiguous() && keys.size(0) == labels.numel() && dense.size(0) == labels.numel(),
              "uniform_synth shapes: keys [B, F], dense [B, n], labels [B]");
  c10::hip::HIPGuardMasqueradingAsCUDA g(keys.device());
  minips_k::uniform_synth((uint64_t)seed, (uint64_t)step, keys.size(0), (int)keys.size(1), (uint64_t)rows,
                          (int)dense.size(1), ptr<float>(dense), ptr<int64_t>(keys), ptr<float>(labels),
                          stream_of(keys));
}

void check_ln(const at::Tensor& t, int64_t C, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.stride(1) == 1 && t.size(1) >= C && t.stride(0) % 4 == 0, n,
              " must be a row-major GPU matrix with >= C columns and a leading dim % 4 == 0");
  check_dtype(t, at::kBFloat16, n);
}

void layernorm_fwd(const at::Tensor& x, int64_t C, const at::Tensor& gamma, const at::Tensor& beta, double eps,
                   at::Tensor& y, at::Tensor& mean, at::Tensor& rstd) {
  TORCH_CHECK(C % 4 == 0 && C <= 1024, "layernorm: C % 4 == 0 and C <= 1024");
  check_ln(x, C, "x");
  check_ln(y, C, "y");
  TORCH_CHECK(y.size(0) == x.size(0) && mean.numel() == x.size(0) && rstd.numel() == x.size(0), "layernorm rows");
  check_gpu(gamma, "gamma");
  check_gpu(beta, "beta");
  check_dtype(gamma, at::kBFloat16, "gamma");
  check_dtype(beta, at::kBFloat16, "beta");
  check_dtype(mean, at::kFloat, "mean");
  check_dtype(rstd, at::kFloat, "rstd");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  minips_k::layernorm_fwd(ptr<bf16_t>(x), (int)x.stride(0), x.size(0), (int)C, ptr<bf16_t>(gamma), ptr<bf16_t>(beta),
                          (float)eps, ptr<bf16_t>(y), (int)y.stride(0), ptr<float>(mean), ptr<float>(rstd),
                          stream_of(x));
}

void layernorm_bwd(const at::Tensor& x, const at::Tensor& dy, int64_t C, const at::Tensor& gamma,
                   const at::Tensor& mean, const at::Tensor& rstd, at::Tensor& dx, at::Tensor& dgamma,
                   at::Tensor& dbeta, bool accumulate) {
  TORCH_CHECK(C % 4 == 0 && C <= 1024, "layernorm: C % 4 == 0 and C <= 1024");
  check_ln(x, C, "x");
  check_ln(dy, C, "dy");
  check_ln(dx, C, "dx");
  const int64_t M = x.size(0);
  TORCH_CHECK(dy.size(0) == M && dx.size(0) == M && mean.numel() == M && rstd.numel() == M, "layernorm_bwd rows");
  check_dtype(gamma, at::kBFloat16, "gamma");
  check_dtype(dgamma, at::kFloat, "dgamma");
  check_dtype(dbeta, at::kFloat, "dbeta");
  TORCH_CHECK(gamma.numel() >= C && dgamma.numel() >= C && dbeta.numel() >= C, "layernorm_bwd params");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor partial = at::empty({(int64_t)minips_k::layernorm_bwd_blocks(M) * 2 * C}, x.options().dtype(at::kFloat));
  minips_k::layernorm_bwd(ptr<bf16_t>(x), (int)x.stride(0), ptr<bf16_t>(dy), (int)dy.stride(0), M, (int)C,
                          ptr<bf16_t>(gamma), ptr<float>(mean), ptr<float>(rstd), ptr<bf16_t>(dx), (int)dx.stride(0),
                          ptr<float>(dgamma), ptr<float>(dbeta), ptr<float>(partial), accumulate, stream_of(x));
}

void softmax_xent(at::Tensor& logits, int64_t V, const at::Tensor& labels, double scale, at::Tensor& loss_sum,
                  const c10::optional<at::Tensor>& correct) {
  check_gpu(logits, "logits");
  check_gpu(labels, "labels");
  check_dtype(logits, at::kBFloat16, "logits");
  check_dtype(labels, at::kLong, "labels");
  TORCH_CHECK(logits.dim() == 2 && logits.size(1) >= V && labels.numel() == logits.size(0), "softmax_xent shapes");
  float* c = opt_ptr<float>(correct, at::kFloat, "correct");
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  minips_k::softmax_xent(ptr<bf16_t>(logits), (int)logits.size(1), logits.size(0), (int)V, ptr<int64_t>(labels),
                         (float)scale, ptr<float>(loss_sum), c, stream_of(logits));
}

void causal_softmax_fwd(const at::Tensor& S, int64_t T, at::Tensor& P) {
  check_gpu(S, "S");
  check_gpu(P, "P");
  TORCH_CHECK(S.numel() == P.numel() && S.numel() % (T * T) == 0, "causal_softmax shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(S.device());
  minips_k::causal_softmax_fwd(ptr<float>(S), S.numel() / T, (int)T, ptr<bf16_t>(P), stream_of(S));
}

void causal_softmax_bwd(const at::Tensor& P, const at::Tensor& dP, int64_t T, double scale, at::Tensor& dS) {
  check_gpu(P, "P");
  check_gpu(dP, "dP");
  check_gpu(dS, "dS");
  TORCH_CHECK(P.numel() == dP.numel() && P.numel() == dS.numel() && P.numel() % (T * T) == 0, "shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(P.device());
  minips_k::causal_softmax_bwd(ptr<bf16_t>(P), ptr<float>(dP), P.numel() / T, (int)T, (float)scale, ptr<bf16_t>(dS),
                               stream_of(P));
}

void gelu_bwd(const at::Tensor& dh, const at::Tensor& u, at::Tensor& du) {
  TORCH_CHECK(dh.numel() == u.numel() && du.numel() == u.numel(), "gelu_bwd sizes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(u.device());
  minips_k::gelu_bwd(ptr<bf16_t>(dh), ptr<bf16_t>(u), u.numel(), ptr<bf16_t>(du), stream_of(u));
}

void add_bf16(const at::Tensor& a, const at::Tensor& b, at::Tensor& out) {
  TORCH_CHECK(a.numel() == b.numel() && out.numel() == a.numel(), "add sizes");
  check_gpu(a, "a");
  check_gpu(b, "b");
  check_gpu(out, "out");
  c10::hip::HIPGuardMasqueradingAsCUDA g(a.device());
  minips_k::add_bf16(ptr<bf16_t>(a), ptr<bf16_t>(b), a.numel(), ptr<bf16_t>(out), stream_of(a));
}

void check_rows(const at::Tensor& t, int64_t rows, int64_t cols, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.stride(1) == 1 && t.size(0) == rows && t.size(1) >= cols &&
                  t.stride(0) % 8 == 0,
              n, " must be a [", rows, ", >=", cols, "] row-major GPU matrix with a leading dim % 8 == 0");
  check_dtype(t, at::kBFloat16, n);
}

void attn_fwd(const at::Tensor& qkv, int64_t B, int64_t T, int64_t H, double scale, at::Tensor& O, at::Tensor& lse) {
  const int64_t d = H * 64;
  check_rows(qkv, B * T, 3 * d, "qkv");
  check_rows(O, B * T, d, "O");
  check_gpu(lse, "lse");
  check_dtype(lse, at::kFloat, "lse");
  TORCH_CHECK(lse.numel() >= B * H * T, "lse too small");
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  minips_k::attn_fwd(ptr<bf16_t>(qkv), (int)qkv.stride(0), (int)B, (int)T, (int)H, (int)d, (float)scale,
                     ptr<bf16_t>(O), (int)O.stride(0), ptr<float>(lse), stream_of(qkv));
}

void attn_bwd(const at::Tensor& qkv, const at::Tensor& O, const at::Tensor& dO, const at::Tensor& lse,
              at::Tensor& delta,
              int64_t B, int64_t T, int64_t H, double scale, at::Tensor& dqkv) {
  const int64_t d = H * 64;
  check_rows(qkv, B * T, 3 * d, "qkv");
  check_rows(O, B * T, d, "O");
  check_rows(dO, B * T, d, "dO");
  check_rows(dqkv, B * T, 3 * d, "dqkv");
  check_dtype(lse, at::kFloat, "lse");
  check_dtype(delta, at::kFloat, "delta");
  TORCH_CHECK(lse.is_cuda() && delta.is_cuda() && lse.numel() >= B * H * T && delta.numel() >= B * H * T,
              "lse/delta too small");
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  minips_k::attn_bwd(ptr<bf16_t>(qkv), (int)qkv.stride(0), ptr<bf16_t>(O), (int)O.stride(0), ptr<bf16_t>(dO),
                     (int)dO.stride(0), ptr<float>(lse), ptr<float>(delta), (int)B, (int)T, (int)H, (int)d,
                     (float)scale, ptr<bf16_t>(dqkv), (int)dqkv.stride(0), stream_of(qkv));
}

void hash_slots(at::Tensor& tab_keys, const at::Tensor& q, at::Tensor& slots, at::Tensor& vals, double init_scale,
                int64_t seed, at::Tensor& counters, const c10::optional<at::Tensor>& n_dev) {
  for (const at::Tensor* t : {(const at::Tensor*)&tab_keys, &q, (const at::Tensor*)&slots, (const at::Tensor*)&vals,
                              (const at::Tensor*)&counters})
    check_gpu(*t, "hash arg");
  check_dtype(tab_keys, at::kLong, "tab_keys");
  check_dtype(q, at::kLong, "q");
  check_dtype(slots, at::kLong, "slots");
  check_dtype(vals, at::kFloat, "vals");
  check_dtype(counters, at::kInt, "counters");
  TORCH_CHECK(vals.dim() == 2 && vals.size(0) == tab_keys.numel() && vals.is_contiguous(), "vals [cap, W]");
  TORCH_CHECK(slots.numel() >= q.numel() && counters.numel() >= 2, "hash_slots sizes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  minips_k::hash_slots(reinterpret_cast<unsigned long long*>(tab_keys.data_ptr()), tab_keys.numel(), ptr<int64_t>(q),
                       q.numel(), ptr<int64_t>(slots), ptr<float>(vals), (int)vals.size(1), (float)init_scale,
                       (uint64_t)seed, ptr<int>(counters), stream_of(q), count_ptr(n_dev));
}

void hash_rehash(const at::Tensor& old_keys, const at::Tensor& old_vals, const c10::optional<at::Tensor>& old_state,
                 at::Tensor& new_keys, at::Tensor& new_vals, const c10::optional<at::Tensor>& new_state,
                 at::Tensor& counters) {
  check_dtype(old_keys, at::kLong, "old_keys");
  check_dtype(new_keys, at::kLong, "new_keys");
  TORCH_CHECK(old_vals.size(0) == old_keys.numel() && new_vals.size(0) == new_keys.numel() &&
                  old_vals.size(1) == new_vals.size(1),
              "rehash shapes");
  TORCH_CHECK(old_state.has_value() == new_state.has_value(), "state on both sides or neither");
  c10::hip::HIPGuardMasqueradingAsCUDA g(old_keys.device());
  minips_k::hash_rehash(reinterpret_cast<const unsigned long long*>(old_keys.data_ptr()), ptr<float>(old_vals),
                        old_state.has_value() ? ptr<float>(*old_state) : nullptr, old_keys.numel(),
                        reinterpret_cast<unsigned long long*>(new_keys.data_ptr()), ptr<float>(new_vals),
                        new_state.has_value() ? ptr<float>(*new_state) : nullptr, new_keys.numel(),
                        (int)new_vals.size(1), ptr<int>(counters), stream_of(old_keys));
}

void embed_fwd(const at::Tensor& wte, const at::Tensor& wpe, const at::Tensor& tok, int64_t T, at::Tensor& out) {
  for (const at::Tensor* t : {&wte, &wpe, &tok, (const at::Tensor*)&out}) check_gpu(*t, "embed arg");
  check_dtype(wte, at::kBFloat16, "wte");
  check_dtype(wpe, at::kBFloat16, "wpe");
  check_dtype(tok, at::kLong, "tok");
  check_dtype(out, at::kBFloat16, "out");
  const int64_t C = wte.size(1), M = tok.numel();
  TORCH_CHECK(C % 8 == 0 && wpe.size(1) == C && wpe.size(0) >= T && out.dim() == 2 && out.stride(1) == 1 &&
                  out.size(0) == M && out.size(1) >= C && out.stride(0) % 8 == 0,
              "embed_fwd shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(wte.device());
  minips_k::embed_fwd(ptr<bf16_t>(wte), ptr<bf16_t>(wpe), ptr<int64_t>(tok), M, (int)T, (int)C, ptr<bf16_t>(out),
                      (int)out.stride(0), stream_of(wte));
}

void embed_bwd(const at::Tensor& dx, const at::Tensor& tok, int64_t T, at::Tensor& dwte, at::Tensor& dwpe) {
  for (const at::Tensor* t : {&dx, &tok, (const at::Tensor*)&dwte, (const at::Tensor*)&dwpe}) check_gpu(*t,
                                                                                                        "embed arg");
  check_dtype(dx, at::kBFloat16, "dx");
  check_dtype(tok, at::kLong, "tok");
  check_dtype(dwte, at::kFloat, "dwte");
  check_dtype(dwpe, at::kFloat, "dwpe");
  const int64_t C = dwte.size(1), M = tok.numel();
  TORCH_CHECK(C % 2 == 0 && dwpe.size(1) == C && dwpe.size(0) >= T && dx.dim() == 2 && dx.stride(1) == 1 &&
                  dx.size(0) == M && dx.size(1) >= C && dx.stride(0) % 2 == 0,
              "embed_bwd shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(dx.device());
  minips_k::embed_bwd(ptr<bf16_t>(dx), (int)dx.stride(0), ptr<int64_t>(tok), M, (int)T, (int)C, ptr<float>(dwte),
                      ptr<float>(dwpe), stream_of(dx));
}

void dlrm_interact_fwd(const at::Tensor& V, int64_t NV, int64_t D, int64_t dense_idx, at::Tensor& out) {
  check_gpu(V, "V");
  check_gpu(out, "out");
  const int64_t B = V.numel() / (NV * D);
  TORCH_CHECK(out.size(0) == B && out.size(1) >= D + NV * (NV - 1) / 2, "interaction out shape");
  TORCH_CHECK(dense_idx >= 0 && dense_idx < NV, "dense_idx");
  c10::hip::HIPGuardMasqueradingAsCUDA g(V.device());
  minips_k::dlrm_interact_fwd(ptr<bf16_t>(V), B, (int)NV, (int)D, (int)dense_idx, ptr<bf16_t>(out), (int)out.size(1),
                              stream_of(V));
}

void dlrm_interact_bwd(const at::Tensor& V, int64_t NV, int64_t D, int64_t dense_idx, const at::Tensor& dout,
                       at::Tensor& dV, at::Tensor& d_dense) {
  check_gpu(V, "V");
  check_gpu(dout, "dout");
  check_gpu(dV, "dV");
  check_gpu(d_dense, "d_dense");
  const int64_t B = V.numel() / (NV * D);
  TORCH_CHECK(dV.numel() == V.numel() && dout.size(0) == B && d_dense.numel() == B * D, "interaction bwd shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(V.device());
  if (dV.scalar_type() == at::kBFloat16) {
    minips_k::dlrm_interact_bwd_bf16(ptr<bf16_t>(V), B, (int)NV, (int)D, (int)dense_idx, ptr<bf16_t>(dout),
                                     (int)dout.size(1), ptr<bf16_t>(dV), ptr<bf16_t>(d_dense), stream_of(V));
    return;
  }
  check_dtype(dV, at::kFloat, "dV");
  minips_k::dlrm_interact_bwd(ptr<bf16_t>(V), B, (int)NV, (int)D, (int)dense_idx, ptr<bf16_t>(dout), (int)dout.size(1),
                              ptr<float>(dV), ptr<bf16_t>(d_dense), stream_of(V));
}

// --- one-sided shards over xGMI (minips_amd/ps/onesided.py) -------------------------------------
// A hipMalloc'd, zero-filled buffer exported for IPC: (uint8 tensor owning it, 64-byte handle).
// kind: 0 coarse-grained (hipMalloc), 1 fine-grained (shards / pull copies / control lines: coherent
// for peer reads and system-scope atomics), 2 uncached (inboxes: written by peers, read once by the
// owner). The memory model of these buffers is written down in csrc/kernels/onesided.hip.
std::tuple<at::Tensor, py::bytes> ipc_alloc(int64_t nbytes, int64_t device, int64_t kind) {
  TORCH_CHECK(nbytes > 0, "ipc_alloc: nbytes must be > 0");
  c10::hip::HIPGuardMasqueradingAsCUDA g(at::Device(at::kCUDA, (c10::DeviceIndex)device));
  void* p = nullptr;
  if (kind == 0) {
    TORCH_CHECK(hipMalloc(&p, (size_t)nbytes) == hipSuccess, "ipc_alloc: hipMalloc of ", nbytes, " bytes failed");
  } else {
    TORCH_CHECK(hipExtMallocWithFlags(&p, (size_t)nbytes,
                                      kind == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached) == hipSuccess,
                "ipc_alloc: hipExtMallocWithFlags(", kind == 1 ? "fine-grained" : "uncached", ") of ", nbytes,
                " bytes failed");
  }
  TORCH_CHECK(hipMemset(p, 0, (size_t)nbytes) == hipSuccess, "ipc_alloc: hipMemset failed");
  hipIpcMemHandle_t h;
  TORCH_CHECK(hipIpcGetMemHandle(&h, p) == hipSuccess, "ipc_alloc: hipIpcGetMemHandle failed");
  auto t = torch::from_blob(p, {nbytes}, [](void* q) { (void)hipFree(q); },
                            at::TensorOptions().dtype(at::kByte).device(at::kCUDA, (c10::DeviceIndex)device));
  return {t, py::bytes(reinterpret_cast<const char*>(&h), sizeof(h))};
}

// Maps a peer's exported buffer into this process (peer access enabled lazily); the tensor owns
// the mapping (closed when it is freed).
at::Tensor ipc_open(py::bytes handle, int64_t nbytes, int64_t device) {
  const std::string hs = handle;
  TORCH_CHECK(hs.size() == sizeof(hipIpcMemHandle_t), "ipc_open: bad handle size ", hs.size());
  hipIpcMemHandle_t h;
  std::memcpy(&h, hs.data(), sizeof(h));
  c10::hip::HIPGuardMasqueradingAsCUDA g(at::Device(at::kCUDA, (c10::DeviceIndex)device));
  void* p = nullptr;
  TORCH_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess,
              "ipc_open: hipIpcOpenMemHandle failed");
  return torch::from_blob(p, {nbytes}, [](void* q) { (void)hipIpcCloseMemHandle(q); },
                          at::TensorOptions().dtype(at::kByte).device(at::kCUDA, (c10::DeviceIndex)device));
}

void check_long_dev(const at::Tensor& t, const char* name) {
  check_gpu(t, name);
  check_dtype(t, at::kLong, name);
}

const int64_t* opt_count(const c10::optional<at::Tensor>& n_dev) {
  if (!n_dev || !n_dev->defined()) return nullptr;
  check_long_dev(*n_dev, "n_dev");
  TORCH_CHECK(n_dev->numel() >= 1, "n_dev must hold a count");
  return ptr<int64_t>(*n_dev);
}

// Requester -> owners push of one clock (onesided.hip): uniq/counts/U_dev of the plan, fp32
// gradient rows [>= n, W], inbox = [P] int64 addresses of every owner's inbox as mapped here.
void ps_push_rows(const at::Tensor& uniq, const at::Tensor& counts, const c10::optional<at::Tensor>& U_dev,
                  int64_t n, const at::Tensor& g, const at::Tensor& inbox, int64_t slot_off, int64_t cap) {
  check_long_dev(uniq, "uniq");
  check_long_dev(counts, "counts");
  check_long_dev(inbox, "inbox");
  check_gpu(g, "grads");
  check_dtype(g, at::kFloat, "grads");
  const int64_t P = inbox.numel();
  TORCH_CHECK(P >= 1 && P <= minips_k::kPsMaxWorld, "inbox must list 1..16 owners");
  TORCH_CHECK(counts.numel() >= P, "counts must have >= P entries");
  TORCH_CHECK(n >= 0 && uniq.numel() >= n && g.dim() == 2 && g.size(0) >= n, "push: uniq/grads shorter than n");
  TORCH_CHECK(n <= cap && slot_off >= 0, "push: n exceeds the inbox slot capacity");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  minips_k::ps_push_rows(ptr<int64_t>(uniq), ptr<int64_t>(counts), opt_count(U_dev), n, ptr<float>(g),
                         (int)g.size(1), ptr<int64_t>(inbox), (int)P, slot_off, cap, stream_of(g));
}

void ps_push_dense(at::Tensor& grad, const at::Tensor& inbox, int64_t data_off, int64_t S,
                   const std::vector<std::tuple<at::Tensor, int64_t, int64_t, int64_t>>& slabs) {
  check_gpu(grad, "grad");
  check_dtype(grad, at::kFloat, "grad");
  check_gpu(inbox, "inbox");
  TORCH_CHECK(grad.numel() >= inbox.numel() * S, "grad: >= P * S floats");
  // (slab [nsplit * plane] fp32, nsplit, plane, offset of its region in grad), as adam_apply's
  minips_k::AdamSlabs sl;
  TORCH_CHECK(slabs.size() <= 4, "ps_push_dense: at most 4 slab regions");
  for (const auto& t : slabs) {
    const at::Tensor& p = std::get<0>(t);
    const int64_t ns = std::get<1>(t), plane = std::get<2>(t), off = std::get<3>(t);
    check_gpu(p, "slab");
    check_dtype(p, at::kFloat, "slab");
    TORCH_CHECK(ns >= 1 && p.numel() >= ns * plane && off >= 0 && off + plane <= inbox.numel() * S,
                "ps_push_dense slab bounds");
    sl.p[sl.n] = ptr<float>(p);
    sl.nsplit[sl.n] = (int)ns;
    sl.plane[sl.n] = plane;
    sl.len[sl.n] = plane;
    sl.off[sl.n] = off;
    ++sl.n;
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(grad.device());
  minips_k::ps_push_dense(ptr<float>(grad), ptr<int64_t>(inbox), (int)inbox.numel(), data_off, S, stream_of(grad),
                          sl.n ? &sl : nullptr);
}

void ps_set_headers(const at::Tensor& inbox, int64_t slot_off, int64_t value) {
  check_long_dev(inbox, "inbox");
  TORCH_CHECK(inbox.numel() >= 1 && inbox.numel() <= minips_k::kPsMaxWorld, "inbox must list 1..16 owners");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(inbox.device());
  minips_k::ps_set_headers(ptr<int64_t>(inbox), (int)inbox.numel(), slot_off, value, stream_of(inbox));
}

void ps_gather_rows(const at::Tensor& bases, const at::Tensor& bounds, const at::Tensor& keys,
                    const c10::optional<at::Tensor>& n_dev, int64_t W, at::Tensor& out) {
  check_long_dev(bases, "bases");
  check_long_dev(bounds, "bounds");
  check_long_dev(keys, "keys");
  check_gpu(out, "out");
  TORCH_CHECK(bounds.numel() == bases.numel() + 1, "bounds must have P+1 entries");
  TORCH_CHECK(bases.numel() >= 1 && bases.numel() <= minips_k::kPsMaxWorld, "1..16 owners");
  const int64_t n = keys.numel();
  TORCH_CHECK(out.dim() == 2 && out.size(0) >= n && out.size(1) == W, "out must be [>= n, W]");
  const bool bf = out.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || out.scalar_type() == at::kFloat, "out must be fp32 or bf16");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(keys.device());
  minips_k::ps_gather_rows(ptr<int64_t>(bases), ptr<int64_t>(bounds), (int)bases.numel(), ptr<int64_t>(keys), n,
                           opt_count(n_dev), (int)W, out.data_ptr(), bf, stream_of(keys));
}

void ps_gather_rows_bf16tab(const at::Tensor& bases, const at::Tensor& bounds, const at::Tensor& keys,
                            const c10::optional<at::Tensor>& n_dev, int64_t W, at::Tensor& out) {
  check_long_dev(bases, "bases");
  check_long_dev(bounds, "bounds");
  check_long_dev(keys, "keys");
  check_gpu(out, "out");
  TORCH_CHECK(bounds.numel() == bases.numel() + 1, "bounds must have P+1 entries");
  TORCH_CHECK(bases.numel() >= 1 && bases.numel() <= minips_k::kPsMaxWorld, "1..16 owners");
  const int64_t n = keys.numel();
  TORCH_CHECK(out.dim() == 2 && out.size(0) >= n && out.size(1) == W && out.is_contiguous(), "out must be [>= n, W]");
  const bool bf = out.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || out.scalar_type() == at::kFloat, "out must be fp32 or bf16");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(keys.device());
  minips_k::ps_gather_rows_bf16tab(ptr<int64_t>(bases), ptr<int64_t>(bounds), (int)bases.numel(), ptr<int64_t>(keys),
                                   n, opt_count(n_dev), (int)W, out.data_ptr(), bf, stream_of(keys));
}

void ps_hash_gather(const at::Tensor& hkeys, const at::Tensor& hvals, const at::Tensor& bounds, int64_t cap,
                    const at::Tensor& keys, const c10::optional<at::Tensor>& n_dev, int64_t W, at::Tensor& out) {
  check_long_dev(hkeys, "hkeys");
  check_long_dev(hvals, "hvals");
  check_long_dev(bounds, "bounds");
  check_long_dev(keys, "keys");
  check_gpu(out, "out");
  TORCH_CHECK(hkeys.numel() == hvals.numel() && bounds.numel() == hkeys.numel() + 1, "P owners, P+1 bounds");
  const int64_t n = keys.numel();
  TORCH_CHECK(out.dim() == 2 && out.size(0) >= n && out.size(1) == W && out.is_contiguous(), "out must be [>= n, W]");
  const bool bf = out.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || out.scalar_type() == at::kFloat, "out must be fp32 or bf16");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(keys.device());
  minips_k::ps_hash_gather(ptr<int64_t>(hkeys), ptr<int64_t>(hvals), ptr<int64_t>(bounds), (int)hkeys.numel(), cap,
                           ptr<int64_t>(keys), n, opt_count(n_dev), (int)W, out.data_ptr(), bf, stream_of(keys));
}

// dst[o * shard_bytes, ...) = srcs[o][0, shard_bytes) for the listed owners (one kernel)
void ps_pull(const at::Tensor& srcs, const std::vector<int64_t>& owners, int64_t shard_bytes, at::Tensor& dst) {
  check_long_dev(srcs, "srcs");
  check_gpu(dst, "dst");
  TORCH_CHECK(owners.size() <= (size_t)minips_k::kPsMaxWorld, "<= 16 owners");
  TORCH_CHECK(dst.is_contiguous() && dst.numel() * dst.element_size() >= srcs.numel() * shard_bytes, "dst too small");
  uint64_t packed = 0;
  for (size_t i = 0; i < owners.size(); ++i) {
    TORCH_CHECK(owners[i] >= 0 && owners[i] < srcs.numel(), "owner out of range");
    packed |= (uint64_t)owners[i] << (4 * i);
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dst.device());
  minips_k::ps_pull(ptr<int64_t>(srcs), packed, (int)owners.size(), shard_bytes, dst.data_ptr(), stream_of(dst));
}

// Reader side of the per-owner locks: `locks` [P] int64 device addresses of the owners' lock words,
// `held` / `err` raw device addresses (a slot of the reader's held ring, the rank's error word).
void ps_read_lock(const at::Tensor& locks, int64_t held, int64_t err) {
  check_long_dev(locks, "locks");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(locks.device());
  minips_k::ps_read_lock(ptr<int64_t>(locks), (int)locks.numel(), reinterpret_cast<uint32_t*>(held),
                         reinterpret_cast<uint32_t*>(err), stream_of(locks));
}

void ps_read_unlock(const at::Tensor& locks, int64_t held) {
  check_long_dev(locks, "locks");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(locks.device());
  minips_k::ps_read_unlock(ptr<int64_t>(locks), (int)locks.numel(), reinterpret_cast<uint32_t*>(held),
                           stream_of(locks));
}

// A host-resident, device-mapped 32-bit word (hipHostMalloc, coherent): the rank's error word of the
// one-sided protocol (a device spin that timed out sets a bit; the host reads it with no sync).
class HostWord {
 public:
  HostWord() {
    TORCH_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_), 64, hipHostMallocMapped | hipHostMallocCoherent) ==
                    hipSuccess,
                "HostWord: hipHostMalloc");
    *h_ = 0;
    TORCH_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_), h_, 0) == hipSuccess, "HostWord: device ptr");
  }
  ~HostWord() { (void)hipHostFree(h_); }
  int64_t value() const { return (int64_t)__atomic_load_n(h_, __ATOMIC_ACQUIRE); }
  void clear() { __atomic_store_n(h_, 0u, __ATOMIC_RELEASE); }
  int64_t device_ptr() const { return reinterpret_cast<int64_t>(d_); }

 private:
  uint32_t* h_ = nullptr;
  uint32_t* d_ = nullptr;
};

// A same-device stream-ordering event: no timing, no system-scope fence (hipEventDisableSystemFence).
// The fork / join events of a step order streams of ONE device, which needs agent scope only; the
// default event's system-scope release on every record cost the W&D step's main queue 7-9 us per
// fork (rocprofv3 timeline, profiles/r4).
class FastEvent {
 public:
  FastEvent() {
    TORCH_CHECK(hipEventCreateWithFlags(&ev_, hipEventDisableTiming | hipEventDisableSystemFence) == hipSuccess,
                "FastEvent: hipEventCreateWithFlags");
  }
  ~FastEvent() {
    if (ev_) (void)hipEventDestroy(ev_);
  }
  void record(int64_t stream) {
    TORCH_CHECK(hipEventRecord(ev_, reinterpret_cast<hipStream_t>(stream)) == hipSuccess, "FastEvent: record");
  }
  void wait(int64_t stream) {
    TORCH_CHECK(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), ev_, 0) == hipSuccess, "FastEvent: wait");
  }
  bool query() { return hipEventQuery(ev_) == hipSuccess; }
  void synchronize() { TORCH_CHECK(hipEventSynchronize(ev_) == hipSuccess, "FastEvent: synchronize"); }

 private:
  hipEvent_t ev_ = nullptr;
};

// A recorded launch sequence over two streams (0: the step's compute stream, 1: its side stream),
// replayed from C++ with no per-launch validation, argument conversion or Python dispatch. The
// recording IS the first execution: every op below launches on the current stream (which must be
// one of the list's two) and appends its validated launch; fork() orders the two streams with an
// event the list owns. run() replays the whole sequence onto the streams it is given. The list
// holds every tensor a launch addresses (operands and its own split-K planes), so no recorded
// address can be freed and handed to another buffer while the list lives; callers key lists by
// the buffers they address and record again when those change. Replaces ~25 binding calls of the
// W&D dense forward / backward per step (ops.gemm's argument conversion is 4-6 us of host each).
class LaunchList {
 public:
  LaunchList(int64_t main, int64_t side)
      : rec_{reinterpret_cast<hipStream_t>(main), reinterpret_cast<hipStream_t>(side)} {}
  ~LaunchList() {
    for (hipEvent_t e : events_) (void)hipEventDestroy(e);
  }
  LaunchList(const LaunchList&) = delete;
  LaunchList& operator=(const LaunchList&) = delete;

  void gemm(const at::Tensor& A, const at::Tensor& B, at::Tensor& C, int64_t M, int64_t N, int64_t K, bool a_km,
            bool b_kn, int64_t epi, const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& mask,
            const c10::optional<at::Tensor>& colsum, double alpha, int64_t split_k,
            const c10::optional<at::Tensor>& perm, int64_t seg, int64_t tile) {
    c10::hip::HIPGuardMasqueradingAsCUDA gd(A.device());
    at::Tensor slab;
    GemmLaunch g = prepare_gemm(A, B, C, M, N, K, a_km, b_kn, epi, bias, mask, colsum, alpha, split_k, 1, 1, 0, 0, 0,
                                {}, perm, seg, slab);
    g.tile = check_tile(tile);
    const int k = slot(A);
    g.launch(rec_[k]);
    for (const auto* t : {&bias, &mask, &colsum, &perm})
      if (t->has_value() && (*t)->defined()) keep_.push_back(**t);
    hold({A, B, C, slab});
    ops_.push_back([g, k](const hipStream_t* s) { g.launch(s[k]); });
  }

  int64_t gemm_slab(const at::Tensor& A, const at::Tensor& B, at::Tensor& slab, int64_t M, int64_t N, int64_t K,
                    bool a_km, bool b_kn, int64_t split_k) {
    check_gpu(A, "A");
    check_gpu(B, "B");
    check_gpu(slab, "slab");
    check_dtype(A, at::kBFloat16, "A");
    check_dtype(B, at::kBFloat16, "B");
    check_dtype(slab, at::kFloat, "slab");
    TORCH_CHECK(A.dim() == 2 && B.dim() == 2, "2-D operands");
    TORCH_CHECK(slab.numel() >= split_k * M * N, "slab: >= split_k * M * N floats");
    c10::hip::HIPGuardMasqueradingAsCUDA gd(A.device());
    const bf16_t *a = ptr<bf16_t>(A), *b = ptr<bf16_t>(B);
    float* p = ptr<float>(slab);
    const int lda = (int)A.stride(0), ldb = (int)B.stride(0), m = (int)M, n = (int)N, kk = (int)K, sk = (int)split_k;
    const int k = slot(A);
    const int nsplit = minips_k::gemm_slab(a, b, p, m, n, kk, lda, ldb, a_km, b_kn, sk, rec_[k]);
    hold({A, B, slab});
    ops_.push_back(
        [=](const hipStream_t* s) { (void)minips_k::gemm_slab(a, b, p, m, n, kk, lda, ldb, a_km, b_kn, sk, s[k]); });
    return nsplit;
  }

  void colsum_bf16(const at::Tensor& x, at::Tensor& out) {
    c10::hip::HIPGuardMasqueradingAsCUDA gd(x.device());
    at::Tensor slab;
    const ColsumLaunch c = prepare_colsum(x, out, slab);
    const int k = slot(x);
    c.launch(rec_[k]);
    hold({x, out, slab});
    ops_.push_back([c, k](const hipStream_t* s) { c.launch(s[k]); });
  }

  void wd_head_fold(int64_t B, int64_t Hd, at::Tensor& dw, at::Tensor& db, at::Tensor& loss_sum,
                    const c10::optional<at::Tensor>& dH_colsum) {
    c10::hip::HIPGuardMasqueradingAsCUDA gd(dw.device());
    const HeadFoldLaunch f = prepare_head_fold(B, Hd, dw, db, loss_sum, dH_colsum);
    const int k = slot(dw);
    f.launch(rec_[k]);
    hold({dw, db, loss_sum});
    if (dH_colsum.has_value()) hold({*dH_colsum});
    ops_.push_back([f, k](const hipStream_t* s) { f.launch(s[k]); });
  }

  // stream ``dst`` waits for the work issued so far on stream ``src`` (raw stream handles of the
  // recording: the list's two streams)
  void fork(int64_t src, int64_t dst) {
    const int a = slot_raw(reinterpret_cast<hipStream_t>(src)), b = slot_raw(reinterpret_cast<hipStream_t>(dst));
    TORCH_CHECK(a != b, "LaunchList.fork: one stream");
    hipEvent_t ev = nullptr;
    TORCH_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventDisableSystemFence) == hipSuccess,
                "LaunchList: hipEventCreateWithFlags");
    events_.push_back(ev);
    auto op = [ev, a, b](const hipStream_t* s) {
      TORCH_CHECK(hipEventRecord(ev, s[a]) == hipSuccess, "LaunchList: event record");
      TORCH_CHECK(hipStreamWaitEvent(s[b], ev, 0) == hipSuccess, "LaunchList: stream wait");
    };
    op(rec_);
    ops_.push_back(op);
  }

  void run(int64_t main, int64_t side) {
    const hipStream_t s[2] = {reinterpret_cast<hipStream_t>(main), reinterpret_cast<hipStream_t>(side)};
    for (const auto& op : ops_) op(s);
  }

  int64_t size() const { return (int64_t)ops_.size(); }

 private:
  int slot_raw(hipStream_t st) const {
    for (int i = 0; i < 2; ++i)
      if (st == rec_[i]) return i;
    TORCH_CHECK(false, "LaunchList: an op on a stream that is neither the list's compute nor its side stream");
    return 0;
  }
  int slot(const at::Tensor& t) const { return slot_raw(stream_of(t)); }
  void hold(std::initializer_list<at::Tensor> ts) {
    for (const auto& t : ts)
      if (t.defined()) keep_.push_back(t);
  }

  hipStream_t rec_[2];
  std::vector<std::function<void(const hipStream_t*)>> ops_;
  std::vector<at::Tensor> keep_;
  std::vector<hipEvent_t> events_;
};

// pos[members[m]] = m: where the dgrad's permuted-rows epilogue puts each lookup's gradient row.
at::Tensor emb_csr_positions(const at::Tensor& members) {
  check_gpu(members, "members");
  check_dtype(members, at::kInt, "members");
  at::Tensor pos = at::empty_like(members);
  c10::hip::HIPGuardMasqueradingAsCUDA g(members.device());
  minips_k::emb_csr_positions(members.data_ptr<int>(), members.numel(), pos.data_ptr<int>(), stream_of(members));
  return pos;
}

// The rank's native RCCL data plane (csrc/comm/rccl_comm.h) over torch tensors: each call is one
// enqueue on the tensors' current HIP stream (minips_amd/ps/comm.py Comm uses it for every
// collective of the step when the backend is RCCL).
int rccl_dtype(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kChar: case at::kByte: case at::kBool: return minips::RcclComm::kI8;
    case at::kInt: return minips::RcclComm::kI32;
    case at::kLong: return minips::RcclComm::kI64;
    case at::kHalf: return minips::RcclComm::kF16;
    case at::kBFloat16: return minips::RcclComm::kBF16;
    case at::kFloat: return minips::RcclComm::kF32;
    case at::kDouble: return minips::RcclComm::kF64;
    default: TORCH_CHECK(false, "rccl: dtype ", t.scalar_type());
  }
  return 0;
}

class PyRccl {
 public:
  // (id: the 128 raw bytes of the unique id; pybind converts Python bytes to std::string before
  // the GIL is released around the communicator's rendezvous)
  PyRccl(const std::string& lib, const std::string& id, int64_t world, int64_t rank, int64_t device, double timeout_s,
         bool teardown)
      : c_(lib, id, (int)world, (int)rank, (int)device, timeout_s, teardown) {}
  // out / inp: row-major [rows, ...] (a row = one element of a 1-D tensor); splits in rows
  void all_to_all_v(const at::Tensor& out, const at::Tensor& inp, const std::vector<int64_t>& recv,
                    const std::vector<int64_t>& send) {
    check_gpu(out, "out");
    check_gpu(inp, "inp");
    TORCH_CHECK(out.scalar_type() == inp.scalar_type(), "rccl all_to_all_v: dtypes differ");
    const int64_t row = inp.dim() > 1 ? inp[0].numel() * inp.element_size() : inp.element_size();
    int64_t ns = 0, nr = 0;
    for (int64_t v : send) ns += v;
    for (int64_t v : recv) nr += v;
    TORCH_CHECK(ns * row <= inp.numel() * inp.element_size() && nr * row <= out.numel() * out.element_size(),
                "rccl all_to_all_v: splits exceed the buffers");
    const hipStream_t s = stream_of(inp);
    py::gil_scoped_release rel;
    c_.AllToAllV(inp.data_ptr(), send, out.data_ptr(), recv, row, s);
  }
  void all_to_all(const at::Tensor& out, const at::Tensor& inp) {
    check_gpu(out, "out");
    check_gpu(inp, "inp");
    const int64_t nb = inp.numel() * inp.element_size();
    TORCH_CHECK(nb % c_.world() == 0 && out.numel() * out.element_size() == nb, "rccl all_to_all: equal blocks");
    const hipStream_t s = stream_of(inp);
    py::gil_scoped_release rel;
    c_.AllToAll(inp.data_ptr(), out.data_ptr(), nb / c_.world(), s);
  }
  void reduce_scatter(const at::Tensor& out, const at::Tensor& inp) {
    check_gpu(out, "out");
    check_gpu(inp, "inp");
    TORCH_CHECK(inp.numel() == out.numel() * c_.world() && inp.scalar_type() == out.scalar_type(),
                "rccl reduce_scatter: inp = world x out");
    const hipStream_t s = stream_of(inp);
    py::gil_scoped_release rel;
    c_.ReduceScatter(inp.data_ptr(), out.data_ptr(), out.numel(), rccl_dtype(out), s);
  }
  void all_gather(const at::Tensor& out, const at::Tensor& inp) {
    check_gpu(out, "out");
    check_gpu(inp, "inp");
    TORCH_CHECK(out.numel() == inp.numel() * c_.world() && inp.scalar_type() == out.scalar_type(),
                "rccl all_gather: out = world x inp");
    const hipStream_t s = stream_of(inp);
    py::gil_scoped_release rel;
    c_.AllGather(inp.data_ptr(), out.data_ptr(), inp.numel(), rccl_dtype(inp), s);
  }
  void all_reduce(const at::Tensor& t, int64_t op) {
    check_gpu(t, "t");
    const hipStream_t s = stream_of(t);
    py::gil_scoped_release rel;
    c_.AllReduce(t.data_ptr(), t.data_ptr(), t.numel(), rccl_dtype(t), (int)op, s);
  }
  std::string async_error() { return c_.AsyncError(); }
  void abort(const std::string& why) { c_.Abort(why); }
  bool aborted() const { return c_.aborted(); }

 private:
  minips::RcclComm c_;
};

// The owner side of the asynchronous PS on a GPU rank: minips::AsyncServer (the server thread,
// csrc/runtime/async_server.h) driving a HipApplier (the optimizer kernels on the owner's own
// stream). Table buffers are passed as raw device addresses; the Python table keeps them alive
// and stops the server before freeing them.
class GpuAsyncServer {
 public:
  GpuAsyncServer(const std::string& board, int64_t world, int64_t rank, int64_t tables, int64_t device)
      : device_((int)device), applier_((int)device, (int)tables),
        server_(board, (int)world, (int)rank, (int)tables, &applier_) {
    pub_ = std::thread([this] { PublishLoop(); });
  }
  ~GpuAsyncServer() {
    {
      std::lock_guard<std::mutex> lk(pmu_);
      pstop_ = true;
    }
    pcv_.notify_all();
    if (pub_.joinable()) pub_.join();
    server_.Stop();
  }

  // Requester side: publish sent[t] = c once the work issued so far on the tensor's current
  // stream (the clock's pushes) has completed -- an event waited for by a native thread, so no
  // Python thread (and no GIL hand-off) sits between the GPU and the board.
  void publish_after(int64_t t, int64_t c, const at::Tensor& on) {
    check_gpu(on, "stream tensor");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(on.device());
    hipEvent_t e;
    TORCH_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess, "publish_after: event");
    TORCH_CHECK(hipEventRecord(e, stream_of(on)) == hipSuccess, "publish_after: record");
    {
      std::lock_guard<std::mutex> lk(pmu_);
      pq_.push_back({e, (int)t, c});
      ++queued_;
    }
    pcv_.notify_one();
  }
  int64_t published() const { return published_.load(); }
  int64_t queued() {
    std::lock_guard<std::mutex> lk(pmu_);
    return queued_;
  }

  void set_error_word(int64_t err) { applier_.SetErrorWord(reinterpret_cast<uint32_t*>(err)); }

  void add_sparse(int64_t t, int64_t opt, int64_t table, int64_t ld, int64_t W, int64_t state, int64_t state2,
                  int64_t D1, int64_t base, double lr, double eps, int64_t cap, int64_t inbox, int64_t slot_bytes,
                  int64_t depth, int64_t bf16, int64_t seed, int64_t hash_cap, int64_t hkeys, int64_t lock, int64_t rs,
                  bool coalesce) {
    TORCH_CHECK(cap % 2 == 0 && slot_bytes % 256 == 0 && depth >= 1, "sparse inbox layout");
    TORCH_CHECK(slot_bytes >= minips_k::kPsSlotHeader + cap * (8 + 4 * W), "sparse inbox slot too small");
    TORCH_CHECK(opt == minips_k::kPsAdd || opt == minips_k::kPsSgd || opt == minips_k::kPsRowwiseAdagrad,
                "sparse optimizer ", opt);
    TORCH_CHECK(opt != minips_k::kPsRowwiseAdagrad || state != 0, "row-wise Adagrad needs its state");
    minips_k::PsSparseDesc d;
    d.opt = (int)opt;
    d.table = reinterpret_cast<float*>(table);
    d.ld = ld;
    d.W = (int)W;
    d.state = reinterpret_cast<float*>(state);
    d.state2 = reinterpret_cast<float*>(state2);
    d.D1 = (int)D1;
    d.base = base;
    d.lr = (float)lr;
    d.eps = (float)eps;
    d.cap = cap;
    d.inbox = reinterpret_cast<char*>(inbox);
    d.slot_bytes = slot_bytes;
    d.depth = (int)depth;
    d.bf16 = (int)bf16;
    d.seed = (uint32_t)seed;
    d.hash_cap = hash_cap;
    d.hkeys = reinterpret_cast<unsigned long long*>(hkeys);
    d.lock = reinterpret_cast<uint32_t*>(lock);
    d.flush = lock ? reinterpret_cast<uint32_t*>(lock) + 1 : nullptr;
    TORCH_CHECK(!bf16 || (W == 16 || W == 32 || W == 64), "bf16 rows hold 16, 32 or 64 values");
    TORCH_CHECK(hash_cap == 0 || ((hash_cap & (hash_cap - 1)) == 0 && hkeys), "hash capacity: a power of two");
    d.rs = reinterpret_cast<void*>(rs);
    TORCH_CHECK(!coalesce || opt != minips_k::kPsRowwiseAdagrad || hash_cap != 0 || rs != 0,
                "clock-coalesced row-wise Adagrad needs its (stamp, index) table");
    TORCH_CHECK(cap < (int64_t)INT32_MAX, "sparse inbox capacity");
    TORCH_CHECK(rs == 0 || (W % 4 == 0 && W <= 64), "clock-coalesced sparse rows: W % 4 == 0, W <= 64");
    applier_.SetSparse((int)t, d);
    server_.SetCoalesce((int)t, coalesce);
    server_.Enable((int)t);
  }

  void add_dense(int64_t t, int64_t opt, int64_t w, int64_t m, int64_t v, int64_t wb, int64_t n, double lr, double b1,
                 double b2, double eps, double wd, int64_t step, int64_t inbox, int64_t slot_bytes, int64_t depth,
                 int64_t lock, int64_t sum, int64_t sum_active, bool coalesce) {
    TORCH_CHECK(slot_bytes % 256 == 0 && depth >= 1 && n % 4 == 0, "dense inbox layout");
    TORCH_CHECK(slot_bytes >= minips_k::kPsSlotHeader + 4 * n, "dense inbox slot too small");
    TORCH_CHECK(opt != minips_k::kPsRowwiseAdagrad, "dense optimizer ", opt);
    TORCH_CHECK((opt != minips_k::kPsAdam || (m && v)) && (opt != minips_k::kPsAdagrad || m), "optimizer state");
    minips_k::PsDenseDesc d;
    d.opt = (int)opt;
    d.w = reinterpret_cast<float*>(w);
    d.m = reinterpret_cast<float*>(m);
    d.v = reinterpret_cast<float*>(v);
    d.wb = reinterpret_cast<bf16_t*>(wb);
    d.n = n;
    d.lr = (float)lr;
    d.b1 = (float)b1;
    d.b2 = (float)b2;
    d.eps = (float)eps;
    d.wd = (float)wd;
    d.step = step;
    d.inbox = reinterpret_cast<char*>(inbox);
    d.slot_bytes = slot_bytes;
    d.depth = (int)depth;
    d.lock = reinterpret_cast<uint32_t*>(lock);
    d.flush = lock ? reinterpret_cast<uint32_t*>(lock) + 1 : nullptr;
    d.sum = reinterpret_cast<float*>(sum);
    d.sum_active = reinterpret_cast<int64_t*>(sum_active);
    TORCH_CHECK(!coalesce || opt == minips_k::kPsAdd || opt == minips_k::kPsSgd || (sum && sum_active),
                "clock-coalesced Adam / Adagrad needs the sum buffer");
    applier_.SetDense((int)t, d);
    server_.SetCoalesce((int)t, coalesce);
    server_.Enable((int)t);
  }

  int64_t step(int64_t t) const { return applier_.Step((int)t); }
  void set_step(int64_t t, int64_t s) { applier_.SetStep((int)t, s); }
  void start() { server_.Start(); }
  void stop() { server_.Stop(); }
  void pause() { server_.Pause(); }
  void resume() { server_.Resume(); }
  bool running() const { return server_.Running(); }
  std::string error() const { return server_.Error(); }
  void set_log(bool on) { server_.SetLog(on); }
  std::vector<int64_t> take_log() { return server_.TakeLog(); }
  int64_t applied() const { return server_.Applied(); }
  int64_t batches() const { return server_.Batches(); }
  std::string publish_error() {
    std::lock_guard<std::mutex> lk(pmu_);
    return perr_;
  }

 private:
  struct Pub {
    hipEvent_t e;
    int t;
    int64_t c;
  };
  void PublishLoop() {
    (void)hipSetDevice(device_);
    for (;;) {
      Pub p;
      {
        std::unique_lock<std::mutex> lk(pmu_);
        pcv_.wait(lk, [&] { return pstop_ || !pq_.empty(); });
        if (pq_.empty()) return;  // stop requested and nothing left
        p = pq_.front();
        pq_.pop_front();
      }
      const hipError_t err = hipEventSynchronize(p.e);
      (void)hipEventDestroy(p.e);
      {
        std::lock_guard<std::mutex> lk(pmu_);
        if (err != hipSuccess && perr_.empty()) perr_ = std::string("publish: ") + hipGetErrorString(err);
        // never publish a clock whose pushes did not complete, nor any later one
        if (!perr_.empty()) continue;
      }
      server_.board().PublishSent(p.t, p.c);
      published_.fetch_add(1);
    }
  }

  int device_;
  minips_k::HipApplier applier_;
  minips::AsyncServer server_;
  std::thread pub_;
  std::mutex pmu_;
  std::condition_variable pcv_;
  std::deque<Pub> pq_;
  bool pstop_ = false;
  int64_t queued_ = 0;
  std::atomic<int64_t> published_{0};
  std::string perr_;
};

void kmeans_assign_csr(const at::Tensor& rowptr, const at::Tensor& cols, const at::Tensor& vals, const at::Tensor& C,
                       at::Tensor& cnorm, at::Tensor& assign, const c10::optional<at::Tensor>& dist) {
  for (const at::Tensor* t : {&rowptr, &cols, &vals, &C, (const at::Tensor*)&cnorm, (const at::Tensor*)&assign})
    check_gpu(*t, "kmeans_csr arg");
  check_dtype(rowptr, at::kLong, "rowptr");
  check_dtype(cols, at::kLong, "cols");
  check_dtype(vals, at::kFloat, "vals");
  check_dtype(C, at::kFloat, "C");
  check_dtype(cnorm, at::kFloat, "cnorm");
  check_dtype(assign, at::kInt, "assign");
  const int64_t n = rowptr.numel() - 1;
  TORCH_CHECK(C.dim() == 2 && cnorm.numel() == C.size(0) && assign.numel() == n && cols.numel() == vals.numel(),
              "kmeans_csr shapes");
  float* dp = opt_ptr<float>(dist, at::kFloat, "dist");
  if (dp) TORCH_CHECK(dist->numel() == n, "dist must be [n]");
  c10::hip::HIPGuardMasqueradingAsCUDA g(C.device());
  minips_k::kmeans_assign_csr(ptr<int64_t>(rowptr), ptr<int64_t>(cols), ptr<float>(vals), n, ptr<float>(C),
                              (int)C.size(0), C.size(1), ptr<float>(cnorm), ptr<int32_t>(assign), dp, stream_of(C));
}

void kmeans_csr_accum(const at::Tensor& rowptr, const at::Tensor& cols, const at::Tensor& vals,
                      const at::Tensor& assign, at::Tensor& sums) {
  for (const at::Tensor* t : {&rowptr, &cols, &vals, &assign, (const at::Tensor*)&sums}) check_gpu(*t,
                                                                                                   "kmeans_csr arg");
  check_dtype(vals, at::kFloat, "vals");
  check_dtype(sums, at::kFloat, "sums");
  check_dtype(assign, at::kInt, "assign");
  TORCH_CHECK(sums.dim() == 2 && assign.numel() == rowptr.numel() - 1, "kmeans_csr_accum shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(sums.device());
  minips_k::kmeans_csr_accum(ptr<int64_t>(rowptr), ptr<int64_t>(cols), ptr<float>(vals), rowptr.numel() - 1,
                             ptr<int32_t>(assign), sums.size(1), ptr<float>(sums), stream_of(sums));
}

}  // namespace


PYBIND11_MODULE(_kernels, m) {
  m.doc() = "minips_amd gfx950 HIP kernels";
  m.attr("EPI_STORE_F32") = (int)minips_k::kEpiStoreF32;
  m.attr("EPI_ATOMIC_F32") = (int)minips_k::kEpiAtomicF32;
  m.attr("EPI_BIAS_RELU_BF16") = (int)minips_k::kEpiBiasReluBf16;
  m.attr("EPI_BIAS_BF16") = (int)minips_k::kEpiBiasBf16;
  m.attr("EPI_STORE_BF16") = (int)minips_k::kEpiStoreBf16;
  m.attr("EPI_RELU_MASK_BF16") = (int)minips_k::kEpiReluMaskBf16;
  m.attr("EPI_BIAS_GELU_BF16") = (int)minips_k::kEpiBiasGeluBf16;
  m.attr("EPI_BIAS_GELU_AUX_BF16") = (int)minips_k::kEpiBiasGeluAuxBf16;
  m.attr("EPI_GELU_GRAD_BF16") = (int)minips_k::kEpiGeluGradBf16;
  m.def("gemm", &gemm, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("M"), py::arg("N"), py::arg("K"),
        py::arg("a_km"), py::arg("b_kn"), py::arg("epi"), py::arg("bias"), py::arg("mask"), py::arg("colsum"),
        py::arg("alpha") = 1.0, py::arg("split_k") = 1, py::arg("batch") = 1, py::arg("inner") = 1,
        py::arg("lda") = 0, py::arg("ldb") = 0, py::arg("ldc") = 0, py::arg("strides") = std::vector<int64_t>(),
        py::arg("perm") = py::none(), py::arg("seg") = 0, py::arg("tile") = 0);
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("layernorm_bwd", &layernorm_bwd);
  m.def("softmax_xent", &softmax_xent);
  m.def("new_stream", &new_stream);
  m.def("causal_softmax_fwd", &causal_softmax_fwd);
  m.def("causal_softmax_bwd", &causal_softmax_bwd);
  m.def("gelu_bwd", &gelu_bwd);
  m.def("add_bf16", &add_bf16);
  m.def("dlrm_interact_fwd", &dlrm_interact_fwd);
  m.def("dlrm_interact_bwd", &dlrm_interact_bwd);
  m.def("unique_bucketize", &unique_bucketize, py::arg("keys"), py::arg("bounds"), py::arg("F") = 1,
        py::arg("route_mult") = 0, py::arg("route_n") = 0, py::arg("extra_zero_ints") = 0,
        py::arg("csr_counts") = false);
  m.def("gather_rows", &gather_rows, py::arg("table"), py::arg("keys"), py::arg("base"), py::arg("out"),
        py::arg("n_dev") = py::none());
  m.def("scatter_add_rows", &scatter_add_rows);
  m.def("lookup_rows", &lookup_rows);
  m.def("embed_fwd", &embed_fwd);
  m.def("hash_slots", &hash_slots, py::arg("tab_keys"), py::arg("q"), py::arg("slots"), py::arg("vals"),
        py::arg("init_scale"), py::arg("seed"), py::arg("counters"), py::arg("n_dev") = py::none());
  m.def("hash_rehash", &hash_rehash);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd);
  m.def("embed_bwd", &embed_bwd);
  m.def("sparse_rowwise_adagrad", &sparse_rowwise_adagrad, py::arg("table"), py::arg("state"), py::arg("state2"),
        py::arg("D1"), py::arg("keys"), py::arg("base"), py::arg("grads"), py::arg("lr"), py::arg("eps"),
        py::arg("n_dev") = py::none(), py::arg("zero_g") = false);
  m.def("sparse_sgd", &sparse_sgd, py::arg("table"), py::arg("keys"), py::arg("base"), py::arg("grads"),
        py::arg("scale"), py::arg("n_dev") = py::none());
  m.def("embedding_bag_fwd", &embedding_bag_fwd);
  m.def("embedding_bag_bwd", &embedding_bag_bwd);
  m.def("wd_assemble", &wd_assemble, py::arg("dense"), py::arg("rows"), py::arg("inv"), py::arg("F"),
        py::arg("D"), py::arg("X"), py::arg("wide_logit"), py::arg("ones_col") = -1, py::arg("zero") = py::none());
  m.def("wd_head", &wd_head, py::arg("H"), py::arg("w"), py::arg("b0"), py::arg("wide_logit"), py::arg("labels"),
        py::arg("dH"), py::arg("dw"), py::arg("db"), py::arg("dwide"), py::arg("loss_sum"), py::arg("dH_colsum"),
        py::arg("grad_scale"), py::arg("defer_fold") = false);
  m.def("wd_head_fold", &wd_head_fold);
  m.def("wd_assemble_tab", &wd_assemble_tab);
  m.def("owner_slots", &owner_slots, py::arg("own_inv"), py::arg("splits"), py::arg("cap"));
  m.def("owner_rows_adagrad", &owner_rows_adagrad, py::arg("table"), py::arg("state"), py::arg("state2"),
        py::arg("D1"), py::arg("keys"), py::arg("n"), py::arg("n_dev"), py::arg("base"), py::arg("recv"),
        py::arg("P"), py::arg("slots"), py::arg("lr"), py::arg("eps"));
  m.def("owner_push_adagrad", &owner_push_adagrad, py::arg("table"), py::arg("state"), py::arg("state2"),
        py::arg("D1"), py::arg("keys"), py::arg("base"), py::arg("recv"), py::arg("splits"), py::arg("rs"),
        py::arg("stamp"), py::arg("lr"), py::arg("eps"));
  m.def("wd_emb_backward", &wd_emb_backward, py::arg("dX"), py::arg("dwide"), py::arg("inv"), py::arg("F"),
        py::arg("D"), py::arg("grad_rows"), py::arg("x_off") = 0, py::arg("members") = py::none(),
        py::arg("memrow") = py::none(), py::arg("sorted_rows") = false);
  m.def("colsum_bf16", &colsum_bf16);
  m.def("plan_sorted", &plan_sorted, py::arg("keys"), py::arg("col_base"), py::arg("col_bits"),
        py::arg("col_bits_host"), py::arg("route_mult"), py::arg("route_n"), py::arg("bounds"),
        py::arg("with_positions") = false);
  m.def("emb_build_csr", &emb_build_csr, py::arg("inv"), py::arg("F"), py::arg("U"), py::arg("zeroed") = py::none(),
        py::arg("counts_ready") = false);
  m.def("adam_apply", &adam_apply, py::arg("w"), py::arg("m"), py::arg("v"), py::arg("g"), py::arg("lr"),
        py::arg("beta1"), py::arg("beta2"), py::arg("eps"), py::arg("weight_decay"), py::arg("step"),
        py::arg("grad_scale"), py::arg("w_bf16"), py::arg("step_dev") = py::none(), py::arg("zero_g") = false,
        py::arg("slabs") = std::vector<std::tuple<at::Tensor, int64_t, int64_t, int64_t>>());
  m.def("gemm_slab", &gemm_slab);
  m.def("sgd_apply", &sgd_apply);
  m.def("adagrad_apply", &adagrad_apply);
  m.def("cast_f32_bf16", &cast_f32_bf16);
  m.def("lr_sparse_step", &lr_sparse_step);
  m.def("kmeans_assign", &kmeans_assign);
  m.def("kmeans_split3", &kmeans_split3);
  m.def("kmeans_argmin", &kmeans_argmin);
  m.def("criteo_synth", &criteo_synth);
  m.def("multi_copy", &multi_copy);
  m.def("slab_pack", &slab_pack);
  m.def("emu_sum_slices", &emu_sum_slices);
  m.def("emu_rebase", &emu_rebase);
  m.def("wire_spin", [](int64_t ticks, int64_t blocks, int64_t stream) {
    minips_k::wire_spin((int)ticks, (int)blocks,
                       stream ? reinterpret_cast<hipStream_t>(stream)
                              : c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
  });
  m.def("clock_probe", &clock_probe, py::arg("out"), py::arg("spin_ticks") = 2000, py::arg("stream") = 0);
  m.def("bitmap_plan", &bitmap_plan, py::arg("keys"), py::arg("bounds"), py::arg("num_rows"), py::arg("route_mult"),
        py::arg("route_n"), py::arg("oor") = py::none());
  m.def("uniform_synth", &uniform_synth);
  m.def("ipc_alloc", &ipc_alloc, py::arg("nbytes"), py::arg("device"), py::arg("kind") = 0);
  m.def("kmeans_assign_csr", &kmeans_assign_csr);
  m.def("kmeans_csr_accum", &kmeans_csr_accum);
  m.def("ipc_open", &ipc_open);
  m.def("ps_push_rows", &ps_push_rows, py::arg("uniq"), py::arg("counts"), py::arg("U_dev"), py::arg("n"),
        py::arg("g"), py::arg("inbox"), py::arg("slot_off"), py::arg("cap"));
  m.def("ps_set_headers", &ps_set_headers);
  m.def("ps_push_dense", &ps_push_dense, py::arg("grad"), py::arg("inbox"), py::arg("data_off"), py::arg("S"),
        py::arg("slabs") = std::vector<std::tuple<at::Tensor, int64_t, int64_t, int64_t>>());
  m.def("ps_gather_rows_bf16tab", &ps_gather_rows_bf16tab, py::arg("bases"), py::arg("bounds"), py::arg("keys"),
        py::arg("n_dev"), py::arg("W"), py::arg("out"));
  m.def("ps_hash_gather", &ps_hash_gather, py::arg("hkeys"), py::arg("hvals"), py::arg("bounds"), py::arg("cap"),
        py::arg("keys"), py::arg("n_dev"), py::arg("W"), py::arg("out"));
  m.def("ps_pull", &ps_pull);
  m.def("ps_set_fences", [](bool on) { minips_k::ps_set_fences(on); });
  m.def("ps_read_lock", &ps_read_lock);
  m.def("ps_read_unlock", &ps_read_unlock);
  m.attr("PS_CTRL_BYTES") = minips_k::kPsCtrlBytes;
  m.attr("PS_CTRL_LINE") = minips_k::kPsCtrlLine;
  m.attr("PS_HELD_SLOTS") = minips_k::kPsHeldSlots;
  m.def("rccl_unique_id", [](const std::string& lib) { return py::bytes(minips::RcclComm::UniqueId(lib)); });
  py::class_<PyRccl>(m, "Rccl")
      .def(py::init<const std::string&, const std::string&, int64_t, int64_t, int64_t, double, bool>(),
           py::arg("lib"), py::arg("unique_id"), py::arg("world"), py::arg("rank"), py::arg("device"),
           py::arg("timeout_s") = 60.0, py::arg("teardown") = false, py::call_guard<py::gil_scoped_release>())
      .def("all_to_all_v", &PyRccl::all_to_all_v)
      .def("all_to_all", &PyRccl::all_to_all)
      .def("reduce_scatter", &PyRccl::reduce_scatter)
      .def("all_gather", &PyRccl::all_gather)
      .def("all_reduce", &PyRccl::all_reduce)
      .def("async_error", &PyRccl::async_error)
      .def("abort", &PyRccl::abort, py::arg("why") = "aborted by the caller",
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("aborted", &PyRccl::aborted);
  py::class_<LaunchList>(m, "LaunchList")
      .def(py::init<int64_t, int64_t>())
      .def("gemm", &LaunchList::gemm)
      .def("gemm_slab", &LaunchList::gemm_slab)
      .def("colsum_bf16", &LaunchList::colsum_bf16)
      .def("wd_head_fold", &LaunchList::wd_head_fold)
      .def("fork", &LaunchList::fork)
      .def("run", &LaunchList::run)
      .def("size", &LaunchList::size);
  py::class_<FastEvent>(m, "FastEvent")
      .def(py::init<>())
      .def("record", &FastEvent::record)
      .def("wait", &FastEvent::wait)
      .def("query", &FastEvent::query)
      .def("synchronize", &FastEvent::synchronize);
  py::class_<HostWord>(m, "HostWord")
      .def(py::init<>())
      .def_property_readonly("value", &HostWord::value)
      .def("clear", &HostWord::clear)
      .def_property_readonly("device_ptr", &HostWord::device_ptr);
  m.def("emb_csr_positions", &emb_csr_positions);
  m.def("sparse_apply_bf16", &sparse_apply_bf16);
  m.attr("EPI_PERM_ROWS_BF16") = (int)minips_k::kEpiPermRowsBf16;
  m.def("ps_gather_rows", &ps_gather_rows, py::arg("bases"), py::arg("bounds"), py::arg("keys"), py::arg("n_dev"),
        py::arg("W"), py::arg("out"));
  m.attr("PS_ADD") = (int)minips_k::kPsAdd;
  m.attr("PS_SGD") = (int)minips_k::kPsSgd;
  m.attr("PS_ROWWISE_ADAGRAD") = (int)minips_k::kPsRowwiseAdagrad;
  m.attr("PS_ADAGRAD") = (int)minips_k::kPsAdagrad;
  m.attr("PS_ADAM") = (int)minips_k::kPsAdam;
  py::class_<GpuAsyncServer>(m, "AsyncServer")
      .def(py::init<const std::string&, int64_t, int64_t, int64_t, int64_t>(), py::arg("board"), py::arg("world"),
           py::arg("rank"), py::arg("tables"), py::arg("device"))
      .def("add_sparse", &GpuAsyncServer::add_sparse, py::arg("t"), py::arg("opt"), py::arg("table"), py::arg("ld"),
           py::arg("W"), py::arg("state"), py::arg("state2"), py::arg("D1"), py::arg("base"), py::arg("lr"),
           py::arg("eps"), py::arg("cap"), py::arg("inbox"), py::arg("slot_bytes"), py::arg("depth"), py::arg("bf16"),
           py::arg("seed"), py::arg("hash_cap"), py::arg("hkeys"), py::arg("lock"), py::arg("rs") = 0,
           py::arg("coalesce") = false)
      .def("set_error_word", &GpuAsyncServer::set_error_word)
      .def("publish_after", &GpuAsyncServer::publish_after)
      .def_property_readonly("published", &GpuAsyncServer::published)
      .def_property_readonly("queued", &GpuAsyncServer::queued)
      .def("publish_error", &GpuAsyncServer::publish_error)
      .def("add_dense", &GpuAsyncServer::add_dense, py::arg("t"), py::arg("opt"), py::arg("w"), py::arg("m"),
           py::arg("v"), py::arg("wb"), py::arg("n"), py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"),
           py::arg("wd"), py::arg("step"), py::arg("inbox"), py::arg("slot_bytes"), py::arg("depth"), py::arg("lock"),
           py::arg("sum") = 0, py::arg("sum_active") = 0, py::arg("coalesce") = false)
      .def("step", &GpuAsyncServer::step)
      .def("set_step", &GpuAsyncServer::set_step)
      .def("start", &GpuAsyncServer::start)
      .def("stop", &GpuAsyncServer::stop, py::call_guard<py::gil_scoped_release>())
      .def("pause", &GpuAsyncServer::pause, py::call_guard<py::gil_scoped_release>())
      .def("resume", &GpuAsyncServer::resume)
      .def("running", &GpuAsyncServer::running)
      .def("error", &GpuAsyncServer::error)
      .def("set_log", &GpuAsyncServer::set_log)
      .def("take_log", &GpuAsyncServer::take_log)
      .def_property_readonly("applied", &GpuAsyncServer::applied)
      .def_property_readonly("batches", &GpuAsyncServer::batches);
}
