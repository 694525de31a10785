// Torch-facing bindings of the gfx950 kernels (module minips_amd._kernels).
// Every op validates device/dtype/shape/contiguity on the host BEFORE launching, so a bad
// shape raises a Python exception instead of faulting the GPU, and launches on the current
// HIP stream of the tensor's device (graph-capture safe: no allocation or sync in here).
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/extension.h>

#include "../kernels/kernels.h"

namespace {

using minips_k::bf16_t;

hipStream_t stream_of(const at::Tensor& t) { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream(); }

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

// C = A . B with layout flags; see gemm.hip. Returns nothing (C preallocated).
void gemm(const at::Tensor& A, const at::Tensor& B, at::Tensor& C, int64_t M, int64_t N, int64_t K, bool a_km,
          bool b_kn, int64_t epi, const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& mask,
          const c10::optional<at::Tensor>& colsum, double alpha, int64_t split_k) {
  check_gpu(A, "A");
  check_gpu(B, "B");
  check_gpu(C, "C");
  check_dtype(A, at::kBFloat16, "A");
  check_dtype(B, at::kBFloat16, "B");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "gemm operands must be 2-D");
  const int64_t a_rows = a_km ? K : M, a_cols = a_km ? M : K;
  const int64_t b_rows = b_kn ? K : N, b_cols = b_kn ? N : K;
  TORCH_CHECK(A.size(0) == a_rows && A.size(1) >= a_cols, "A shape ", A.sizes(), " vs M,N,K=", M, ",", N, ",", K);
  TORCH_CHECK(B.size(0) == b_rows && B.size(1) >= b_cols, "B shape ", B.sizes(), " vs M,N,K=", M, ",", N, ",", K);
  TORCH_CHECK(C.size(0) == M && C.size(1) >= N, "C shape ", C.sizes(), " vs M,N=", M, ",", N);
  TORCH_CHECK(A.size(1) % 8 == 0 && B.size(1) % 8 == 0, "leading dims must be multiples of 8 (16-byte rows)");
  TORCH_CHECK(K % 8 == 0, "K must be a multiple of 8");
  if (a_km) TORCH_CHECK(M % 8 == 0, "KM layout needs M % 8 == 0");
  if (b_kn) TORCH_CHECK(N % 8 == 0, "KN layout needs N % 8 == 0");
  const bool f32_out = epi == minips_k::kEpiStoreF32 || epi == minips_k::kEpiAtomicF32;
  check_dtype(C, f32_out ? at::kFloat : at::kBFloat16, "C");
  const bf16_t* bias_p = opt_ptr<bf16_t>(bias, at::kBFloat16, "bias");
  if (bias_p) TORCH_CHECK(bias->numel() >= N, "bias too short");
  const bf16_t* mask_p = opt_ptr<bf16_t>(mask, at::kBFloat16, "mask");
  int ldmask = 0;
  if (mask_p) {
    TORCH_CHECK(mask->dim() == 2 && mask->size(0) == M && mask->size(1) >= N, "mask shape ", mask->sizes());
    ldmask = (int)mask->size(1);
  }
  if (epi == minips_k::kEpiReluMaskBf16) TORCH_CHECK(mask_p, "relu-mask epilogue needs mask");
  float* colsum_p = opt_ptr<float>(colsum, at::kFloat, "colsum");
  if (colsum_p) TORCH_CHECK(colsum->numel() >= N, "colsum too short");
  c10::hip::HIPGuardMasqueradingAsCUDA g(A.device());
  minips_k::gemm_bf16(ptr<bf16_t>(A), ptr<bf16_t>(B), C.data_ptr(), (int)M, (int)N, (int)K, (int)A.size(1),
                      (int)B.size(1), (int)C.size(1), a_km, b_kn, (int)epi, bias_p, mask_p, ldmask, colsum_p,
                      (float)alpha, (int)split_k, stream_of(A));
}

// Returns (unique keys grouped by owner [n] (first U valid), inverse [n], counts [P]).
std::vector<at::Tensor> unique_bucketize(const at::Tensor& keys, const at::Tensor& bounds, int64_t F) {
  check_gpu(keys, "keys");
  check_gpu(bounds, "bounds");
  check_dtype(keys, at::kLong, "keys");
  check_dtype(bounds, at::kLong, "bounds");
  TORCH_CHECK(bounds.dim() == 1 && bounds.numel() >= 2, "bounds must be [P+1]");
  const int64_t n = keys.numel();
  const int P = (int)bounds.numel() - 1;
  int64_t cap = 1024;
  while (cap < 2 * n) cap <<= 1;
  auto opts = keys.options();
  auto table_keys = at::empty({cap}, opts), table_pos = at::empty({cap}, opts);
  auto slot = at::empty({n}, opts), flags = at::empty({n}, opts.dtype(at::kInt));
  auto counts = at::empty({P}, opts), cursor = at::empty({P}, opts);
  auto out_keys = at::empty({n}, opts), inverse = at::empty({n}, opts);
  c10::hip::HIPGuardMasqueradingAsCUDA g(keys.device());
  TORCH_CHECK(F >= 1 && n % F == 0, "unique_bucketize: numel must be a multiple of F");
  minips_k::unique_bucketize(ptr<int64_t>(keys), n, (int)F, ptr<int64_t>(bounds), P, ptr<int64_t>(table_keys),
                             ptr<int64_t>(table_pos), cap, ptr<int64_t>(slot), ptr<int32_t>(flags),
                             ptr<int64_t>(counts), ptr<int64_t>(cursor), ptr<int64_t>(out_keys), ptr<int64_t>(inverse),
                             stream_of(keys));
  return {out_keys, inverse, counts};
}

void gather_rows(const at::Tensor& table, const at::Tensor& keys, int64_t base, at::Tensor& out) {
  check_gpu(keys, "keys");
  check_gpu(out, "out");
  TORCH_CHECK(table.is_cuda() && table.dim() == 2 && table.stride(1) == 1, "table must be a row-major GPU matrix");
  check_dtype(table, at::kFloat, "table");
  check_dtype(keys, at::kLong, "keys");
  const int64_t n = keys.numel();
  TORCH_CHECK(out.dim() == 2 && out.size(0) >= n, "out shape ", out.sizes());
  const int D = (int)out.size(1);
  TORCH_CHECK(D <= table.size(1), "out row wider than table row");
  TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16, "out must be fp32 or bf16");
  c10::hip::HIPGuardMasqueradingAsCUDA g(keys.device());
  minips_k::gather_rows(ptr<float>(table), table.stride(0), ptr<int64_t>(keys), n, base, D, out.data_ptr(),
                        out.scalar_type() == at::kBFloat16, stream_of(keys));
}

void scatter_add_rows(const at::Tensor& src, const at::Tensor& idx, at::Tensor& acc) {
  check_gpu(src, "src");
  check_gpu(idx, "idx");
  check_gpu(acc, "acc");
  check_dtype(src, at::kFloat, "src");
  check_dtype(acc, at::kFloat, "acc");
  check_dtype(idx, at::kLong, "idx");
  TORCH_CHECK(src.dim() == 2 && acc.dim() == 2 && src.size(1) == acc.size(1), "row widths differ");
  TORCH_CHECK(idx.numel() == src.size(0), "idx/src length mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA g(src.device());
  minips_k::scatter_add_rows(ptr<float>(src), src.size(0), (int)src.size(1), ptr<int64_t>(idx), ptr<float>(acc),
                             stream_of(src));
}

void sparse_rowwise_adagrad(at::Tensor& table, at::Tensor& state, const c10::optional<at::Tensor>& state2, int64_t D1,
                            const at::Tensor& keys, int64_t base, const at::Tensor& grads, double lr, double eps) {
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
                                   (float)lr, (float)eps, stream_of(table));
}

void sparse_sgd(at::Tensor& table, const at::Tensor& keys, int64_t base, const at::Tensor& grads, double scale) {
  TORCH_CHECK(table.is_cuda() && table.dim() == 2 && table.stride(1) == 1, "table must be a row-major GPU matrix");
  check_gpu(keys, "keys");
  check_gpu(grads, "grads");
  TORCH_CHECK(grads.dim() == 2 && grads.size(0) == keys.numel() && grads.size(1) <= table.size(1), "grads shape");
  c10::hip::HIPGuardMasqueradingAsCUDA g(table.device());
  minips_k::sparse_sgd(ptr<float>(table), table.stride(0), ptr<int64_t>(keys), keys.numel(), base,
                       (int)grads.size(1), ptr<float>(grads), (float)scale, stream_of(table));
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
                 at::Tensor& X, at::Tensor& wide_logit, int64_t ones_col) {
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
                        (int)ones_col, stream_of(X));
}

void wd_head(const at::Tensor& H, const at::Tensor& w, const at::Tensor& b0, const at::Tensor& wide_logit,
             const at::Tensor& labels, at::Tensor& dH, at::Tensor& dw, at::Tensor& db, at::Tensor& dwide,
             at::Tensor& loss_sum, const c10::optional<at::Tensor>& dH_colsum, double grad_scale) {
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
                    ptr<float>(dwide), ptr<float>(loss_sum), cs, (float)grad_scale, stream_of(H));
}

void wd_emb_backward(const at::Tensor& dX, const at::Tensor& dwide, const at::Tensor& inv, int64_t F, int64_t D,
                     at::Tensor& grad_rows) {
  check_gpu(dX, "dX");
  check_gpu(dwide, "dwide");
  check_gpu(inv, "inv");
  check_gpu(grad_rows, "grad_rows");
  check_dtype(dX, at::kFloat, "dX");
  check_dtype(grad_rows, at::kFloat, "grad_rows");
  const int64_t B = dX.size(0);
  TORCH_CHECK(inv.numel() == B * F && dX.size(1) >= F * D && grad_rows.size(1) > D, "shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(dX.device());
  minips_k::wd_emb_backward(ptr<float>(dX), (int)dX.size(1), ptr<float>(dwide), ptr<int64_t>(inv), B, (int)F, (int)D,
                            ptr<float>(grad_rows), (int)grad_rows.size(1), stream_of(dX));
}

void adam_apply(at::Tensor& w, at::Tensor& m, at::Tensor& v, const at::Tensor& g, double lr, double beta1,
                double beta2, double eps, double weight_decay, int64_t step, double grad_scale,
                const c10::optional<at::Tensor>& w_bf16) {
  for (auto* t : {&w, &m, &v}) {
    check_gpu(*t, "adam state");
    check_dtype(*t, at::kFloat, "adam state");
  }
  check_gpu(g, "g");
  check_dtype(g, at::kFloat, "g");
  TORCH_CHECK(w.numel() == m.numel() && w.numel() == v.numel() && w.numel() == g.numel(), "adam sizes differ");
  bf16_t* wb = opt_ptr<bf16_t>(w_bf16, at::kBFloat16, "w_bf16");
  if (wb) TORCH_CHECK(w_bf16->numel() == w.numel(), "w_bf16 size");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(w.device());
  minips_k::adam_apply(ptr<float>(w), ptr<float>(m), ptr<float>(v), ptr<float>(g), w.numel(), (float)lr, (float)beta1,
                       (float)beta2, (float)eps, (float)weight_decay, (int)step, (float)grad_scale, wb, stream_of(w));
}

void sgd_apply(at::Tensor& w, const at::Tensor& g, double lr, double grad_scale, const c10::optional<at::Tensor>& w_bf16) {
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
  check_dtype(w, at::kFloat, "w");
  check_dtype(vals, at::kFloat, "vals");
  TORCH_CHECK(rowptr.numel() == labels.numel() + 1, "rowptr must be [B+1]");
  float* d = opt_ptr<float>(delta, at::kFloat, "delta");
  if (d) TORCH_CHECK(delta->numel() == w.numel(), "delta must match w");
  float* c = opt_ptr<float>(correct, at::kFloat, "correct");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(w.device());
  minips_k::lr_sparse_step(ptr<int64_t>(rowptr), ptr<int64_t>(cols), ptr<float>(vals), ptr<float>(labels),
                           labels.numel(), ptr<float>(w), (float)alpha, d, c, stream_of(w));
}

void kmeans_assign(const at::Tensor& X, const at::Tensor& C, at::Tensor& assign, const c10::optional<at::Tensor>& dist) {
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

void criteo_synth(int64_t seed, int64_t step, const at::Tensor& cards, const at::Tensor& offsets, const at::Tensor& w,
                  at::Tensor& dense, at::Tensor& keys, at::Tensor& labels) {
  for (const at::Tensor* t : {&cards, &offsets, &w, (const at::Tensor*)&dense, (const at::Tensor*)&keys, (const at::Tensor*)&labels}) check_gpu(*t, "criteo_synth arg");
  check_dtype(keys, at::kLong, "keys");
  check_dtype(cards, at::kLong, "cards");
  const int64_t B = labels.numel();
  const int F = (int)cards.numel();
  TORCH_CHECK(keys.numel() == B * F && dense.size(0) == B && w.numel() == dense.size(1), "criteo_synth shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(keys.device());
  minips_k::criteo_synth((uint64_t)seed, (uint64_t)step, B, F, ptr<int64_t>(cards), ptr<int64_t>(offsets),
                         (int)dense.size(1), ptr<float>(w), ptr<float>(dense), ptr<int64_t>(keys), ptr<float>(labels),
                         stream_of(keys));
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
  m.def("gemm", &gemm);
  m.def("unique_bucketize", &unique_bucketize, py::arg("keys"), py::arg("bounds"), py::arg("F") = 1);
  m.def("gather_rows", &gather_rows);
  m.def("scatter_add_rows", &scatter_add_rows);
  m.def("sparse_rowwise_adagrad", &sparse_rowwise_adagrad);
  m.def("sparse_sgd", &sparse_sgd);
  m.def("embedding_bag_fwd", &embedding_bag_fwd);
  m.def("embedding_bag_bwd", &embedding_bag_bwd);
  m.def("wd_assemble", &wd_assemble, py::arg("dense"), py::arg("rows"), py::arg("inv"), py::arg("F"), py::arg("D"), py::arg("X"), py::arg("wide_logit"), py::arg("ones_col") = -1);
  m.def("wd_head", &wd_head);
  m.def("wd_emb_backward", &wd_emb_backward);
  m.def("adam_apply", &adam_apply);
  m.def("sgd_apply", &sgd_apply);
  m.def("adagrad_apply", &adagrad_apply);
  m.def("cast_f32_bf16", &cast_f32_bf16);
  m.def("lr_sparse_step", &lr_sparse_step);
  m.def("kmeans_assign", &kmeans_assign);
  m.def("criteo_synth", &criteo_synth);
}
