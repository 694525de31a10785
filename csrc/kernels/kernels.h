// Host-callable launchers of the gfx950 kernels (raw pointers + stream; no torch types).
// The torch-facing validation layer is csrc/bindings/ops_py.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace minips_k {

typedef uint16_t bf16_t;

// ------------------------------------------------------------------ GEMM (gemm.hip)
enum GemmEpilogue {
  kEpiStoreF32 = 0,      // C fp32 = alpha*acc
  kEpiAtomicF32 = 1,     // C fp32 += alpha*acc (split-K weight gradients)
  kEpiBiasReluBf16 = 2,  // C bf16 = relu(acc + bias)
  kEpiBiasBf16 = 3,      // C bf16 = acc + bias
  kEpiStoreBf16 = 4,     // C bf16 = acc
  kEpiReluMaskBf16 = 5,  // C bf16 = acc * (mask > 0); colsum[n] += sum_m C
  kEpiBiasGeluBf16 = 6,  // C bf16 = gelu_tanh(acc + bias)
  kEpiBiasGeluAuxBf16 = 7,  // C bf16 = gelu_tanh(u), mask(aux) bf16 = u = acc + bias (saved for bwd)
  kEpiGeluGradBf16 = 8,     // C bf16 = acc * gelu'(mask)  (mask = saved pre-activation u)
  // C bf16 = acc, row segments permuted: output (row, col) with s = col / seg lands at
  // C[perm[row * (N / seg) + s] * seg + col % seg] -- the embedding dgrad writes every lookup's
  // gradient row straight into the planner's row-sorted order (seg = D, seg % 8 == 0)
  kEpiPermRowsBf16 = 9,
  // C fp32 += alpha*acc without atomics: chosen by the launcher for an accumulating GEMM that is
  // not split over K (every output element has exactly one writer), e.g. GPT-2's LM-head weight
  // gradient (38.6M fp32 outputs: memory-side atomics cost it 1.75 ms/step)
  kEpiAccumF32 = 10,
  // C bf16 = gelu_tanh(u), aux bf16 = gelu'(u), u = acc + bias: the backward multiplies by the stored
  // derivative (kEpiMulAuxBf16) instead of re-evaluating tanh of the saved pre-activation
  kEpiBiasGeluDAuxBf16 = 13,
  kEpiMulAuxBf16 = 14,  // C bf16 = acc * mask(aux)
};
void gemm_bf16(const bf16_t* A, const bf16_t* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
               bool a_km, bool b_kn, int epi, const bf16_t* bias, const bf16_t* mask, int ldmask, float* colsum,
               float alpha, int split_k, hipStream_t s);
// Batched form: `batch` GEMMs, z = blockIdx.y; operand offsets are (z / inner) * s_outer +
// (z % inner) * s_inner elements (e.g. attention heads inside a [B*T, H*dh] activation).
void gemm_bf16_batched(const bf16_t* A, const bf16_t* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                       bool a_km, bool b_kn, int epi, const bf16_t* bias, const bf16_t* mask, int ldmask,
                       float* colsum, float alpha, int split_k, int batch, int inner, int64_t sa_o, int64_t sa_i,
                       int64_t sb_o, int64_t sb_i, int64_t sc_o, int64_t sc_i, hipStream_t s,
                       float* slab = nullptr,  // split-K workspace [split_k][M][N] (atomic epilogue only)
                       const int* perm = nullptr, int seg = 0,  // kEpiPermRowsBf16
                       int colsum_ld = 1,  // colsum[col * colsum_ld]
                       int tile = 0);      // EpiArgs::tile

// ------------------------------------------------------------------ sparse keys (sparse.hip)
// Hash-based dedupe + owner bucketing of int64 keys in 3 launches (no sort):
//   insert: open-addressing insert; first inserter of a key counts it for its owner shard
//   assign: per unique key, position = offset[owner] + cursor (keys grouped by owner)
//   inverse: inverse[i] = position of keys[i]
// `bounds` [P+1] are the shard key ranges (owner = upper_bound(bounds, key) - 1); P=1 with
// bounds {0, 2^63} makes it a plain unique. Work buffers are provided by the caller:
// table_keys/table_pos [cap] (cap power of two >= 2n), slot [n], flags [n], counts [P+1]
// (counts[P] = total unique on return),
// cursor [P] (all state re-initialised inside).
// keys may be a [B, F] batch (F > 1): tiles are then taken feature-major for better dedupe.
// route_mult != 0 dedupes the ROUTED keys key * route_mult mod route_n (uniq holds routed keys).
// extra_zero_bytes: when table_keys | counts | cursor are one buffer, that many more bytes after
// cursor are zeroed by the same memset (a workspace for a following op, e.g. emb_build_csr).
// counter shards of unique_bucketize's zero buffer for P owners (table | counts | total | 2*S*P | extra)
int ub_shards(int P);
// Bitmap planning of a bounded key space [0, num_keys_space) (bitmap.hip): sorted unique keys,
// inverse, per-owner counts (counts[P] = U) and U on the device. ws: bitmap_plan_workspace_words().
int64_t bitmap_plan_workspace_words(int64_t num_keys_space);
// oor (nullable, device int64): += the number of keys outside [0, num_keys_space) after routing
// (they get inverse 0; the caller checks the counter at its next host sync and raises).
void bitmap_plan(const int64_t* keys, int64_t n, int64_t num_keys_space, const int64_t* bounds, int P,
                 uint64_t rmult, uint64_t rn, int64_t* ws, int64_t* uniq, int64_t* inverse, int64_t* counts,
                 int64_t* U, hipStream_t s, int64_t* oor = nullptr);
void unique_bucketize(const int64_t* keys, int64_t n, int F, const int64_t* bounds, int P, int64_t* table_keys,
                      int64_t* table_pos, int64_t cap, int64_t* slot, int32_t* flags, int64_t* counts,
                      int64_t* cursor, int64_t* out_keys, int64_t* inverse, hipStream_t s, uint64_t route_mult = 0,
                      uint64_t route_n = 0, int64_t extra_zero_bytes = 0, int* csr_counts = nullptr);

// Row gather from a shard: out[i, :] = table[keys[i] - base, :] with dtype conversion.
// table fp32 [R, D] row stride ld; out fp32 or bf16 [n, D].
// n_dev (nullable, here and below): device-side row count <= n (n then only sizes the grid),
// so a table op can consume a count produced on the GPU without a host round trip.
void gather_rows(const float* table, int64_t ld, const int64_t* keys, int64_t n, int64_t base, int D, void* out,
                 bool out_bf16, hipStream_t s, const int64_t* n_dev = nullptr);
// Lookup: out[b, f*D:(f+1)*D] = rows[inv[b*F+f], 0:D]  (bf16; D % 8 == 0).
void lookup_rows(const bf16_t* rows, int row_stride, const int64_t* inv, int64_t B, int F, int D, bf16_t* out, int ldo,
                 hipStream_t s);
// Scatter-add rows: acc[idx[i], :] += src[i, :] (fp32, float atomics, 2 rows per wave-instr).
// Owner side of a multi-rank sparse push (sparse.hip): received rows are grouped by requester
// (segment s = rows [off[s], off[s+1])); slots[u * P + s] = the received row of requester s for
// owned unique row u (own_inv[i] = u), -1 when s did not push u (cap rows, memset first).
constexpr int kOwnerMaxP = 16;
struct OwnerSegs {
  int64_t off[kOwnerMaxP + 1];
};
void owner_slots(const int64_t* own_inv, int64_t M, const OwnerSegs& segs, int P, int* slots, int64_t cap,
                 hipStream_t s);
// Row-wise Adagrad of owned rows keys[0, min(n, *n_dev)) with the gradient = the sum, in requester
// order, of their received rows recv[slots[u * P + s]] (fp32 or bf16 [M, D]): one pass, no atomics.
void owner_rows_adagrad(float* table, int64_t ld, float* state, float* state2, int D1, const int64_t* keys, int64_t n,
                        const int64_t* n_dev, int64_t base, int D, const void* recv, bool recv_bf16, int P,
                        const int* slots, float lr, float eps, hipStream_t s);
// owner_mark + owner_apply: the direct-addressed owner apply of one push (rs: [rows_local * P]
// int2 {stamp, received row}, persistent; stamp: this push's number, >= 0, increasing)
void owner_push_adagrad(float* table, int64_t ld, float* state, float* state2, int D1, const int64_t* keys, int64_t M,
                        int64_t base, int64_t rows_local, int D, const void* recv, bool recv_bf16,
                        const OwnerSegs& segs, int P, void* rs, int stamp, float lr, float eps, hipStream_t s);
void scatter_add_rows(const float* src, int64_t n, int D, const int64_t* idx, float* acc, hipStream_t s);
void scatter_add_rows_bf16(const bf16_t* src, int64_t n, int D, const int64_t* idx, float* acc, hipStream_t s);
// Row-wise Adagrad on a shard (one accumulator per row, DLRM style):
//   s[row] += mean(g^2); w[row,:] -= lr * g / (sqrt(s[row]) + eps)
// Columns [D1, D) may use a second accumulator state2 (D1 = D: single group).
void sparse_rowwise_adagrad(float* table, int64_t ld, float* state, float* state2, int D1, const int64_t* keys,
                            int64_t n, int64_t base, int D, const float* grads, float lr, float eps, hipStream_t s,
                            const int64_t* n_dev = nullptr, bool zero_g = false);  // zero_g: clear grads after
// Plain SGD on rows: w[row,:] += scale * g  (the reference's "w += delta" server apply)
void sparse_sgd(float* table, int64_t ld, const int64_t* keys, int64_t n, int64_t base, int D, const float* grads,
                float scale, hipStream_t s, const int64_t* n_dev = nullptr);

// EmbeddingBag (sum/mean) over an [R, D] table (fp32 or bf16 rows via gathered buffer):
//   out[b, :] = pool_{j in bag b} rows[idx[j], :]   offsets [B+1]
void embedding_bag_fwd(const float* rows, const int64_t* idx, const int64_t* offsets, int64_t B, int D, bool mean,
                       float* out, hipStream_t s);
void embedding_bag_bwd(const float* grad_out, const int64_t* idx, const int64_t* offsets, int64_t B, int D,
                       bool mean, float* grad_rows, hipStream_t s);

// ------------------------------------------------------------------ Wide&Deep (widedeep.hip)
// Builds the deep-tower input X [B, ldx] bf16 = [F embeddings of width D | n_dense dense
// features | zero pad]: columns [f*D, (f+1)*D) hold row inv[b*F+f] of the pulled rows
// (bf16 [U, row_stride]), columns [F*D, F*D+n_dense) the dense features (fp32 [B, n_dense]).
// wide_logit[b] = sum_f rows[inv[b*F+f], D] (the wide weight lives in column D of a row).
// Column ones_col (>= 0) is set to 1.0: the bias input of a bias-folded first layer.
// zero_out (nullable): one float the kernel sets to 0 (the step's loss accumulator, so the step
// needs no separate fill kernel before the head's atomics)
void wd_assemble(const float* dense, int n_dense, const bf16_t* rows, int row_stride, const int64_t* inv, int64_t B,
                 int F, int D, bf16_t* X, int ldx, float* wide_logit, int ones_col, hipStream_t s,
                 float* zero_out = nullptr);
// Head (last Linear Hd->1 + BCE-with-logits, fwd and bwd fused):
//   z = H[b,:].w + b0 + wide[b]; dz = (sigmoid(z) - y) * grad_scale
//   dH = dz * w * (H > 0) (bf16), dw += dz*H, db += dz, dH_colsum += dH, dwide[b] = dz,
//   loss_sum += BCE(z, y)
void wd_assemble_tab(const float* dense, int n_dense, const float* tab, int64_t tab_ld, const int64_t* uniq,
                     int64_t base, const int64_t* inv, int64_t B, int F, int D, bf16_t* X, int ldx,
                     float* wide_logit, int ones_col, hipStream_t s, float* zero_out,
                     const int32_t* rowidx = nullptr);  // rowidx: lookup j's row + base (plan_sorted)
void wd_head(const bf16_t* H, int64_t B, int Hd, const bf16_t* w, const bf16_t* b0, const float* wide_logit,
             const float* labels, bf16_t* dH, float* dw, float* db, float* dwide, float* loss_sum, float* dH_colsum,
             float grad_scale, hipStream_t s, bool defer_fold = false);
// defer_fold: the head leaves its per-block partial rows in a per-device slab and wd_head_fold
// (same B / Hd, a later kernel on any stream ordered after it, before the next head of the
// device) adds their totals into dw / db / loss_sum / dH_colsum.
void wd_head_fold(int64_t B, int Hd, float* dw, float* db, float* loss_sum, float* dH_colsum, hipStream_t s);
// Embedding backward: grad_rows[inv[b*F+f], 0:D] += dX[b, f*D : (f+1)*D] (fp32 dX, ld ldx),
// grad_rows[inv[b*F+f], D] += dwide[b] when dwide != null (grad_rows fp32 [U, row_stride],
// pre-zeroed).
void wd_emb_backward(const float* dX, int ldx, const float* dwide, const int64_t* inv, int64_t B, int F, int D,
                     float* grad_rows, int row_stride, hipStream_t s);
// Segment-sum form of the embedding backward: out[u] = sum over lookups j with inv[j] == u for
// every row u < U (columns [0, D) the lookups' dX values, column D the samples' dwide, [D+1,
// row_stride) zero), written exactly once per row in a fixed summation order (deterministic, no
// atomics, no zero-fill): lookups are grouped by row (count / scan / fill) and summed piecewise,
// rows cut by piece boundaries finished by a second kernel over the pieces' partials. out: fp32
// or bf16 (out_bf16) [U, row_stride]. ws: (3U + 2 + 2*B*F + U/1024) int32; part:
// emb_seg_part_floats(B*F, D) floats.
void emb_backward_segment(const void* dX, bool bf16, int ldx, const float* dwide, const int64_t* inv, int64_t B, int F,
                          int D, void* out, bool out_bf16, int row_stride, int U, int* ws, float* part, hipStream_t s);
int64_t emb_seg_part_floats(int64_t total, int D);
// The two halves of emb_backward_segment: the lookup CSR (depends on inv only; ws: counts[U] |
// cursor[U] | offsets[U+1] | tiles[U/1024+1]; members/memrow [B*F]) and the segmented sum.
// zeroed_cc (nullable): a pre-zeroed 2U-int block used for counts|cursor (ws then starts at offsets).
void emb_build_csr(const int64_t* inv, int64_t B, int F, int U, int* ws, int* members, int* memrow, hipStream_t s,
                   int* zeroed_cc = nullptr, bool counts_ready = false);
// sorted_rows: dX is [B*F, D] in the CSR's member order (dX row m = the gradient of lookup
// members[m], written there by the dgrad GEMM's kEpiPermRowsBf16 epilogue): the segment sums read
// it as one contiguous stream instead of gathering 2*D-byte pieces of [B, F*D] rows.
void emb_backward_csr(const void* dX, bool bf16, int ldx, const float* dwide, int64_t B, int F, int D,
                      const int* members, const int* memrow, void* out, bool out_bf16, int row_stride, float* part,
                      hipStream_t s, bool sorted_rows = false);
// pos[members[m]] = m (n entries): where each lookup's gradient row goes in member order.
void emb_csr_positions(const int* members, int64_t n, int* pos, hipStream_t s);
void wd_emb_backward_bf16(const bf16_t* dX, int ldx, const float* dwide, const int64_t* inv, int64_t B, int F, int D,
                          float* grad_rows, int row_stride, hipStream_t s);
// Sort-based key planning of a [B, F] batch with disjoint column key ranges (plan.hip): keys of
// column f lie in [col_base[f], col_base[f] + 2^col_bits[f]), 1 <= col_bits[f] <= 32 (device
// arrays); P owners with routed-key bounds [P+1] (1 <= P <= 16). ws: int32 [7*B*F + F + 4 +
// 2*ceil(B*F/1024)*P], ukey: int64 [B*F]. Outputs: uniq [B*F] (first U valid, routed, grouped
// by owner), inv [B*F], the lookup CSR members/memrow [B*F] int32, counts [P+1] = {per owner, U}.
void plan_sorted(const int64_t* keys, int B, int F, const int64_t* col_base, const int32_t* col_bits,
                 uint64_t route_mult, uint64_t route_n, const int64_t* bounds, int P, int32_t* ws, int64_t* ukey,
                 int64_t* uniq, int64_t* inv, int32_t* members, int32_t* memrow, int64_t* counts, hipStream_t s,
                 int32_t* pos = nullptr, int32_t* rowstart = nullptr, int32_t* rowidx = nullptr);
// plan_sorted's int32 workspace for n = B * F lookups; owner bits of the sort key for P owners
int64_t plan_sorted_ws_ints(int64_t n, int F, int P);
int plan_owner_bits(int P);
// (pos, nullable: pos[members[m]] = m, emb_csr_positions fused; rowstart, nullable, one owner only:
// rowstart[u] = first member of row u, rowstart[U] = B*F)
// out[c] += column sums of x (bf16 [M, N], row stride ld; N, ld multiples of 8): a bias gradient.
// slab: colsum_chunks(M, N) * ceil(N / 64) * 64 floats of scratch (the blocks' partial rows).
void colsum_bf16(const bf16_t* x, int64_t M, int N, int ld, float* out, float* slab, hipStream_t s);
int64_t colsum_chunks(int64_t M, int N);

// ------------------------------------------------------------------ optimizers (optim.hip)
// Fused Adam(W) on an fp32 master shard; optionally writes the bf16 copy for all-gather.
// active (nullable, device): the kernel does nothing when *active == 0 (an empty async push).
// slabs (nullable): split-K weight-gradient planes left unreduced (gemm_slab): element off + e of
// the gradient gets sum_z p[z * plane + e] for e < len (offsets / lengths / planes multiples of 4).
struct AdamSlabs {
  int n = 0;
  const float* p[4] = {nullptr, nullptr, nullptr, nullptr};
  int64_t off[4] = {0, 0, 0, 0}, len[4] = {0, 0, 0, 0}, plane[4] = {0, 0, 0, 0};
  int nsplit[4] = {0, 0, 0, 0};
};
// several ranks: out = g + the split-K planes of its regions, g cleared (the reduce-scatter input)
void slab_pack(float* g, float* out, int64_t n, const AdamSlabs* slabs, hipStream_t s);
void adam_apply(float* w, float* m, float* v, const float* g, int64_t n, float lr, float beta1, float beta2,
                float eps, float weight_decay, int step, float grad_scale, bf16_t* w_bf16, hipStream_t s,
                const int* step_dev = nullptr, bool zero_g = false, const int64_t* active = nullptr,
                const AdamSlabs* slabs = nullptr);
// split-K GEMM whose K slices stay in their fp32 slab planes [nsplit][M][N] (no reduce launch):
// the consumer folds them (adam_apply slabs). Returns nsplit.
int gemm_slab(const bf16_t* A, const bf16_t* B, float* slab, int M, int N, int K, int lda, int ldb, bool a_km,
              bool b_kn, int split_k, hipStream_t s);
void sgd_apply(float* w, const float* g, int64_t n, float lr, float grad_scale, bf16_t* w_bf16, hipStream_t s,
               const int64_t* active = nullptr);
void adagrad_apply(float* w, float* acc, const float* g, int64_t n, float lr, float eps, float grad_scale,
                   bf16_t* w_bf16, hipStream_t s, const int64_t* active = nullptr);
void cast_f32_bf16(const float* x, bf16_t* y, int64_t n, hipStream_t s);
void cast_bf16_f32(const bf16_t* x, float* y, int64_t n, hipStream_t s);

// ------------------------------------------------------------------ LR / K-Means (ml.hip)
// Sparse logistic regression over a CSR batch whose columns are positions into the pulled
// weight vector w [U]: p_i = sigmoid(sum_j w[col_j] x_j); delta[col_j] += alpha*x_j*(y_i - p_i)
// (labels < 0 treated as 0, lr_example.cpp:291-312). Optional correct-count for accuracy.
void lr_sparse_step(const int64_t* rowptr, const int64_t* cols, const float* vals, const float* labels, int64_t B,
                    const float* w, float alpha, float* delta, float* correct, hipStream_t s);
// K-Means assignment: X [n, d] fp32, C [k, d] fp32 -> assign [n] (int32), min dist [n].
// MFMA assignment pieces (ops.kmeans_assign): hi/lo bf16 split (+ squared row norms) and the
// argmin over a GEMM-produced S = X.C^T (fp32 [n, k]).
void kmeans_split3(const float* src, int64_t r, int d, bf16_t* out, int ld, int order, float* norms, hipStream_t s);
void kmeans_argmin(const float* S, int64_t n, int k, const float* cn, const float* xn, int32_t* assign, float* dist,
                   hipStream_t s);
void kmeans_assign(const float* X, int64_t n, int d, const float* C, int k, int32_t* assign, float* dist,
                   hipStream_t s);

// ------------------------------------------------------------------ dense-model kernels (nn.hip)
void layernorm_fwd(const bf16_t* x, int ldx, int64_t M, int C, const bf16_t* gamma, const bf16_t* beta, float eps,
                   bf16_t* y, int ldy, float* mean, float* rstd, hipStream_t s);
// partial: scratch of layernorm_bwd_blocks(M) * 2 * C floats (per-block dgamma/dbeta partials).
int layernorm_bwd_blocks(int64_t M);
void layernorm_bwd(const bf16_t* x, int ldx, const bf16_t* dy, int lddy, int64_t M, int C, const bf16_t* gamma,
                   const float* mean, const float* rstd, bf16_t* dx, int lddx, float* dgamma, float* dbeta,
                   float* partial, bool accumulate_dx, hipStream_t s);
// In place: logits [M, ld] bf16 become (softmax - onehot) * scale; loss_sum += sum CE.
void softmax_xent(bf16_t* logits, int ld, int64_t M, int V, const int64_t* labels, float scale, float* loss_sum,
                  float* correct, hipStream_t s);
void causal_softmax_fwd(const float* S, int64_t rows, int T, bf16_t* P, hipStream_t s);
void causal_softmax_bwd(const bf16_t* P, const float* dP, int64_t rows, int T, float scale, bf16_t* dS,
                        hipStream_t s);
void gelu_bwd(const bf16_t* dh, const bf16_t* u, int64_t n, bf16_t* du, hipStream_t s);
void add_bf16(const bf16_t* a, const bf16_t* b, int64_t n, bf16_t* out, hipStream_t s);
// GPU hash-table shard (hashtable.hip): tab_keys EMPTY = ~0; counters[0] += inserts,
// counters[1] += failed lookups (table full); slot -1 for those.
// n_dev (optional, device int64): only q[0, *n_dev) are looked up / inserted; the rest get slot -1.
void hash_slots(unsigned long long* tab_keys, int64_t cap, const int64_t* q, int64_t n, int64_t* slots, float* vals,
                int W, float init_scale, uint64_t seed, int* counters, hipStream_t s, const int64_t* n_dev = nullptr);
void hash_rehash(const unsigned long long* old_keys, const float* old_vals, const float* old_state, int64_t old_cap,
                 unsigned long long* new_keys, float* new_vals, float* new_state, int64_t new_cap, int W, int* counters,
                 hipStream_t s);
// Fused causal attention, head dim 64 (attention.hip). qkv [B*T][ldq] holds Q|K|V (each dmodel
// = H*64 columns); O/dO/dqkv row-major with head h at column h*64; lse/delta [B*H*T] fp32.
void attn_fwd(const bf16_t* qkv, int ldq, int B, int T, int H, int dmodel, float scale, bf16_t* O, int ldo, float* lse,
              hipStream_t s);
void attn_bwd(const bf16_t* qkv, int ldq, const bf16_t* O, int ldo, const bf16_t* dO, int lddo, const float* lse,
              float* delta, int B, int T, int H, int dmodel, float scale, bf16_t* dqkv, int lddq, hipStream_t s);
void embed_fwd(const bf16_t* wte, const bf16_t* wpe, const int64_t* tok, int64_t M, int T, int C, bf16_t* out, int ldo,
               hipStream_t s);
void embed_bwd(const bf16_t* dx, int ldx, const int64_t* tok, int64_t M, int T, int C, float* dwte, float* dwpe,
               hipStream_t s);
// DLRM dot interaction of NV vectors of width D per sample (V [B][NV][D] bf16): out[b] =
// [V[b][dense_idx] | V_i.V_j for i > j]. Backward: dV fp32 for all vectors, and the dense
// vector's gradient ReLU-masked by its value as bf16 (feeds the bottom MLP's backward).
void dlrm_interact_fwd(const bf16_t* V, int64_t B, int NV, int D, int dense_idx, bf16_t* out, int ldo, hipStream_t s);
// bf16 dV (half the bytes for the embedding backward that reads it): NV <= 32, D in {16, 32, 64}.
void dlrm_interact_bwd_bf16(const bf16_t* V, int64_t B, int NV, int D, int dense_idx, const bf16_t* dout, int ldo,
                            bf16_t* dV, bf16_t* d_dense, hipStream_t s);
void dlrm_interact_bwd(const bf16_t* V, int64_t B, int NV, int D, int dense_idx, const bf16_t* dout, int ldo,
                       float* dV, bf16_t* d_dense, hipStream_t s);

// ------------------------------------------------------------------ synthetic data (data.hip)
// DLRM batch: keys uniform in [0, rows), dense N(0,1), labels = dense[:, 0] > 0 (data.hip).
void uniform_synth(uint64_t seed, uint64_t step, int64_t B, int F, uint64_t rows, int n_dense, float* dense,
                   int64_t* keys, float* labels, hipStream_t s);
// out[0] = shader-clock cycles, out[1] = 100 MHz real-time ticks over ~spin_ticks (one wave; diagnostics)
void clock_probe(int64_t* out, int spin_ticks, hipStream_t s);
void wire_spin(int spin_ticks, int blocks, hipStream_t s);
void emu_sum_slices(const float* in, float* out, int64_t n, int P, hipStream_t s);
void emu_rebase(int64_t* keys, int64_t n, int64_t step, int P, int64_t base, hipStream_t s);
// up to 16 device-to-device copies in one launch: pair t copies n16[t] 16-byte vectors then tail[t]
// bytes (src / dst 16-byte aligned when n16 > 0); start[] = exclusive prefix of n16 + tail
constexpr int kMultiCopyMax = 16;
struct MultiCopyArgs {
  const void* src[kMultiCopyMax];
  void* dst[kMultiCopyMax];
  int64_t n16[kMultiCopyMax];
  int64_t tail[kMultiCopyMax];
  int64_t start[kMultiCopyMax + 1];
  int n;
};
void multi_copy(const MultiCopyArgs& a, hipStream_t s);
void criteo_synth(uint64_t seed, uint64_t step, const int64_t* step_dev, int64_t B, int F, const int64_t* cards,
                  const int64_t* offsets, int n_dense, const float* w, float* dense, int64_t* keys, float* labels,
                  hipStream_t s);

// ------------------------------------------------------------------ bf16 table rows (bf16rows.hip)
// Row gather from a bf16 table [R, ld] (D in {16, 32, 64}) to bf16 or fp32 out [n, D].
void gather_rows_bf16tab(const bf16_t* table, int64_t ld, const int64_t* keys, int64_t n, int64_t base, int D,
                         void* out, bool out_bf16, hipStream_t s, const int64_t* n_dev = nullptr);
// Apply fp32 gradient rows to bf16 table rows with stochastic rounding: opt 0 row-wise Adagrad
// (fp32 state / state2, column split D1), opt 1 w += scale * g. `step` / `seed` key the rounding.
void sparse_apply_bf16tab(int opt, bf16_t* table, int64_t ld, float* state, float* state2, int D1, const int64_t* keys,
                          int64_t n, int64_t base, int D, const float* grads, float lr, float eps, float scale,
                          uint32_t step, uint32_t seed, hipStream_t s, const int64_t* n_dev = nullptr);

// (the asynchronous PS path over xGMI -- push / gather / owner apply -- is declared in onesided.h)

// ------------------------------------------------------------------ fp64 parity tables (f64.hip, ml.hip)
void gather_rows_f64(const double* table, int W, const int64_t* keys, int64_t base, int64_t n, const int64_t* n_dev,
                     double* out, hipStream_t s);
void scatter_add_rows_f64(const double* src, const int64_t* idx, int64_t n, int W, double* acc, hipStream_t s);
void sparse_add_f64(double* table, int W, const int64_t* keys, int64_t base, const double* grads, int64_t n,
                    double scale, const int64_t* n_dev, hipStream_t s);
void lr_sparse_step_f64(const int64_t* rowptr, const int64_t* cols, const float* vals, const float* labels, int64_t B,
                        const double* w, double alpha, double* delta, float* correct, hipStream_t s);

// ------------------------------------------------------------------ sparse K-Means (ml.hip)
void kmeans_assign_csr(const int64_t* rowptr, const int64_t* cols, const float* vals, int64_t n, const float* C,
                       int k, int64_t d, float* cnorm, int32_t* assign, float* dist, hipStream_t s);
void kmeans_csr_accum(const int64_t* rowptr, const int64_t* cols, const float* vals, int64_t n, const int32_t* assign,
                      int64_t d, float* sums, hipStream_t s);

}  // namespace minips_k
