// Asynchronous PS over xGMI: push / gather launchers and the owner-side applier of the
// AsyncServer thread (csrc/kernels/onesided.hip, csrc/runtime/async_server.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <vector>

#include "../runtime/async_server.h"

namespace minips_k {

typedef uint16_t bf16_t;

constexpr int kPsMaxWorld = 16;
constexpr int64_t kPsSlotHeader = 64;

enum PsOptimizer { kPsAdd = 0, kPsSgd = 1, kPsRowwiseAdagrad = 2, kPsAdagrad = 3, kPsAdam = 4 };

// Requester -> owners: unique keys uniq[0, U) (U = *U_dev, <= n) grouped by owner with counts[P]
// rows per owner, gradient rows g [>= U, W] fp32; owner o's slot starts at inbox[o] + slot_off.
void ps_push_rows(const int64_t* uniq, const int64_t* counts, const int64_t* U_dev, int64_t n, const float* g, int W,
                  const int64_t* inbox, int P, int64_t slot_off, int64_t cap, hipStream_t s);
// Every owner's slot header := value (0: a clock without an Add; a dense push marks its slot 1).
void ps_set_headers(const int64_t* inbox, int P, int64_t slot_off, int64_t value, hipStream_t s);
// out[i] = row of keys[i] (i < min(n, *n_dev)) from its owner's fp32 shard at bases[o]
// ([rows_o, W]); out fp32 or bf16 [n, W].
void ps_gather_rows(const int64_t* bases, const int64_t* bounds, int P, const int64_t* keys, int64_t n,
                    const int64_t* n_dev, int W, void* out, bool out_bf16, hipStream_t s);

// Owner-side descriptors. `inbox` is this owner's inbox buffer: requester r's slot k at
// inbox + (r * depth + k) * slot_bytes.
struct PsSparseDesc {
  int opt = kPsRowwiseAdagrad;
  float* table = nullptr;
  int64_t ld = 0;
  int W = 0;
  float* state = nullptr;
  float* state2 = nullptr;
  int D1 = 0;
  int64_t base = 0;
  float lr = 0.f, eps = 1e-8f;
  int64_t cap = 0;
  char* inbox = nullptr;
  int64_t slot_bytes = 0;
  int depth = 1;
};

struct PsDenseDesc {
  int opt = kPsAdam;
  float* w = nullptr;
  float* m = nullptr;
  float* v = nullptr;
  bf16_t* wb = nullptr;  // the pull copy peers read (bf16), written by the apply
  int64_t n = 0;
  float lr = 0.f, b1 = 0.9f, b2 = 0.999f, eps = 1e-8f, wd = 0.f;
  int64_t step = 0;
  char* inbox = nullptr;
  int64_t slot_bytes = 0;
  int depth = 1;
};

class HipApplier : public minips::Applier {
 public:
  HipApplier(int device, int tables);
  ~HipApplier() override;
  void SetSparse(int t, const PsSparseDesc& d);
  void SetDense(int t, const PsDenseDesc& d);
  int64_t Step(int t) const { return descs_.at(t).step.load(); }
  void SetStep(int t, int64_t s) { descs_.at(t).step.store(s); }
  void ThreadInit() override;
  void Apply(int t, int r, int64_t c) override;
  void Flush() override;

 private:
  struct Desc {
    int kind = -1;  // 0 sparse, 1 dense
    PsSparseDesc sp;
    PsDenseDesc dn;
    std::atomic<int64_t> step{0};
  };
  int dev_;
  hipStream_t stream_ = nullptr;
  std::vector<Desc> descs_;
};

}  // namespace minips_k
