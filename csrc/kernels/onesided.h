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
struct AdamSlabs;  // (kernels.h) split-K planes folded by ps_push_dense

constexpr int kPsMaxWorld = 16;
constexpr int64_t kPsSlotHeader = 64;

enum PsOptimizer { kPsAdd = 0, kPsSgd = 1, kPsRowwiseAdagrad = 2, kPsAdagrad = 3, kPsAdam = 4 };

// Requester -> owners: unique keys uniq[0, U) (U = *U_dev, <= n) grouped by owner with counts[P]
// rows per owner, gradient rows g [>= U, W] fp32; owner o's slot starts at inbox[o] + slot_off.
void ps_push_rows(const int64_t* uniq, const int64_t* counts, const int64_t* U_dev, int64_t n, const float* g, int W,
                  const int64_t* inbox, int P, int64_t slot_off, int64_t cap, hipStream_t s);
// Every owner's slot header := value (0: a clock without an Add; a dense push marks its slot 1).
void ps_set_headers(const int64_t* inbox, int P, int64_t slot_off, int64_t value, hipStream_t s);
// dense push: grad[o * S, (o + 1) * S) -> inbox[o] + data_off for every owner o, grad cleared
void ps_push_dense(float* grad, const int64_t* inbox, int P, int64_t data_off, int64_t S, hipStream_t s,
                   const AdamSlabs* slabs = nullptr);
// out[i] = row of keys[i] (i < min(n, *n_dev)) from its owner's fp32 shard at bases[o]
// ([rows_o, W]); out fp32 or bf16 [n, W].
void ps_gather_rows(const int64_t* bases, const int64_t* bounds, int P, const int64_t* keys, int64_t n,
                    const int64_t* n_dev, int W, void* out, bool out_bf16, hipStream_t s);

// out[i] = row of keys[i] from a bf16 shard (rows of W bf16, W in {16, 32, 64}).
void ps_gather_rows_bf16tab(const int64_t* bases, const int64_t* bounds, int P, const int64_t* keys, int64_t n,
                            const int64_t* n_dev, int W, void* out, bool out_bf16, hipStream_t s);
// Map storage: out[i] = the row of keys[i] in its owner's open-addressing table (hkeys[o], hvals[o]:
// device addresses of owner o's key array [cap] and rows [cap, W] fp32), zeros when absent (the
// reference's default-insert 0, server/map_storage.hpp:21-26).
void ps_hash_gather(const int64_t* hkeys, const int64_t* hvals, const int64_t* bounds, int P, int64_t cap,
                    const int64_t* keys, int64_t n, const int64_t* n_dev, int W, void* out, bool out_bf16,
                    hipStream_t s);
// Pull copies of a dense table: for every owner o in `owners` (a list of `count` 4-bit owner ids),
// dst[o * shard_bytes ...] = srcs[o][0, shard_bytes) (srcs: device table of P addresses).
void ps_pull(const int64_t* srcs, uint64_t owners, int count, int64_t shard_bytes, void* dst, hipStream_t s);

// ---- per-owner reader / writer lock (the consistency of one-sided reads, see onesided.hip) ----
constexpr uint32_t kPsWriter = 0x80000000u;  // lock word: bit 31 the owner's writer, bits 0..30 readers
constexpr int kPsCtrlLine = 64;              // control buffer: one 64-byte line per table
constexpr int kPsCtrlBytes = 64 * 64;        // 16 table lines + the flush counters
constexpr int kPsHeldSlots = 256;            // reader-side ring of "locks held" masks
enum PsLockError : uint32_t { kPsErrReadLock = 1, kPsErrWriteLock = 2, kPsErrHashFull = 4 };
// Reader: take the read lock of every owner (ascending order), record the ones taken in *held.
void ps_read_lock(const int64_t* locks, int P, uint32_t* held, uint32_t* err, hipStream_t s);
// false: every owner is on this device (one rank): no system-scope fence launches
void ps_set_fences(bool on);
void ps_read_unlock(const int64_t* locks, int P, uint32_t* held, hipStream_t s);
// Owner: announce the writer, wait for the readers to drain / flush every XCD's L2, then release.
void ps_write_lock(uint32_t* lock, uint32_t* err, hipStream_t s);
void ps_write_unlock(uint32_t* lock, uint32_t* flush_count, hipStream_t s);

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
  int bf16 = 0;                 // rows stored in bf16 (stochastic rounding; fp32 pushes and state)
  uint32_t seed = 0;            //   ... the rounding stream's seed
  int64_t hash_cap = 0;         // > 0: Map storage -- open addressing over hkeys[hash_cap], rows in table
  unsigned long long* hkeys = nullptr;
  uint32_t* lock = nullptr;     // this owner's lock word of the table (+ its flush counter)
  uint32_t* flush = nullptr;
  void* rs = nullptr;           // clock-coalesced row-wise Adagrad: int2 [rows_local * P] (stamp, index)
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
  uint32_t* lock = nullptr;
  uint32_t* flush = nullptr;
  float* sum = nullptr;          // clock-coalesced Adam / Adagrad: the clock's summed gradient [n]
  int64_t* sum_active = nullptr;  //   ... and its number of active pushes (device word)
};

class HipApplier : public minips::Applier {
 public:
  HipApplier(int device, int tables);
  ~HipApplier() override;
  void SetSparse(int t, const PsSparseDesc& d);
  void SetDense(int t, const PsDenseDesc& d);
  int64_t Step(int t) const { return descs_.at(t).step.load(); }
  void SetStep(int t, int64_t s) { descs_.at(t).step.store(s); }
  void SetErrorWord(uint32_t* err) { err_ = err; }
  void ThreadInit() override;
  void BeginTable(int t) override;
  void Apply(int t, int r, int64_t c) override;
  void ApplyClock(int t, int64_t c, int world) override;
  void EndTable(int t) override;
  uint64_t Submit() override;
  void Wait(uint64_t ticket) override;
  void Flush() override;

 private:
  struct Desc {
    int kind = -1;  // 0 sparse, 1 dense
    PsSparseDesc sp;
    PsDenseDesc dn;
    std::atomic<int64_t> step{0};  // Adam steps (dense) / applies (bf16 rows: the rounding stream)
    int64_t stamp = 0;             // clock-coalesced sparse applies issued (the rs table's stamps)
  };
  int dev_;
  hipStream_t stream_ = nullptr;
  std::vector<Desc> descs_;
  uint32_t* err_ = nullptr;
  static constexpr int kEvents = 8;  // batches in flight at most (the server keeps <= 2)
  hipEvent_t events_[kEvents] = {};
  uint64_t submitted_ = 0;
};

}  // namespace minips_k
