// Progress board of the asynchronous parameter server (minips_amd/ps/onesided.py): the ranks of
// one node share a /dev/shm segment that records, per table,
//
//   sent[t][r]        clocks requester r has finished for table t: the pushes of its clocks
//                     < sent have landed in every owner's inbox (published after the push
//                     kernels completed)
//   applied[t][o][r]  clocks of requester r that owner o's server thread has applied to its
//                     shard of table t (published after the apply kernels completed)
//
// and everything the asynchronous protocol decides is a predicate over these numbers:
//
//   owner o has work          sent[t][r] > applied[t][o][r] for some r
//   SSP Get at clock c        min_{o,r} applied[t][o][r] >= c - s: every worker's pushes of its
//                             clocks < c - s are in every shard -- the reference's "a Get waits
//                             while progress > min_clock + staleness" (server/consistency/
//                             ssp_model.cpp:58-85) with the server-side apply of SSPModel::Add
//                             (:54-56) happening on the owner
//   inbox slot reuse          requester r may write its clock-c push into slot c % depth once
//                             min_o applied[t][o][r] >= c - depth + 1
//   dense pull freshness      owner o's shard changed iff sum_r applied[t][o][r] changed
//
// The ProgressTracker role (server/util/progress_tracker.{hpp,cpp}: per-worker progress and the
// min clock) is this table of counters; there is no message round trip, a rank reads it with a
// few loads. Waiters sleep on one shared futex word (the epoch) that every publish bumps.
//
// Layout: 64-byte header, then sent as one 64-byte line per (table, rank) (each line has a single
// writer), then applied as one 128-byte row per (table, owner) (written only by that owner).
#pragma once

#include <atomic>
#include <cstdint>
#include <string>
#include <vector>

namespace minips {

class PSBoard {
 public:
  static constexpr int kMaxWorld = 16;
  static constexpr int kMaxTables = 16;

  // Maps (creating if absent) /dev/shm/<name>; every rank of the job passes the same world/tables.
  PSBoard(const std::string& name, int world, int rank, int tables, double attach_timeout_s = 30.0);
  ~PSBoard();
  PSBoard(const PSBoard&) = delete;
  PSBoard& operator=(const PSBoard&) = delete;

  int world() const { return world_; }
  int rank() const { return rank_; }
  int tables() const { return tables_; }

  // requester side
  void PublishSent(int table, int64_t clock);
  int64_t Sent(int table, int rank) const;
  int64_t MinSent(int table) const;
  // owner side (this rank is the owner)
  void PublishApplied(int table, int requester, int64_t clock);
  void PublishAppliedRow(int table, int64_t clock);  // every requester's entry (restore / reset)
  int64_t Applied(int table, int owner, int requester) const;
  int64_t MinApplied(int table) const;                       // min over owners and requesters
  int64_t MinAppliedFrom(int table, int requester) const;    // min over owners
  int64_t OwnerVersion(int table, int owner) const;          // sum over requesters
  int64_t Pending(int table) const;  // clocks sent to this rank (as owner) and not applied yet

  // Blocking waits (futex sleep on the epoch, GIL released by the bindings). They return the
  // seconds waited, or -1 if the condition still does not hold after `timeout_s` (> 0) -- the
  // caller decides whether that is a failure (and can check the server's error in between) --
  // or -2 once the board is aborted.
  double WaitMinApplied(int table, int64_t target, double timeout_s);
  double WaitAppliedFrom(int table, int requester, int64_t target, double timeout_s);
  double WaitSentAtLeast(int table, int rank, int64_t target, double timeout_s);
  // Server: sleep until the epoch differs from `seen` (or `max_s` passed); returns the new epoch.
  uint32_t WaitEpoch(uint32_t seen, double max_s);
  uint32_t Epoch() const { return hdr_->epoch.load(std::memory_order_acquire); }
  void Wake();  // bump the epoch and wake every sleeper (shutdown, pause)

  // Reader / writer lock per (table, owner) for the CPU data path (GPU ranks keep their lock words
  // in the owners' HBM, csrc/kernels/onesided.hip): a reader takes every owner's read lock in
  // ascending order, the owner's server thread takes its own write lock around a batch of applies,
  // so no read sees half of a batch. Writer preference (a waiting writer blocks new readers).
  bool ReadLock(int table, double timeout_s);  // false (nothing held) on timeout / abort
  void ReadUnlock(int table);
  bool WriteLock(int table, double timeout_s);
  void WriteUnlock(int table);
  // Job-wide abort word: a rank that knows the set cannot finish (a peer died, the supervisor
  // restarts everyone) sets it; every wait on this board then gives up at once (returns -2).
  void SetAbort(uint32_t code);
  uint32_t Aborted() const { return hdr_->abort.load(std::memory_order_acquire); }

  std::vector<int64_t> SnapshotSent(int table) const;
  std::vector<int64_t> SnapshotApplied(int table) const;  // [owner][requester] row-major
  uint64_t Wakeups() const { return wakeups_; }
  void Unlink();
  const std::string& Name() const { return name_; }

 private:
  struct Header {
    uint64_t magic;
    int32_t world, tables;
    std::atomic<uint32_t> epoch;  // futex word
    std::atomic<uint32_t> abort;
    char pad[40];
  };
  struct LockLine {
    std::atomic<uint32_t> word;  // bit 31 writer, bits 0..30 readers
    char pad[60];
  };
  struct SentLine {
    std::atomic<int64_t> clock;
    char pad[56];
  };
  struct AppliedRow {
    std::atomic<int64_t> clock[kMaxWorld];
  };
  template <typename Pred>
  double WaitUntil(Pred pred, double timeout_s);
  void Bump();

  Header* hdr_ = nullptr;
  SentLine* sent_ = nullptr;
  AppliedRow* applied_ = nullptr;
  LockLine* locks_ = nullptr;
  size_t bytes_ = 0;
  int world_, rank_, tables_;
  std::string name_;
  uint64_t wakeups_ = 0;
};

}  // namespace minips
