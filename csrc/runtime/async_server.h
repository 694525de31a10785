// Server thread of the asynchronous parameter server: the owner side of every SSP / ASP table on
// one rank (minips_amd/ps/onesided.py).
//
// Parity: server/server_thread.cpp:23-61 (an actor that pops requests and dispatches them to the
// table's model) and server/consistency/{ssp,asp}_model.cpp (Add applies at the server as soon
// as it arrives: ssp_model.cpp:54-56, asp_model.cpp:18-21). Requests are not messages here: a
// requester writes its clock's (key, gradient row) batch straight into an inbox slot in the
// owner's HBM (one slot ring per requester) and bumps its `sent` counter on the PSBoard; this
// thread sleeps on the board's futex, finds (table, requester, clock) triples with sent > applied,
// has the Applier run the optimizer on them (row-wise Adagrad / Adam / SGD with the owner's own
// optimizer state), waits for that device work and publishes `applied`. Gets never come here:
// they read the owner's rows one-sidedly, gated on `applied` (PSBoard).
//
// Apply order inside one wake-up: clock-major, requesters interleaved (r0 c, r1 c, ..., r0 c+1,
// ...), per table -- recorded in the apply log when enabled, so a test can replay the exact order.
//
// Pipelining: the thread does not wait for a batch's device work. It hands (ticket, what the batch
// applied) to a publisher thread, which waits for the ticket and then publishes `applied`, and
// scans for the next batch right away (up to kInFlight batches issued and unpublished), so the
// applies of consecutive batches queue back to back on the owner's stream. `issued_` remembers
// what is in flight; Pause() drains the pipeline.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ps_board.h"

namespace minips {

class Applier {
 public:
  virtual ~Applier() = default;
  virtual void ThreadInit() {}  // called once on the server thread (e.g. bind the device)
  // Brackets of one table's applies in a batch (the GPU applier takes the owner's write lock of
  // the table there, so no one-sided read sees half of the batch).
  virtual void BeginTable(int /*t*/) {}
  virtual void EndTable(int /*t*/) {}
  // Issue the apply of requester `r`'s clock `c` of table `t` (inbox slot c % depth); may return
  // before the work completed.
  virtual void Apply(int t, int r, int64_t c) = 0;
  // Issue ONE apply of clock `c` of table `t` that covers every requester's slot (a table served
  // clock-coalesced, AsyncServer::SetCoalesce): the rows of the P pushes summed per key in
  // requester order, one optimizer step per row per clock. The default applies the P pushes one
  // by one (exact for the linear add / SGD rules).
  virtual void ApplyClock(int t, int64_t c, int world) {
    for (int r = 0; r < world; ++r) Apply(t, r, c);
  }
  // Mark the end of a batch: Wait(ticket) returns once every apply issued before Submit completed
  // and is visible to every rank. The default is synchronous (the work is done when Submit returns).
  virtual uint64_t Submit() {
    Flush();
    return 0;
  }
  virtual void Wait(uint64_t /*ticket*/) {}
  // Complete every issued apply: the updated rows must be visible to every rank afterwards.
  virtual void Flush() = 0;
};

class AsyncServer {
 public:
  AsyncServer(const std::string& board_name, int world, int rank, int tables, Applier* applier);
  ~AsyncServer();
  AsyncServer(const AsyncServer&) = delete;
  AsyncServer& operator=(const AsyncServer&) = delete;

  void Enable(int table);  // serve `table` from now on (its descriptors exist)
  // Clock-coalesced service of `table` (SSP tables with a stateful optimizer): clock c is applied
  // once every requester sent it, as one Applier::ApplyClock, and published for all requesters
  // together. The reference's SSP server applies each Add on arrival as `+=`
  // (server/consistency/ssp_model.cpp:54-56) -- linear in the pushes, so P pushes of a clock sum
  // to the BSP update; a row-wise Adagrad / Adam step per push is not (each push would be its own
  // scale-invariant step: a key every rank pushed moved up to ~2.8x a BSP step at 4 ranks). Set
  // before Enable.
  void SetCoalesce(int table, bool on);
  void Start();
  void Stop();
  // Pause: returns once no apply is in flight and none will start until Resume() (a consistent
  // point of this owner's shards for a checkpoint snapshot or a restore).
  void Pause();
  void Resume();
  bool Running() const { return running_.load(); }
  std::string Error() const;
  void SetLog(bool on);
  std::vector<int64_t> TakeLog();  // flat (table, requester, clock) triples in apply order
  int64_t Applied() const { return applies_.load(); }
  int64_t Batches() const { return batches_.load(); }
  PSBoard& board() { return board_; }

 private:
  void Loop();
  void PublishLoop();
  struct Batch {
    uint64_t ticket;
    std::vector<int64_t> pub;  // (table, requester, clock) triples to publish
    int64_t applies;
    std::vector<int64_t> logged;
  };
  static constexpr int kInFlight = 2;

  PSBoard board_;
  Applier* applier_;
  const int world_, rank_, tables_;
  std::vector<std::atomic<bool>> enabled_, coalesce_;
  std::thread th_;
  std::atomic<bool> stop_{false}, running_{false};
  std::atomic<int64_t> applies_{0}, batches_{0};
  mutable std::mutex mu_;
  std::condition_variable cv_;
  bool pause_req_ = false, paused_ = false;
  std::string error_;
  bool log_on_ = false;
  std::vector<int64_t> log_;
  // pipeline (guarded by mu_): batches issued, not yet published; issued_[t * world + r]
  std::deque<Batch> inflight_;
  std::vector<int64_t> issued_;
  bool resync_ = true;  // re-read issued_ from the board (start, resume: a restore may rewind it)
  bool loop_done_ = false;
  std::condition_variable pcv_;
  std::thread pub_;
};

}  // namespace minips
