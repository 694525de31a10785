#include "async_server.h"

#include <algorithm>
#include <climits>
#include <exception>

#include "base.h"
#include "trace.h"

namespace minips {

AsyncServer::AsyncServer(const std::string& board_name, int world, int rank, int tables, Applier* applier)
    : board_(board_name, world, rank, tables), applier_(applier), world_(world), rank_(rank), tables_(tables),
      enabled_(tables), coalesce_(tables), issued_((size_t)tables * world, 0) {
  MINIPS_CHECK(applier_ != nullptr, "async server: no applier");
  for (auto& e : enabled_) e.store(false);
  for (auto& e : coalesce_) e.store(false);
}

void AsyncServer::SetCoalesce(int table, bool on) {
  MINIPS_CHECK(table >= 0 && table < tables_, "async server: table " << table);
  MINIPS_CHECK(!enabled_[table].load(), "async server: SetCoalesce before Enable (table " << table << ")");
  coalesce_[table].store(on, std::memory_order_release);
}

AsyncServer::~AsyncServer() { Stop(); }

void AsyncServer::Enable(int table) {
  MINIPS_CHECK(table >= 0 && table < tables_, "async server: table " << table);
  {
    // the table's counters may be ahead of issued_ (a table registered after earlier traffic)
    std::lock_guard<std::mutex> lk(mu_);
    resync_ = true;
  }
  enabled_[table].store(true, std::memory_order_release);
  board_.Wake();
}

void AsyncServer::Start() {
  if (running_.exchange(true)) return;
  stop_.store(false);
  {
    std::lock_guard<std::mutex> lk(mu_);
    resync_ = true;
    loop_done_ = false;
  }
  pub_ = std::thread([this] { PublishLoop(); });
  th_ = std::thread([this] { Loop(); });
}

void AsyncServer::Stop() {
  if (!th_.joinable() && !pub_.joinable()) return;
  stop_.store(true);
  {
    std::lock_guard<std::mutex> lk(mu_);
    pause_req_ = false;
  }
  cv_.notify_all();
  pcv_.notify_all();
  board_.Wake();
  if (th_.joinable()) th_.join();  // the publisher then drains what was issued and exits
  pcv_.notify_all();
  if (pub_.joinable()) pub_.join();
  running_.store(false);
}

void AsyncServer::Pause() {
  std::unique_lock<std::mutex> lk(mu_);
  pause_req_ = true;
  lk.unlock();
  board_.Wake();
  pcv_.notify_all();
  lk.lock();
  cv_.wait(lk, [&] { return paused_ || !running_.load() || !error_.empty(); });
}

void AsyncServer::Resume() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    pause_req_ = false;
  }
  cv_.notify_all();
}

std::string AsyncServer::Error() const {
  std::lock_guard<std::mutex> lk(mu_);
  return error_;
}

void AsyncServer::SetLog(bool on) {
  std::lock_guard<std::mutex> lk(mu_);
  log_on_ = on;
}

std::vector<int64_t> AsyncServer::TakeLog() {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<int64_t> out;
  out.swap(log_);
  return out;
}

void AsyncServer::Loop() {
  struct Todo {
    int t, r;
    int64_t from, to;
  };
  std::vector<Todo> todo;
  try {
    applier_->ThreadInit();
    while (!stop_.load()) {
      bool log_on;
      {
        std::unique_lock<std::mutex> lk(mu_);
        if (pause_req_) {
          // a consistent point: nothing issued and unpublished, nothing starts until Resume
          pcv_.wait(lk, [&] { return inflight_.empty() || stop_.load() || !error_.empty(); });
          paused_ = true;
          cv_.notify_all();
          cv_.wait(lk, [&] { return !pause_req_ || stop_.load(); });
          paused_ = false;
          resync_ = true;  // a restore may have rewound the board
          if (stop_.load()) break;
        }
        // at most kInFlight batches issued and not yet published
        pcv_.wait(lk, [&] { return (int)inflight_.size() < kInFlight || stop_.load() || pause_req_; });
        if (stop_.load()) break;
        if (pause_req_) continue;
        if (resync_) {  // the pipeline is empty here (start / resume / enable)
          if (inflight_.empty()) {
            for (int t = 0; t < tables_; ++t)
              for (int r = 0; r < world_; ++r) issued_[(size_t)t * world_ + r] = board_.Applied(t, rank_, r);
            resync_ = false;
          } else {
            pcv_.wait(lk, [&] { return inflight_.empty() || stop_.load(); });
            continue;
          }
        }
        log_on = log_on_;
      }
      // read the epoch BEFORE scanning: a publish after the scan changes it, so the sleep below
      // returns at once instead of missing that work
      const uint32_t epoch = board_.Epoch();
      todo.clear();
      for (int t = 0; t < tables_; ++t) {
        if (!enabled_[t].load(std::memory_order_acquire)) continue;
        if (coalesce_[t].load(std::memory_order_relaxed)) {
          // whole clocks only: every requester sent them (issued_ is the same for every requester)
          const int64_t a = issued_[(size_t)t * world_];
          int64_t s = INT64_MAX;
          for (int r = 0; r < world_; ++r) s = std::min(s, board_.Sent(t, r));
          if (s > a) todo.push_back({t, -1, a, s});
          continue;
        }
        for (int r = 0; r < world_; ++r) {
          const int64_t a = issued_[(size_t)t * world_ + r], s = board_.Sent(t, r);
          if (s > a) todo.push_back({t, r, a, s});
        }
      }
      if (todo.empty()) {
        board_.WaitEpoch(epoch, 0.05);
        continue;
      }
      Batch b;
      b.applies = 0;
      TraceRange range("ps.owner.issue");  // the batch's lock / apply / unlock launches
      for (int t = 0; t < tables_; ++t) {
        bool begun = false;
        for (int64_t k = 0;; ++k) {
          bool any = false;
          for (const Todo& w : todo) {
            if (w.t != t || w.from + k >= w.to) continue;
            if (!begun) {
              applier_->BeginTable(t);
              begun = true;
            }
            any = true;
            if (w.r < 0) {  // a coalesced clock: every requester's slot in one apply
              applier_->ApplyClock(t, w.from + k, world_);
              b.applies += world_;
              if (log_on)
                for (int r = 0; r < world_; ++r) b.logged.insert(b.logged.end(), {(int64_t)t, (int64_t)r, w.from + k});
              continue;
            }
            applier_->Apply(t, w.r, w.from + k);
            ++b.applies;
            if (log_on) b.logged.insert(b.logged.end(), {(int64_t)t, (int64_t)w.r, w.from + k});
          }
          if (!any) break;
        }
        if (begun) applier_->EndTable(t);
      }
      b.ticket = applier_->Submit();
      for (const Todo& w : todo) {
        for (int r = w.r < 0 ? 0 : w.r; r < (w.r < 0 ? world_ : w.r + 1); ++r) {
          issued_[(size_t)w.t * world_ + r] = w.to;
          b.pub.insert(b.pub.end(), {(int64_t)w.t, (int64_t)r, w.to});
        }
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        inflight_.push_back(std::move(b));
      }
      pcv_.notify_all();
    }
  } catch (const std::exception& e) {
    std::lock_guard<std::mutex> lk(mu_);
    error_ = e.what();
  } catch (...) {
    std::lock_guard<std::mutex> lk(mu_);
    error_ = "unknown error in the async server thread";
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    paused_ = false;
    loop_done_ = true;
  }
  pcv_.notify_all();
  cv_.notify_all();
  board_.Wake();
}

// Publishes the batches in issue order once their device work completed (their rows are visible
// to every rank), then wakes the waiters of the board.
void AsyncServer::PublishLoop() {
  for (;;) {
    Batch* b = nullptr;
    {
      std::unique_lock<std::mutex> lk(mu_);
      pcv_.wait(lk, [&] { return !inflight_.empty() || loop_done_; });
      if (inflight_.empty()) break;  // the loop ended and everything issued is published
      b = &inflight_.front();        // stays in the deque (only this thread pops)
    }
    bool ok = true;
    TraceRange range("ps.owner.publish");  // wait for the batch's device work, then publish it
    try {
      applier_->Wait(b->ticket);
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> lk(mu_);
      if (error_.empty()) error_ = e.what();
      ok = false;
    }
    if (ok) {  // never publish a batch whose device work failed
      for (size_t i = 0; i + 2 < b->pub.size(); i += 3)
        board_.PublishApplied((int)b->pub[i], (int)b->pub[i + 1], b->pub[i + 2]);
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (ok) {
        applies_.fetch_add(b->applies);
        batches_.fetch_add(1);
        if (!b->logged.empty()) log_.insert(log_.end(), b->logged.begin(), b->logged.end());
      }
      inflight_.pop_front();
      if (!ok) {
        inflight_.clear();  // nothing later may be published either
        stop_.store(true);
      }
    }
    pcv_.notify_all();
    cv_.notify_all();
  }
  cv_.notify_all();
  running_.store(false);
}

}  // namespace minips
