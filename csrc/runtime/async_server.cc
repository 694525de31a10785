#include "async_server.h"

#include <exception>

#include "base.h"

namespace minips {

AsyncServer::AsyncServer(const std::string& board_name, int world, int rank, int tables, Applier* applier)
    : board_(board_name, world, rank, tables), applier_(applier), world_(world), rank_(rank), tables_(tables),
      enabled_(tables) {
  MINIPS_CHECK(applier_ != nullptr, "async server: no applier");
  for (auto& e : enabled_) e.store(false);
}

AsyncServer::~AsyncServer() { Stop(); }

void AsyncServer::Enable(int table) {
  MINIPS_CHECK(table >= 0 && table < tables_, "async server: table " << table);
  enabled_[table].store(true, std::memory_order_release);
  board_.Wake();
}

void AsyncServer::Start() {
  if (running_.exchange(true)) return;
  stop_.store(false);
  th_ = std::thread([this] { Loop(); });
}

void AsyncServer::Stop() {
  if (!th_.joinable()) return;
  stop_.store(true);
  {
    std::lock_guard<std::mutex> lk(mu_);
    pause_req_ = false;
  }
  cv_.notify_all();
  board_.Wake();
  th_.join();
  running_.store(false);
}

void AsyncServer::Pause() {
  std::unique_lock<std::mutex> lk(mu_);
  pause_req_ = true;
  lk.unlock();
  board_.Wake();
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
        log_on = log_on_;
        if (pause_req_) {
          paused_ = true;
          cv_.notify_all();
          cv_.wait(lk, [&] { return !pause_req_ || stop_.load(); });
          paused_ = false;
          if (stop_.load()) break;
        }
      }
      // read the epoch BEFORE scanning: a publish after the scan changes it, so the sleep below
      // returns at once instead of missing that work
      const uint32_t epoch = board_.Epoch();
      todo.clear();
      for (int t = 0; t < tables_; ++t) {
        if (!enabled_[t].load(std::memory_order_acquire)) continue;
        for (int r = 0; r < world_; ++r) {
          const int64_t a = board_.Applied(t, rank_, r), s = board_.Sent(t, r);
          if (s > a) todo.push_back({t, r, a, s});
        }
      }
      if (todo.empty()) {
        board_.WaitEpoch(epoch, 0.05);
        continue;
      }
      std::vector<int64_t> logged;
      int64_t n = 0;
      for (int t = 0; t < tables_; ++t) {
        for (int64_t k = 0;; ++k) {
          bool any = false;
          for (const Todo& w : todo) {
            if (w.t != t || w.from + k >= w.to) continue;
            any = true;
            applier_->Apply(t, w.r, w.from + k);
            ++n;
            if (log_on) logged.insert(logged.end(), {(int64_t)t, (int64_t)w.r, w.from + k});
          }
          if (!any) break;
        }
      }
      applier_->Flush();  // the device work is complete: the rows are visible to every rank
      for (const Todo& w : todo) board_.PublishApplied(w.t, w.r, w.to);
      applies_.fetch_add(n);
      batches_.fetch_add(1);
      if (!logged.empty()) {
        std::lock_guard<std::mutex> lk(mu_);
        log_.insert(log_.end(), logged.begin(), logged.end());
      }
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
  }
  running_.store(false);
  cv_.notify_all();
  board_.Wake();
}

}  // namespace minips
