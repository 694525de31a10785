#include "worker.h"

namespace minips {

void CallbackRunner::RegisterRecvHandle(uint32_t app_tid, uint32_t model_id, const std::function<void(Message&)>& h) {
  std::lock_guard<std::mutex> lk(mu_);
  recv_handle_[app_tid][model_id] = h;
}

void CallbackRunner::RegisterRecvFinishHandle(uint32_t app_tid, uint32_t model_id, const std::function<void()>& h) {
  std::lock_guard<std::mutex> lk(mu_);
  recv_finish_handle_[app_tid][model_id] = h;
}

void CallbackRunner::NewRequest(uint32_t app_tid, uint32_t model_id, uint32_t expected_responses) {
  std::lock_guard<std::mutex> lk(mu_);
  tracker_[app_tid][model_id] = {expected_responses, 0};
}

void CallbackRunner::WaitRequest(uint32_t app_tid, uint32_t model_id) {
  std::unique_lock<std::mutex> lk(mu_);
  auto done = [&] {
    auto& t = tracker_[app_tid][model_id];
    return t.first <= t.second;
  };
  if (timeout_s_ > 0) {
    MINIPS_CHECK(CondWaitFor(cond_, lk, timeout_s_, done),
                 "request of thread " << app_tid << " table " << model_id << " timed out");
  } else {
    cond_.wait(lk, done);
  }
}

void CallbackRunner::AddResponse(uint32_t app_tid, uint32_t model_id, Message& msg) {
  std::function<void(Message&)> handle;
  std::function<void()> finish;
  bool last;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto& t = tracker_[app_tid][model_id];
    last = t.first == t.second + 1;
    auto hit = recv_handle_[app_tid].find(model_id);
    if (hit != recv_handle_[app_tid].end()) handle = hit->second;
    if (last) {
      auto fit = recv_finish_handle_[app_tid].find(model_id);
      if (fit != recv_finish_handle_[app_tid].end()) finish = fit->second;
    }
  }
  if (handle) handle(msg);
  if (last && finish) finish();
  {
    std::lock_guard<std::mutex> lk(mu_);
    tracker_[app_tid][model_id].second += 1;
  }
  if (last) cond_.notify_all();
}

void CallbackRunner::NewCheckPoint(uint32_t expected_responses) {
  std::lock_guard<std::mutex> lk(mu_);
  checkpoint_expected_ = expected_responses;
  checkpoint_current_ = 0;
}

void CallbackRunner::WaitCheckPoint() {
  std::unique_lock<std::mutex> lk(mu_);
  auto done = [&] { return checkpoint_expected_ <= checkpoint_current_; };
  if (timeout_s_ > 0) {
    MINIPS_CHECK(CondWaitFor(cond_, lk, timeout_s_, done), "checkpoint timed out");
  } else {
    cond_.wait(lk, done);
  }
}

void CallbackRunner::CheckPointResponse() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    checkpoint_current_ += 1;
  }
  cond_.notify_all();
}

void CallbackRunner::ForceCompleteAll() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& a : tracker_)
      for (auto& m : a.second) m.second.second = std::max(m.second.second, m.second.first);
    for (auto& a : recv_finish_handle_)
      for (auto& m : a.second) m.second = nullptr;
    checkpoint_current_ = std::max(checkpoint_current_, checkpoint_expected_);
  }
  cond_.notify_all();
}

void CallbackRunner::DecrementExpected(uint32_t lost) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& a : tracker_)
      for (auto& m : a.second) m.second.first = m.second.first > lost ? m.second.first - lost : 0;
    checkpoint_expected_ = checkpoint_expected_ > lost ? checkpoint_expected_ - lost : 0;
  }
  cond_.notify_all();
}

void WorkerThread::Main() {
  while (true) {
    Message msg;
    work_queue_.WaitAndPop(&msg);
    if (msg.meta.flag == Flag::kExit) break;
    try {
      if (msg.meta.flag == Flag::kCheckpoint) {
        CheckPointResponse();
      } else {
        AddResponse((uint32_t)msg.meta.recver, (uint32_t)msg.meta.model_id, msg);
      }
    } catch (const std::exception& e) {
      MINIPS_LOG(2, "worker helper " << id_ << ": " << e.what());
    }
  }
}

}  // namespace minips
