// Worker side: completion tracking (callback runner / worker helper thread) and the
// per-(thread, table) KV client API.
//
// Parity:
//   AbstractCallbackRunner -> worker/abstract_callback_runner.hpp:9-44
//   WorkerThread           -> worker/worker_thread.{hpp,cpp} (tracker_[tid][model] =
//                             {expected, current}; RollBackWorker force-completes). The
//                             reference reads the handle maps outside its mutex
//                             (worker_thread.cpp:91-94); here every map access is locked.
//   KVClientTable<Val>     -> worker/kv_client_table.hpp (Get blocks; Add/Clock async;
//                             CheckPoint blocks; replies re-assembled by sorting slices by
//                             first key). Reply values are read as Val, not always double.
#pragma once

#include <algorithm>
#include <map>

#include "base.h"
#include "ids.h"
#include "message.h"

namespace minips {

class AbstractCallbackRunner {
 public:
  virtual ~AbstractCallbackRunner() = default;
  virtual void RegisterRecvHandle(uint32_t app_tid, uint32_t model_id, const std::function<void(Message&)>& h) = 0;
  virtual void RegisterRecvFinishHandle(uint32_t app_tid, uint32_t model_id, const std::function<void()>& h) = 0;
  virtual void NewRequest(uint32_t app_tid, uint32_t model_id, uint32_t expected_responses) = 0;
  virtual void WaitRequest(uint32_t app_tid, uint32_t model_id) = 0;
  virtual void AddResponse(uint32_t app_tid, uint32_t model_id, Message& msg) = 0;
  virtual void NewCheckPoint(uint32_t expected_responses) = 0;
  virtual void WaitCheckPoint() = 0;
  virtual void CheckPointResponse() = 0;
};

// In-process callback runner (also the completion engine inside WorkerThread).
class CallbackRunner : public AbstractCallbackRunner {
 public:
  void RegisterRecvHandle(uint32_t app_tid, uint32_t model_id, const std::function<void(Message&)>& h) override;
  void RegisterRecvFinishHandle(uint32_t app_tid, uint32_t model_id, const std::function<void()>& h) override;
  void NewRequest(uint32_t app_tid, uint32_t model_id, uint32_t expected_responses) override;
  void WaitRequest(uint32_t app_tid, uint32_t model_id) override;
  void AddResponse(uint32_t app_tid, uint32_t model_id, Message& msg) override;
  void NewCheckPoint(uint32_t expected_responses) override;
  void WaitCheckPoint() override;
  void CheckPointResponse() override;
  // Force-complete every outstanding request and drop finish handles (rollback).
  void ForceCompleteAll();
  // A node was removed: each outstanding request expects `lost` fewer replies.
  void DecrementExpected(uint32_t lost);
  void SetTimeout(double seconds) { timeout_s_ = seconds; }

 private:
  std::mutex mu_;
  std::condition_variable cond_;
  std::map<uint32_t, std::map<uint32_t, std::pair<uint32_t, uint32_t>>> tracker_;
  std::map<uint32_t, std::map<uint32_t, std::function<void(Message&)>>> recv_handle_;
  std::map<uint32_t, std::map<uint32_t, std::function<void()>>> recv_finish_handle_;
  uint32_t checkpoint_expected_ = 0, checkpoint_current_ = 0;
  double timeout_s_ = 0;  // 0 = wait forever
};

class WorkerThread : public Actor, public CallbackRunner {
 public:
  explicit WorkerThread(uint32_t id) : Actor(id) {}
  void RollBackWorker() { ForceCompleteAll(); }
  void Update(uint32_t lost_servers) { DecrementExpected(lost_servers); }

 protected:
  void Main() override;
};

template <typename Val>
class KVClientTable {
 public:
  KVClientTable(uint32_t app_thread_id, uint32_t model_id, ThreadsafeQueue<Message>* sender_queue,
                const AbstractPartitionManager* partition_manager, AbstractCallbackRunner* callback_runner)
      : app_thread_id_(app_thread_id),
        model_id_(model_id),
        sender_queue_(sender_queue),
        partition_manager_(partition_manager),
        callback_runner_(callback_runner) {
    callback_runner_->RegisterRecvHandle(app_thread_id_, model_id_, [this](Message& m) { HandleMsg_(m); });
  }

  // Keys must be sorted ascending (range partitioning + reply re-assembly rely on it).
  void Get(const std::vector<Key>& keys, std::vector<Val>* vals) { Get_(SArray<Key>(keys), vals); }
  void Get(const SArray<Key>& keys, std::vector<Val>* vals) { Get_(keys, vals); }
  void Add(const std::vector<Key>& keys, const std::vector<Val>& vals) { Add_(SArray<Key>(keys), SArray<Val>(vals)); }
  void Add(const SArray<Key>& keys, const SArray<Val>& vals) { Add_(keys, vals); }

  void Clock() {
    for (uint32_t server : partition_manager_->GetServerThreadIds()) {
      Message m;
      m.meta.sender = app_thread_id_;
      m.meta.recver = server;
      m.meta.model_id = model_id_;
      m.meta.flag = Flag::kClock;
      sender_queue_->Push(m);
    }
  }

  void CheckPoint() {
    const auto& servers = partition_manager_->GetServerThreadIds();
    callback_runner_->NewCheckPoint((uint32_t)servers.size());
    for (uint32_t server : servers) {
      Message m;
      m.meta.sender = app_thread_id_;
      m.meta.recver = server;
      m.meta.model_id = model_id_;
      m.meta.flag = Flag::kCheckpoint;
      sender_queue_->Push(m);
    }
    callback_runner_->WaitCheckPoint();
  }

  void HeartBeat(int node_id, bool quit = false) {
    int master = partition_manager_->GetMasterNodeId();
    if (master < 0) return;
    Message m;
    m.meta.sender = node_id;
    m.meta.recver = master;
    m.meta.flag = quit ? Flag::kQuitHeartBeat : Flag::kHeartBeat;
    sender_queue_->Push(m);
  }

 private:
  void Send_(const SArray<Key>& keys, const SArray<char>& vals, int server, Flag flag) {
    Message m;
    m.meta.sender = app_thread_id_;
    m.meta.recver = server;
    m.meta.model_id = model_id_;
    m.meta.flag = flag;
    m.AddData(keys);
    if (flag == Flag::kAdd) m.data.push_back(vals);
    sender_queue_->Push(m);
  }

  void Add_(const SArray<Key>& keys, const SArray<Val>& vals) {
    MINIPS_CHECK(keys.size() == vals.size(), "Add: keys/vals mismatch " << keys.size() << "/" << vals.size());
    std::vector<std::tuple<int, Keys, SArray<char>>> sliced;
    partition_manager_->SliceBytes(keys, SArray<char>(vals), &sliced);
    for (auto& s : sliced) Send_(std::get<1>(s), std::get<2>(s), std::get<0>(s), Flag::kAdd);
  }

  void Get_(const SArray<Key>& keys, std::vector<Val>* vals) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      recv_kvs_.clear();
    }
    std::vector<std::pair<int, Keys>> sliced;
    partition_manager_->Slice(keys, &sliced);
    callback_runner_->RegisterRecvFinishHandle(app_thread_id_, model_id_, [this, vals] { HandleFinish_(vals); });
    callback_runner_->NewRequest(app_thread_id_, model_id_, (uint32_t)sliced.size());
    for (auto& s : sliced) Send_(s.second, SArray<char>(), s.first, Flag::kGet);
    callback_runner_->WaitRequest(app_thread_id_, model_id_);
    if (sliced.empty()) vals->clear();
  }

  void HandleMsg_(Message& msg) {
    MINIPS_CHECK(msg.data.size() == 2, "Get reply must carry [keys, vals]");
    std::lock_guard<std::mutex> lk(mu_);
    recv_kvs_.push_back({SArray<Key>(msg.data[0]), SArray<Val>(msg.data[1])});
  }

  void HandleFinish_(std::vector<Val>* vals) {
    std::lock_guard<std::mutex> lk(mu_);
    size_t total = 0;
    for (auto& kv : recv_kvs_) total += kv.second.size();
    std::sort(recv_kvs_.begin(), recv_kvs_.end(), [](const auto& a, const auto& b) {
      Key ka = a.first.empty() ? 0 : a.first[0];
      Key kb = b.first.empty() ? 0 : b.first[0];
      return ka < kb;
    });
    vals->resize(total);
    size_t off = 0;
    for (auto& kv : recv_kvs_) {
      if (kv.second.size()) std::memcpy(vals->data() + off, kv.second.data(), kv.second.size() * sizeof(Val));
      off += kv.second.size();
    }
  }

  uint32_t app_thread_id_;
  uint32_t model_id_;
  ThreadsafeQueue<Message>* sender_queue_;
  const AbstractPartitionManager* partition_manager_;
  AbstractCallbackRunner* callback_runner_;
  std::mutex mu_;
  std::vector<std::pair<SArray<Key>, SArray<Val>>> recv_kvs_;
};

}  // namespace minips
