// Control/data message protocol and the Actor base.
//
// Parity: Flag enum keeps the reference's 13 values in the same order
// (base/message.hpp:15-29); Meta keeps {sender, recver, model_id, failed_node_id, flag}
// (base/message.hpp:34-52) and -- unlike the reference (comm/mailbox.cpp:333-344) -- the
// wire format carries failed_node_id. Actor mirrors base/actor_model.hpp:13-34.
#pragma once

#include "base.h"

namespace minips {

enum class Flag : char {
  kExit = 0,
  kBarrier,
  kResetWorkerInModel,
  kClock,
  kAdd,
  kGet,
  kForceQuit,
  kCheckpoint,
  kHeartBeat,
  kQuitHeartBeat,
  kRollBack,
  kScale,
  kScaleRollback,
};
constexpr int kNumFlags = 13;
const char* FlagName(Flag f);

struct Meta {
  int32_t sender = -1;
  int32_t recver = -1;
  int32_t model_id = -1;
  int32_t failed_node_id = -1;
  Flag flag = Flag::kExit;
  std::string DebugString() const;
};

struct Message {
  Meta meta;
  std::vector<SArray<char>> data;

  template <typename V>
  void AddData(const SArray<V>& v) {
    data.push_back(SArray<char>(v));
  }
  std::string DebugString() const;
};

// An actor owns one thread that runs Main() over its work queue.
class Actor {
 public:
  explicit Actor(uint32_t id) : id_(id) {}
  virtual ~Actor() = default;
  void Start() { thread_ = std::thread([this] { Main(); }); }
  void Stop() {
    Message m;
    m.meta.flag = Flag::kExit;
    work_queue_.Push(m);
    if (thread_.joinable()) thread_.join();
  }
  ThreadsafeQueue<Message>* GetWorkQueue() { return &work_queue_; }
  uint32_t GetId() const { return id_; }

 protected:
  virtual void Main() = 0;
  uint32_t id_;
  ThreadsafeQueue<Message> work_queue_;
  std::thread thread_;
};

}  // namespace minips
