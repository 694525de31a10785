// Server side: progress tracking, pending buffers, storages, consistency models and the
// server actor.
//
// Parity:
//   ProgressTracker  -> server/util/progress_tracker.{hpp,cpp} (unique-min advance rule,
//                       DeleteNode by tid range, text Dump/Restore "min_clock:<r100> tid:<r100>")
//   PendingBuffer    -> server/util/pending_buffer.{hpp,cpp}
//   AbstractStorage  -> server/abstract_storage.hpp (template method Add/Get)
//   MapStorage       -> server/map_storage.hpp     (default-insert 0 on Get)
//   VectorStorage    -> server/vector_storage.hpp  ("<local_idx>:<val> " text dump; the
//                       reference's mis-parsing Restore is fixed)
//   BSP/SSP/ASPModel -> server/consistency/*       (identical gating rules; all three now
//                       answer kCheckpoint so CheckPoint() cannot hang under BSP/ASP)
//   ServerThread     -> server/server_thread.{hpp,cpp}
#pragma once

#include <map>
#include <unordered_map>

#include "base.h"
#include "message.h"
#include "node.h"

namespace minips {

class ProgressTracker {
 public:
  void Init(const std::vector<uint32_t>& tids);
  // Returns the new min clock when it advanced, -1 otherwise.
  int AdvanceAndGetChangedMinClock(int tid);
  int GetProgress(int tid) const;
  int GetMinClock() const { return min_clock_; }
  int GetNumThreads() const { return (int)progresses_.size(); }
  bool IsUniqueMin(int tid) const;
  bool CheckThreadValid(int tid) const { return progresses_.count(tid) > 0; }
  // Removes every tid of node_id; returns the new min clock if it advanced, else -1.
  int DeleteNode(uint32_t node_id);
  int Update(int failed_node_id, const std::vector<Node>& nodes);
  static int32_t RoundHundred(int32_t input);
  // round_hundred=true reproduces the reference's RoundHundred rounding in the file.
  void Dump(const std::string& path, bool round_hundred = true) const;
  // scale_node_id >= 0 clones every entry onto that node's tids (progress_tracker.hpp:112-118).
  void Restore(const std::string& path, int scale_node_id = -1);
  std::string DebugString() const;
  const std::map<int, int>& Progresses() const { return progresses_; }

 private:
  std::map<int, int> progresses_;
  int min_clock_ = 0;
};

class PendingBuffer {
 public:
  void Push(int clock, const Message& msg) { buffer_[clock].push_back(msg); }
  std::vector<Message> Pop(int clock);
  std::vector<Message> PopAll();
  void EraseAll() { buffer_.clear(); }
  int Size(int clock) const;
  int TotalSize() const;

 private:
  std::map<int, std::vector<Message>> buffer_;  // ordered: FlushAll replays in clock order
};

// Where a storage/model writes its checkpoint; filled from Context by the engine.
struct CheckpointConfig {
  bool toggle = false;
  std::string prefix;
  int my_id = 0;
  int local_server_index = 0;  // disambiguates multiple server threads per node
  int model_id = 0;
  std::string ParamsFile() const;
  std::string ProgressFile() const;
  std::string WorkerConfigFile() const;
  static CheckpointConfig FromContext(int local_server_index, int model_id);
};

class AbstractStorage {
 public:
  virtual ~AbstractStorage() = default;
  void Add(const Message& msg);
  Message Get(const Message& msg);
  virtual void SubAdd(const SArray<Key>& keys, const SArray<char>& vals) = 0;
  virtual SArray<char> SubGet(const SArray<Key>& keys) = 0;
  virtual void FinishIter() {}
  virtual void Dump(const CheckpointConfig& cfg) = 0;
  virtual void Restore(const CheckpointConfig& cfg) = 0;
  virtual void Update(const Range& range) = 0;
  virtual size_t ValueSize() const = 0;
};

template <typename Val>
class MapStorage : public AbstractStorage {
 public:
  void SubAdd(const SArray<Key>& keys, const SArray<char>& vals) override {
    SArray<Val> v(vals);
    MINIPS_CHECK(keys.size() == v.size(), "keys/vals size mismatch " << keys.size() << "/" << v.size());
    for (size_t i = 0; i < keys.size(); ++i) storage_[keys[i]] += v[i];
  }
  SArray<char> SubGet(const SArray<Key>& keys) override {
    SArray<Val> r(keys.size());
    for (size_t i = 0; i < keys.size(); ++i) r[i] = storage_[keys[i]];
    return SArray<char>(r);
  }
  void Dump(const CheckpointConfig& cfg) override;
  void Restore(const CheckpointConfig& cfg) override;
  void Update(const Range&) override {}
  size_t ValueSize() const override { return sizeof(Val); }
  size_t Size() const { return storage_.size(); }

 private:
  std::unordered_map<Key, Val> storage_;
};

template <typename Val>
class VectorStorage : public AbstractStorage {
 public:
  explicit VectorStorage(const Range& range) : range_(range), storage_(range.size(), Val()) {}
  void SubAdd(const SArray<Key>& keys, const SArray<char>& vals) override {
    SArray<Val> v(vals);
    MINIPS_CHECK(keys.size() == v.size(), "keys/vals size mismatch");
    for (size_t i = 0; i < keys.size(); ++i) {
      MINIPS_CHECK(keys[i] >= range_.begin() && keys[i] < range_.end(),
                   "key " << keys[i] << " outside [" << range_.begin() << "," << range_.end() << ")");
      storage_[keys[i] - range_.begin()] += v[i];
    }
  }
  SArray<char> SubGet(const SArray<Key>& keys) override {
    SArray<Val> r(keys.size());
    for (size_t i = 0; i < keys.size(); ++i) {
      MINIPS_CHECK(keys[i] >= range_.begin() && keys[i] < range_.end(), "key " << keys[i] << " outside range");
      r[i] = storage_[keys[i] - range_.begin()];
    }
    return SArray<char>(r);
  }
  void Dump(const CheckpointConfig& cfg) override;
  void Restore(const CheckpointConfig& cfg) override;
  void Update(const Range& range) override {
    std::vector<Val> n(range.size(), Val());
    for (uint64_t k = std::max(range.begin(), range_.begin()); k < std::min(range.end(), range_.end()); ++k)
      n[k - range.begin()] = storage_[k - range_.begin()];
    storage_.swap(n);
    range_ = range;
  }
  size_t ValueSize() const override { return sizeof(Val); }
  const std::vector<Val>& Data() const { return storage_; }
  const Range& GetRange() const { return range_; }

 private:
  Range range_;
  std::vector<Val> storage_;
};

class AbstractModel {
 public:
  virtual ~AbstractModel() = default;
  virtual void Clock(Message& msg) = 0;
  virtual void Add(Message& msg) = 0;
  virtual void Get(Message& msg) = 0;
  virtual int GetProgress(int tid) = 0;
  virtual void ResetWorker(Message& msg) = 0;
  virtual void Dump(Message& msg) = 0;
  virtual void Restore() = 0;
  virtual void Update(int failed_node_id, const std::vector<Node>& nodes, const Range& range) = 0;
  virtual int GetPendingSize() const { return 0; }
};

// Shared plumbing of the three consistency models.
class ModelBase : public AbstractModel {
 public:
  ModelBase(uint32_t model_id, std::unique_ptr<AbstractStorage>&& storage, ThreadsafeQueue<Message>* reply_queue,
            CheckpointConfig ckpt)
      : model_id_(model_id), storage_(std::move(storage)), reply_queue_(reply_queue), ckpt_(ckpt) {}
  int GetProgress(int tid) override { return tracker_.GetProgress(tid); }
  void ResetWorker(Message& msg) override;
  void Dump(Message& msg) override;
  AbstractStorage* storage() { return storage_.get(); }
  ProgressTracker& tracker() { return tracker_; }

 protected:
  void ReplyGet(const Message& req) { reply_queue_->Push(storage_->Get(req)); }
  virtual bool SkipTrackerInitOnReset() const { return false; }
  uint32_t model_id_;
  std::unique_ptr<AbstractStorage> storage_;
  ThreadsafeQueue<Message>* reply_queue_;
  CheckpointConfig ckpt_;
  ProgressTracker tracker_;
};

class BSPModel : public ModelBase {
 public:
  using ModelBase::ModelBase;
  void Clock(Message& msg) override;
  void Add(Message& msg) override;
  void Get(Message& msg) override;
  void Restore() override;
  void Update(int failed_node_id, const std::vector<Node>& nodes, const Range& range) override;
  int GetGetPendingSize() const { return (int)get_buffer_.size(); }
  int GetAddPendingSize() const { return (int)add_buffer_.size(); }
  int GetPendingSize() const override { return (int)(get_buffer_.size() + add_buffer_.size()); }

 private:
  void AdvanceSuperstep();
  std::vector<Message> add_buffer_;
  std::vector<Message> get_buffer_;
};

class SSPModel : public ModelBase {
 public:
  SSPModel(uint32_t model_id, std::unique_ptr<AbstractStorage>&& storage, int staleness,
           ThreadsafeQueue<Message>* reply_queue, CheckpointConfig ckpt, bool restore_on_start = false);
  void Clock(Message& msg) override;
  void Add(Message& msg) override;
  void Get(Message& msg) override;
  void Restore() override;
  void Update(int failed_node_id, const std::vector<Node>& nodes, const Range& range) override;
  int GetPendingSize(int progress) const { return buffer_.Size(progress); }
  int GetPendingSize() const override { return buffer_.TotalSize(); }
  int staleness() const { return staleness_; }

 protected:
  bool SkipTrackerInitOnReset() const override { return restored_; }

 private:
  void Flush(int updated_min_clock);
  void FlushAll();
  int staleness_;
  bool restored_ = false;
  PendingBuffer buffer_;
};

class ASPModel : public ModelBase {
 public:
  using ModelBase::ModelBase;
  void Clock(Message& msg) override;
  void Add(Message& msg) override;
  void Get(Message& msg) override;
  void Restore() override;
  void Update(int failed_node_id, const std::vector<Node>& nodes, const Range& range) override;
};

class ServerThread : public Actor {
 public:
  explicit ServerThread(uint32_t id) : Actor(id) {}
  void RegisterModel(uint32_t model_id, std::unique_ptr<AbstractModel>&& model);
  AbstractModel* GetModel(uint32_t model_id);
  void UpdateModel(int failed_node_id, const std::vector<Node>& nodes, const Range& range);
  void RollbackModel();
  // Counts of dispatched messages by flag (test observability).
  int DispatchCount(Flag f) const { return dispatch_count_[static_cast<int>(f)].load(); }

 protected:
  void Main() override;

 private:
  std::mutex mu_;  // guards models_ against rollback from the mailbox thread
  std::map<uint32_t, std::unique_ptr<AbstractModel>> models_;
  std::atomic<int> dispatch_count_[kNumFlags] = {};
};

}  // namespace minips
