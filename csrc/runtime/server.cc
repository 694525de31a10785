#include "server.h"

#include <algorithm>
#include <cmath>
#include <fstream>

#include "fs.h"
#include <iomanip>

#include "checkpoint.h"
#include "config.h"
#include "ids.h"

namespace minips {

// ------------------------------------------------------------------------------ tracker
void ProgressTracker::Init(const std::vector<uint32_t>& tids) {
  progresses_.clear();
  for (auto t : tids) progresses_[(int)t] = 0;
  min_clock_ = 0;
}

bool ProgressTracker::IsUniqueMin(int tid) const {
  auto it = progresses_.find(tid);
  MINIPS_CHECK(it != progresses_.end(), "unknown tid " << tid);
  if (it->second != min_clock_) return false;
  int n = 0;
  for (auto& kv : progresses_) {
    if (kv.second == min_clock_ && ++n > 1) return false;
  }
  return true;
}

int ProgressTracker::AdvanceAndGetChangedMinClock(int tid) {
  MINIPS_CHECK(CheckThreadValid(tid), "tid:" << tid);
  if (IsUniqueMin(tid)) {
    min_clock_ += 1;
    progresses_[tid] += 1;
    return min_clock_;
  }
  progresses_[tid] += 1;
  return -1;
}

int ProgressTracker::GetProgress(int tid) const {
  auto it = progresses_.find(tid);
  MINIPS_CHECK(it != progresses_.end(), "unknown tid " << tid);
  return it->second;
}

int ProgressTracker::DeleteNode(uint32_t node_id) {
  int result = -1;
  const int lo = (int)(node_id * SimpleIdMapper::kMaxThreadsPerNode);
  const int hi = (int)((node_id + 1) * SimpleIdMapper::kMaxThreadsPerNode);
  for (auto it = progresses_.begin(); it != progresses_.end();) {
    if (it->first >= lo && it->first < hi) {
      if (IsUniqueMin(it->first)) {
        min_clock_ += 1;
        result = min_clock_;
      }
      MINIPS_LOG(0, "worker " << it->first << " of failed node " << node_id << " dropped at clock " << it->second);
      it = progresses_.erase(it);
    } else {
      ++it;
    }
  }
  return result;
}

int ProgressTracker::Update(int failed_node_id, const std::vector<Node>&) {
  if (failed_node_id < 0) return -1;
  return DeleteNode((uint32_t)failed_node_id);
}

int32_t ProgressTracker::RoundHundred(int32_t input) { return 100 * (int32_t)std::round(input / 100.0); }

void ProgressTracker::Dump(const std::string& path, bool round_hundred) const {
  GeneralOfstream out(path);
  MINIPS_CHECK(out.good(), "cannot write " << path);
  auto f = [&](int v) { return round_hundred ? RoundHundred(v) : v; };
  out << "min_clock" << ":" << f(min_clock_) << " ";
  for (auto& kv : progresses_) out << kv.first << ":" << f(kv.second) << " ";
  out.close();
  MINIPS_CHECK(out.good(), "write failed " << path);
}

void ProgressTracker::Restore(const std::string& path, int scale_node_id) {
  GeneralIfstream in(path);
  MINIPS_CHECK(in.good(), "cannot read " << path);
  std::string tok;
  while (in >> tok) {
    auto c = tok.find(':');
    if (c == std::string::npos) continue;
    std::string k = tok.substr(0, c);
    int v = std::stoi(tok.substr(c + 1));
    if (k == "min_clock") {
      min_clock_ = v;
    } else {
      int tid = std::stoi(k);
      progresses_[tid] = v;
      if (scale_node_id >= 0) {
        int mid = scale_node_id * (int)SimpleIdMapper::kMaxThreadsPerNode
            + tid % (int)SimpleIdMapper::kMaxThreadsPerNode;
        progresses_[mid] = v;
      }
    }
  }
}

std::string ProgressTracker::DebugString() const {
  std::ostringstream os;
  os << "min_clock=" << min_clock_;
  for (auto& kv : progresses_) os << " " << kv.first << ":" << kv.second;
  return os.str();
}

// ------------------------------------------------------------------------------ pending buffer
std::vector<Message> PendingBuffer::Pop(int clock) {
  std::vector<Message> r;
  auto it = buffer_.find(clock);
  if (it != buffer_.end()) {
    r = std::move(it->second);
    buffer_.erase(it);
  }
  return r;
}
std::vector<Message> PendingBuffer::PopAll() {
  std::vector<Message> r;
  for (auto& kv : buffer_)
    for (auto& m : kv.second) r.push_back(std::move(m));
  buffer_.clear();
  return r;
}
int PendingBuffer::Size(int clock) const {
  auto it = buffer_.find(clock);
  return it == buffer_.end() ? 0 : (int)it->second.size();
}
int PendingBuffer::TotalSize() const {
  int n = 0;
  for (auto& kv : buffer_) n += (int)kv.second.size();
  return n;
}

// ------------------------------------------------------------------------------ checkpoint cfg
static std::string Suffix(const CheckpointConfig& c) {
  std::string s = std::to_string(c.my_id);
  if (c.model_id > 0) s += "_t" + std::to_string(c.model_id);
  if (c.local_server_index > 0) s += "_s" + std::to_string(c.local_server_index);
  return s;
}
std::string CheckpointConfig::ParamsFile() const { return prefix + "server_params_" + Suffix(*this); }
std::string CheckpointConfig::ProgressFile() const { return prefix + "server_progress_" + Suffix(*this); }
std::string CheckpointConfig::WorkerConfigFile() const { return prefix + "worker_config_" + std::to_string(my_id); }
CheckpointConfig CheckpointConfig::FromContext(int local_server_index, int model_id) {
  CheckpointConfig c;
  auto& ctx = Context::Get();
  c.toggle = ctx.get_bool("checkpoint_toggle");
  c.prefix = ctx.get_string("checkpoint_file_prefix");
  c.my_id = ctx.get_int32("my_id");
  c.local_server_index = local_server_index;
  c.model_id = model_id;
  return c;
}

// ------------------------------------------------------------------------------ storage
void AbstractStorage::Add(const Message& msg) {
  MINIPS_CHECK(msg.data.size() == 2, "Add expects [keys, vals], got " << msg.data.size());
  SubAdd(SArray<Key>(msg.data[0]), msg.data[1]);
}

Message AbstractStorage::Get(const Message& msg) {
  MINIPS_CHECK(msg.data.size() == 1, "Get expects [keys], got " << msg.data.size());
  Message reply;
  reply.meta.sender = msg.meta.recver;
  reply.meta.recver = msg.meta.sender;
  reply.meta.model_id = msg.meta.model_id;
  reply.meta.flag = msg.meta.flag;
  SArray<Key> keys(msg.data[0]);
  reply.AddData(keys);
  reply.data.push_back(SubGet(keys));
  return reply;
}

template <typename Val>
static void WriteVal(std::ostream& os, Val v) {
  if (std::is_floating_point<Val>::value)
    os << std::setprecision(std::numeric_limits<Val>::max_digits10) << v;
  else
    os << v;
}
template <typename Val>
static Val ParseVal(const std::string& s) {
  if (std::is_floating_point<Val>::value) return (Val)std::stod(s);
  return (Val)std::stoll(s);
}

template <typename Val>
void MapStorage<Val>::Dump(const CheckpointConfig& cfg) {
  if (!cfg.toggle) return;
  EnsureParentDir(cfg.ParamsFile());
  GeneralOfstream out(cfg.ParamsFile());
  MINIPS_CHECK(out.good(), "cannot write " << cfg.ParamsFile());
  std::vector<Key> keys;
  for (auto& kv : storage_) keys.push_back(kv.first);
  std::sort(keys.begin(), keys.end());
  for (Key k : keys) {
    out << k << ":";
    WriteVal(out, storage_[k]);
    out << " ";
  }
  out.close();
  MINIPS_CHECK(out.good(), "write failed " << cfg.ParamsFile());
}
template <typename Val>
void MapStorage<Val>::Restore(const CheckpointConfig& cfg) {
  GeneralIfstream in(cfg.ParamsFile());
  MINIPS_CHECK(in.good(), "cannot read " << cfg.ParamsFile());
  storage_.clear();
  std::string tok;
  while (in >> tok) {
    auto c = tok.find(':');
    if (c == std::string::npos) continue;
    storage_[(Key)std::stoull(tok.substr(0, c))] = ParseVal<Val>(tok.substr(c + 1));
  }
}

template <typename Val>
void VectorStorage<Val>::Dump(const CheckpointConfig& cfg) {
  if (!cfg.toggle) return;
  EnsureParentDir(cfg.ParamsFile());
  GeneralOfstream out(cfg.ParamsFile());
  MINIPS_CHECK(out.good(), "cannot write " << cfg.ParamsFile());
  // Reference format (server/vector_storage.hpp:54-73): one line, "<local_idx>:<val> " for
  // every non-zero entry.
  for (size_t i = 0; i < storage_.size(); ++i) {
    if (storage_[i] != Val()) {
      out << i << ":";
      WriteVal(out, storage_[i]);
      out << " ";
    }
  }
  out.close();
  MINIPS_CHECK(out.good(), "write failed " << cfg.ParamsFile());
}
template <typename Val>
void VectorStorage<Val>::Restore(const CheckpointConfig& cfg) {
  GeneralIfstream in(cfg.ParamsFile());
  MINIPS_CHECK(in.good(), "cannot read " << cfg.ParamsFile());
  std::fill(storage_.begin(), storage_.end(), Val());
  std::string tok;
  while (in >> tok) {
    auto c = tok.find(':');
    if (c == std::string::npos) continue;
    size_t idx = std::stoull(tok.substr(0, c));
    MINIPS_CHECK(idx < storage_.size(), "checkpoint index " << idx << " out of range " << storage_.size());
    storage_[idx] = ParseVal<Val>(tok.substr(c + 1));
  }
}

template class MapStorage<double>;
template class MapStorage<float>;
template class MapStorage<int>;
template class MapStorage<int64_t>;
template class VectorStorage<double>;
template class VectorStorage<float>;
template class VectorStorage<int>;
template class VectorStorage<int64_t>;

// ------------------------------------------------------------------------------ models
void ModelBase::ResetWorker(Message& msg) {
  MINIPS_CHECK(msg.data.size() == 1, "ResetWorker expects [tids]");
  if (!SkipTrackerInitOnReset()) {
    SArray<uint32_t> tids(msg.data[0]);
    tracker_.Init(tids.ToVector());
  }
  Message reply;
  reply.meta.model_id = model_id_;
  reply.meta.sender = msg.meta.recver;
  reply.meta.recver = msg.meta.sender;
  reply.meta.flag = Flag::kResetWorkerInModel;
  reply_queue_->Push(reply);
}

void ModelBase::Dump(Message& msg) {
  if (ckpt_.toggle) {
    storage_->Dump(ckpt_);
    EnsureParentDir(ckpt_.ProgressFile());
    tracker_.Dump(ckpt_.ProgressFile(), /*round_hundred=*/false);
    if (ckpt_.local_server_index == 0 && ckpt_.model_id == 0)
      DumpConfigData(ckpt_.WorkerConfigFile(), Context::Get().GetIterationMap());
  }
  Message reply;
  reply.meta.recver = msg.meta.sender;
  reply.meta.sender = msg.meta.recver;
  reply.meta.flag = msg.meta.flag;
  reply.meta.model_id = msg.meta.model_id;
  reply_queue_->Push(reply);
}

// BSP: Adds are buffered until the min clock advances; Gets from a worker that already
// clocked wait for the superstep to close (bsp_model.cpp:14-56).
void BSPModel::Clock(Message& msg) {
  int updated = tracker_.AdvanceAndGetChangedMinClock(msg.meta.sender);
  int progress = tracker_.GetProgress(msg.meta.sender);
  MINIPS_CHECK(progress <= tracker_.GetMinClock() + 1,
               "BSP progress " << progress << " > min_clock+1 " << tracker_.GetMinClock() + 1);
  if (updated != -1) AdvanceSuperstep();
}

void BSPModel::AdvanceSuperstep() {
  for (auto& a : add_buffer_) storage_->Add(a);
  add_buffer_.clear();
  for (auto& g : get_buffer_) ReplyGet(g);
  get_buffer_.clear();
  storage_->FinishIter();
}

void BSPModel::Add(Message& msg) {
  MINIPS_CHECK(tracker_.CheckThreadValid(msg.meta.sender), "unknown sender " << msg.meta.sender);
  int progress = tracker_.GetProgress(msg.meta.sender);
  MINIPS_CHECK(progress == tracker_.GetMinClock(), "BSP add from worker at clock " << progress
                                                       << " while the table is at " << tracker_.GetMinClock());
  add_buffer_.push_back(msg);
}

void BSPModel::Get(Message& msg) {
  MINIPS_CHECK(tracker_.CheckThreadValid(msg.meta.sender), "unknown sender " << msg.meta.sender);
  int progress = tracker_.GetProgress(msg.meta.sender);
  if (progress == tracker_.GetMinClock() + 1) {
    get_buffer_.push_back(msg);
  } else if (progress == tracker_.GetMinClock()) {
    ReplyGet(msg);
  } else {
    MINIPS_CHECK(false, "BSP get from worker at clock " << progress << " while the table is at "
                                                                << tracker_.GetMinClock());
  }
}

void BSPModel::Restore() {
  storage_->Restore(ckpt_);
  tracker_.Restore(ckpt_.ProgressFile());
  add_buffer_.clear();  // adds of the interrupted superstep are replayed by the workers
  for (auto& g : get_buffer_) ReplyGet(g);
  get_buffer_.clear();
}

void BSPModel::Update(int failed_node_id, const std::vector<Node>& nodes, const Range& range) {
  storage_->Update(range);
  if (tracker_.Update(failed_node_id, nodes) != -1) AdvanceSuperstep();
}

SSPModel::SSPModel(uint32_t model_id, std::unique_ptr<AbstractStorage>&& storage, int staleness,
                   ThreadsafeQueue<Message>* reply_queue, CheckpointConfig ckpt, bool restore_on_start)
    : ModelBase(model_id, std::move(storage), reply_queue, ckpt), staleness_(staleness) {
  if (restore_on_start) Restore();
}

void SSPModel::Clock(Message& msg) {
  int updated = tracker_.AdvanceAndGetChangedMinClock(msg.meta.sender);
  if (updated != -1) Flush(updated);
}

void SSPModel::Flush(int updated_min_clock) {
  for (auto& req : buffer_.Pop(updated_min_clock)) ReplyGet(req);
  storage_->FinishIter();
}

void SSPModel::FlushAll() {
  auto reqs = buffer_.PopAll();
  for (auto& r : reqs) ReplyGet(r);
  storage_->FinishIter();
}

void SSPModel::Add(Message& msg) { storage_->Add(msg); }

// SSP gate (ssp_model.cpp:58-85): a Get from a worker more than `staleness` clocks ahead of
// the slowest is parked under clock (progress - staleness) and released when the min
// clock reaches it.
void SSPModel::Get(Message& msg) {
  int tid = msg.meta.sender;
  MINIPS_CHECK(tracker_.CheckThreadValid(tid), "unknown sender " << tid);
  int progress = tracker_.GetProgress(tid);
  int min_clock = tracker_.GetMinClock();
  if (progress > min_clock + staleness_) {
    buffer_.Push(progress - staleness_, msg);
  } else {
    ReplyGet(msg);
  }
}

void SSPModel::Restore() {
  storage_->Restore(ckpt_);
  tracker_.Restore(ckpt_.ProgressFile());
  restored_ = true;
  FlushAll();
  MINIPS_LOG(0, "SSPModel restored, min_clock=" << tracker_.GetMinClock());
}

void SSPModel::Update(int failed_node_id, const std::vector<Node>& nodes, const Range& range) {
  storage_->Update(range);
  int r = tracker_.Update(failed_node_id, nodes);
  if (r != -1) Flush(r);
}

void ASPModel::Clock(Message& msg) { tracker_.AdvanceAndGetChangedMinClock(msg.meta.sender); }
void ASPModel::Add(Message& msg) { storage_->Add(msg); }
void ASPModel::Get(Message& msg) { ReplyGet(msg); }
void ASPModel::Restore() {
  storage_->Restore(ckpt_);
  tracker_.Restore(ckpt_.ProgressFile());
}
void ASPModel::Update(int failed_node_id, const std::vector<Node>& nodes, const Range& range) {
  storage_->Update(range);
  tracker_.Update(failed_node_id, nodes);
}

// ------------------------------------------------------------------------------ server thread
void ServerThread::RegisterModel(uint32_t model_id, std::unique_ptr<AbstractModel>&& model) {
  std::lock_guard<std::mutex> lk(mu_);
  models_[model_id] = std::move(model);
}

AbstractModel* ServerThread::GetModel(uint32_t model_id) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = models_.find(model_id);
  return it == models_.end() ? nullptr : it->second.get();
}

void ServerThread::UpdateModel(int failed_node_id, const std::vector<Node>& nodes, const Range& range) {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& kv : models_) kv.second->Update(failed_node_id, nodes, range);
}

void ServerThread::RollbackModel() {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& kv : models_) kv.second->Restore();
}

void ServerThread::Main() {
  while (true) {
    Message msg;
    work_queue_.WaitAndPop(&msg);
    if (msg.meta.flag == Flag::kExit) break;
    std::lock_guard<std::mutex> lk(mu_);
    auto it = models_.find((uint32_t)msg.meta.model_id);
    if (it == models_.end()) {
      MINIPS_LOG(1, "server " << id_ << ": unknown model_id " << msg.meta.model_id << ", dropping "
                              << msg.meta.DebugString());
      continue;
    }
    dispatch_count_[static_cast<int>(msg.meta.flag)]++;
    AbstractModel* model = it->second.get();
    try {
      switch (msg.meta.flag) {
        case Flag::kClock: model->Clock(msg); break;
        case Flag::kAdd: model->Add(msg); break;
        case Flag::kGet: model->Get(msg); break;
        case Flag::kResetWorkerInModel: model->ResetWorker(msg); break;
        case Flag::kCheckpoint: model->Dump(msg); break;
        default: MINIPS_CHECK(false, "server " << id_ << " cannot handle " << FlagName(msg.meta.flag));
      }
    } catch (const std::exception& e) {
      MINIPS_LOG(2, "server " << id_ << ": " << e.what());
    }
  }
}

}  // namespace minips
