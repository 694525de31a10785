// Implementations for base.h / message.h / node.h / config.h / ids.h.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>

#include "fs.h"
#include <iomanip>

#include "config.h"
#include "ids.h"
#include "message.h"
#include "node.h"

namespace minips {

// ------------------------------------------------------------------------------ logging
namespace {
std::mutex g_log_mu;
}
int VerboseLevel() {
  static int v = [] {
    const char* s = std::getenv("GLOG_v");  // glog's names (the reference logs through glog)
    return s ? std::atoi(s) : 0;
  }();
  return v;
}
void LogLine(int level, const std::string& line) {
  static int min_level = [] {
    const char* s = std::getenv("GLOG_minloglevel");
    return s ? std::atoi(s) : 0;
  }();
  if (level < min_level) return;
  static const char kTag[] = {'I', 'W', 'E'};
  auto now = std::chrono::system_clock::now().time_since_epoch();
  double ts = std::chrono::duration<double>(now).count();
  std::lock_guard<std::mutex> lk(g_log_mu);
  std::fprintf(stderr, "%c%.6f minips] %s\n", kTag[std::min(level, 2)], ts, line.c_str());
}

// ------------------------------------------------------------------------------ message
const char* FlagName(Flag f) {
  static const char* kNames[kNumFlags] = {
      "kExit",      "kBarrier",      "kResetWorkerInModel", "kClock",    "kAdd",
      "kGet",       "kForceQuit",    "kCheckpoint",         "kHeartBeat", "kQuitHeartBeat",
      "kRollBack",  "kScale",        "kScaleRollback"};
  int i = static_cast<int>(f);
  return (i >= 0 && i < kNumFlags) ? kNames[i] : "kUnknown";
}

std::string Meta::DebugString() const {
  std::ostringstream os;
  os << "Meta{sender=" << sender << ", recver=" << recver << ", model_id=" << model_id
     << ", failed_node_id=" << failed_node_id << ", flag=" << FlagName(flag) << "}";
  return os.str();
}

std::string Message::DebugString() const {
  std::ostringstream os;
  os << meta.DebugString() << " data:[";
  for (size_t i = 0; i < data.size(); ++i) os << (i ? "," : "") << data[i].size() << "B";
  os << "]";
  return os.str();
}

// ------------------------------------------------------------------------------ node
std::string Node::DebugString() const {
  std::ostringstream os;
  os << "Node{id=" << id << ", host=" << hostname << ", port=" << port << ", is_master=" << is_master
     << ", gpu=" << gpu << "}";
  return os.str();
}

std::vector<Node> ParseFile(const std::string& path) {
  GeneralIfstream in(path);
  MINIPS_CHECK(in.good(), "cannot open hostfile " << path);
  std::vector<Node> nodes;
  std::string line;
  while (std::getline(in, line)) {
    // strip comments/whitespace
    auto hash = line.find('#');
    if (hash != std::string::npos) line = line.substr(0, hash);
    line.erase(std::remove_if(line.begin(), line.end(), [](char c) { return std::isspace((unsigned char)c); }),
               line.end());
    if (line.empty()) continue;
    std::vector<std::string> parts;
    std::stringstream ss(line);
    std::string tok;
    while (std::getline(ss, tok, ':')) parts.push_back(tok);
    MINIPS_CHECK(parts.size() == 3 || parts.size() == 4, "bad hostfile line '" << line << "'");
    Node n;
    n.id = static_cast<uint32_t>(std::stoul(parts[0]));
    n.hostname = parts[1];
    n.port = std::stoi(parts[2]);
    if (parts.size() == 4) n.gpu = std::stoi(parts[3]);
    nodes.push_back(n);
  }
  return nodes;
}

Node SelectMaster(std::vector<Node>& nodes, int heartbeat_interval) {
  Node master;
  master.is_master = false;
  if (heartbeat_interval <= 0) return master;
  for (auto it = nodes.begin(); it != nodes.end(); ++it) {
    if (it->id == 1) {
      master = *it;
      master.is_master = true;
      nodes.erase(it);
      return master;
    }
  }
  return master;
}

bool CheckValidNodeIds(const std::vector<Node>& nodes) {
  for (auto& n : nodes)
    if (n.id >= SimpleIdMapper::kMaxNodeId) return false;
  return true;
}

bool CheckUniquePort(std::vector<Node>& nodes) {
  std::set<std::pair<std::string, int>> seen;
  for (auto& n : nodes)
    if (!seen.insert({n.hostname, n.port}).second) return false;
  return true;
}

Node GetNodeById(const std::vector<Node>& nodes, uint32_t id) {
  for (auto& n : nodes)
    if (n.id == id) return n;
  MINIPS_CHECK(false, "node " << id << " not found");
  return Node();
}

bool CheckConsecutiveIds(const std::vector<Node>& nodes) {
  for (size_t i = 0; i < nodes.size(); ++i)
    if (nodes[i].id != i) return false;
  return true;
}

bool HasNode(const std::vector<Node>& nodes, uint32_t id) {
  for (auto& n : nodes)
    if (n.id == id) return true;
  return false;
}

// ------------------------------------------------------------------------------ context
Context& Context::Get() {
  static Context ctx;
  return ctx;
}

Context::Context() { ResetToDefaults(); }

void Context::ResetToDefaults() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    flags_.clear();
    iteration_map_.clear();
  }
  // Flags the library reads, same names as the reference.
  Define("my_id", Type::kInt, "0", "node id of this process (checkpoint file suffix)");
  Define("config_file", Type::kString, "", "hostfile: id:host:port[:gpu] per line");
  Define("checkpoint_toggle", Type::kBool, "false", "enable checkpoint dumps");
  Define("checkpoint_file_prefix", Type::kString, "/tmp/minips_ckpt/", "checkpoint dump prefix");
  Define("checkpoint_raw_prefix", Type::kString, "/tmp/minips_ckpt/", "data reload prefix");
  Define("use_weight_file", Type::kBool, "false", "resume from checkpoint (relaunch mode)");
  Define("heartbeat_interval", Type::kInt, "0", "seconds; <=0 disables the master");
  Define("relaunch_cmd", Type::kString, "", "shell prefix; failed node id appended");
  Define("num_servers_per_node", Type::kInt, "1", "server threads (shards) per node");
  Define("num_workers_per_node", Type::kInt, "1", "worker threads per node");
  Define("num_dims", Type::kInt, "0", "parameter dimension for getRanges()");
  Define("scale", Type::kBool, "false", "this process is a scale-out node");
  Define("scale_node_id", Type::kInt, "-1", "id of the scale-out node");
  Define("has_scale_node", Type::kBool, "false", "a scale-out node joined");
  Define("scale_file", Type::kString, "/tmp/minips_scale", "scale node description file");
  // North-star additions.
  Define("dtype", Type::kString, "bf16", "compute dtype of the GPU data plane");
  Define("optimizer", Type::kString, "sgd", "server-side optimizer");
  Define("bucket_mb", Type::kInt, "64", "dense collective bucket size (MB)");
  Define("num_gpus", Type::kInt, "1", "GPU ranks per node");
  Define("key_bits", Type::kInt, "64", "key width");
  Define("barrier_timeout_s", Type::kDouble, "600", "barrier / request timeout (seconds)");
}

Context& Context::Define(const std::string& name, Type type, const std::string& default_value,
                         const std::string& help) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = flags_.find(name);
  if (it != flags_.end()) {
    MINIPS_CHECK(it->second.type == type, "flag " << name << " redefined with another type");
    return *this;
  }
  flags_[name] = Entry{type, default_value, default_value, help};
  return *this;
}

bool Context::Has(const std::string& name) const {
  std::lock_guard<std::mutex> lk(mu_);
  return flags_.count(name) > 0;
}

const Context::Entry& Context::Find(const std::string& name) const {
  auto it = flags_.find(name);
  MINIPS_CHECK(it != flags_.end(), "unknown flag '" << name << "'");
  return it->second;
}

std::string Context::get_string(const std::string& name) const {
  std::lock_guard<std::mutex> lk(mu_);
  return Find(name).value;
}
int32_t Context::get_int32(const std::string& name) const { return static_cast<int32_t>(get_int64(name)); }
int64_t Context::get_int64(const std::string& name) const {
  std::lock_guard<std::mutex> lk(mu_);
  const Entry& e = Find(name);
  MINIPS_CHECK(e.type == Type::kInt || e.type == Type::kDouble, "flag " << name << " is not numeric");
  return e.value.empty() ? 0 : std::stoll(e.value);
}
bool Context::get_bool(const std::string& name) const {
  std::lock_guard<std::mutex> lk(mu_);
  const Entry& e = Find(name);
  const std::string& v = e.value;
  return v == "1" || v == "true" || v == "True" || v == "yes";
}
double Context::get_double(const std::string& name) const {
  std::lock_guard<std::mutex> lk(mu_);
  const Entry& e = Find(name);
  return e.value.empty() ? 0.0 : std::stod(e.value);
}

void Context::set(const std::string& name, const std::string& value) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = flags_.find(name);
  MINIPS_CHECK(it != flags_.end(), "unknown flag '" << name << "'");
  if (it->second.type == Type::kInt) {
    size_t pos = 0;
    (void)std::stoll(value, &pos);
    MINIPS_CHECK(pos == value.size(), "flag " << name << " expects an int, got '" << value << "'");
  } else if (it->second.type == Type::kDouble) {
    size_t pos = 0;
    (void)std::stod(value, &pos);
    MINIPS_CHECK(pos == value.size(), "flag " << name << " expects a number, got '" << value << "'");
  } else if (it->second.type == Type::kBool) {
    MINIPS_CHECK(value == "0" || value == "1" || value == "true" || value == "false" || value == "True" ||
                     value == "False",
                 "flag " << name << " expects a bool, got '" << value << "'");
  }
  it->second.value = value;
}

void Context::set(const std::string& name, double value) {
  std::ostringstream os;
  os << std::setprecision(17) << value;
  set(name, os.str());
}

std::vector<std::string> Context::ParseArgs(int argc, const char* const* argv, bool allow_unknown) {
  std::vector<std::string> args;
  for (int i = 1; i < argc; ++i) args.push_back(argv[i]);
  return ParseArgs(args, allow_unknown);
}

std::vector<std::string> Context::ParseArgs(const std::vector<std::string>& args, bool allow_unknown) {
  std::vector<std::string> rest;
  for (size_t i = 0; i < args.size(); ++i) {
    const std::string& a = args[i];
    if (a.rfind("--", 0) != 0 && !(a.rfind("-", 0) == 0 && a.size() > 1 && !std::isdigit((unsigned char)a[1]))) {
      rest.push_back(a);
      continue;
    }
    std::string body = a.substr(a.rfind("--", 0) == 0 ? 2 : 1);
    std::string name, value;
    bool has_value = false;
    auto eq = body.find('=');
    if (eq != std::string::npos) {
      name = body.substr(0, eq);
      value = body.substr(eq + 1);
      has_value = true;
    } else {
      name = body;
    }
    if (!Has(name)) {
      if (!has_value && name.rfind("no", 0) == 0 && Has(name.substr(2))) {
        set(name.substr(2), std::string("false"));
        continue;
      }
      MINIPS_CHECK(allow_unknown, "unknown flag --" << name);
      rest.push_back(a);
      continue;
    }
    Type t;
    {
      std::lock_guard<std::mutex> lk(mu_);
      t = flags_[name].type;
    }
    if (!has_value) {
      if (t == Type::kBool) {
        value = "true";
      } else {
        MINIPS_CHECK(i + 1 < args.size(), "flag --" << name << " needs a value");
        value = args[++i];
      }
    }
    set(name, value);
  }
  return rest;
}

std::map<std::string, std::string> Context::Snapshot() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::map<std::string, std::string> m;
  for (auto& kv : flags_) m[kv.first] = kv.second.value;
  return m;
}

std::string Context::Help() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::ostringstream os;
  for (auto& kv : flags_)
    os << "  --" << kv.first << " (default '" << kv.second.default_value << "') " << kv.second.help << "\n";
  return os.str();
}

void Context::SetIteration(int worker_id, int iteration) {
  std::lock_guard<std::mutex> lk(mu_);
  iteration_map_[worker_id] = iteration;
}
int Context::GetIteration(int worker_id) const {
  std::lock_guard<std::mutex> lk(mu_);
  int wid = worker_id;
  // Under scale-out the new node's workers map onto the originals (context.hpp:44-47).
  auto sit = flags_.find("scale");
  if (sit != flags_.end() && (sit->second.value == "true" || sit->second.value == "1")) {
    int wpn = std::stoi(flags_.at("num_workers_per_node").value);
    if (wpn > 0) wid = worker_id % wpn;
  }
  auto it = iteration_map_.find(wid);
  return it == iteration_map_.end() ? 0 : it->second;
}
std::map<int, int> Context::GetIterationMap() const {
  std::lock_guard<std::mutex> lk(mu_);
  return iteration_map_;
}
void Context::SetIterationMap(const std::map<int, int>& m) {
  std::lock_guard<std::mutex> lk(mu_);
  iteration_map_ = m;
}

// ------------------------------------------------------------------------------ id mapper
void SimpleIdMapper::Init(int num_server_threads_per_node, int skip_node_id) {
  std::lock_guard<std::mutex> lk(mu_);
  MINIPS_CHECK(num_server_threads_per_node > 0, "need >= 1 server thread");
  MINIPS_CHECK(num_server_threads_per_node <= (int)kWorkerHelperThreadId, "too many server threads");
  for (const auto& node : nodes_) {
    MINIPS_CHECK(node.id < kMaxNodeId, "node id " << node.id << " >= " << kMaxNodeId);
    if (skip_node_id >= 0 && (int)node.id == skip_node_id) continue;
    auto& servers = node2server_[node.id];
    servers.clear();
    for (int i = 0; i < num_server_threads_per_node; ++i) servers.push_back(node.id * kMaxThreadsPerNode + i);
    node2worker_helper_[node.id] = {node.id * kMaxThreadsPerNode + kWorkerHelperThreadId};
  }
}

void SimpleIdMapper::Update(const std::vector<Node>& nodes, int num_server_threads_per_node, int skip_node_id) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    nodes_ = nodes;
    node2server_.clear();
    node2worker_helper_.clear();
    node2worker_.clear();
  }
  Init(num_server_threads_per_node, skip_node_id);
}

uint32_t SimpleIdMapper::AllocateWorkerThread(uint32_t node_id) {
  std::lock_guard<std::mutex> lk(mu_);
  MINIPS_CHECK(node2worker_helper_.count(node_id), "node " << node_id << " has no worker helper");
  auto& used = node2worker_[node_id];
  for (uint32_t i = kMaxBgThreadsPerNode; i < kMaxThreadsPerNode; ++i) {
    uint32_t tid = i + node_id * kMaxThreadsPerNode;
    if (!used.count(tid)) {
      used.insert(tid);
      return tid;
    }
  }
  MINIPS_CHECK(false, "no free worker thread id on node " << node_id);
  return 0;
}

void SimpleIdMapper::DeallocateWorkerThread(uint32_t node_id, uint32_t tid) {
  std::lock_guard<std::mutex> lk(mu_);
  MINIPS_CHECK(node2worker_helper_.count(node_id), "node " << node_id << " unknown");
  auto& used = node2worker_[node_id];
  MINIPS_CHECK(used.count(tid), "tid " << tid << " not allocated");
  used.erase(tid);
}

std::vector<uint32_t> SimpleIdMapper::GetServerThreadsForId(uint32_t node_id) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = node2server_.find(node_id);
  return it == node2server_.end() ? std::vector<uint32_t>() : it->second;
}
std::vector<uint32_t> SimpleIdMapper::GetWorkerHelperThreadsForId(uint32_t node_id) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = node2worker_helper_.find(node_id);
  return it == node2worker_helper_.end() ? std::vector<uint32_t>() : it->second;
}
std::vector<uint32_t> SimpleIdMapper::GetWorkerThreadsForId(uint32_t node_id) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = node2worker_.find(node_id);
  if (it == node2worker_.end()) return {};
  return {it->second.begin(), it->second.end()};
}
std::vector<uint32_t> SimpleIdMapper::GetAllServerThreads() {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<uint32_t> r;
  for (auto& kv : node2server_) r.insert(r.end(), kv.second.begin(), kv.second.end());
  return r;
}

// ------------------------------------------------------------------------------ worker spec
void WorkerSpec::Init(const std::vector<WorkerAlloc>& worker_alloc) {
  for (const auto& a : worker_alloc) {
    MINIPS_CHECK(a.node_id < SimpleIdMapper::kMaxNodeId, "bad node id");
    MINIPS_CHECK(a.num_workers < SimpleIdMapper::kMaxThreadsPerNode - SimpleIdMapper::kMaxBgThreadsPerNode,
                 "too many workers");
    for (uint32_t i = 0; i < a.num_workers; ++i) {
      worker_to_node_[num_workers_] = a.node_id;
      node_to_workers_[a.node_id].push_back(num_workers_);
      num_workers_ += 1;
    }
  }
}
bool WorkerSpec::HasLocalWorkers(uint32_t node_id) const { return node_to_workers_.count(node_id) > 0; }
const std::vector<uint32_t>& WorkerSpec::GetLocalWorkers(uint32_t node_id) const {
  auto it = node_to_workers_.find(node_id);
  MINIPS_CHECK(it != node_to_workers_.end(), "node " << node_id << " has no workers");
  return it->second;
}
const std::vector<uint32_t>& WorkerSpec::GetLocalThreads(uint32_t node_id) const {
  auto it = node_to_threads_.find(node_id);
  MINIPS_CHECK(it != node_to_threads_.end(), "node " << node_id << " has no threads");
  return it->second;
}
std::vector<uint32_t> WorkerSpec::GetAllThreadIds() const {
  std::vector<uint32_t> r;
  for (auto& kv : thread_to_worker_) r.push_back(kv.first);
  return r;
}
void WorkerSpec::InsertWorkerIdThreadId(uint32_t worker_id, uint32_t thread_id) {
  MINIPS_CHECK(!worker_to_thread_.count(worker_id), "worker " << worker_id << " already mapped");
  MINIPS_CHECK(!thread_to_worker_.count(thread_id), "thread " << thread_id << " already mapped");
  MINIPS_CHECK(worker_to_node_.count(worker_id), "worker " << worker_id << " unknown");
  worker_to_thread_[worker_id] = thread_id;
  thread_to_worker_[thread_id] = worker_id;
  node_to_threads_[worker_to_node_[worker_id]].push_back(thread_id);
}

// ------------------------------------------------------------------------------ partition
RangePartitionManager::RangePartitionManager(const std::vector<uint32_t>& server_thread_ids,
                                             const std::vector<Range>& ranges, int master_node_id)
    : AbstractPartitionManager(server_thread_ids, master_node_id), ranges_(ranges) {
  MINIPS_CHECK(ranges_.size() == server_thread_ids_.size(),
               "ranges (" << ranges_.size() << ") != servers (" << server_thread_ids_.size() << ")");
}

template <typename F>
void RangePartitionManager::ForEachSlice(const Keys& keys, F&& f) const {
  if (ranges_.empty()) return;
  const Key* it = std::lower_bound(keys.begin(), keys.end(), (Key)ranges_[0].begin());
  size_t start = it - keys.begin();
  for (size_t i = 0; i < ranges_.size(); ++i) {
    it = std::lower_bound(it, keys.end(), (Key)ranges_[i].end());
    size_t end = it - keys.begin();
    if (end > start) f(i, start, end);
    start = end;
  }
}

void RangePartitionManager::Slice(const Keys& keys, std::vector<std::pair<int, Keys>>* sliced) const {
  sliced->reserve(ranges_.size());
  ForEachSlice(keys, [&](size_t i, size_t b, size_t e) {
    sliced->push_back({(int)server_thread_ids_[i], keys.segment(b, e)});
  });
}

void RangePartitionManager::Slice(const KVPairs& kvs, std::vector<std::pair<int, KVPairs>>* sliced) const {
  sliced->reserve(ranges_.size());
  size_t ratio = kvs.first.empty() ? 1 : kvs.second.size() / kvs.first.size();
  ForEachSlice(kvs.first, [&](size_t i, size_t b, size_t e) {
    KVPairs kv;
    kv.first = kvs.first.segment(b, e);
    kv.second = kvs.second.segment(b * ratio, e * ratio);
    sliced->push_back({(int)server_thread_ids_[i], std::move(kv)});
  });
}

void RangePartitionManager::SliceBytes(const Keys& keys, const SArray<char>& vals,
                                       std::vector<std::tuple<int, Keys, SArray<char>>>* sliced) const {
  sliced->reserve(ranges_.size());
  size_t ratio = keys.empty() ? 0 : vals.size() / keys.size();
  MINIPS_CHECK(keys.empty() || vals.size() % keys.size() == 0, "values not a multiple of keys");
  ForEachSlice(keys, [&](size_t i, size_t b, size_t e) {
    sliced->emplace_back((int)server_thread_ids_[i], keys.segment(b, e),
                         vals.empty() ? SArray<char>() : vals.segment(b * ratio, e * ratio));
  });
}

void RangePartitionManager::Update(const std::vector<Range>& ranges, const std::vector<uint32_t>& server_thread_ids) {
  MINIPS_CHECK(ranges.size() == server_thread_ids.size(), "ranges/servers mismatch");
  ranges_ = ranges;
  server_thread_ids_ = server_thread_ids;
}

std::vector<Range> EvenRanges(uint64_t num_dims, uint32_t parts) {
  MINIPS_CHECK(parts > 0, "need >= 1 part");
  // Same split as the reference getRanges(): equal floor-sized ranges, the last one takes
  // the remainder (keeps checkpoint local indices compatible).
  std::vector<Range> r;
  uint64_t step = num_dims / parts;
  for (uint32_t i = 0; i + 1 < parts; ++i) r.emplace_back(step * i, step * (i + 1));
  r.emplace_back(step * (parts - 1), num_dims);
  return r;
}

}  // namespace minips
