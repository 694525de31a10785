#include "engine.h"

#include <cstdlib>

#include "checkpoint.h"

namespace minips {

namespace {
int64_t NowMs() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
// heartbeat period: heartbeat_interval seconds, overridable in ms for tests.
int64_t HeartbeatPeriodMs() {
  auto& ctx = Context::Get();
  if (ctx.Has("heartbeat_interval_ms") && ctx.get_int64("heartbeat_interval_ms") > 0)
    return ctx.get_int64("heartbeat_interval_ms");
  return (int64_t)ctx.get_int32("heartbeat_interval") * 1000;
}
}  // namespace

Engine::Engine(const Node& node, const std::vector<Node>& nodes, const Node& master, const Node& scale_node)
    : node_(node), nodes_(nodes), master_(master), scale_node_(scale_node) {
  has_scale_node_ = scale_node_.port > 0;
  Context::Get().Define("heartbeat_interval_ms", Context::Type::kInt, "0", "test override of heartbeat period");
}

Engine::~Engine() {
  if (heartbeat_running_) StopHeartbeatThread();
}

void Engine::StartEverything(int num_server_threads_per_node) {
  CreateIdMapper(num_server_threads_per_node);
  CreateMailbox();
  StartMailbox();
  StartSender();
  StartServerThreads();
  StartWorkerThreads();
  StartHeartbeatThread();
  MINIPS_VLOG(1, "engine " << node_.id << " started");
}

void Engine::CreateIdMapper(int num_server_threads_per_node) {
  num_server_threads_per_node_ = num_server_threads_per_node;
  id_mapper_.reset(new SimpleIdMapper(node_, nodes_));
  int skip = Context::Get().get_bool("scale") ? Context::Get().get_int32("scale_node_id") : -1;
  id_mapper_->Init(num_server_threads_per_node, skip);
}

void Engine::CreateMailbox() { mailbox_.reset(new Mailbox(node_, nodes_, id_mapper_.get(), this)); }

void Engine::StartMailbox() {
  MINIPS_CHECK(mailbox_, "mailbox not created");
  mailbox_->Start(master_.is_master ? &master_ : nullptr, has_scale_node_ ? &scale_node_ : nullptr);
}

void Engine::StartSender() {
  sender_.reset(new Sender(mailbox_.get()));
  sender_->Start();
}

void Engine::StartServerThreads() {
  for (uint32_t tid : id_mapper_->GetServerThreadsForId(node_.id)) {
    std::unique_ptr<ServerThread> st(new ServerThread(tid));
    mailbox_->RegisterQueue(tid, st->GetWorkQueue());
    st->Start();
    server_thread_group_.push_back(std::move(st));
  }
  MINIPS_VLOG(1, "server threads started on node " << node_.id);
}

void Engine::StartWorkerThreads() {
  auto helpers = id_mapper_->GetWorkerHelperThreadsForId(node_.id);
  MINIPS_CHECK(helpers.size() == 1, "expected one worker helper on node " << node_.id);
  worker_thread_.reset(new WorkerThread(helpers[0]));
  double t = Context::Get().get_double("barrier_timeout_s");
  worker_thread_->SetTimeout(t);
  mailbox_->RegisterQueue(helpers[0], worker_thread_->GetWorkQueue());
  worker_thread_->Start();
}

void Engine::StartHeartbeatThread() {
  if (!master_.is_master) return;
  int64_t period = HeartbeatPeriodMs();
  if (period <= 0) return;
  heartbeat_running_ = true;
  heartbeat_thread_ = std::thread([this, period] {
    if (Context::Get().get_bool("scale")) SendScale();
    SendHeartBeat(false);  // announce immediately (recovering nodes trigger rollback on it)
    while (heartbeat_running_) {
      std::unique_lock<std::mutex> lk(hb_mu_);
      CondWaitFor(hb_cond_, lk, period / 1000.0, [this] { return !heartbeat_running_; });
      if (!heartbeat_running_) break;
      lk.unlock();
      SendHeartBeat(false);
    }
    SendHeartBeat(true);
  });
}

void Engine::StopHeartbeatThread() {
  if (!heartbeat_running_) return;
  {
    std::lock_guard<std::mutex> lk(hb_mu_);
    heartbeat_running_ = false;
  }
  hb_cond_.notify_all();
  if (heartbeat_thread_.joinable()) heartbeat_thread_.join();
}

void Engine::SendHeartBeat(bool quit) {
  if (!master_.is_master || !mailbox_) return;
  Message m;
  m.meta.sender = (int32_t)node_.id;
  m.meta.recver = (int32_t)master_.id;
  m.meta.flag = quit ? Flag::kQuitHeartBeat : Flag::kHeartBeat;
  mailbox_->Send(m);
}

void Engine::SendScale() {
  if (!master_.is_master) return;
  Message m;
  m.meta.sender = (int32_t)node_.id;
  m.meta.recver = (int32_t)master_.id;
  m.meta.flag = Flag::kScale;
  mailbox_->Send(m);
}

void Engine::RollBack(int failed_node_id) {
  for (auto& n : GetNodes()) {
    Message m;
    m.meta.sender = failed_node_id;
    m.meta.recver = (int32_t)n.id;
    m.meta.failed_node_id = failed_node_id;
    m.meta.flag = Flag::kRollBack;
    mailbox_->Send(m);
  }
}

void Engine::ScaleRollBack(int scale_node_id) {
  for (auto& n : GetNodes()) {
    Message m;
    m.meta.sender = scale_node_id;
    m.meta.recver = (int32_t)n.id;
    m.meta.flag = Flag::kScaleRollback;
    mailbox_->Send(m);
  }
}

void Engine::StopEverything() {
  StopHeartbeatThread();
  if (sender_) sender_->Flush();
  StopMailbox(true);
  StopSender();
  StopServerThreads();
  StopWorkerThreads();
  MINIPS_VLOG(1, "engine " << node_.id << " stopped");
}

void Engine::StopMailbox(bool barrier) {
  MINIPS_CHECK(mailbox_, "no mailbox");
  mailbox_->Stop(barrier);
}
void Engine::StopSender() {
  if (sender_) sender_->Stop();
}
void Engine::StopServerThreads() {
  for (auto& s : server_thread_group_) s->Stop();
}
void Engine::StopWorkerThreads() {
  if (worker_thread_) worker_thread_->Stop();
}

void Engine::Barrier() { mailbox_->Barrier(); }
void Engine::ForceQuit() { mailbox_->ForceQuit(node_.id); }

std::vector<Node> Engine::GetNodes() {
  std::lock_guard<std::mutex> lk(nodes_mu_);
  return nodes_;
}

void Engine::RegisterPartitionManager(uint32_t table_id, std::unique_ptr<AbstractPartitionManager>&& pm) {
  partition_manager_map_[table_id] = std::move(pm);
}

AbstractPartitionManager* Engine::GetPartitionManager(uint32_t table) {
  auto it = partition_manager_map_.find(table);
  return it == partition_manager_map_.end() ? nullptr : it->second.get();
}

std::vector<Range> Engine::getRanges() {
  auto& ctx = Context::Get();
  uint32_t spn = (uint32_t)ctx.get_int32("num_servers_per_node");
  uint64_t dims = (uint64_t)ctx.get_int64("num_dims");
  uint32_t total = (uint32_t)GetNodes().size() * spn;
  if (ctx.get_bool("scale")) total -= spn;
  return EvenRanges(dims, total);
}

std::vector<uint32_t> Engine::AllocateWorkers(const std::vector<WorkerAlloc>& alloc, WorkerSpec* spec) {
  *spec = WorkerSpec(alloc);
  std::vector<uint32_t> allocated;
  for (auto& kv : spec->GetNodeToWorkers()) {
    for (uint32_t w : kv.second) {
      uint32_t tid = id_mapper_->AllocateWorkerThread(kv.first);
      spec->InsertWorkerIdThreadId(w, tid);
      allocated.push_back(tid);
    }
  }
  return allocated;
}

void Engine::InitTable(uint32_t table_id, const std::vector<uint32_t>& worker_ids) {
  auto local_servers = id_mapper_->GetServerThreadsForId(node_.id);
  int count = (int)local_servers.size();
  if (count == 0) return;
  uint32_t id = id_mapper_->AllocateWorkerThread(node_.id);
  ThreadsafeQueue<Message> queue;
  mailbox_->RegisterQueue(id, &queue);
  Message reset;
  reset.meta.flag = Flag::kResetWorkerInModel;
  reset.meta.model_id = (int32_t)table_id;
  reset.meta.sender = (int32_t)id;
  reset.AddData(SArray<uint32_t>(worker_ids));
  for (uint32_t s : local_servers) {
    reset.meta.recver = (int32_t)s;
    sender_->GetMessageQueue()->Push(reset);
  }
  double timeout = Context::Get().get_double("barrier_timeout_s");
  while (count > 0) {
    Message reply;
    MINIPS_CHECK(queue.WaitAndPopFor(&reply, timeout), "InitTable timed out");
    MINIPS_CHECK(reply.meta.flag == Flag::kResetWorkerInModel, "unexpected reply " << FlagName(reply.meta.flag));
    MINIPS_CHECK(reply.meta.model_id == (int32_t)table_id, "reply for wrong table");
    --count;
  }
  mailbox_->DeregisterQueue(id);
  id_mapper_->DeallocateWorkerThread(node_.id, id);
}

void Engine::Run(const MLTask& task) {
  MINIPS_CHECK(task.IsSetup(), "task not set up");
  WorkerSpec spec;
  auto allocated = AllocateWorkers(task.GetWorkerAlloc(), &spec);
  const auto& tables = task.GetTables();
  for (auto t : tables) InitTable(t, spec.GetAllThreadIds());
  if (!Context::Get().get_bool("use_weight_file")) mailbox_->Barrier();
  std::vector<std::string> errors;
  std::mutex err_mu;
  if (spec.HasLocalWorkers(node_.id)) {
    const auto& threads = spec.GetLocalThreads(node_.id);
    const auto& workers = spec.GetLocalWorkers(node_.id);
    std::map<uint32_t, AbstractPartitionManager*> pm_map;
    for (auto t : tables) {
      auto* pm = GetPartitionManager(t);
      MINIPS_CHECK(pm, "table " << t << " not created");
      pm_map[t] = pm;
    }
    std::vector<std::thread> group;
    for (size_t i = 0; i < threads.size(); ++i) {
      mailbox_->RegisterQueue(threads[i], worker_thread_->GetWorkQueue());
      Info info;
      info.thread_id = threads[i];
      info.worker_id = workers[i];
      info.node_id = node_.id;
      info.send_queue = sender_->GetMessageQueue();
      info.partition_manager_map = pm_map;
      info.callback_runner = worker_thread_.get();
      group.emplace_back([&task, info, &errors, &err_mu] {
        try {
          task.RunLambda(info);
        } catch (const std::exception& e) {
          std::lock_guard<std::mutex> lk(err_mu);
          errors.push_back(e.what());
        }
      });
    }
    for (auto& t : group) t.join();
    for (auto tid : threads) mailbox_->DeregisterQueue(tid);
  }
  if (sender_) sender_->Flush();  // the workers' last Adds/Clocks leave before the barrier
  mailbox_->Barrier();
  for (auto& kv : spec.GetNodeToWorkers()) {
    (void)kv;
  }
  for (auto tid : allocated) id_mapper_->DeallocateWorkerThread(id_mapper_->GetNodeIdForThread(tid), tid);
  MINIPS_CHECK(errors.empty(), "worker task failed: " << errors[0]);
}

void Engine::RollBackServer() {
  for (auto& s : server_thread_group_) s->RollbackModel();
}
void Engine::RollBackWorker() { worker_thread_->RollBackWorker(); }

void Engine::SetNeedRollBack(bool need) {
  if (need) {
    std::lock_guard<std::mutex> lk(mu_);
    rollback_counter_ = 0;
    recover_end_ = false;
  }
}
bool Engine::IsNeedRollBack() { return rollback_counter_.load() < Context::Get().get_int32("num_workers_per_node"); }
void Engine::IncRollBackCount() { rollback_counter_ += 1; }
void Engine::RecoverEnd() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    recover_end_ = true;
  }
  recover_cond_.notify_all();
}
void Engine::WaitRecover() {
  std::unique_lock<std::mutex> lk(mu_);
  recover_cond_.wait(lk, [this] { return recover_end_; });
}

void Engine::SetScaleNode(const Node& n) {
  scale_node_ = n;
  has_scale_node_ = true;
  Context::Get().set("has_scale_node", true);
  Context::Get().set("scale_node_id", (int)n.id);
  if (mailbox_) mailbox_->SetScaleNode(n);
}

void Engine::OnForceQuit(uint32_t node_id) {
  std::lock_guard<std::mutex> lk(nodes_mu_);
  nodes_.erase(std::remove_if(nodes_.begin(), nodes_.end(), [&](const Node& n) { return n.id == node_id; }),
               nodes_.end());
}

// Survivor side of the recovery protocol (comm/mailbox.cpp:172-191).
void Engine::OnRollBack(int failed_node_id) {
  if (failed_node_id == (int)node_.id) return;  // the relaunched node restores on its own
  auto& ctx = Context::Get();
  CheckpointConfig c = CheckpointConfig::FromContext(0, 0);
  try {
    ctx.SetIterationMap(LoadConfigData(c.WorkerConfigFile()));
  } catch (const std::exception& e) {
    MINIPS_LOG(1, "rollback: no worker config: " << e.what());
  }
  SetNeedRollBack(true);
  RollBackServer();
  RollBackWorker();
  CheckFaultTolerance(5, "node " + std::to_string(node_.id) + " rolled back for failed node " +
                             std::to_string(failed_node_id));
}

void Engine::OnScaleRollBack(const Node& n) {
  try {
    Node scale = LoadScaleFile(Context::Get().get_string("scale_file"));
    mailbox_->ConnectTo(scale);
    SetScaleNode(scale);
  } catch (const std::exception& e) {
    MINIPS_LOG(2, "scale rollback failed: " << e.what());
    return;
  }
  OnRollBack((int)n.id);
}

void Engine::UpdateAndRestart(int failed_node_id) {
  {
    std::lock_guard<std::mutex> lk(nodes_mu_);
    nodes_.erase(std::remove_if(nodes_.begin(), nodes_.end(),
                                [&](const Node& n) { return (int)n.id == failed_node_id; }),
                 nodes_.end());
  }
  auto nodes = GetNodes();
  auto ranges = getRanges();
  mailbox_->Update(nodes);
  id_mapper_->Update(nodes, num_server_threads_per_node_);
  auto local = id_mapper_->GetServerThreadsForId(node_.id);
  auto all = id_mapper_->GetAllServerThreads();
  for (size_t i = 0; i < server_thread_group_.size() && i < local.size(); ++i) {
    auto pos = std::find(all.begin(), all.end(), local[i]) - all.begin();
    server_thread_group_[i]->UpdateModel(failed_node_id, nodes, ranges.at(pos));
  }
  worker_thread_->Update((uint32_t)num_server_threads_per_node_);
  for (auto& kv : partition_manager_map_) kv.second->Update(ranges, all);
}

// ------------------------------------------------------------------------------ master
MasterThread::MasterThread(uint32_t id, Master* master, const std::vector<Node>& nodes)
    : Actor(id), master_(master), nodes_(nodes) {
  Init();
}

void MasterThread::Init() {
  std::lock_guard<std::mutex> lk(mu_);
  int64_t now = NowMs();
  for (auto& n : nodes_) heartbeats_[n.id] = now;
}

int64_t MasterThread::LastHeartbeatMs(uint32_t node_id) {
  std::lock_guard<std::mutex> lk(mu_);
  return heartbeats_[node_id];
}
std::map<uint32_t, int64_t> MasterThread::Heartbeats() {
  std::lock_guard<std::mutex> lk(mu_);
  return heartbeats_;
}
void MasterThread::SetRecoveringNodeId(int id) {
  std::lock_guard<std::mutex> lk(mu_);
  recovering_node_id_ = id;
}
int MasterThread::GetRecoveringNodeId() {
  std::lock_guard<std::mutex> lk(mu_);
  return recovering_node_id_;
}
bool MasterThread::AllQuit() {
  std::lock_guard<std::mutex> lk(mu_);
  return quit_nodes_.size() >= nodes_.size();
}
void MasterThread::WaitAllQuit() {
  std::unique_lock<std::mutex> lk(mu_);
  quit_cond_.wait(lk, [this] { return quit_nodes_.size() >= nodes_.size(); });
}

void MasterThread::Main() {
  while (true) {
    Message msg;
    work_queue_.WaitAndPop(&msg);
    if (msg.meta.flag == Flag::kExit) break;
    if (msg.meta.flag == Flag::kQuitHeartBeat) {
      std::lock_guard<std::mutex> lk(mu_);
      quit_nodes_.insert((uint32_t)msg.meta.sender);
      if (quit_nodes_.size() >= nodes_.size()) {
        MINIPS_LOG(0, "[Master] all nodes quit");
        quit_cond_.notify_all();
      }
    } else if (msg.meta.flag == Flag::kHeartBeat) {
      bool rollback = false;
      {
        std::lock_guard<std::mutex> lk(mu_);
        heartbeats_[(uint32_t)msg.meta.sender] = NowMs();
        if (msg.meta.sender == recovering_node_id_) {
          recovering_node_id_ = -1;
          rollback = true;
        }
      }
      if (rollback) {
        MINIPS_LOG(0, "[Master] node " << msg.meta.sender << " is back, broadcasting rollback");
        master_->RollBack(msg.meta.sender);
      }
      MINIPS_VLOG(1, "[Master] heartbeat from node " << msg.meta.sender);
    } else if (msg.meta.flag == Flag::kScale) {
      master_->ScaleRollBack(msg.meta.sender);
    }
  }
}

HeartBeatCheckThread::HeartBeatCheckThread(MasterThread* mt, const std::vector<Node>& nodes, int interval_s,
                                           std::string relaunch_cmd)
    : mt_(mt), nodes_(nodes), interval_s_(interval_s), relaunch_cmd_(std::move(relaunch_cmd)) {}

void HeartBeatCheckThread::Start() {
  running_ = true;
  thread_ = std::thread([this] { Main(); });
}

void HeartBeatCheckThread::Stop() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    running_ = false;
  }
  cond_.notify_all();
  if (thread_.joinable()) thread_.join();
}

std::vector<int> HeartBeatCheckThread::Detected() {
  std::lock_guard<std::mutex> lk(mu_);
  return detected_;
}

// A node silent for more than 3 periods is declared failed: log Phase 2, run
// `relaunch_cmd <id>`, and mark it recovering (one recovery at a time).
void HeartBeatCheckThread::Main() {
  int64_t period = HeartbeatPeriodMs();
  if (period <= 0) period = (int64_t)interval_s_ * 1000;
  if (period <= 0) return;
  while (true) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      CondWaitFor(cond_, lk, period / 1000.0, [this] { return !running_; });
      if (!running_) return;
    }
    if (mt_->AllQuit()) return;
    if (mt_->GetRecoveringNodeId() >= 0) continue;
    auto hb = mt_->Heartbeats();
    int64_t now = NowMs();
    for (auto& n : nodes_) {
      if (now - hb[n.id] > 3 * period) {
        CheckFaultTolerance(2, "node " + std::to_string(n.id) + " missed heartbeats");
        {
          std::lock_guard<std::mutex> lk(mu_);
          detected_.push_back((int)n.id);
        }
        if (!relaunch_cmd_.empty()) {
          std::string cmd = relaunch_cmd_ + std::to_string(n.id);
          int rc = std::system(cmd.c_str());
          CheckFaultTolerance(3, "relaunch '" + cmd + "' rc=" + std::to_string(rc));
        }
        mt_->SetRecoveringNodeId((int)n.id);
        break;
      }
    }
  }
}

Master::Master(const Node& master_node, const std::vector<Node>& nodes) : master_node_(master_node), nodes_(nodes) {
  // The master runs only a mailbox + sender (no servers/workers) (master/master.hpp:22-27).
  engine_.reset(new Engine(master_node_, nodes_));
  engine_->CreateIdMapper(1);
  engine_->CreateMailbox();
  engine_->StartMailbox();
  engine_->StartSender();
  master_thread_.reset(new MasterThread(master_node_.id, this, nodes_));
  engine_->GetMailbox()->RegisterQueue(master_node_.id, master_thread_->GetWorkQueue());
  master_thread_->Start();
  auto& ctx = Context::Get();
  check_thread_.reset(new HeartBeatCheckThread(master_thread_.get(), nodes_, ctx.get_int32("heartbeat_interval"),
                                               ctx.get_string("relaunch_cmd")));
  check_thread_->Start();
}

Master::~Master() { StopMaster(); }

void Master::RollBack(int failed_node_id) {
  rollbacks_ += 1;
  engine_->RollBack(failed_node_id);
}

void Master::ScaleRollBack(int scale_node_id) { engine_->ScaleRollBack(scale_node_id); }

bool Master::WaitAllQuit(double timeout_s) {
  auto* mt = master_thread_.get();
  auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  while (!mt->AllQuit()) {
    if (timeout_s > 0 && std::chrono::steady_clock::now() > deadline) return false;
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  return true;
}

void Master::StopMaster() {
  if (stopped_) return;
  stopped_ = true;
  check_thread_->Stop();
  engine_->StopMailbox(false);
  engine_->StopSender();
  master_thread_->Stop();
}

}  // namespace minips
