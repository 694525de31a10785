// Per-process orchestrator (Engine), user task (MLTask / Info) and the failure-detecting
// master.
//
// Parity:
//   Engine         -> driver/engine.{hpp,cpp}: StartEverything (id mapper -> mailbox ->
//                     sender -> server threads -> worker helper -> heartbeat), CreateTable,
//                     InitTable (kResetWorkerInModel), Run(MLTask), Barrier, ForceQuit,
//                     StopEverything, getRanges, rollback helpers, dump callback.
//   MLTask / Info  -> driver/ml_task.hpp, driver/info.hpp
//   Master         -> master/master.hpp; MasterThread -> master/master_thread.{hpp,cpp};
//                     HeartBeatCheckThread -> master/heartbeat_check_thread.{hpp,cpp}
// The master signals completion through WaitAllQuit() instead of calling exit(0).
#pragma once

#include <map>
#include <memory>

#include "comm.h"
#include "config.h"
#include "ids.h"
#include "server.h"
#include "worker.h"

namespace minips {

enum class ModelType { SSP = 0, BSP = 1, ASP = 2 };
enum class StorageType { Map = 0, Vector = 1 };

struct Info {
  uint32_t thread_id = 0;
  uint32_t worker_id = 0;
  uint32_t node_id = 0;
  ThreadsafeQueue<Message>* send_queue = nullptr;
  std::map<uint32_t, AbstractPartitionManager*> partition_manager_map;
  AbstractCallbackRunner* callback_runner = nullptr;

  template <typename Val>
  std::unique_ptr<KVClientTable<Val>> CreateKVClientTable(uint32_t table_id) const {
    auto it = partition_manager_map.find(table_id);
    MINIPS_CHECK(it != partition_manager_map.end(), "table " << table_id << " not found");
    return std::unique_ptr<KVClientTable<Val>>(
        new KVClientTable<Val>(thread_id, table_id, send_queue, it->second, callback_runner));
  }
};

class MLTask {
 public:
  void SetLambda(const std::function<void(const Info&)>& f) { func_ = f; }
  void RunLambda(const Info& info) const { func_(info); }
  void SetWorkerAlloc(const std::vector<WorkerAlloc>& a) { worker_alloc_ = a; }
  const std::vector<WorkerAlloc>& GetWorkerAlloc() const { return worker_alloc_; }
  void SetTables(const std::vector<uint32_t>& t) { tables_ = t; }
  const std::vector<uint32_t>& GetTables() const { return tables_; }
  bool IsSetup() const { return func_ && !worker_alloc_.empty() && !tables_.empty(); }

 private:
  std::function<void(const Info&)> func_;
  std::vector<WorkerAlloc> worker_alloc_;
  std::vector<uint32_t> tables_;
};

class Engine : public MailboxHooks {
 public:
  // `master` with is_master=false means "no master". `scale_node` with port<=0 = none.
  Engine(const Node& node, const std::vector<Node>& nodes, const Node& master = Node(),
         const Node& scale_node = Node());
  ~Engine() override;

  void StartEverything(int num_server_threads_per_node = 1);
  void CreateIdMapper(int num_server_threads_per_node = 1);
  void CreateMailbox();
  void StartMailbox();
  void StartSender();
  void StartServerThreads();
  void StartWorkerThreads();
  void StartHeartbeatThread();
  void StopEverything();
  void StopHeartbeatThread();
  void StopMailbox(bool barrier = true);
  void StopSender();
  void StopServerThreads();
  void StopWorkerThreads();

  void Barrier();
  void ForceQuit();
  void Run(const MLTask& task);
  void InitTable(uint32_t table_id, const std::vector<uint32_t>& worker_ids);

  template <typename Val>
  uint32_t CreateTable(std::unique_ptr<AbstractPartitionManager>&& pm, ModelType model_type,
                       StorageType storage_type, int staleness = 0);
  template <typename Val>
  uint32_t CreateTable(const std::vector<Range>& ranges, ModelType model_type, StorageType storage_type,
                       int staleness = 0) {
    auto servers = id_mapper_->GetAllServerThreads();
    std::unique_ptr<AbstractPartitionManager> pm(
        new RangePartitionManager(servers, ranges, master_.is_master ? (int)master_.id : -1));
    return CreateTable<Val>(std::move(pm), model_type, storage_type, staleness);
  }

  std::vector<Range> getRanges();
  void SendHeartBeat(bool quit = false);
  void SendScale();
  // Broadcast a rollback for `failed_node_id` (used by the master).
  void RollBack(int failed_node_id);
  void ScaleRollBack(int scale_node_id);
  void RollBackServer();
  void RollBackWorker();
  void SetNeedRollBack(bool need);
  bool IsNeedRollBack();
  void IncRollBackCount();
  void RecoverEnd();
  void WaitRecover();
  void SetDumpCallback(const std::function<void()>& f) { dump_callback_ = f; }
  void RunDumpCallback() {
    if (dump_callback_) dump_callback_();
  }
  void SetRestarter(const std::function<void()>& f) { restarter_ = f; }
  void SetScaleNode(const Node& n);
  // Elastic shrink (reference's UpdateAndRestart): drop `failed_node_id`, re-range tables.
  void UpdateAndRestart(int failed_node_id);

  // MailboxHooks
  void OnForceQuit(uint32_t node_id) override;
  void OnRollBack(int failed_node_id) override;
  void OnCheckpoint() override { RunDumpCallback(); }
  void OnScaleRollBack(const Node& scale_node) override;

  const Node& GetNode() const { return node_; }
  std::vector<Node> GetNodes();
  Mailbox* GetMailbox() { return mailbox_.get(); }
  ThreadsafeQueue<Message>* GetSendQueue() { return sender_ ? sender_->GetMessageQueue() : nullptr; }
  SimpleIdMapper* GetIdMapper() { return id_mapper_.get(); }
  AbstractPartitionManager* GetPartitionManager(uint32_t table);
  ServerThread* GetServerThread(size_t i) { return server_thread_group_.at(i).get(); }
  size_t NumServerThreads() const { return server_thread_group_.size(); }
  WorkerThread* GetWorkerThread() { return worker_thread_.get(); }
  uint32_t NumTables() const { return model_count_; }
  int RollBackCount() const { return rollback_counter_.load(); }

 private:
  void RegisterPartitionManager(uint32_t table_id, std::unique_ptr<AbstractPartitionManager>&& pm);
  std::vector<uint32_t> AllocateWorkers(const std::vector<WorkerAlloc>& alloc, WorkerSpec* spec);

  Node node_;
  std::vector<Node> nodes_;
  Node master_;
  Node scale_node_;
  bool has_scale_node_ = false;
  int num_server_threads_per_node_ = 1;

  std::unique_ptr<SimpleIdMapper> id_mapper_;
  std::unique_ptr<Mailbox> mailbox_;
  std::unique_ptr<Sender> sender_;
  std::vector<std::unique_ptr<ServerThread>> server_thread_group_;
  std::unique_ptr<WorkerThread> worker_thread_;
  std::map<uint32_t, std::unique_ptr<AbstractPartitionManager>> partition_manager_map_;
  std::vector<int> table_value_size_;
  uint32_t model_count_ = 0;

  std::thread heartbeat_thread_;
  std::atomic<bool> heartbeat_running_{false};
  std::mutex hb_mu_;
  std::condition_variable hb_cond_;

  std::function<void()> dump_callback_;
  std::function<void()> restarter_;
  std::atomic<int> rollback_counter_{1 << 30};
  std::mutex mu_;
  std::condition_variable recover_cond_;
  bool recover_end_ = false;
  std::mutex nodes_mu_;
};

// ---------------------------------------------------------------------------------------
// Master (failure detector). Runs on the node whose id is 1 (base/node_utils.cpp:19-32).
// ---------------------------------------------------------------------------------------
class Master;

class MasterThread : public Actor {
 public:
  MasterThread(uint32_t id, Master* master, const std::vector<Node>& nodes);
  void Init();
  int64_t LastHeartbeatMs(uint32_t node_id);
  std::map<uint32_t, int64_t> Heartbeats();
  void SetRecoveringNodeId(int id);
  int GetRecoveringNodeId();
  bool AllQuit();
  void WaitAllQuit();

 protected:
  void Main() override;

 private:
  Master* master_;
  std::vector<Node> nodes_;
  std::mutex mu_;
  std::condition_variable quit_cond_;
  std::map<uint32_t, int64_t> heartbeats_;
  std::set<uint32_t> quit_nodes_;
  int recovering_node_id_ = -1;
};

class HeartBeatCheckThread {
 public:
  HeartBeatCheckThread(MasterThread* mt, const std::vector<Node>& nodes, int interval_s, std::string relaunch_cmd);
  void Start();
  void Stop();
  std::vector<int> Detected();

 private:
  void Main();
  MasterThread* mt_;
  std::vector<Node> nodes_;
  int interval_s_;
  std::string relaunch_cmd_;
  std::atomic<bool> running_{false};
  std::thread thread_;
  std::mutex mu_;
  std::condition_variable cond_;
  std::vector<int> detected_;
};

class Master {
 public:
  Master(const Node& master_node, const std::vector<Node>& nodes);
  ~Master();
  void RollBack(int failed_node_id);
  void ScaleRollBack(int scale_node_id);
  // Blocks until every node sent kQuitHeartBeat (or timeout_s elapses; <=0 = forever).
  bool WaitAllQuit(double timeout_s = 0);
  void StopMaster();
  MasterThread* GetMasterThread() { return master_thread_.get(); }
  HeartBeatCheckThread* GetCheckThread() { return check_thread_.get(); }
  int RollBackCount() const { return rollbacks_.load(); }

 private:
  Node master_node_;
  std::vector<Node> nodes_;
  std::unique_ptr<Engine> engine_;
  std::unique_ptr<MasterThread> master_thread_;
  std::unique_ptr<HeartBeatCheckThread> check_thread_;
  std::atomic<int> rollbacks_{0};
  bool stopped_ = false;
};

// ---------------------------------------------------------------------------------------
template <typename Val>
uint32_t Engine::CreateTable(std::unique_ptr<AbstractPartitionManager>&& pm, ModelType model_type,
                             StorageType storage_type, int staleness) {
  uint32_t table_id = model_count_++;
  auto* rpm = dynamic_cast<RangePartitionManager*>(pm.get());
  const auto& server_ids = pm->GetServerThreadIds();
  auto local_servers = id_mapper_->GetServerThreadsForId(node_.id);
  bool use_weight_file = Context::Get().get_bool("use_weight_file");
  for (size_t li = 0; li < local_servers.size(); ++li) {
    uint32_t tid = local_servers[li];
    std::unique_ptr<AbstractStorage> storage;
    if (storage_type == StorageType::Map) {
      storage.reset(new MapStorage<Val>());
    } else {
      MINIPS_CHECK(rpm, "Vector storage needs a RangePartitionManager");
      auto pos = std::find(server_ids.begin(), server_ids.end(), tid) - server_ids.begin();
      MINIPS_CHECK(pos < (long)server_ids.size(), "server " << tid << " missing from partition manager");
      storage.reset(new VectorStorage<Val>(rpm->GetRanges()[pos]));
    }
    CheckpointConfig ckpt = CheckpointConfig::FromContext((int)li, (int)table_id);
    ThreadsafeQueue<Message>* reply = sender_->GetMessageQueue();
    std::unique_ptr<AbstractModel> model;
    switch (model_type) {
      case ModelType::SSP:
        model.reset(new SSPModel(table_id, std::move(storage), staleness, reply, ckpt, use_weight_file));
        break;
      case ModelType::BSP:
        model.reset(new BSPModel(table_id, std::move(storage), reply, ckpt));
        break;
      case ModelType::ASP:
        model.reset(new ASPModel(table_id, std::move(storage), reply, ckpt));
        break;
    }
    server_thread_group_.at(li)->RegisterModel(table_id, std::move(model));
  }
  RegisterPartitionManager(table_id, std::move(pm));
  table_value_size_.push_back((int)sizeof(Val));
  return table_id;
}

}  // namespace minips
