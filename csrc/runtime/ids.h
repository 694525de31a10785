// Thread-id arithmetic, worker spec, ML task and range partitioning.
//
// Parity:
//   SimpleIdMapper        -> driver/simple_id_mapper.{hpp,cpp} (same id layout:
//                            node*1000 + [0,n) servers, node*1000+50 worker helper,
//                            node*1000 + [100,1000) user worker threads)
//   WorkerSpec            -> driver/worker_spec.{hpp,cpp}
//   WorkerAlloc / MLTask  -> driver/ml_task.hpp:12-66
//   Abstract/RangePartitionManager -> base/abstract_partition_manager.hpp,
//                            base/range_partition_manager.hpp:24-66
#pragma once

#include <functional>
#include <map>
#include <set>
#include <vector>

#include "base.h"
#include "node.h"

namespace minips {

class AbstractIdMapper {
 public:
  virtual ~AbstractIdMapper() = default;
  virtual uint32_t GetNodeIdForThread(uint32_t tid) = 0;
};

class SimpleIdMapper : public AbstractIdMapper {
 public:
  static constexpr uint32_t kMaxNodeId = 1000;
  static constexpr uint32_t kMaxThreadsPerNode = 1000;
  static constexpr uint32_t kMaxBgThreadsPerNode = 100;
  static constexpr uint32_t kWorkerHelperThreadId = 50;

  SimpleIdMapper(Node node, const std::vector<Node>& nodes) : node_(node), nodes_(nodes) {}
  uint32_t GetNodeIdForThread(uint32_t tid) override { return tid / kMaxThreadsPerNode; }
  // `skip_node_id` >= 0 excludes that node from server creation (the scale-out node).
  void Init(int num_server_threads_per_node, int skip_node_id = -1);
  void Update(const std::vector<Node>& nodes, int num_server_threads_per_node, int skip_node_id = -1);
  uint32_t AllocateWorkerThread(uint32_t node_id);
  void DeallocateWorkerThread(uint32_t node_id, uint32_t tid);
  std::vector<uint32_t> GetServerThreadsForId(uint32_t node_id);
  std::vector<uint32_t> GetWorkerHelperThreadsForId(uint32_t node_id);
  std::vector<uint32_t> GetWorkerThreadsForId(uint32_t node_id);
  std::vector<uint32_t> GetAllServerThreads();

 private:
  std::mutex mu_;
  Node node_;
  std::vector<Node> nodes_;
  std::map<uint32_t, std::vector<uint32_t>> node2server_;
  std::map<uint32_t, std::vector<uint32_t>> node2worker_helper_;
  std::map<uint32_t, std::set<uint32_t>> node2worker_;
};

struct WorkerAlloc {
  uint32_t node_id;
  uint32_t num_workers;
};

class WorkerSpec {
 public:
  WorkerSpec() = default;
  explicit WorkerSpec(const std::vector<WorkerAlloc>& worker_alloc) { Init(worker_alloc); }
  bool HasLocalWorkers(uint32_t node_id) const;
  const std::vector<uint32_t>& GetLocalWorkers(uint32_t node_id) const;
  const std::vector<uint32_t>& GetLocalThreads(uint32_t node_id) const;
  std::map<uint32_t, std::vector<uint32_t>> GetNodeToWorkers() const { return node_to_workers_; }
  std::vector<uint32_t> GetAllThreadIds() const;
  void InsertWorkerIdThreadId(uint32_t worker_id, uint32_t thread_id);
  uint32_t GetNumWorkers() const { return num_workers_; }
  uint32_t GetThreadId(uint32_t worker_id) const { return worker_to_thread_.at(worker_id); }
  uint32_t GetWorkerId(uint32_t thread_id) const { return thread_to_worker_.at(thread_id); }

 private:
  void Init(const std::vector<WorkerAlloc>& worker_alloc);
  uint32_t num_workers_ = 0;
  std::map<uint32_t, std::vector<uint32_t>> node_to_workers_;
  std::map<uint32_t, std::vector<uint32_t>> node_to_threads_;
  std::map<uint32_t, uint32_t> worker_to_thread_;
  std::map<uint32_t, uint32_t> thread_to_worker_;
  std::map<uint32_t, uint32_t> worker_to_node_;
};

class AbstractPartitionManager {
 public:
  AbstractPartitionManager(const std::vector<uint32_t>& server_thread_ids, int master_node_id = -1)
      : server_thread_ids_(server_thread_ids), master_node_id_(master_node_id) {}
  virtual ~AbstractPartitionManager() = default;
  size_t GetNumServers() const { return server_thread_ids_.size(); }
  const std::vector<uint32_t>& GetServerThreadIds() const { return server_thread_ids_; }
  int GetMasterNodeId() const { return master_node_id_; }

  // Keys must be sorted ascending. Only non-empty slices are emitted.
  virtual void Slice(const Keys& keys, std::vector<std::pair<int, Keys>>* sliced) const = 0;
  virtual void Slice(const KVPairs& kvs, std::vector<std::pair<int, KVPairs>>* sliced) const = 0;
  // Generic byte-valued version (vals.size() must be a multiple of keys.size()).
  virtual void SliceBytes(const Keys& keys, const SArray<char>& vals,
                          std::vector<std::tuple<int, Keys, SArray<char>>>* sliced) const = 0;
  virtual void Update(const std::vector<Range>& ranges, const std::vector<uint32_t>& server_thread_ids) = 0;

 protected:
  std::vector<uint32_t> server_thread_ids_;
  int master_node_id_;
};

class RangePartitionManager : public AbstractPartitionManager {
 public:
  RangePartitionManager(const std::vector<uint32_t>& server_thread_ids, const std::vector<Range>& ranges,
                        int master_node_id = -1);
  const std::vector<Range>& GetRanges() const { return ranges_; }
  void Slice(const Keys& keys, std::vector<std::pair<int, Keys>>* sliced) const override;
  void Slice(const KVPairs& kvs, std::vector<std::pair<int, KVPairs>>* sliced) const override;
  void SliceBytes(const Keys& keys, const SArray<char>& vals,
                  std::vector<std::tuple<int, Keys, SArray<char>>>* sliced) const override;
  void Update(const std::vector<Range>& ranges, const std::vector<uint32_t>& server_thread_ids) override;

 private:
  template <typename F>
  void ForEachSlice(const Keys& keys, F&& f) const;
  std::vector<Range> ranges_;
};

// Evenly split [0, num_dims) into `parts` contiguous ranges (driver/engine.hpp:158-172).
std::vector<Range> EvenRanges(uint64_t num_dims, uint32_t parts);

}  // namespace minips
