// Shared helpers of the native example apps (LR, K-Means, basic): flag parsing through the
// typed Context registry, hostfile/master setup, synthetic libsvm-like data.
#pragma once

#include <cmath>
#include <cstdio>
#include <fstream>
#include <random>
#include <set>

#include "../runtime/checkpoint.h"
#include "../runtime/config.h"
#include "../runtime/engine.h"

namespace minips_app {

using minips::Context;
using minips::Master;
using minips::ModelType;
using minips::Node;
using minips::ParseFile;
using minips::StorageType;
using minips::SVMItem;


inline void DefineCommonFlags() {
  auto& c = Context::Get();
  c.Define("input", Context::Type::kString, "", "libsvm input (local path); empty = synthetic");
  c.Define("kModelType", Context::Type::kString, "SSP", "ASP/SSP/BSP");
  c.Define("kStorageType", Context::Type::kString, "Vector", "Map/Vector");
  c.Define("batch_size", Context::Type::kInt, "100", "samples per iteration per worker");
  c.Define("num_iters", Context::Type::kInt, "1000", "iterations");
  c.Define("kStaleness", Context::Type::kInt, "1", "SSP staleness");
  c.Define("kSpeculation", Context::Type::kInt, "5", "extra pre-sampled batches");
  c.Define("num_local_load_thread", Context::Type::kInt, "4", "parser threads");
  c.Define("with_injected_straggler", Context::Type::kBool, "false", "5% chance of a U(0,100) ms sleep");
  c.Define("alpha", Context::Type::kDouble, "0.1", "learning rate");
  c.Define("init_dump", Context::Type::kBool, "false", "dump the loaded data for recovery");
  c.Define("report_prefix", Context::Type::kString, "", "append `iter\\tms` lines here");
  c.Define("report_interval", Context::Type::kInt, "0", "report every N iterations");
  c.Define("synthetic_rows", Context::Type::kInt, "2000", "synthetic samples per node");
  c.Define("synthetic_nnz", Context::Type::kInt, "20", "synthetic non-zeros per sample");
}

inline ModelType ParseModelType(const std::string& s) {
  if (s == "BSP") return ModelType::BSP;
  if (s == "ASP") return ModelType::ASP;
  return ModelType::SSP;
}
inline StorageType ParseStorageType(const std::string& s) { return s == "Map" ? StorageType::Map
                                                           : StorageType::Vector; }

// Webspam-shaped synthetic samples with a sparse linear teacher (labels +1/-1).
inline std::vector<SVMItem> SyntheticData(int rows, int64_t dims, int nnz, uint64_t seed) {
  std::mt19937_64 rng(seed);
  std::vector<double> teacher(std::min<int64_t>(dims, 1 << 20));
  std::normal_distribution<double> nd;
  for (auto& t : teacher) t = nd(rng);
  std::uniform_int_distribution<int64_t> fid(0, dims - 1);
  std::uniform_real_distribution<double> val(0.0, 1.0);
  std::vector<SVMItem> data(rows);
  for (auto& it : data) {
    std::set<int64_t> ids;
    while ((int)ids.size() < nnz) ids.insert(fid(rng));
    double z = 0;
    for (auto id : ids) {
      double v = val(rng);
      it.x.emplace_back(id, v);
      z += v * teacher[id % teacher.size()];
    }
    it.y = z > 0 ? 1 : -1;
  }
  return data;
}

// Parses the hostfile, selects the master (node 1 when heartbeat_interval > 0).
inline bool SetupNodes(Node* my_node, std::vector<Node>* nodes, Node* master) {
  auto& c = Context::Get();
  *nodes = ParseFile(c.get_string("config_file"));
  MINIPS_CHECK(CheckValidNodeIds(*nodes), "invalid node ids");
  *master = SelectMaster(*nodes, c.get_int32("heartbeat_interval"));
  int my_id = c.get_int32("my_id");
  if (master->is_master && (int)master->id == my_id) {
    *my_node = *master;
    return true;  // this process is the master
  }
  *my_node = GetNodeById(*nodes, (uint32_t)my_id);
  return false;
}

inline int RunMasterIfNeeded(const Node& master, const std::vector<Node>& nodes) {
  Master m(master, nodes);
  m.WaitAllQuit();
  m.StopMaster();
  MINIPS_LOG(0, "[Master] exiting");
  return 0;
}

inline void Report(const std::string& path, int iter, long long ms, double extra = NAN) {
  if (path.empty()) return;
  std::ofstream out(path, std::ios::app);
  out << iter << "\t";
  if (!std::isnan(extra)) out << extra << "\t";
  out << ms << "\n";
}

}  // namespace minips_app
