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
  c.Define("input", Context::Type::kString, "", "libsvm input: path/dir/comma list, file://, webhdfs:// or hdfs:// "
           "URL (a bare path is read from HDFS when --hdfs_namenode is set); empty = synthetic");
  c.Define("hdfs_namenode", Context::Type::kString, "", "HDFS namenode host for bare --input paths");
  c.Define("hdfs_namenode_port", Context::Type::kInt, "9000", "namenode RPC port (libhdfs3)");
  c.Define("hdfs_http_port", Context::Type::kInt, "0", "namenode HTTP port: > 0 reads through WebHDFS");
  c.Define("assigner_master_port", Context::Type::kInt, "0",
           "> 0: node 0 serves locality-aware block assignment on this port (HDFSBlockAssigner); "
           "0: static byte-range shards");
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

// The app's libsvm input (lib/abstract_data_loader.hpp): static shards, or blocks handed out by
// the locality-aware assigner that node 0 serves on --assigner_master_port.
inline std::vector<SVMItem> LoadAppData(const std::vector<Node>& nodes, int my_index) {
  auto& c = Context::Get();
  std::string input = c.get_string("input");
  const std::string nn = c.get_string("hdfs_namenode");
  if (!nn.empty() && input.find("://") == std::string::npos) {
    const int http = c.get_int32("hdfs_http_port");
    input = (http > 0 ? "webhdfs://" + nn + ":" + std::to_string(http)
                      : "hdfs://" + nn + ":" + std::to_string(c.get_int32("hdfs_namenode_port"))) +
            (input.empty() || input[0] != '/' ? "/" : "") + input;
  }
  minips::LoadOptions opt;
  opt.rank = my_index;
  opt.num_ranks = (int)nodes.size();
  opt.num_threads = c.get_int32("num_local_load_thread");
  const int port = c.get_int32("assigner_master_port");
  std::unique_ptr<minips::BlockAssignerServer> server;
  if (port > 0) {
    if (my_index == 0) {
      server.reset(new minips::BlockAssignerServer(port));
      server->Start();
    }
    opt.assigner = nodes[0].hostname + ":" + std::to_string(port);
    opt.host = nodes[my_index].hostname;  // the hostfile names hosts as HDFS reports datanodes
  }
  auto data = minips::LoadLibsvmFile(input, opt, true);
  if (server) {  // serve until every loader thread of every node has exited (kExit)
    if (!server->WaitDone(600)) MINIPS_LOG(1, "block assigner: not every loader exited");
    MINIPS_LOG(0, "block assigner: " << server->LocalServed() << " local / " << server->RemoteServed()
                                     << " remote blocks");
    server->Stop();
  }
  return data;
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
