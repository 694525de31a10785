// Sparse logistic regression on the native PS runtime (BASELINE config 1: CPU, TCP control +
// data plane; e.g. 2 worker threads + 1 server thread per node).
//
// Behaviour follows the reference app (apps/logistic_regression/lr_example.cpp:97-431):
// libsvm (or synthetic webspam-shaped) data sharded by node; one double table of num_dims
// keys range-partitioned over all server threads; per worker: pre-sampled mini-batches
// (sorted unique keys), Get -> LR gradient -> Add -> Clock; worker 0 checkpoints every 100
// iterations (--checkpoint_toggle); rollback on kRollBack; straggler injection; final
// accuracy on the local data. The master (node id 1 when --heartbeat_interval > 0) detects
// failed nodes and relaunches them through --relaunch_cmd.
#include <atomic>
#include <chrono>
#include <set>

#include "app_common.h"

using namespace minips;
using namespace minips_app;

static double TestAccuracy(const std::vector<double>& w, const std::vector<SVMItem>& data) {
  if (data.empty()) return 0;
  int correct = 0;
  for (auto& it : data) {
    double z = 0;
    for (auto& f : it.x)
      if (f.first < (int64_t)w.size()) z += w[f.first] * f.second;
    double p = 1.0 / (1.0 + std::exp(-z));
    double y = it.y < 0 ? 0 : it.y;
    correct += ((p > 0.5) == (y > 0.5)) ? 1 : 0;
  }
  return (double)correct / data.size();
}

int main(int argc, char** argv) {
  DefineCommonFlags();
  auto& ctx = Context::Get();
  ctx.ParseArgs(argc, argv);
  Node me, master;
  std::vector<Node> nodes;
  if (SetupNodes(&me, &nodes, &master)) return RunMasterIfNeeded(master, nodes);

  const int64_t num_dims = ctx.get_int64("num_dims") > 0 ? ctx.get_int64("num_dims") : 100000;
  ctx.set("num_dims", (int64_t)num_dims);
  const int my_index = (int)(std::find(nodes.begin(), nodes.end(), me) - nodes.begin());
  const bool recovering = ctx.get_bool("use_weight_file");
  std::vector<SVMItem> data;
  CheckpointConfig ck = CheckpointConfig::FromContext(0, 0);
  if (recovering) {
    CheckFaultTolerance(3, "node " + std::to_string(me.id) + " restarting");
    data = LoadSVMData(ck.prefix + "worker_" + std::to_string(me.id));
  } else if (!ctx.get_string("input").empty()) {
    data = LoadAppData(nodes, my_index);
  } else {
    data = SyntheticData(ctx.get_int32("synthetic_rows"), num_dims, ctx.get_int32("synthetic_nnz"), 17 + me.id);
  }

  Engine engine(me, nodes, master);
  engine.StartEverything(ctx.get_int32("num_servers_per_node"));
  if (data.empty()) {  // graceful degradation: a node without data leaves (lr_example.cpp:145-152)
    MINIPS_LOG(1, "node " << me.id << " has no data, force quit");
    engine.ForceQuit();
    engine.StopEverything();
    return 0;
  }
  if (recovering) {
    try {
      ctx.SetIterationMap(LoadConfigData(ck.WorkerConfigFile()));
    } catch (const std::exception&) {
    }
  }
  auto table_id = engine.CreateTable<double>(engine.getRanges(), ParseModelType(ctx.get_string("kModelType")),
                                             ParseStorageType(ctx.get_string("kStorageType")),
                                             ctx.get_int32("kStaleness"));
  if (ctx.get_bool("init_dump") && ctx.get_bool("checkpoint_toggle")) DumpSVMData(ck.prefix + "worker_"
                                                                                  + std::to_string(me.id), data);
  if (recovering) CheckFaultTolerance(4, "node " + std::to_string(me.id) + " restored its shard");

  MLTask task;
  std::vector<WorkerAlloc> alloc;
  for (auto& n : nodes) alloc.push_back({n.id, (uint32_t)ctx.get_int32("num_workers_per_node")});
  task.SetWorkerAlloc(alloc);
  task.SetTables({table_id});
  const int num_iters = ctx.get_int32("num_iters");
  const int wpn = ctx.get_int32("num_workers_per_node");
  const double alpha = ctx.get_double("alpha");
  std::atomic<double> final_acc{0};
  task.SetLambda([&](const Info& info) {
    BatchDataSampler sampler(&data, ctx.get_int32("batch_size"), 1000 + info.worker_id);
    std::vector<std::vector<Key>> future_keys;
    std::vector<std::vector<const SVMItem*>> future_ptrs;
    for (int i = 0; i < num_iters + ctx.get_int32("kSpeculation"); ++i) {
      sampler.RandomStartPoint();
      future_keys.push_back(sampler.PrepareNextBatch());
      future_ptrs.push_back(sampler.GetDataPtrs());
    }
    auto table = info.CreateKVClientTable<double>(table_id);
    std::mt19937_64 rng(info.worker_id * 7919 + 1);
    std::uniform_real_distribution<double> u01(0, 1);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<double> params;
    bool after_checkpoint = false;
    for (int i = ctx.GetIteration(info.worker_id); i < num_iters; ++i) {
      auto& keys = future_keys[i];
      if (keys.empty()) {
        table->Clock();
        continue;
      }
      table->Get(keys, &params);
      if (engine.IsNeedRollBack()) {
        engine.IncRollBackCount();
        if (info.worker_id % wpn == 0) {
          engine.Barrier();
          engine.RecoverEnd();
        } else {
          engine.WaitRecover();
        }
        if (info.worker_id == 0) after_checkpoint = true;
        i = ctx.GetIteration(info.worker_id) - 1;
        continue;
      }
      std::vector<double> deltas(keys.size(), 0.0);
      for (const SVMItem* it : future_ptrs[i]) {
        double y = it->y < 0 ? 0 : it->y;
        double z = 0;
        size_t j = 0;
        for (auto& f : it->x) {
          while (keys[j] < (Key)f.first) ++j;
          z += params[j] * f.second;
        }
        double p = 1.0 / (1.0 + std::exp(-z));
        j = 0;
        for (auto& f : it->x) {
          while (keys[j] < (Key)f.first) ++j;
          deltas[j] += alpha * f.second * (y - p);
        }
      }
      table->Add(keys, deltas);
      table->Clock();
      if (i > 0 && i % 100 == 0 && info.worker_id == 0 && ctx.get_bool("checkpoint_toggle")) {
        if (after_checkpoint) {
          after_checkpoint = false;
        } else {
          auto c0 = std::chrono::steady_clock::now();
          table->CheckPoint();
          MINIPS_LOG(0, "[CheckPoint] iteration " << i << " took "
                                                 << std::chrono::duration_cast<std::chrono::milliseconds>(
                                                        std::chrono::steady_clock::now() - c0)
                                                        .count()
                                                 << " ms");
        }
      }
      if (i > 0 && i % 10 == 0 && info.worker_id % wpn == 0)
        MINIPS_VLOG(1, "Current iteration=" << i << " on node=" << me.id);
      int rep = ctx.get_int32("report_interval");
      if (rep > 0 && i > 0 && i % rep == 0 && info.worker_id == 0)
        Report(ctx.get_string("report_prefix"), i,
               std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count());
      if (ctx.get_bool("with_injected_straggler") && u01(rng) < 0.05)
        std::this_thread::sleep_for(std::chrono::milliseconds((int)(u01(rng) * 100)));
      ctx.SetIteration(info.worker_id, i + 1);
    }
    auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
    if (info.worker_id % wpn == 0) {
      std::vector<Key> all(num_dims);
      for (int64_t k = 0; k < num_dims; ++k) all[k] = (Key)k;
      table->Get(all, &params);
      double acc = TestAccuracy(params, data);
      final_acc = acc;
      MINIPS_LOG(0, "The accuracy is " << acc << " on node=" << me.id);
    }
    MINIPS_LOG(0, "Total training time: " << ms << " ms on worker: " << info.worker_id);
  });
  engine.Run(task);
  engine.StopEverything();
  std::printf("{\"app\": \"lr\", \"node\": %u, \"accuracy\": %.4f}\n", me.id, final_acc.load());
  return 0;
}
