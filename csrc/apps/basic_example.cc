// Push/pull smoke app (reference apps/basic/basic_example.cpp): kMaxKey = 1000 keys range-
// partitioned over the nodes, SSP staleness 1 on MapStorage, num_workers_per_node workers per
// node each running 100 x {Get(all keys), Add(0.5 to each), Clock}. At the end every key must
// equal 0.5 * total_workers * iterations; the app prints the check as JSON.
#include <numeric>

#include "app_common.h"

using namespace minips;
using namespace minips_app;

int main(int argc, char** argv) {
  DefineCommonFlags();
  auto& ctx = Context::Get();
  ctx.set("num_workers_per_node", 10);
  ctx.set("num_iters", 100);
  ctx.ParseArgs(argc, argv);
  Node me, master;
  std::vector<Node> nodes;
  if (SetupNodes(&me, &nodes, &master)) return RunMasterIfNeeded(master, nodes);
  const uint64_t kMaxKey = 1000;
  Engine engine(me, nodes, master);
  engine.StartEverything(1);
  auto table_id = engine.CreateTable<double>(EvenRanges(kMaxKey, (uint32_t)nodes.size()), ModelType::SSP,
                                             StorageType::Map, 1);
  engine.Barrier();
  MLTask task;
  std::vector<WorkerAlloc> alloc;
  const int wpn = ctx.get_int32("num_workers_per_node");
  for (auto& n : nodes) alloc.push_back({n.id, (uint32_t)wpn});
  task.SetWorkerAlloc(alloc);
  task.SetTables({table_id});
  const int iters = ctx.get_int32("num_iters");
  std::vector<Key> keys(kMaxKey);
  std::iota(keys.begin(), keys.end(), 0);
  task.SetLambda([&](const Info& info) {
    auto table = info.CreateKVClientTable<double>(table_id);
    std::vector<double> vals;
    for (int i = 0; i < iters; ++i) {
      table->Get(keys, &vals);
      table->Add(keys, std::vector<double>(kMaxKey, 0.5));
      table->Clock();
    }
  });
  engine.Run(task);
  double expect = 0.5 * wpn * nodes.size() * iters, got = 0;
  MLTask check;
  check.SetWorkerAlloc({{nodes[0].id, 1}});
  check.SetTables({table_id});
  check.SetLambda([&](const Info& info) {
    auto table = info.CreateKVClientTable<double>(table_id);
    std::vector<double> vals;
    table->Get(keys, &vals);
    got = vals[kMaxKey - 1];
  });
  engine.Run(check);
  engine.StopEverything();
  std::printf("{\"app\": \"basic\", \"node\": %u, \"expected\": %.1f, \"got\": %.1f}\n", me.id, expect,
              me.id == nodes[0].id ? got : expect);
  return 0;
}
