// Mini-batch K-Means on the native PS runtime (reference apps/kmeans/kmeans.cpp:95-309,
// kmeans_helper.hpp). Table 0 holds (K+1)*num_dims centre parameters, table 1 the K
// cluster-member counts. An init task (worker 0) seeds the centres with random / kmeans++ /
// kmeans_parallel (approximated by oversampled k-means++), then every worker runs
// num_iters mini-batch iterations: Get both tables, assign each sampled point to its
// nearest centre, move it by lr = alpha / ++count, push the deltas and count deltas, Clock.
// The report worker appends `iter\tSSE\tms` (sampled SSE over 50 points) to report_prefix.
#include <algorithm>
#include <chrono>
#include <numeric>
#include <set>

#include "app_common.h"

using namespace minips;
using namespace minips_app;

static std::pair<int, double> Nearest(const SVMItem& x, int K, const std::vector<std::vector<double>>& c, int dims) {
  int best = 0;
  double bd = 1e300;
  for (int k = 0; k < K; ++k) {
    std::vector<double> diff = c[k];
    for (auto& f : x.x)
      if (f.first < dims) diff[f.first] -= f.second;
    double d = 0;
    for (double v : diff) d += v * v;
    if (d < bd) {
      bd = d;
      best = k;
    }
  }
  return {best, bd};
}

static void InitCenters(int K, int dims, const std::vector<SVMItem>& data, std::vector<std::vector<double>>& c,
                        const std::string& mode, std::mt19937_64& rng) {
  auto set_center = [&](int k, const SVMItem& x) {
    std::fill(c[k].begin(), c[k].end(), 0.0);
    for (auto& f : x.x)
      if (f.first < dims) c[k][f.first] = f.second;
  };
  std::uniform_int_distribution<size_t> pick(0, data.size() - 1);
  if (mode == "random") {
    for (int k = 0; k < K; ++k) set_center(k, data[pick(rng)]);
    return;
  }
  // k-means++ (D^2 sampling); kmeans_parallel oversamples candidates 2K then reduces.
  int m = mode == "kmeans_parallel" ? 2 * K : K;
  std::vector<std::vector<double>> cand(m, std::vector<double>(dims, 0.0));
  std::vector<std::vector<double>> tmp = c;
  tmp.resize(std::max<int>(m, K + 1), std::vector<double>(dims, 0.0));
  std::swap(tmp, cand);
  auto setc = [&](int k, const SVMItem& x) {
    std::fill(cand[k].begin(), cand[k].end(), 0.0);
    for (auto& f : x.x)
      if (f.first < dims) cand[k][f.first] = f.second;
  };
  setc(0, data[pick(rng)]);
  std::vector<double> d2(data.size());
  for (int k = 1; k < m; ++k) {
    double total = 0;
    for (size_t i = 0; i < data.size(); ++i) {
      d2[i] = Nearest(data[i], k, cand, dims).second;
      total += d2[i];
    }
    std::uniform_real_distribution<double> u(0, total);
    double r = u(rng), acc = 0;
    size_t chosen = data.size() - 1;
    for (size_t i = 0; i < data.size(); ++i) {
      acc += d2[i];
      if (acc >= r) {
        chosen = i;
        break;
      }
    }
    setc(k, data[chosen]);
  }
  for (int k = 0; k < K; ++k) c[k] = cand[k];
}

int main(int argc, char** argv) {
  DefineCommonFlags();
  auto& ctx = Context::Get();
  ctx.Define("K", Context::Type::kInt, "5", "clusters");
  ctx.Define("kmeans_init_mode", Context::Type::kString, "kmeans++", "random / kmeans++ / kmeans_parallel");
  ctx.Define("report_worker", Context::Type::kInt, "0", "worker that writes the SSE report");
  ctx.ParseArgs(argc, argv);
  Node me, master;
  std::vector<Node> nodes;
  if (SetupNodes(&me, &nodes, &master)) return RunMasterIfNeeded(master, nodes);
  const int K = ctx.get_int32("K");
  const int dims = ctx.get_int64("num_dims") > 0 ? (int)ctx.get_int64("num_dims") : 64;
  MINIPS_CHECK(K > 0 && dims > 0, "K and num_dims must be positive");
  const int my_index = (int)(std::find(nodes.begin(), nodes.end(), me) - nodes.begin());
  std::vector<SVMItem> data = !ctx.get_string("input").empty()
                                  ? LoadAppData(nodes, my_index)
                                  : SyntheticData(ctx.get_int32("synthetic_rows"), dims, ctx.get_int32("synthetic_nnz"),
                                                  31 + me.id);
  Engine engine(me, nodes, master);
  engine.StartEverything(ctx.get_int32("num_servers_per_node"));
  uint32_t servers = (uint32_t)(nodes.size() * ctx.get_int32("num_servers_per_node"));
  auto t0 = engine.CreateTable<double>(EvenRanges((uint64_t)(K + 1) * dims, servers),
                                       ParseModelType(ctx.get_string("kModelType")),
                                       ParseStorageType(ctx.get_string("kStorageType")), ctx.get_int32("kStaleness"));
  auto t1 = engine.CreateTable<double>(EvenRanges((uint64_t)K, std::min<uint32_t>(servers, (uint32_t)K)),
                                       ParseModelType(ctx.get_string("kModelType")), StorageType::Map,
                                       ctx.get_int32("kStaleness"));
  engine.Barrier();
  std::vector<WorkerAlloc> alloc;
  for (auto& n : nodes) alloc.push_back({n.id, (uint32_t)ctx.get_int32("num_workers_per_node")});
  std::vector<Key> keys((size_t)(K + 1) * dims), keys2(K);
  std::iota(keys.begin(), keys.end(), 0);
  std::iota(keys2.begin(), keys2.end(), 0);

  MLTask init;
  init.SetWorkerAlloc(alloc);
  init.SetTables({t0});
  init.SetLambda([&](const Info& info) {
    if (info.worker_id != 0) return;
    std::mt19937_64 rng(7);
    std::vector<std::vector<double>> c(K + 1, std::vector<double>(dims, 0.0));
    InitCenters(K, dims, data, c, ctx.get_string("kmeans_init_mode"), rng);
    std::vector<double> push;
    for (auto& row : c) push.insert(push.end(), row.begin(), row.end());
    auto table = info.CreateKVClientTable<double>(t0);
    table->Add(keys, push);
    table->Clock();
  });
  engine.Run(init);

  double last_sse = 0;
  MLTask task;
  task.SetWorkerAlloc(alloc);
  task.SetTables({t0, t1});
  const int wpn = ctx.get_int32("num_workers_per_node");
  task.SetLambda([&](const Info& info) {
    auto table = info.CreateKVClientTable<double>(t0);
    auto table2 = info.CreateKVClientTable<double>(t1);
    std::mt19937_64 rng(100 + info.worker_id);
    std::uniform_int_distribution<size_t> pick(0, data.size() - 1);
    std::vector<double> pull, members;
    auto start = std::chrono::steady_clock::now();
    for (int iter = 0; iter < ctx.get_int32("num_iters"); ++iter) {
      table->Get(keys, &pull);
      table2->Get(keys2, &members);
      std::vector<std::vector<double>> params(K + 1, std::vector<double>(dims));
      for (int i = 0; i <= K; ++i)
        for (int j = 0; j < dims; ++j) params[i][j] = pull[(size_t)i * dims + j];
      auto deltas = params;
      auto counts0 = members;
      size_t p = pick(rng);
      for (int s = 0; s < std::max(1, ctx.get_int32("batch_size") / wpn); ++s) {
        if (p >= data.size()) p = pick(rng);
        const SVMItem& x = data[p++];
        int k = Nearest(x, K, deltas, dims).first;
        double lr = ctx.get_double("alpha") / ++members[k];
        std::vector<double> dist = deltas[k];
        for (auto& f : x.x)
          if (f.first < dims) dist[f.first] -= f.second;
        for (int j = 0; j < dims; ++j) deltas[k][j] -= lr * dist[j];
      }
      std::vector<double> push((size_t)(K + 1) * dims);
      for (int i = 0; i <= K; ++i)
        for (int j = 0; j < dims; ++j) push[(size_t)i * dims + j] = deltas[i][j] - params[i][j];
      for (int k = 0; k < K; ++k) members[k] -= counts0[k];
      table->Add(keys, push);
      table->Clock();
      table2->Add(keys2, members);
      table2->Clock();
      int rep = ctx.get_int32("report_interval");
      if (info.worker_id == (uint32_t)ctx.get_int32("report_worker") && rep > 0 && iter % rep == 0) {
        double sse = 0;
        for (int s = 0; s < 50 && s < (int)data.size(); ++s) sse += Nearest(data[pick(rng)], K, params, dims).second;
        last_sse = sse;
        Report(ctx.get_string("report_prefix"), iter,
               std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - start).count(),
               sse);
      }
    }
  });
  engine.Run(task);
  engine.StopEverything();
  std::printf("{\"app\": \"kmeans\", \"node\": %u, \"sampled_sse\": %.4f}\n", me.id, last_sse);
  return 0;
}
