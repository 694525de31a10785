#include "checkpoint.h"

#include <memory>

#include "io.h"

#include <sys/stat.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <fstream>

#include "fs.h"
#include <iomanip>
#include <set>
#include <thread>

namespace minips {

void EnsureParentDir(const std::string& path) {
  if (!IsLocalUrl(path)) {  // remote file systems: mkdir -p of the parent through the FileSystem
    const Url u = ParseUrl(path);
    const auto s = u.path.rfind('/');
    if (s != std::string::npos && s > 0) {
      Url parent = u;
      parent.path = u.path.substr(0, s);
      FileSystem::For(path).MakeDirs(parent.ToString());
    }
    return;
  }
  auto slash = path.rfind('/');
  if (slash == std::string::npos || slash == 0) return;
  std::string dir = path.substr(0, slash);
  // mkdir -p
  std::string cur;
  for (size_t i = 0; i < dir.size(); ++i) {
    cur += dir[i];
    if ((dir[i] == '/' && i > 0) || i + 1 == dir.size()) {
      if (mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) {
        MINIPS_CHECK(false, "mkdir " << cur << " failed errno=" << errno);
      }
    }
  }
}

void DumpSVMData(const std::string& path, const std::vector<SVMItem>& data) {
  EnsureParentDir(path);
  GeneralOfstream out(path);
  MINIPS_CHECK(out.good(), "cannot write " << path);
  out << std::setprecision(17);
  for (auto& it : data) {
    out << it.y;
    for (auto& f : it.x) out << " " << f.first << ":" << f.second;
    out << "\n";
  }
  out.close();
  MINIPS_CHECK(out.good(), "write failed " << path);
}

std::vector<SVMItem> LoadSVMData(const std::string& path) { return LoadLibsvmFile(path, 0, 1, 4, false); }

void DumpConfigData(const std::string& path, const std::map<int, int>& iteration_map) {
  EnsureParentDir(path);
  GeneralOfstream out(path);
  MINIPS_CHECK(out.good(), "cannot write " << path);
  for (auto& kv : iteration_map) out << kv.first << ":" << kv.second << " ";
  out.close();
  MINIPS_CHECK(out.good(), "write failed " << path);
}

std::map<int, int> LoadConfigData(const std::string& path) {
  GeneralIfstream in(path);
  MINIPS_CHECK(in.good(), "cannot read " << path);
  std::map<int, int> m;
  std::string tok;
  while (in >> tok) {
    auto c = tok.find(':');
    if (c == std::string::npos) continue;
    m[std::stoi(tok.substr(0, c))] = std::stoi(tok.substr(c + 1));
  }
  return m;
}

void DumpScaleFile(const std::string& path, const Node& node) {
  EnsureParentDir(path);
  GeneralOfstream out(path);
  MINIPS_CHECK(out.good(), "cannot write " << path);
  out << node.id << ":" << node.hostname << ":" << node.port;
  if (node.gpu >= 0) out << ":" << node.gpu;
  out << "\n";
  out.close();
  MINIPS_CHECK(out.good(), "write failed " << path);
}

Node LoadScaleFile(const std::string& path) {
  auto nodes = ParseFile(path);
  MINIPS_CHECK(!nodes.empty(), "empty scale file " << path);
  return nodes[0];
}

bool ParseLibsvm(const char* line, size_t len, SVMItem* out, bool one_based) {
  out->x.clear();
  const char* p = line;
  const char* end = line + len;
  auto skip_ws = [&] {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
  };
  skip_ws();
  if (p >= end) return false;
  char* q = nullptr;
  out->y = std::strtod(p, &q);
  if (q == p) return false;
  p = q;
  while (true) {
    skip_ws();
    if (p >= end) break;
    long long idx = std::strtoll(p, &q, 10);
    if (q == p || q >= end || *q != ':') break;
    p = q + 1;
    double v = std::strtod(p, &q);
    if (q == p) break;
    p = q;
    out->x.emplace_back(one_based ? idx - 1 : idx, v);
  }
  return true;
}

std::vector<SVMItem> LoadLibsvmFile(const std::string& path, const LoadOptions& opt, bool one_based) {
  // Blocks of every input (a path, a directory or a comma list; local, webhdfs:// or hdfs://)
  // are handed out statically (rank r of n) or by the locality-aware block assigner, and parsed
  // by `opt.num_threads` loader threads (io.h ForEachLine); results are kept per block and
  // concatenated in block order, so the order is deterministic for a given assignment.
  const int threads = std::max(1, opt.num_threads);
  std::vector<std::map<int, std::vector<SVMItem>>> per_thread(threads);
  ForEachLine(path, opt, [&](const FileBlock& b, const char* l, size_t n, int t) {
    SVMItem item;
    if (ParseLibsvm(l, n, &item, one_based)) per_thread[t][b.id].push_back(std::move(item));
  });
  std::map<int, std::vector<SVMItem>*> order;
  for (auto& m : per_thread)
    for (auto& kv : m) order[kv.first] = &kv.second;
  std::vector<SVMItem> all;
  for (auto& kv : order)
    for (auto& it : *kv.second) all.push_back(std::move(it));
  return all;
}

std::vector<SVMItem> LoadLibsvmFile(const std::string& path, int shard, int num_shards, int num_threads,
                                    bool one_based) {
  LoadOptions opt;
  opt.rank = shard;
  opt.num_ranks = num_shards;
  opt.num_threads = num_threads;
  return LoadLibsvmFile(path, opt, one_based);
}

BatchDataSampler::BatchDataSampler(const std::vector<SVMItem>* data, int batch_size, uint64_t seed)
    : data_(data), batch_size_(batch_size), rng_(seed) {
  MINIPS_CHECK(data_ && !data_->empty(), "sampler needs data");
  MINIPS_CHECK(batch_size_ > 0, "batch size must be positive");
}

void BatchDataSampler::RandomStartPoint() { current_ = rng_() % data_->size(); }

std::vector<Key> BatchDataSampler::PrepareNextBatch() {
  batch_ptrs_.clear();
  std::set<Key> keys;
  for (int i = 0; i < batch_size_; ++i) {
    const SVMItem& it = (*data_)[current_];
    batch_ptrs_.push_back(&it);
    for (auto& f : it.x) keys.insert((Key)f.first);
    current_ = (current_ + 1) % data_->size();
  }
  return std::vector<Key>(keys.begin(), keys.end());
}

void CheckFaultTolerance(int phase, const std::string& detail) {
  static const char* kPhase[] = {"", "Phase1", "Phase2 detect failure", "Phase3 restart", "Phase4 recover",
                                 "Phase5 others recovered"};
  long long ts = std::chrono::duration_cast<std::chrono::milliseconds>(
                     std::chrono::system_clock::now().time_since_epoch())
                     .count();
  const char* name = (phase >= 1 && phase <= 5) ? kPhase[phase] : "Phase?";
  MINIPS_LOG(0, "[Fault Tolerance][Phase" << phase << "][" << ts << "] " << name << (detail.empty() ? "" : ": ")
                                           << detail);
}

}  // namespace minips
