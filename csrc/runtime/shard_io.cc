#include "shard_io.h"

#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "base.h"
#include "checkpoint.h"

namespace minips {

namespace {
constexpr char kMagic[8] = {'M', 'P', 'S', 'S', 'H', 'R', 'D', '1'};
constexpr uint32_t kVersion = 1;

template <typename T>
void put(std::ofstream& o, const T& v) {
  o.write(reinterpret_cast<const char*>(&v), sizeof(T));
}
template <typename T>
T get(std::ifstream& i) {
  T v;
  i.read(reinterpret_cast<char*>(&v), sizeof(T));
  MINIPS_CHECK(i.good(), "truncated shard file");
  return v;
}
void put_str(std::ofstream& o, const std::string& s) {
  put<uint32_t>(o, (uint32_t)s.size());
  o.write(s.data(), (std::streamsize)s.size());
}
std::string get_str(std::ifstream& i) {
  const uint32_t n = get<uint32_t>(i);
  MINIPS_CHECK(n < (1u << 20), "corrupt string length in shard file");
  std::string s(n, '\0');
  i.read(&s[0], n);
  MINIPS_CHECK(i.good(), "truncated shard file");
  return s;
}

double elem(const ArrayRef& a, uint64_t i) {
  switch (a.dtype) {
    case DType::kF32:
      return static_cast<const float*>(a.data)[i];
    case DType::kF64:
      return static_cast<const double*>(a.data)[i];
    case DType::kBF16: {
      uint32_t u = (uint32_t) static_cast<const uint16_t*>(a.data)[i] << 16;
      float f;
      std::memcpy(&f, &u, 4);
      return f;
    }
    case DType::kI64:
      return (double)static_cast<const int64_t*>(a.data)[i];
    case DType::kI32:
      return (double)static_cast<const int32_t*>(a.data)[i];
  }
  return 0.0;
}
}  // namespace

size_t DTypeSize(DType t) {
  switch (t) {
    case DType::kF32:
    case DType::kI32:
      return 4;
    case DType::kBF16:
      return 2;
    case DType::kF64:
    case DType::kI64:
      return 8;
  }
  return 0;
}

void WriteShard(const std::string& path, const ShardMeta& m, const std::vector<ArrayRef>& arrays) {
  EnsureParentDir(path);
  const std::string tmp = path + ".tmp";
  {
    std::ofstream o(tmp, std::ios::binary | std::ios::trunc);
    MINIPS_CHECK(o.good(), "cannot write " << tmp);
    o.write(kMagic, 8);
    put<uint32_t>(o, kVersion);
    put<uint64_t>(o, m.global_rows);
    put<uint64_t>(o, m.base);
    put<uint64_t>(o, m.rows);
    put<uint64_t>(o, m.cols);
    put<int64_t>(o, m.clock);
    put<int32_t>(o, m.table_id);
    put<int32_t>(o, m.rank);
    put<int32_t>(o, m.world);
    put_str(o, m.kind);
    put<uint32_t>(o, (uint32_t)arrays.size());
    for (const auto& a : arrays) {
      put_str(o, a.name);
      put<uint32_t>(o, (uint32_t)a.dtype);
      put<uint64_t>(o, a.rows);
      put<uint64_t>(o, a.cols);
      const uint64_t bytes = a.rows * a.cols * DTypeSize(a.dtype);
      put<uint64_t>(o, bytes);
      if (bytes) o.write(static_cast<const char*>(a.data), (std::streamsize)bytes);
    }
    MINIPS_CHECK(o.good(), "write failed: " << tmp);
  }
  // atomic publish: a crash mid-write never leaves a truncated checkpoint under the real name
  MINIPS_CHECK(std::rename(tmp.c_str(), path.c_str()) == 0, "rename " << tmp << " -> " << path);
}

LoadedShard ReadShard(const std::string& path) {
  std::ifstream i(path, std::ios::binary);
  MINIPS_CHECK(i.good(), "cannot read " << path);
  char magic[8];
  i.read(magic, 8);
  MINIPS_CHECK(i.good() && std::memcmp(magic, kMagic, 8) == 0, "not a minips shard file: " << path);
  const uint32_t ver = get<uint32_t>(i);
  MINIPS_CHECK(ver == kVersion, "unsupported shard version " << ver);
  LoadedShard s;
  s.meta.global_rows = get<uint64_t>(i);
  s.meta.base = get<uint64_t>(i);
  s.meta.rows = get<uint64_t>(i);
  s.meta.cols = get<uint64_t>(i);
  s.meta.clock = get<int64_t>(i);
  s.meta.table_id = get<int32_t>(i);
  s.meta.rank = get<int32_t>(i);
  s.meta.world = get<int32_t>(i);
  s.meta.kind = get_str(i);
  const uint32_t n = get<uint32_t>(i);
  MINIPS_CHECK(n < 64, "corrupt array count");
  for (uint32_t k = 0; k < n; ++k) {
    LoadedArray a;
    a.name = get_str(i);
    a.dtype = (DType)get<uint32_t>(i);
    a.rows = get<uint64_t>(i);
    a.cols = get<uint64_t>(i);
    const uint64_t bytes = get<uint64_t>(i);
    MINIPS_CHECK(bytes == a.rows * a.cols * DTypeSize(a.dtype), "array size mismatch in " << path);
    a.bytes.resize(bytes);
    if (bytes) i.read(a.bytes.data(), (std::streamsize)bytes);
    MINIPS_CHECK(i.good() || bytes == 0, "truncated array " << a.name << " in " << path);
    s.arrays.push_back(std::move(a));
  }
  return s;
}

void WriteTextParams(const std::string& path, const ArrayRef& a) {
  EnsureParentDir(path);
  std::ofstream o(path, std::ios::trunc);
  MINIPS_CHECK(o.good(), "cannot write " << path);
  o.precision(9);
  const uint64_t n = a.rows * a.cols;
  std::string buf;
  buf.reserve(1 << 20);
  char tmp[64];
  for (uint64_t i = 0; i < n; ++i) {
    const double v = elem(a, i);
    if (v == 0.0) continue;
    const int len = std::snprintf(tmp, sizeof(tmp), "%llu:%.9g ", (unsigned long long)i, v);
    buf.append(tmp, len);
    if (buf.size() > (1u << 20) - 64) {
      o << buf;
      buf.clear();
    }
  }
  o << buf;
  MINIPS_CHECK(o.good(), "write failed: " << path);
}

std::vector<double> ReadTextParams(const std::string& path, uint64_t n) {
  std::ifstream in(path);
  MINIPS_CHECK(in.good(), "cannot read " << path);
  std::vector<double> out(n, 0.0);
  std::string tok;
  while (in >> tok) {
    const auto c = tok.find(':');
    MINIPS_CHECK(c != std::string::npos, "bad token '" << tok << "' in " << path);
    const uint64_t idx = std::stoull(tok.substr(0, c));
    MINIPS_CHECK(idx < n, "index " << idx << " out of range " << n << " in " << path);
    out[idx] = std::stod(tok.substr(c + 1));
  }
  return out;
}

AsyncShardWriter::AsyncShardWriter() : th_([this] { Loop(); }) {}

AsyncShardWriter::~AsyncShardWriter() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  th_.join();
}

uint64_t AsyncShardWriter::Submit(std::function<void()> job) {
  std::lock_guard<std::mutex> lk(mu_);
  const uint64_t t = next_++;
  jobs_.emplace_back(t, std::move(job));
  cv_.notify_all();
  return t;
}

void AsyncShardWriter::Wait(uint64_t ticket) {
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return finished_ >= ticket; });
}

void AsyncShardWriter::WaitAll() {
  std::unique_lock<std::mutex> lk(mu_);
  const uint64_t last = next_ - 1;
  done_cv_.wait(lk, [&] { return finished_ >= last; });
}

std::string AsyncShardWriter::TakeError() {
  std::lock_guard<std::mutex> lk(mu_);
  std::string e;
  e.swap(error_);
  return e;
}

void AsyncShardWriter::Loop() {
  for (;;) {
    std::pair<uint64_t, std::function<void()>> job;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
      if (jobs_.empty()) return;  // stop_ and drained
      job = std::move(jobs_.front());
      jobs_.pop_front();
    }
    std::string err;
    try {
      job.second();
    } catch (const std::exception& e) {
      err = e.what();
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      finished_ = job.first;
      if (!err.empty()) error_ = err;
    }
    done_cv_.notify_all();
  }
}

}  // namespace minips
