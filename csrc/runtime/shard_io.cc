#include "shard_io.h"

#include <fcntl.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <fstream>

#include "fs.h"
#include <sstream>
#include <stdexcept>

#include "base.h"
#include "checkpoint.h"

namespace minips {

namespace {
constexpr char kMagic[8] = {'M', 'P', 'S', 'S', 'H', 'R', 'D', '1'};
constexpr uint32_t kVersion = 2;
constexpr uint64_t kAlign = 4096;
std::atomic<uint64_t> g_bytes_read{0};

uint64_t AlignUp(uint64_t v) { return (v + kAlign - 1) / kAlign * kAlign; }

void PWriteAll(int fd, const void* src, uint64_t n, uint64_t off, const std::string& what) {
  const char* p = static_cast<const char*>(src);
  while (n > 0) {
    const ssize_t w = ::pwrite(fd, p, (size_t)std::min<uint64_t>(n, 1ull << 30), (off_t)off);
    if (w < 0 && errno == EINTR) continue;
    MINIPS_CHECK(w > 0, "pwrite failed on " << what << ": " << std::strerror(errno));
    p += w;
    off += (uint64_t)w;
    n -= (uint64_t)w;
  }
}

void PReadAll(int fd, void* dst, uint64_t n, uint64_t off, const std::string& what) {
  char* p = static_cast<char*>(dst);
  while (n > 0) {
    const ssize_t r = ::pread(fd, p, (size_t)std::min<uint64_t>(n, 1ull << 30), (off_t)off);
    if (r < 0 && errno == EINTR) continue;
    MINIPS_CHECK(r > 0, "pread failed / truncated " << what << ": " << (r < 0 ? std::strerror(errno) : "eof"));
    p += r;
    off += (uint64_t)r;
    n -= (uint64_t)r;
    g_bytes_read += (uint64_t)r;
  }
}

// Header image: magic, version, meta, n, [name, dtype, rows, cols, bytes, offset]...
std::string HeaderImage(const ShardMeta& m, const std::vector<ArrayDesc>& arrays) {
  std::ostringstream o(std::ios::binary);
  auto put = [&](const auto& v) { o.write(reinterpret_cast<const char*>(&v), sizeof(v)); };
  auto put_s = [&](const std::string& s) {
    put((uint32_t)s.size());
    o.write(s.data(), (std::streamsize)s.size());
  };
  o.write(kMagic, 8);
  put(kVersion);
  put(m.global_rows);
  put(m.base);
  put(m.rows);
  put(m.cols);
  put(m.clock);
  put(m.table_id);
  put(m.rank);
  put(m.world);
  put_s(m.kind);
  put((uint32_t)arrays.size());
  for (const auto& a : arrays) {
    put_s(a.name);
    put((uint32_t)a.dtype);
    put(a.rows);
    put(a.cols);
    put(a.bytes);
    put(a.offset);
  }
  return o.str();
}

// Assigns 4 KiB aligned offsets after a header of the final size.
void LayoutArrays(const ShardMeta& m, std::vector<ArrayDesc>& arrays) {
  for (auto& a : arrays) a.bytes = a.rows * a.cols * DTypeSize(a.dtype);
  uint64_t off = AlignUp(HeaderImage(m, arrays).size());
  for (auto& a : arrays) {
    a.offset = off;
    off = AlignUp(off + a.bytes);
  }
}

template <typename T>
T get(std::ifstream& i) {
  T v;
  i.read(reinterpret_cast<char*>(&v), sizeof(T));
  MINIPS_CHECK(i.good(), "truncated shard file");
  return v;
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
  std::vector<ArrayDesc> desc;
  for (const auto& a : arrays) {
    ArrayDesc d;
    d.name = a.name;
    d.dtype = a.dtype;
    d.rows = a.rows;
    d.cols = a.cols;
    desc.push_back(d);
  }
  ShardFileWriter w(path, m, desc);
  for (size_t k = 0; k < arrays.size(); ++k)
    if (arrays[k].rows) w.WriteRows((int)k, 0, arrays[k].data, arrays[k].rows);
  w.Close();
}

ShardHeader ReadShardHeader(const std::string& path) {
  std::ifstream i(path, std::ios::binary);
  MINIPS_CHECK(i.good(), "cannot read " << path);
  char magic[8];
  i.read(magic, 8);
  MINIPS_CHECK(i.good() && std::memcmp(magic, kMagic, 8) == 0, "not a minips shard file: " << path);
  const uint32_t ver = get<uint32_t>(i);
  // v1 (round-1 trees): the same header fields, but each array's bytes follow its descriptor
  // (no offset field) -- still readable, so old checkpoints restore
  MINIPS_CHECK(ver == kVersion || ver == 1, "unsupported shard version " << ver << " in " << path);
  ShardHeader h;
  h.meta.global_rows = get<uint64_t>(i);
  h.meta.base = get<uint64_t>(i);
  h.meta.rows = get<uint64_t>(i);
  h.meta.cols = get<uint64_t>(i);
  h.meta.clock = get<int64_t>(i);
  h.meta.table_id = get<int32_t>(i);
  h.meta.rank = get<int32_t>(i);
  h.meta.world = get<int32_t>(i);
  h.meta.kind = get_str(i);
  const uint32_t n = get<uint32_t>(i);
  MINIPS_CHECK(n < 64, "corrupt array count in " << path);
  for (uint32_t k = 0; k < n; ++k) {
    ArrayDesc a;
    a.name = get_str(i);
    a.dtype = (DType)get<uint32_t>(i);
    a.rows = get<uint64_t>(i);
    a.cols = get<uint64_t>(i);
    a.bytes = get<uint64_t>(i);
    MINIPS_CHECK(a.bytes == a.rows * a.cols * DTypeSize(a.dtype), "array size mismatch in " << path);
    if (ver == 1) {
      a.offset = (uint64_t)i.tellg();
      i.seekg((std::streamoff)a.bytes, std::ios::cur);
      MINIPS_CHECK(i.good(), "truncated array " << a.name << " in " << path);
    } else {
      a.offset = get<uint64_t>(i);
    }
    h.arrays.push_back(a);
  }
  return h;
}

void ReadRows(const std::string& path, uint64_t offset, uint64_t row_bytes, uint64_t row0, uint64_t nrows, void* dst) {
  if (nrows == 0) return;
  const int fd = ::open(path.c_str(), O_RDONLY);
  MINIPS_CHECK(fd >= 0, "cannot open " << path << ": " << std::strerror(errno));
  try {
    PReadAll(fd, dst, nrows * row_bytes, offset + row0 * row_bytes, path);
  } catch (...) {
    ::close(fd);
    throw;
  }
  ::close(fd);
}

uint64_t ShardBytesRead() { return g_bytes_read.load(); }
void ResetShardBytesRead() { g_bytes_read = 0; }

LoadedShard ReadShard(const std::string& path) {
  const ShardHeader h = ReadShardHeader(path);
  LoadedShard s;
  s.meta = h.meta;
  for (const auto& d : h.arrays) {
    LoadedArray a;
    a.name = d.name;
    a.dtype = d.dtype;
    a.rows = d.rows;
    a.cols = d.cols;
    a.bytes.resize(d.bytes);
    if (d.bytes) ReadRows(path, d.offset, d.cols * DTypeSize(d.dtype), 0, d.rows, a.bytes.data());
    s.arrays.push_back(std::move(a));
  }
  return s;
}

ShardFileWriter::ShardFileWriter(const std::string& path, const ShardMeta& meta, const std::vector<ArrayDesc>& arrays)
    : path_(path), tmp_(path + ".tmp"), arrays_(arrays) {
  EnsureParentDir(path);
  LayoutArrays(meta, arrays_);
  fd_ = ::open(tmp_.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  MINIPS_CHECK(fd_ >= 0, "cannot write " << tmp_ << ": " << std::strerror(errno));
  const std::string hdr = HeaderImage(meta, arrays_);
  PWriteAll(fd_, hdr.data(), hdr.size(), 0, tmp_);
  uint64_t end = AlignUp(hdr.size());
  for (const auto& a : arrays_) end = std::max(end, a.offset + a.bytes);
  MINIPS_CHECK(::ftruncate(fd_, (off_t)end) == 0, "ftruncate " << tmp_);
}

ShardFileWriter::~ShardFileWriter() {
  if (fd_ >= 0) {
    ::close(fd_);
    std::remove(tmp_.c_str());  // never closed: an abandoned checkpoint leaves no file behind
  }
}

void ShardFileWriter::WriteRows(int array, uint64_t row0, const void* src, uint64_t nrows) {
  MINIPS_CHECK(fd_ >= 0, "ShardFileWriter already closed");
  MINIPS_CHECK(array >= 0 && array < (int)arrays_.size(), "bad array index " << array);
  const ArrayDesc& a = arrays_[array];
  MINIPS_CHECK(row0 + nrows <= a.rows, "rows [" << row0 << ", " << row0 + nrows << ") out of range " << a.rows);
  const uint64_t rb = a.cols * DTypeSize(a.dtype);
  PWriteAll(fd_, src, nrows * rb, a.offset + row0 * rb, tmp_);
}

void ShardFileWriter::Close() {
  MINIPS_CHECK(fd_ >= 0, "ShardFileWriter already closed");
  // durable before published: a committed 'latest' must never name data still in the page cache
  // when the machine loses power
  MINIPS_CHECK(::fsync(fd_) == 0, "fsync " << tmp_ << ": " << std::strerror(errno));
  MINIPS_CHECK(::close(fd_) == 0, "close " << tmp_);
  fd_ = -1;
  // atomic publish: a crash mid-write never leaves a truncated checkpoint under the real name
  MINIPS_CHECK(std::rename(tmp_.c_str(), path_.c_str()) == 0, "rename " << tmp_ << " -> " << path_);
  const std::string dir = path_.find('/') == std::string::npos ? "." : path_.substr(0, path_.rfind('/') + 1);
  const int dfd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY);
  if (dfd >= 0) {  // the rename itself (the directory entry) reaches the disk too
    (void)::fsync(dfd);
    ::close(dfd);
  }
}

TextParamsWriter::TextParamsWriter(const std::string& path) : path_(path) {
  EnsureParentDir(path);
  out_.reset(new GeneralOfstream(path));
  MINIPS_CHECK(out_->good(), "cannot write " << path);
  buf_.reserve(1 << 20);
}

TextParamsWriter::~TextParamsWriter() {
  try {
    Close();
  } catch (const std::exception&) {
  }
}

void TextParamsWriter::Append(const ArrayRef& a) {
  MINIPS_CHECK(out_, "TextParamsWriter already closed");
  const uint64_t n = a.rows * a.cols;
  // shortest round-trip precision of the stored type (fp64 tables need 17 digits)
  const char* fmt = a.dtype == DType::kF64 ? "%llu:%.17g " : "%llu:%.9g ";
  char tmp[64];
  for (uint64_t i = 0; i < n; ++i) {
    const double v = elem(a, i);
    if (v == 0.0) continue;
    const int len = std::snprintf(tmp, sizeof(tmp), fmt, (unsigned long long)(next_ + i), v);
    buf_.append(tmp, len);
    if (buf_.size() > (1u << 20) - 64) {
      *out_ << buf_;
      buf_.clear();
    }
  }
  next_ += n;
}

void TextParamsWriter::Close() {
  if (!out_) return;
  *out_ << buf_;
  buf_.clear();
  out_->close();
  const bool ok = out_->good();
  out_.reset();
  MINIPS_CHECK(ok, "write failed: " << path_);
}

void WriteTextParams(const std::string& path, const ArrayRef& a) {
  TextParamsWriter w(path);
  w.Append(a);
  w.Close();
}

std::vector<double> ReadTextParams(const std::string& path, uint64_t n) {
  GeneralIfstream in(path);
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
