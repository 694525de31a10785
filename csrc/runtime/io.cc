#include "io.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <memory>
#include <cstring>
#include <sstream>

namespace minips {

std::vector<std::string> ListInputFiles(const std::string& spec) {
  std::vector<std::string> out;
  std::stringstream ss(spec);
  std::string item;
  while (std::getline(ss, item, ',')) {
    if (item.empty()) continue;
    struct stat st;
    MINIPS_CHECK(::stat(item.c_str(), &st) == 0, "no such input " << item);
    if (S_ISDIR(st.st_mode)) {
      std::vector<std::string> files;
      DIR* d = ::opendir(item.c_str());
      MINIPS_CHECK(d != nullptr, "cannot open directory " << item);
      while (dirent* e = ::readdir(d)) {
        std::string name = e->d_name;
        if (name == "." || name == "..") continue;
        std::string p = item + (item.back() == '/' ? "" : "/") + name;
        struct stat fs;
        if (::stat(p.c_str(), &fs) == 0 && S_ISREG(fs.st_mode)) files.push_back(p);
      }
      ::closedir(d);
      std::sort(files.begin(), files.end());
      out.insert(out.end(), files.begin(), files.end());
    } else {
      out.push_back(item);
    }
  }
  return out;
}

std::vector<FileBlock> SplitFiles(const std::vector<std::string>& paths, uint64_t block_size) {
  MINIPS_CHECK(block_size > 0, "block_size must be positive");
  std::vector<FileBlock> blocks;
  int id = 0;
  for (const auto& p : paths) {
    struct stat st;
    MINIPS_CHECK(::stat(p.c_str(), &st) == 0, "cannot stat " << p);
    const uint64_t n = (uint64_t)st.st_size;
    for (uint64_t off = 0; off < n; off += block_size)
      blocks.push_back(FileBlock{p, off, std::min(block_size, n - off), n, id++});
  }
  return blocks;
}

BlockAssigner::BlockAssigner(std::vector<FileBlock> blocks, int rank, int num_ranks) {
  MINIPS_CHECK(num_ranks >= 1 && rank >= 0 && rank < num_ranks, "bad rank " << rank << "/" << num_ranks);
  for (auto& b : blocks)
    if (b.id % num_ranks == rank) queue_.push_back(std::move(b));
}

std::optional<FileBlock> BlockAssigner::Next() {
  std::lock_guard<std::mutex> lk(mu_);
  if (queue_.empty()) return std::nullopt;
  FileBlock b = std::move(queue_.front());
  queue_.pop_front();
  served_++;
  return b;
}

size_t BlockAssigner::Remaining() {
  std::lock_guard<std::mutex> lk(mu_);
  return queue_.size();
}

MappedFile::MappedFile(const std::string& path) {
  fd_ = ::open(path.c_str(), O_RDONLY);
  MINIPS_CHECK(fd_ >= 0, "cannot open " << path);
  struct stat st;
  MINIPS_CHECK(::fstat(fd_, &st) == 0, "cannot stat " << path);
  size_ = (uint64_t)st.st_size;
  if (size_) {
    void* p = ::mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    MINIPS_CHECK(p != MAP_FAILED, "mmap failed for " << path);
    ::madvise(p, size_, MADV_SEQUENTIAL);
    data_ = static_cast<const char*>(p);
  }
}

MappedFile::~MappedFile() {
  if (data_) ::munmap(const_cast<char*>(data_), size_);
  if (fd_ >= 0) ::close(fd_);
}

LineInputFormat::LineInputFormat(const MappedFile& f, const FileBlock& b)
    : base_(f.data()), pos_(b.offset), end_(b.offset + b.size), file_size_(f.size()) {
  // A line belongs to the block in which it starts: unless this block begins a file or right
  // after a newline, skip the partial first line (the previous block reads it to its end).
  if (pos_ > 0 && pos_ < file_size_ && base_[pos_ - 1] != '\n') {
    const void* nl = std::memchr(base_ + pos_, '\n', file_size_ - pos_);
    pos_ = nl ? (uint64_t)(static_cast<const char*>(nl) - base_) + 1 : file_size_;
  }
}

bool LineInputFormat::Next(const char** line, size_t* len) {
  if (pos_ >= end_ || pos_ >= file_size_) return false;  // lines starting past the block belong to the next
  const void* nl = std::memchr(base_ + pos_, '\n', file_size_ - pos_);
  const uint64_t e = nl ? (uint64_t)(static_cast<const char*>(nl) - base_) : file_size_;
  *line = base_ + pos_;
  *len = (size_t)(e - pos_);
  pos_ = e + 1;
  return true;
}

uint64_t LoadLines(const std::vector<std::string>& paths, uint64_t block_size, int rank, int num_ranks,
                   int num_threads, const std::function<void(const char*, size_t, int)>& udf) {
  BlockAssigner assigner(SplitFiles(paths, block_size), rank, num_ranks);
  std::atomic<uint64_t> lines{0};
  std::vector<std::thread> th;
  std::mutex err_mu;
  std::string err;
  num_threads = std::max(1, num_threads);
  for (int t = 0; t < num_threads; ++t) {
    th.emplace_back([&, t] {
      try {
        std::string cur_path;
        std::unique_ptr<MappedFile> mf;
        while (auto b = assigner.Next()) {  // kBlockRequest
          if (b->path != cur_path) {
            mf.reset(new MappedFile(b->path));
            cur_path = b->path;
          }
          LineInputFormat in(*mf, *b);
          const char* l;
          size_t n;
          while (in.Next(&l, &n)) {
            udf(l, n, t);
            lines++;
          }
        }  // kExit
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> lk(err_mu);
        err = e.what();
      }
    });
  }
  for (auto& x : th) x.join();
  MINIPS_CHECK(err.empty(), "loader failed: " << err);
  return lines.load();
}

}  // namespace minips
