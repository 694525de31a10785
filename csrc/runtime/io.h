// Data ingest over local files (reference io/: HDFSManager, Coordinator, HDFSBlockAssigner,
// HDFSFileSplitter, LineInputFormat; lib/abstract_data_loader.hpp, lib/abstract_aync_data_loader.hpp).
//
//   FileBlock / SplitFiles    files cut into fixed-size byte blocks (hdfs_block_size analogue)
//   BlockAssigner             thread-safe work queue of blocks, handed out one per request
//                             (the assigner's kBlockRequest / kExit protocol, in-process); a
//                             rank takes the blocks b with b % num_ranks == rank ("rank r reads
//                             shard r") and its loader threads pull from that queue
//   MappedFile + LineInputFormat
//                             mmap'd block reader; a line belongs to the block where it STARTS,
//                             so lines straddling a block boundary are read exactly once
//                             (line_input_format.hpp:43-131)
//   LoadLines                 N loader threads x assigner x UDF (AbstractDataLoader::load)
//   AsyncReadBuffer<T>        bounded producer/consumer prefetch queue filled by a background
//                             thread (the reference's empty AbstractAsyncDataLoader, implemented)
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <optional>
#include <string>
#include <thread>
#include <vector>

#include "base.h"

namespace minips {

struct FileBlock {
  std::string path;
  uint64_t offset = 0;
  uint64_t size = 0;
  uint64_t file_size = 0;
  int id = 0;
};

// Cuts every file into blocks of `block_size` bytes (the last block of a file is shorter).
std::vector<FileBlock> SplitFiles(const std::vector<std::string>& paths, uint64_t block_size);
// Expands a path, a directory (all regular files, sorted) or a comma-separated list.
std::vector<std::string> ListInputFiles(const std::string& spec);

class BlockAssigner {
 public:
  BlockAssigner(std::vector<FileBlock> blocks, int rank = 0, int num_ranks = 1);
  std::optional<FileBlock> Next();  // nullopt when this rank's blocks are exhausted
  size_t Remaining();
  int Served() const { return served_.load(); }

 private:
  std::mutex mu_;
  std::deque<FileBlock> queue_;
  std::atomic<int> served_{0};
};

class MappedFile {
 public:
  explicit MappedFile(const std::string& path);
  ~MappedFile();
  MappedFile(const MappedFile&) = delete;
  MappedFile& operator=(const MappedFile&) = delete;
  const char* data() const { return data_; }
  uint64_t size() const { return size_; }

 private:
  const char* data_ = nullptr;
  uint64_t size_ = 0;
  int fd_ = -1;
};

class LineInputFormat {
 public:
  LineInputFormat(const MappedFile& f, const FileBlock& b);
  // Next line (without '\n') of this block; false at the end of the block.
  bool Next(const char** line, size_t* len);

 private:
  const char* base_;
  uint64_t pos_, end_, file_size_;
};

// Runs `udf(line, len, thread_index)` on every line of this rank's blocks with `num_threads`
// loader threads; returns the number of lines.
uint64_t LoadLines(const std::vector<std::string>& paths, uint64_t block_size, int rank, int num_ranks,
                   int num_threads, const std::function<void(const char*, size_t, int)>& udf);

template <typename T>
class AsyncReadBuffer {
 public:
  // `produce(out)` fills one item and returns false at the end of the stream.
  AsyncReadBuffer(std::function<bool(T*)> produce, size_t capacity)
      : produce_(std::move(produce)), capacity_(capacity ? capacity : 1) {
    th_ = std::thread([this] { Loop(); });
  }
  ~AsyncReadBuffer() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  // Blocks for the next item; false at the end of the stream.
  bool Get(T* out) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return !q_.empty() || done_; });
    if (q_.empty()) return false;
    *out = std::move(q_.front());
    q_.pop_front();
    cv_.notify_all();
    return true;
  }
  size_t Buffered() {
    std::lock_guard<std::mutex> lk(mu_);
    return q_.size();
  }

 private:
  void Loop() {
    for (;;) {
      T item;
      bool ok = produce_(&item);
      std::unique_lock<std::mutex> lk(mu_);
      if (!ok) {
        done_ = true;
        cv_.notify_all();
        return;
      }
      cv_.wait(lk, [&] { return q_.size() < capacity_ || stop_; });
      if (stop_) return;
      q_.push_back(std::move(item));
      cv_.notify_all();
    }
  }
  std::function<bool(T*)> produce_;
  size_t capacity_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<T> q_;
  bool done_ = false, stop_ = false;
  std::thread th_;
};

}  // namespace minips
