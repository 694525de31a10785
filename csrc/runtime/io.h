// Data ingest (reference io/: HDFSManager, Coordinator, HDFSBlockAssigner, HDFSFileSplitter,
// LineInputFormat; lib/abstract_data_loader.hpp, lib/abstract_aync_data_loader.hpp).
//
//   ListInputs / SplitInputs  files of a path / directory / comma list on any FileSystem (fs.h:
//                             local, webhdfs://, hdfs://) cut into byte blocks, each carrying the
//                             hosts that store a replica of it (browse_hdfs,
//                             io/hdfs_assigner.cpp:124-155)
//   BlockAssigner             static partition: rank r takes the blocks b with b % n == r
//   LocalityAssigner          the reference's locality rule (io/hdfs_assigner.cpp:160-222): a
//                             requester gets a block stored on its own host while any is left,
//                             otherwise one from the host with the most unassigned blocks; a
//                             chosen block leaves the lists of all its replica hosts
//   BlockAssignerServer       the assigner as a TCP service on the master (HDFSBlockAssigner::
//                             Serve, kBlockRequest=301 / kExit=300; it halts once every loader
//                             thread has exited), one LocalityAssigner per (job id, input url)
//   Coordinator               the loader-side client (io/coordinator.cpp:48-81 ask_master /
//                             notify_master), one connection per loader thread
//   LineInputFormat           line reader over a window of a file; a line belongs to the block
//                             where it STARTS, so lines straddling a block boundary are read
//                             exactly once (line_input_format.hpp:43-131). Local blocks are read
//                             through mmap, remote ones with one ranged read (plus the tail of
//                             the last line) into a buffer.
//   ForEachLine / LoadLines   N loader threads x (static | coordinated) blocks x UDF
//                             (AbstractDataLoader::load, HDFSManager::Run)
//   AsyncReadBuffer<T>        bounded producer/consumer prefetch queue filled by a background
//                             thread (the reference's empty AbstractAsyncDataLoader, implemented)
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <optional>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "base.h"
#include "fs.h"

namespace minips {

struct FileBlock {
  std::string path;  // URL of the file
  uint64_t offset = 0;
  uint64_t size = 0;
  uint64_t file_size = 0;
  int id = 0;
  std::vector<std::string> hosts;  // replica hosts (empty when not located)
};

// Files of a path, a directory (regular files, sorted) or a comma-separated list, any scheme.
std::vector<FileStat> ListInputs(const std::string& spec);
std::vector<std::string> ListInputFiles(const std::string& spec);
// Cuts every file into blocks of `block_size` bytes (0: the file system's block size, HDFS
// dfs.blocksize, else 64 MiB); `locate` fills FileBlock::hosts from the block locations.
std::vector<FileBlock> SplitInputs(const std::vector<FileStat>& files, uint64_t block_size, bool locate = false);
std::vector<FileBlock> SplitFiles(const std::vector<std::string>& paths, uint64_t block_size);

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

class LocalityAssigner {
 public:
  explicit LocalityAssigner(std::vector<FileBlock> blocks);
  // Not thread-safe (the server serialises requests).
  std::optional<FileBlock> Next(const std::string& host);
  size_t Remaining() const { return remaining_; }
  uint64_t LocalServed() const { return local_; }
  uint64_t RemoteServed() const { return remote_; }

 private:
  void Take(int b);
  std::vector<FileBlock> blocks_;
  std::vector<char> taken_;
  std::map<std::string, std::deque<int>> by_host_;  // lazily purged of taken blocks
  std::map<std::string, size_t> left_;              // unassigned blocks per host
  std::deque<int> unlocated_;                       // blocks with no replica host
  size_t remaining_ = 0;
  uint64_t local_ = 0, remote_ = 0;
};

class BlockAssignerServer {
 public:
  static constexpr int32_t kExit = 300;
  static constexpr int32_t kBlockRequest = 301;
  // `port` 0 binds an ephemeral port (Port() tells which).
  explicit BlockAssignerServer(int port = 0);
  ~BlockAssignerServer();
  void Start();
  void Stop();
  int Port() const { return port_; }
  // True once every loader thread announced in the requests has sent kExit.
  bool WaitDone(double timeout_s);
  uint64_t LocalServed() const { return local_.load(); }
  uint64_t RemoteServed() const { return remote_.load(); }

 private:
  void Loop();
  bool Handle(int fd);
  std::string Answer(const std::string& body);
  int listen_fd_ = -1, port_ = 0;
  int wake_[2] = {-1, -1};
  std::thread th_;
  std::atomic<bool> running_{false};
  std::mutex mu_;
  std::condition_variable cv_;
  // (job id, url) -> assigner + rejected-request count (the reference's finish_multi_dict_)
  std::map<std::pair<int, std::string>, std::pair<std::unique_ptr<LocalityAssigner>, int>> jobs_;
  std::set<std::string> finished_;
  int workers_alive_ = -1;
  bool done_ = false;
  std::atomic<uint64_t> local_{0}, remote_{0};
};

class Coordinator {
 public:
  Coordinator(const std::string& master_host, int master_port, std::string name);
  ~Coordinator();
  // kBlockRequest: the next block of input `url` for a loader on `host`; `num_workers` is the
  // total number of loader threads of the job (the server halts after that many kExit).
  std::optional<FileBlock> AskBlock(const std::string& url, const std::string& host, int num_workers, int job_id,
                                    uint64_t block_size);
  void NotifyExit(int job_id);

 private:
  std::string Call(const std::string& payload);
  int fd_ = -1;
  std::string name_;
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
  // `window` holds file bytes [window_offset, window_offset + window_len): the byte before the
  // block (when it has one) through the newline that ends the block's last line (or EOF).
  LineInputFormat(const char* window, uint64_t window_offset, uint64_t window_len, const FileBlock& b);
  LineInputFormat(const MappedFile& f, const FileBlock& b);
  // Next line (without '\n') of this block; false at the end of the block.
  bool Next(const char** line, size_t* len);

 private:
  const char* At(uint64_t file_pos) const { return base_ + (file_pos - win_off_); }
  const char* base_;
  uint64_t win_off_, win_end_, pos_, end_;
};

// Reads one block of a remote file into `buf` as the window LineInputFormat needs.
LineInputFormat ReadBlockWindow(RandomAccessFile* f, const FileBlock& b, std::string* buf);

struct LoadOptions {
  uint64_t block_size = 0;  // 0: local inputs ~4 blocks per thread and rank (>= 64 KiB); remote:
                            // the file system's block size
  int rank = 0, num_ranks = 1;  // static partition (no assigner)
  int num_threads = 4;
  std::string assigner;  // "host:port" of a BlockAssignerServer: coordinated, locality-aware
  std::string host;      // this loader's host for locality ("" = LocalHostName())
  int job_id = 0;
};

// Runs `udf(block, line, len, thread_index)` on every line of the blocks this rank is handed;
// returns the number of lines.
uint64_t ForEachLine(const std::string& inputs, const LoadOptions& opt,
                     const std::function<void(const FileBlock&, const char*, size_t, int)>& udf);
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
