// Checkpoint files of the GPU parameter-server shards.
//
// Every rank writes, per table, one binary sidecar
//     <prefix>server_params_<my_id>_t<table>.bin
// holding a fixed header and named arrays (the parameter rows plus optimizer state), and, when
// requested, the reference's text file <prefix>server_params_<my_id>[_t<table>] with
// "<local_idx>:<val> " for the non-zero entries of the first array (server/vector_storage.hpp:54-73;
// the reference Restore mis-parses that format -- ReadTextParams parses it correctly).
// Writes run on a background thread from host memory the caller keeps alive (pinned staging
// buffers the D2H copies landed in), so a checkpoint overlaps the next training steps.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace minips {

enum class DType : uint32_t { kF32 = 0, kBF16 = 1, kF64 = 2, kI64 = 3, kI32 = 4 };
size_t DTypeSize(DType t);

struct ArrayRef {
  std::string name;
  const void* data = nullptr;  // host memory, valid until the write completes
  DType dtype = DType::kF32;
  uint64_t rows = 0, cols = 1;
};

struct ShardMeta {
  uint64_t global_rows = 0;  // rows of the whole table (dense tables: elements, cols = 1)
  uint64_t base = 0;         // first global row of this shard
  uint64_t rows = 0;         // rows of this shard
  uint64_t cols = 1;
  int64_t clock = 0;         // table clock / optimizer step at the checkpoint
  int32_t table_id = 0;
  int32_t rank = 0;
  int32_t world = 1;
  std::string kind;          // "dense" | "sparse" | "hash"
};

struct LoadedArray {
  std::string name;
  DType dtype;
  uint64_t rows, cols;
  std::vector<char> bytes;
};

struct LoadedShard {
  ShardMeta meta;
  std::vector<LoadedArray> arrays;
};

// Synchronous writers / readers.
void WriteShard(const std::string& path, const ShardMeta& meta, const std::vector<ArrayRef>& arrays);
LoadedShard ReadShard(const std::string& path);
// Reference text format of one array: "<local_idx>:<val> " for non-zero entries, one line.
void WriteTextParams(const std::string& path, const ArrayRef& a);
// Parses the text format back into a dense vector of `n` values (missing entries = 0).
std::vector<double> ReadTextParams(const std::string& path, uint64_t n);

// Background writer: jobs run in submission order on one thread.
class AsyncShardWriter {
 public:
  AsyncShardWriter();
  ~AsyncShardWriter();
  // Returns a ticket; `done` (optional) runs on the writer thread after the job.
  uint64_t Submit(std::function<void()> job);
  void Wait(uint64_t ticket);  // blocks until the job with this ticket finished
  void WaitAll();
  // Error text of the last failed job ("" if none); cleared by the call.
  std::string TakeError();

 private:
  void Loop();
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<std::pair<uint64_t, std::function<void()>>> jobs_;
  uint64_t next_ = 1, finished_ = 0;
  bool stop_ = false;
  std::string error_;
  std::thread th_;
};

}  // namespace minips
