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
//
// Format v2 (scales to multi-hundred-GB shards, e.g. a 10B-row embedding table over 8 GPUs):
// the header lists every array with its file offset (4 KiB aligned), so
//   * a writer streams an array in row chunks (ShardFileWriter::WriteRows -> pwrite) from a
//     bounded pinned ring, never holding a whole shard in host memory;
//   * a reader parses the header only (ReadShardHeader) and preads exactly the rows of the
//     global range it owns (ReadRows), so an N -> M reshard reads each byte once in total
//     instead of every rank reading every file.
// ShardBytesRead() counts the payload bytes read by this process (tests assert read
// amplification with it).
#pragma once

#include <memory>

#include "fs.h"

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

struct ArrayDesc {  // header entry of one array in a v2 shard file
  std::string name;
  DType dtype = DType::kF32;
  uint64_t rows = 0, cols = 1, bytes = 0, offset = 0;
};

struct ShardHeader {
  ShardMeta meta;
  std::vector<ArrayDesc> arrays;
};

struct LoadedShard {
  ShardMeta meta;
  std::vector<LoadedArray> arrays;
};

// Synchronous writers / readers.
void WriteShard(const std::string& path, const ShardMeta& meta, const std::vector<ArrayRef>& arrays);
LoadedShard ReadShard(const std::string& path);  // whole file (small shards, tools)
ShardHeader ReadShardHeader(const std::string& path);
// Reads rows [row0, row0 + nrows) of the array at `offset` (row_bytes each) into dst.
void ReadRows(const std::string& path, uint64_t offset, uint64_t row_bytes, uint64_t row0, uint64_t nrows, void* dst);
uint64_t ShardBytesRead();
void ResetShardBytesRead();

// Streaming writer of one v2 shard file: the header (with every array's offset) is written on
// construction into "<path>.tmp", rows arrive in any order by pwrite, Close() renames the file
// into place (a crash never leaves a truncated file under the real name).
class ShardFileWriter {
 public:
  ShardFileWriter(const std::string& path, const ShardMeta& meta, const std::vector<ArrayDesc>& arrays);
  ~ShardFileWriter();
  void WriteRows(int array, uint64_t row0, const void* src, uint64_t nrows);
  void Close();
  const std::vector<ArrayDesc>& arrays() const { return arrays_; }

 private:
  std::string path_, tmp_;
  std::vector<ArrayDesc> arrays_;
  int fd_ = -1;
};
// Reference text format of one array: "<local_idx>:<val> " for non-zero entries, one line.
void WriteTextParams(const std::string& path, const ArrayRef& a);
// The same format written in pieces (a shard streamed through the checkpoint ring): every
// Append continues the running element index; any FileSystem URL (local, webhdfs://, hdfs://).
class TextParamsWriter {
 public:
  explicit TextParamsWriter(const std::string& path);
  ~TextParamsWriter();
  void Append(const ArrayRef& a);
  void Close();
  uint64_t Elements() const { return next_; }

 private:
  std::string path_;
  std::unique_ptr<GeneralOfstream> out_;
  std::string buf_;
  uint64_t next_ = 0;
};
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
