// File systems behind every path the runtime reads or writes: input data, checkpoints, config,
// hostfiles.
//
// Parity: base/third_party/general_fstream.{hpp,cpp} (one stream type that dispatches
// `hdfs://host:port/path` to HDFS and everything else to the local file system, parse_hdfs_url
// :18-59), base/third_party/hdfs.{hpp,cpp} (libhdfs3 device, connection pool keyed by host:port
// :43-61) and cmake/dep.cmake:3-25 (the optional libhdfs3 probe).
//
// Design (MI355X build):
//   * one FileSystem interface with random-access reads (ReadAt) -- loader threads read whole
//     blocks with one call instead of streaming through a boost device, and block locations are
//     part of the interface (the locality-aware assigner in io.h needs them);
//   * `file://` and plain paths: POSIX pread/mmap;
//   * `webhdfs://host:port/path`: the namenode's WebHDFS REST API spoken directly over a TCP
//     socket (HTTP/1.1, 307 redirects to the datanodes, JSON FileStatus / BlockLocations). This
//     needs no Hadoop client library at all, so HDFS input works in this image;
//   * `hdfs://host:port/path`: the native RPC protocol through libhdfs3 when the library is
//     present. It is probed at run time with dlopen (libhdfs3.so, or $MINIPS_LIBHDFS3) instead of
//     at build time, so the runtime never carries a hard dependency on it; without it, an hdfs://
//     URL fails with a message naming the webhdfs:// alternative (MINIPS_HDFS_HTTP_PORT maps
//     hdfs://host:port to webhdfs://host:<http port> instead when set).
#pragma once

#include <cstdint>
#include <istream>
#include <memory>
#include <ostream>
#include <streambuf>
#include <string>
#include <vector>

#include "base.h"

namespace minips {

struct Url {
  std::string scheme;  // "" (local), "file", "hdfs", "webhdfs", "http"
  std::string host;
  int port = 0;
  std::string path;   // absolute path (no query)
  std::string query;  // after '?', http only
  std::string ToString() const;
};
// `hdfs://nn:9000/a/b`, `webhdfs://nn:9870/a`, `file:///a`, `/a`, `a/b` (relative local).
Url ParseUrl(const std::string& url);

struct FileStat {
  std::string url;  // full URL of the file (same scheme/authority as the query)
  uint64_t size = 0;
  uint64_t block_size = 0;  // the file system's block size (HDFS dfs.blocksize); 0 = none
  bool is_dir = false;
};

struct BlockLocation {
  uint64_t offset = 0, length = 0;
  std::vector<std::string> hosts;  // hosts holding a replica
};

class RandomAccessFile {
 public:
  virtual ~RandomAccessFile() = default;
  virtual uint64_t Size() const = 0;
  // Reads up to n bytes at `offset`; returns the count (short only at end of file).
  virtual size_t ReadAt(uint64_t offset, char* buf, size_t n) = 0;
};

class WritableFile {
 public:
  virtual ~WritableFile() = default;
  virtual void Append(const char* data, size_t n) = 0;
  virtual void Close() = 0;  // flushes; throws on failure
};

class FileSystem {
 public:
  virtual ~FileSystem() = default;
  virtual std::string Name() const = 0;
  virtual FileStat Stat(const std::string& url) = 0;
  virtual bool Exists(const std::string& url) = 0;
  // Regular files of a directory (sorted by name), or the file itself.
  virtual std::vector<FileStat> List(const std::string& url) = 0;
  // Replica hosts of every block of a file (one entry per block, in offset order).
  virtual std::vector<BlockLocation> Locations(const FileStat& f) = 0;
  virtual std::unique_ptr<RandomAccessFile> OpenRead(const std::string& url) = 0;
  virtual std::unique_ptr<WritableFile> OpenWrite(const std::string& url) = 0;
  virtual void MakeDirs(const std::string& url) = 0;
  virtual void Rename(const std::string& from, const std::string& to) = 0;
  virtual void Remove(const std::string& url) = 0;

  // The file system serving `url` (shared instance per scheme + authority).
  static FileSystem& For(const std::string& url);
};

// This host's name as the locality-aware assigner compares it with block replica hosts.
std::string LocalHostName();

// libhdfs3 run-time probe (dlopen); the error text when unavailable.
bool LibHdfs3Available(std::string* why = nullptr);

// general_fstream conveniences.
std::string ReadFileToString(const std::string& url);
void WriteStringToFile(const std::string& url, const std::string& data);
bool IsLocalUrl(const std::string& url);

// general_fstream: std::istream / std::ostream over any FileSystem URL (buffered; the input
// stream also seeks). `good()` is false on a stream whose file could not be opened.
class FsReadBuf : public std::streambuf {
 public:
  explicit FsReadBuf(std::unique_ptr<RandomAccessFile> f, size_t buf = 1 << 20) : f_(std::move(f)), buf_(buf) {}

 protected:
  int_type underflow() override;
  pos_type seekoff(off_type off, std::ios_base::seekdir dir, std::ios_base::openmode) override;
  pos_type seekpos(pos_type pos, std::ios_base::openmode m) override { return seekoff(pos, std::ios_base::beg, m); }

 private:
  std::unique_ptr<RandomAccessFile> f_;
  std::vector<char> buf_;
  uint64_t base_ = 0;  // file offset of buf_[0]
};

class FsWriteBuf : public std::streambuf {
 public:
  explicit FsWriteBuf(std::unique_ptr<WritableFile> f, size_t buf = 1 << 20);
  ~FsWriteBuf() override;
  bool Close();  // false when a write or the flush failed

 protected:
  int_type overflow(int_type c) override;
  int sync() override;

 private:
  bool Drain();
  std::unique_ptr<WritableFile> f_;
  std::vector<char> buf_;
  bool failed_ = false;
};

class GeneralIfstream : public std::istream {
 public:
  explicit GeneralIfstream(const std::string& url);

 private:
  std::unique_ptr<FsReadBuf> sb_;
};

class GeneralOfstream : public std::ostream {
 public:
  explicit GeneralOfstream(const std::string& url);
  ~GeneralOfstream() override;
  void close();

 private:
  std::unique_ptr<FsWriteBuf> sb_;
};

// Bytes moved through the remote (WebHDFS/libhdfs3) backends -- test and metrics hook.
uint64_t RemoteBytesRead();

}  // namespace minips
