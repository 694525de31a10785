#include "io.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <memory>
#include <sstream>

#include "serialization.h"

namespace minips {

// ------------------------------------------------------------------------------------------
// Listing and splitting
// ------------------------------------------------------------------------------------------
std::vector<FileStat> ListInputs(const std::string& spec) {
  std::vector<FileStat> out;
  std::stringstream ss(spec);
  std::string item;
  while (std::getline(ss, item, ',')) {
    if (item.empty()) continue;
    FileSystem& fs = FileSystem::For(item);
    MINIPS_CHECK(fs.Exists(item), "no such input " << item);
    auto files = fs.List(item);
    out.insert(out.end(), files.begin(), files.end());
  }
  return out;
}

std::vector<std::string> ListInputFiles(const std::string& spec) {
  std::vector<std::string> out;
  for (auto& f : ListInputs(spec)) out.push_back(f.url);
  return out;
}

std::vector<FileBlock> SplitInputs(const std::vector<FileStat>& files, uint64_t block_size, bool locate) {
  std::vector<FileBlock> blocks;
  int id = 0;
  for (const auto& f : files) {
    const uint64_t bs = block_size ? block_size : (f.block_size ? f.block_size : (64ull << 20));
    std::vector<BlockLocation> locs;
    if (locate && f.size) locs = FileSystem::For(f.url).Locations(f);
    size_t li = 0;
    for (uint64_t off = 0; off < f.size; off += bs) {
      FileBlock b{f.url, off, std::min(bs, f.size - off), f.size, id++, {}};
      while (li + 1 < locs.size() && locs[li].offset + locs[li].length <= off) ++li;
      if (li < locs.size() && locs[li].offset <= off) b.hosts = locs[li].hosts;
      blocks.push_back(std::move(b));
    }
  }
  return blocks;
}

std::vector<FileBlock> SplitFiles(const std::vector<std::string>& paths, uint64_t block_size) {
  MINIPS_CHECK(block_size > 0, "block_size must be positive");
  std::vector<FileStat> files;
  for (auto& p : paths) files.push_back(FileSystem::For(p).Stat(p));
  return SplitInputs(files, block_size, false);
}

// ------------------------------------------------------------------------------------------
// Assigners
// ------------------------------------------------------------------------------------------
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

LocalityAssigner::LocalityAssigner(std::vector<FileBlock> blocks) : blocks_(std::move(blocks)) {
  taken_.assign(blocks_.size(), 0);
  remaining_ = blocks_.size();
  for (int b = 0; b < (int)blocks_.size(); ++b) {
    if (blocks_[b].hosts.empty()) unlocated_.push_back(b);
    for (auto& h : blocks_[b].hosts) {
      by_host_[h].push_back(b);
      left_[h]++;
    }
  }
}

void LocalityAssigner::Take(int b) {
  taken_[b] = 1;
  remaining_--;
  for (auto& h : blocks_[b].hosts) left_[h]--;  // the block leaves every replica host's list
}

std::optional<FileBlock> LocalityAssigner::Next(const std::string& host) {
  auto pop = [&](std::deque<int>& q) -> int {
    while (!q.empty()) {
      const int b = q.front();
      q.pop_front();
      if (!taken_[b]) return b;
    }
    return -1;
  };
  auto it = by_host_.find(host);
  if (it != by_host_.end()) {
    const int b = pop(it->second);
    if (b >= 0) {
      Take(b);
      local_++;
      return blocks_[b];
    }
  }
  int b = pop(unlocated_);
  if (b < 0) {  // no local block left: take one from the host with the most unassigned blocks
    const std::string* best = nullptr;
    size_t most = 0;
    for (auto& kv : left_)
      if (kv.second > most) {
        most = kv.second;
        best = &kv.first;
      }
    if (best) b = pop(by_host_[*best]);
  }
  if (b < 0) return std::nullopt;
  Take(b);
  remote_++;
  return blocks_[b];
}

// ------------------------------------------------------------------------------------------
// Assigner service (length-prefixed BinStream frames over TCP)
// ------------------------------------------------------------------------------------------
namespace {

bool SendFrame(int fd, const std::string& payload) {
  const uint32_t n = (uint32_t)payload.size();
  std::string buf(reinterpret_cast<const char*>(&n), 4);
  buf += payload;
  const char* p = buf.data();
  size_t left = buf.size();
  while (left > 0) {
    ssize_t w = ::send(fd, p, left, MSG_NOSIGNAL);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return false;
    p += w;
    left -= (size_t)w;
  }
  return true;
}

bool RecvExact(int fd, char* p, size_t n) {
  while (n > 0) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    p += r;
    n -= (size_t)r;
  }
  return true;
}

bool RecvFrame(int fd, std::string* payload) {
  uint32_t n = 0;
  if (!RecvExact(fd, reinterpret_cast<char*>(&n), 4)) return false;
  payload->resize(n);
  return n == 0 || RecvExact(fd, &(*payload)[0], n);
}

std::string ToString(const BinStream& s) { return std::string(s.data(), s.size()); }

}  // namespace

BlockAssignerServer::BlockAssignerServer(int port) : port_(port) {}

BlockAssignerServer::~BlockAssignerServer() { Stop(); }

void BlockAssignerServer::Start() {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  MINIPS_CHECK(listen_fd_ >= 0, "socket() failed");
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_addr.s_addr = htonl(INADDR_ANY);
  addr.sin_port = htons((uint16_t)port_);
  MINIPS_CHECK(::bind(listen_fd_, (sockaddr*)&addr, sizeof(addr)) == 0,
               "block assigner cannot bind port " << port_ << " errno=" << errno);
  MINIPS_CHECK(::listen(listen_fd_, 256) == 0, "listen failed");
  socklen_t len = sizeof(addr);
  ::getsockname(listen_fd_, (sockaddr*)&addr, &len);
  port_ = ntohs(addr.sin_port);
  MINIPS_CHECK(::pipe(wake_) == 0, "pipe failed");
  running_ = true;
  th_ = std::thread([this] { Loop(); });
}

void BlockAssignerServer::Stop() {
  if (!running_.exchange(false)) return;
  char c = 'x';
  (void)!::write(wake_[1], &c, 1);
  th_.join();
  ::close(listen_fd_);
  ::close(wake_[0]);
  ::close(wake_[1]);
}

bool BlockAssignerServer::WaitDone(double timeout_s) {
  std::unique_lock<std::mutex> lk(mu_);
  return CondWaitFor(cv_, lk, timeout_s, [&] { return done_; });
}

void BlockAssignerServer::Loop() {
  std::vector<int> clients;
  while (running_) {
    std::vector<pollfd> fds{{wake_[0], POLLIN, 0}, {listen_fd_, POLLIN, 0}};
    for (int c : clients) fds.push_back({c, POLLIN, 0});
    if (::poll(fds.data(), fds.size(), 1000) < 0) continue;
    if (fds[0].revents) break;
    // requests are answered one at a time, in arrival order (the reference's single ROUTER)
    std::vector<int> keep;
    for (size_t i = 2; i < fds.size(); ++i) {
      const int c = fds[i].fd;
      if (fds[i].revents && !Handle(c)) {
        ::close(c);
        continue;
      }
      keep.push_back(c);
    }
    if (fds[1].revents & POLLIN) {
      int c = ::accept(listen_fd_, nullptr, nullptr);
      if (c >= 0) {
        int one = 1;
        setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        // a client that stalls inside a frame is dropped after 30 s instead of blocking the
        // single-threaded service (every other loader waits on it)
        timeval tv{30, 0};
        setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
        setsockopt(c, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
        keep.push_back(c);
      }
    }
    clients.swap(keep);
  }
  for (int c : clients) ::close(c);
}

bool BlockAssignerServer::Handle(int fd) {
  std::string req;
  if (!RecvFrame(fd, &req)) return false;
  std::string rep;
  try {
    rep = Answer(req);
  } catch (const std::exception& e) {
    BinStream s;
    s << (int32_t)-1 << std::string(e.what());
    rep = ToString(s);
  }
  return SendFrame(fd, rep);
}

std::string BlockAssignerServer::Answer(const std::string& body) {
  BinStream in(body.data(), body.size()), out;
  int32_t type = 0;
  in >> type;
  std::lock_guard<std::mutex> lk(mu_);
  if (type == kExit) {
    std::string name;
    int32_t job = 0;
    in >> name >> job;
    finished_.insert(name);
    if (workers_alive_ > 0 && (int)finished_.size() >= workers_alive_) {
      done_ = true;
      cv_.notify_all();
    }
    out << (int32_t)0;
    return ToString(out);
  }
  MINIPS_CHECK(type == kBlockRequest, "unknown assigner message " << type);
  std::string url, host;
  int32_t num_workers = 0, job = 0;
  uint64_t block_size = 0;
  in >> url >> host >> num_workers >> job >> block_size;
  workers_alive_ = num_workers;  // reset per request (handle_block_request)
  auto key = std::make_pair((int)job, url);
  auto it = jobs_.find(key);
  if (it == jobs_.end()) {  // browse: list + locate the input once per (job, url)
    auto blocks = SplitInputs(ListInputs(url), block_size, true);
    it = jobs_.emplace(key, std::make_pair(std::unique_ptr<LocalityAssigner>(new LocalityAssigner(blocks)), 0)).first;
  }
  LocalityAssigner& a = *it->second.first;
  const uint64_t l0 = a.LocalServed(), r0 = a.RemoteServed();
  auto b = a.Next(host);
  local_ += a.LocalServed() - l0;
  remote_ += a.RemoteServed() - r0;
  if (!b) {
    // every worker has been turned away: the url is fully assigned; forget it so a later pass
    // (next epoch, reload after recovery) browses it again
    if (++it->second.second >= num_workers) jobs_.erase(it);
    out << (int32_t)0;
    return ToString(out);
  }
  out << (int32_t)1 << b->path << b->offset << b->size << b->file_size << (int32_t)b->id;
  return ToString(out);
}

Coordinator::Coordinator(const std::string& master_host, int master_port, std::string name) : name_(std::move(name)) {
  const std::string host = master_host == "localhost" ? "127.0.0.1" : master_host;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(60);
  for (;;) {  // the master may still be starting its assigner
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(master_port).c_str(), &hints, &res) == 0 && res) {
      fd_ = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
      const bool ok = fd_ >= 0 && ::connect(fd_, res->ai_addr, res->ai_addrlen) == 0;
      freeaddrinfo(res);
      if (ok) break;
      if (fd_ >= 0) ::close(fd_);
      fd_ = -1;
    }
    MINIPS_CHECK(std::chrono::steady_clock::now() < deadline,
                 "cannot reach the block assigner at " << master_host << ":" << master_port);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  int one = 1;
  setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

Coordinator::~Coordinator() {
  if (fd_ >= 0) ::close(fd_);
}

std::string Coordinator::Call(const std::string& payload) {
  std::string rep;
  MINIPS_CHECK(SendFrame(fd_, payload) && RecvFrame(fd_, &rep), "block assigner connection lost");
  return rep;
}

std::optional<FileBlock> Coordinator::AskBlock(const std::string& url, const std::string& host, int num_workers,
                                               int job_id, uint64_t block_size) {
  BinStream req;
  req << BlockAssignerServer::kBlockRequest << url << host << (int32_t)num_workers << (int32_t)job_id << block_size;
  const std::string rep = Call(ToString(req));
  BinStream in(rep.data(), rep.size());
  int32_t found = 0;
  in >> found;
  if (found < 0) {
    std::string err;
    in >> err;
    throw CheckError("block assigner: " + err);
  }
  if (!found) return std::nullopt;
  FileBlock b;
  int32_t id = 0;
  in >> b.path >> b.offset >> b.size >> b.file_size >> id;
  b.id = id;
  return b;
}

void Coordinator::NotifyExit(int job_id) {
  BinStream req;
  req << BlockAssignerServer::kExit << name_ << (int32_t)job_id;
  Call(ToString(req));
}

// ------------------------------------------------------------------------------------------
// Block readers
// ------------------------------------------------------------------------------------------
MappedFile::MappedFile(const std::string& url) {
  const std::string path = ParseUrl(url).path;
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

LineInputFormat::LineInputFormat(const char* window, uint64_t window_offset, uint64_t window_len, const FileBlock& b)
    : base_(window), win_off_(window_offset), win_end_(window_offset + window_len), pos_(b.offset),
      end_(b.offset + b.size) {
  // A line belongs to the block in which it starts: unless this block begins a file or right
  // after a newline, skip the partial first line (the previous block reads it to its end).
  if (pos_ > 0 && pos_ < win_end_) {
    MINIPS_CHECK(pos_ - 1 >= win_off_, "block window lacks the byte before the block");
    if (*At(pos_ - 1) != '\n') {
      const void* nl = std::memchr(At(pos_), '\n', win_end_ - pos_);
      pos_ = nl ? (uint64_t)(static_cast<const char*>(nl) - base_) + win_off_ + 1 : win_end_;
    }
  }
}

LineInputFormat::LineInputFormat(const MappedFile& f, const FileBlock& b) : LineInputFormat(f.data(), 0, f.size(), b) {}

bool LineInputFormat::Next(const char** line, size_t* len) {
  if (pos_ >= end_ || pos_ >= win_end_) return false;  // lines starting past the block belong to the next
  const void* nl = std::memchr(At(pos_), '\n', win_end_ - pos_);
  const uint64_t e = nl ? (uint64_t)(static_cast<const char*>(nl) - base_) + win_off_ : win_end_;
  *line = At(pos_);
  *len = (size_t)(e - pos_);
  pos_ = e + 1;
  return true;
}

LineInputFormat ReadBlockWindow(RandomAccessFile* f, const FileBlock& b, std::string* buf) {
  const uint64_t start = b.offset > 0 ? b.offset - 1 : 0;
  const uint64_t fsize = f->Size();
  uint64_t want = std::min(fsize, b.offset + b.size) - start;
  buf->resize(want);
  size_t got = want ? f->ReadAt(start, &(*buf)[0], want) : 0;
  MINIPS_CHECK(got == want, "short read of " << b.path << " @" << start);
  // extend through the newline that ends the last line starting inside the block
  uint64_t scan = (b.offset + b.size > start + 1) ? b.offset + b.size - 1 - start : 0;
  while (start + buf->size() < fsize) {
    if (scan < buf->size() && std::memchr(buf->data() + scan, '\n', buf->size() - scan)) break;
    scan = buf->size();
    const size_t chunk = (size_t)std::min<uint64_t>(64 << 10, fsize - start - buf->size());
    const size_t old = buf->size();
    buf->resize(old + chunk);
    got = f->ReadAt(start + old, &(*buf)[old], chunk);
    MINIPS_CHECK(got == chunk, "short read of " << b.path);
  }
  return LineInputFormat(buf->data(), start, buf->size(), b);
}

// ------------------------------------------------------------------------------------------
// Loader
// ------------------------------------------------------------------------------------------
uint64_t ForEachLine(const std::string& inputs, const LoadOptions& opt,
                     const std::function<void(const FileBlock&, const char*, size_t, int)>& udf) {
  const auto files = ListInputs(inputs);
  bool all_local = true;
  uint64_t total = 0;
  for (auto& f : files) {
    all_local = all_local && IsLocalUrl(f.url);
    total += f.size;
  }
  const int threads = std::max(1, opt.num_threads);
  uint64_t bs = opt.block_size;
  if (bs == 0 && all_local)  // ~4 blocks per loader thread and rank, at least 64 KiB
    bs = std::max<uint64_t>(64 << 10, total / std::max(1, 4 * threads * opt.num_ranks) + 1);
  std::unique_ptr<BlockAssigner> statics;
  std::string master_host;
  int master_port = 0;
  if (opt.assigner.empty()) {
    statics.reset(new BlockAssigner(SplitInputs(files, bs, false), opt.rank, opt.num_ranks));
  } else {
    const size_t c = opt.assigner.rfind(':');
    MINIPS_CHECK(c != std::string::npos, "assigner must be host:port, got " << opt.assigner);
    master_host = opt.assigner.substr(0, c);
    master_port = std::atoi(opt.assigner.c_str() + c + 1);
  }
  const std::string host = opt.host.empty() ? LocalHostName() : opt.host;
  std::atomic<uint64_t> lines{0};
  std::vector<std::thread> th;
  std::mutex err_mu;
  std::string err;
  for (int t = 0; t < threads; ++t) {
    th.emplace_back([&, t] {
      try {
        std::unique_ptr<Coordinator> coord;
        if (!statics)
          coord.reset(new Coordinator(master_host, master_port,
                                      host + "-" + std::to_string(::getpid()) + "-r" + std::to_string(opt.rank) +
                                          "-t" + std::to_string(t)));
        std::string cur;
        std::unique_ptr<MappedFile> mf;
        std::unique_ptr<RandomAccessFile> rf;
        std::string window;
        for (;;) {
          std::optional<FileBlock> b =
              statics ? statics->Next()
                      : coord->AskBlock(inputs, host, threads * opt.num_ranks, opt.job_id, bs);  // kBlockRequest
          if (!b) break;
          const bool local = IsLocalUrl(b->path);
          if (b->path != cur) {
            mf.reset();
            rf.reset();
            if (local) {
              mf.reset(new MappedFile(b->path));
            } else {
              rf = FileSystem::For(b->path).OpenRead(b->path);
            }
            cur = b->path;
          }
          LineInputFormat in = local ? LineInputFormat(*mf, *b) : ReadBlockWindow(rf.get(), *b, &window);
          const char* l;
          size_t n;
          while (in.Next(&l, &n)) {
            udf(*b, l, n, t);
            lines++;
          }
        }
        if (coord) coord->NotifyExit(opt.job_id);  // kExit
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

uint64_t LoadLines(const std::vector<std::string>& paths, uint64_t block_size, int rank, int num_ranks,
                   int num_threads, const std::function<void(const char*, size_t, int)>& udf) {
  std::string spec;
  for (auto& p : paths) spec += (spec.empty() ? "" : ",") + p;
  LoadOptions opt;
  opt.block_size = block_size;
  opt.rank = rank;
  opt.num_ranks = num_ranks;
  opt.num_threads = num_threads;
  return ForEachLine(spec, opt, [&](const FileBlock&, const char* l, size_t n, int t) { udf(l, n, t); });
}

}  // namespace minips
