#include "ps_board.h"

#include <fcntl.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <ctime>
#include <thread>

#include "base.h"

namespace minips {

namespace {

constexpr uint64_t kBoardMagic = 0x4452414f42535041ull;  // "APSBOARD"

long FutexCall(std::atomic<uint32_t>* addr, int op, uint32_t val, const timespec* ts) {
  // shared futex (no FUTEX_PRIVATE_FLAG): the word lives in a segment mapped by several processes
  return ::syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), op, val, ts, nullptr, 0);
}

double Since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace

PSBoard::PSBoard(const std::string& name, int world, int rank, int tables, double attach_timeout_s)
    : world_(world), rank_(rank), tables_(tables), name_(name) {
  MINIPS_CHECK(world >= 1 && world <= kMaxWorld && rank >= 0 && rank < world,
               "ps board: bad rank " << rank << "/" << world << " (at most " << kMaxWorld << " ranks)");
  MINIPS_CHECK(tables >= 1 && tables <= kMaxTables, "ps board: tables " << tables);
  static_assert(sizeof(Header) == 64 && sizeof(SentLine) == 64 && sizeof(AppliedRow) == 128 && sizeof(LockLine) == 64,
                "board layout");
  bytes_ = sizeof(Header) + sizeof(SentLine) * (size_t)tables * world + sizeof(AppliedRow) * (size_t)tables * world +
           sizeof(LockLine) * (size_t)tables * world;
  const std::string path = "/dev/shm/" + name;
  int fd = -1;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(attach_timeout_s);
  // every rank may create: a new segment is zero-filled (all counters 0) and only ever grown to
  // the same size, so the order in which the ranks attach does not matter
  while ((fd = ::open(path.c_str(), O_RDWR | O_CREAT, 0600)) < 0) {
    MINIPS_CHECK(std::chrono::steady_clock::now() < deadline, "ps board: cannot open " << path);
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  struct stat st;
  MINIPS_CHECK(::fstat(fd, &st) == 0, "ps board: fstat " << path);
  if ((size_t)st.st_size < bytes_) MINIPS_CHECK(::ftruncate(fd, (off_t)bytes_) == 0, "ps board: ftruncate");
  void* p = ::mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  MINIPS_CHECK(p != MAP_FAILED, "ps board: mmap " << path);
  hdr_ = static_cast<Header*>(p);
  sent_ = reinterpret_cast<SentLine*>(static_cast<char*>(p) + sizeof(Header));
  applied_ = reinterpret_cast<AppliedRow*>(reinterpret_cast<char*>(sent_) + sizeof(SentLine) * (size_t)tables * world);
  locks_ = reinterpret_cast<LockLine*>(reinterpret_cast<char*>(applied_) + sizeof(AppliedRow) * (size_t)tables * world);
  hdr_->magic = kBoardMagic;
  hdr_->world = world;
  hdr_->tables = tables;
}

PSBoard::~PSBoard() {
  if (hdr_) ::munmap(hdr_, bytes_);
}

void PSBoard::Bump() {
  hdr_->epoch.fetch_add(1, std::memory_order_acq_rel);
  FutexCall(&hdr_->epoch, FUTEX_WAKE, INT_MAX, nullptr);
}

void PSBoard::Wake() { Bump(); }

void PSBoard::PublishSent(int table, int64_t clock) {
  sent_[(size_t)table * world_ + rank_].clock.store(clock, std::memory_order_release);
  Bump();
}

int64_t PSBoard::Sent(int table, int rank) const {
  return sent_[(size_t)table * world_ + rank].clock.load(std::memory_order_acquire);
}

int64_t PSBoard::MinSent(int table) const {
  int64_t m = Sent(table, 0);
  for (int r = 1; r < world_; ++r) m = std::min(m, Sent(table, r));
  return m;
}

void PSBoard::PublishApplied(int table, int requester, int64_t clock) {
  applied_[(size_t)table * world_ + rank_].clock[requester].store(clock, std::memory_order_release);
  Bump();
}

void PSBoard::PublishAppliedRow(int table, int64_t clock) {
  for (int r = 0; r < world_; ++r)
    applied_[(size_t)table * world_ + rank_].clock[r].store(clock, std::memory_order_release);
  Bump();
}

int64_t PSBoard::Applied(int table, int owner, int requester) const {
  return applied_[(size_t)table * world_ + owner].clock[requester].load(std::memory_order_acquire);
}

int64_t PSBoard::MinApplied(int table) const {
  int64_t m = INT64_MAX;
  for (int o = 0; o < world_; ++o)
    for (int r = 0; r < world_; ++r) m = std::min(m, Applied(table, o, r));
  return m;
}

int64_t PSBoard::MinAppliedFrom(int table, int requester) const {
  int64_t m = INT64_MAX;
  for (int o = 0; o < world_; ++o) m = std::min(m, Applied(table, o, requester));
  return m;
}

int64_t PSBoard::OwnerVersion(int table, int owner) const {
  int64_t s = 0;
  for (int r = 0; r < world_; ++r) s += Applied(table, owner, r);
  return s;
}

int64_t PSBoard::Pending(int table) const {
  int64_t n = 0;
  for (int r = 0; r < world_; ++r) n += std::max<int64_t>(0, Sent(table, r) - Applied(table, rank_, r));
  return n;
}

template <typename Pred>
double PSBoard::WaitUntil(Pred pred, double timeout_s) {
  if (pred()) return 0.0;
  const auto t0 = std::chrono::steady_clock::now();
  // a short spin first: the publisher is usually a few microseconds away
  for (int i = 0; i < 2000; ++i) {
    if (pred()) return Since(t0);
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
  for (;;) {
    const uint32_t e = hdr_->epoch.load(std::memory_order_acquire);
    if (pred()) break;  // checked after reading the epoch: no lost wake-up
    if (Aborted()) return -2.0;
    if (timeout_s > 0 && Since(t0) >= timeout_s) return -1.0;
    timespec ts{0, 2000000};  // 2 ms: a bounded sleep also covers a publisher that died mid-publish
    FutexCall(&hdr_->epoch, FUTEX_WAIT, e, &ts);
    ++wakeups_;
  }
  return Since(t0);
}

double PSBoard::WaitMinApplied(int table, int64_t target, double timeout_s) {
  return WaitUntil([&] { return MinApplied(table) >= target; }, timeout_s);
}

double PSBoard::WaitAppliedFrom(int table, int requester, int64_t target, double timeout_s) {
  return WaitUntil([&] { return MinAppliedFrom(table, requester) >= target; }, timeout_s);
}

double PSBoard::WaitSentAtLeast(int table, int rank, int64_t target, double timeout_s) {
  return WaitUntil([&] { return Sent(table, rank) >= target; }, timeout_s);
}

uint32_t PSBoard::WaitEpoch(uint32_t seen, double max_s) {
  uint32_t e = hdr_->epoch.load(std::memory_order_acquire);
  if (e != seen) return e;
  const long ns = std::max<long>(1000, (long)(max_s * 1e9));
  timespec ts{ns / 1000000000L, ns % 1000000000L};
  FutexCall(&hdr_->epoch, FUTEX_WAIT, seen, &ts);
  ++wakeups_;
  return hdr_->epoch.load(std::memory_order_acquire);
}

std::vector<int64_t> PSBoard::SnapshotSent(int table) const {
  std::vector<int64_t> out(world_);
  for (int r = 0; r < world_; ++r) out[r] = Sent(table, r);
  return out;
}

std::vector<int64_t> PSBoard::SnapshotApplied(int table) const {
  std::vector<int64_t> out((size_t)world_ * world_);
  for (int o = 0; o < world_; ++o)
    for (int r = 0; r < world_; ++r) out[(size_t)o * world_ + r] = Applied(table, o, r);
  return out;
}

void PSBoard::SetAbort(uint32_t code) {
  hdr_->abort.store(code ? code : 1u, std::memory_order_release);
  Bump();
}

namespace {
constexpr uint32_t kWriter = 0x80000000u;

template <typename Pred>
bool SpinUntil(Pred pred, double timeout_s, const std::atomic<uint32_t>& abort) {
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0;; ++i) {
    if (pred()) return true;
    if (abort.load(std::memory_order_acquire)) return false;
    if (timeout_s > 0 && Since(t0) >= timeout_s) return false;
    if (i < 1000) {
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
}
}  // namespace

bool PSBoard::ReadLock(int table, double timeout_s) {
  for (int o = 0; o < world_; ++o) {  // ascending owners: no reader waits on a lower lock while holding a higher one
    std::atomic<uint32_t>& w = locks_[(size_t)table * world_ + o].word;
    const bool ok = SpinUntil(
        [&] {
          uint32_t v = w.load(std::memory_order_relaxed);
          return !(v & kWriter) && w.compare_exchange_weak(v, v + 1, std::memory_order_acquire);
        },
        timeout_s, hdr_->abort);
    if (!ok) {
      for (int p = 0; p < o; ++p) locks_[(size_t)table * world_ + p].word.fetch_sub(1, std::memory_order_release);
      return false;
    }
  }
  return true;
}

void PSBoard::ReadUnlock(int table) {
  for (int o = 0; o < world_; ++o) locks_[(size_t)table * world_ + o].word.fetch_sub(1, std::memory_order_release);
}

bool PSBoard::WriteLock(int table, double timeout_s) {
  std::atomic<uint32_t>& w = locks_[(size_t)table * world_ + rank_].word;
  w.fetch_or(kWriter, std::memory_order_acq_rel);  // new readers wait from here on
  if (SpinUntil([&] { return (w.load(std::memory_order_acquire) & ~kWriter) == 0; }, timeout_s, hdr_->abort))
    return true;
  w.fetch_and(~kWriter, std::memory_order_release);
  return false;
}

void PSBoard::WriteUnlock(int table) {
  locks_[(size_t)table * world_ + rank_].word.fetch_and(~kWriter, std::memory_order_release);
}

void PSBoard::Unlink() { ::unlink(("/dev/shm/" + name_).c_str()); }

}  // namespace minips
