#include "clock_board.h"

#include <fcntl.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <climits>
#include <ctime>
#include <thread>

#include "base.h"

namespace minips {

namespace {

constexpr uint64_t kMagic = 0x4d50534b4c4f4342ull;  // "BCOLKSPM"

long Futex(std::atomic<uint32_t>* addr, int op, uint32_t val, const timespec* ts) {
  // shared futex (no FUTEX_PRIVATE_FLAG): the word lives in a segment mapped by several processes
  return ::syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), op, val, ts, nullptr, 0);
}

}  // namespace

ClockBoard::ClockBoard(const std::string& name, int world, int rank, bool create, double attach_timeout_s)
    : world_(world), rank_(rank), name_(name) {
  MINIPS_CHECK(world >= 1 && rank >= 0 && rank < world, "clock board: bad rank " << rank << "/" << world);
  static_assert(sizeof(Slot) == 64 && sizeof(Header) == 64, "one cache line per rank");
  bytes_ = sizeof(Header) + sizeof(Slot) * (size_t)world;
  const std::string path = "/dev/shm/" + name;
  // every rank may create: the segment is zero-filled on creation (clocks 0, epoch 0) and only
  // ever grown to the same size, so the order in which the ranks arrive does not matter
  (void)create;  // only decides who unlinks the name at shutdown (the Python owner)
  int fd = -1;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(attach_timeout_s);
  while ((fd = ::open(path.c_str(), O_RDWR | O_CREAT, 0600)) < 0) {
    MINIPS_CHECK(std::chrono::steady_clock::now() < deadline, "clock board: cannot open " << path);
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  struct stat st;
  MINIPS_CHECK(::fstat(fd, &st) == 0, "clock board: fstat " << path);
  if ((size_t)st.st_size < bytes_) MINIPS_CHECK(::ftruncate(fd, (off_t)bytes_) == 0, "clock board: ftruncate");
  void* p = ::mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  MINIPS_CHECK(p != MAP_FAILED, "clock board: mmap " << path);
  hdr_ = static_cast<Header*>(p);
  slots_ = reinterpret_cast<Slot*>(static_cast<char*>(p) + sizeof(Header));
  hdr_->magic = kMagic;
  hdr_->world = world;
}

ClockBoard::~ClockBoard() {
  if (hdr_) ::munmap(hdr_, bytes_);
}

void ClockBoard::Publish(int64_t clock) {
  slots_[rank_].clock.store(clock, std::memory_order_release);
  hdr_->epoch.fetch_add(1, std::memory_order_acq_rel);
  Futex(&hdr_->epoch, FUTEX_WAKE, INT_MAX, nullptr);
}

int64_t ClockBoard::Get(int rank) const { return slots_[rank].clock.load(std::memory_order_acquire); }

int64_t ClockBoard::MinClock() const {
  int64_t m = Get(0);
  for (int r = 1; r < world_; ++r) m = std::min(m, Get(r));
  return m;
}

std::vector<int64_t> ClockBoard::Snapshot() const {
  std::vector<int64_t> out(world_);
  for (int r = 0; r < world_; ++r) out[r] = Get(r);
  return out;
}

double ClockBoard::WaitMinAtLeast(int64_t target, double timeout_s) {
  if (MinClock() >= target) return 0.0;
  const auto t0 = std::chrono::steady_clock::now();
  // a short spin first: under SSP the slowest rank is usually a few microseconds from publishing
  for (int i = 0; i < 2000; ++i) {
    if (MinClock() >= target) return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
  for (;;) {
    const uint32_t e = hdr_->epoch.load(std::memory_order_acquire);
    if (MinClock() >= target) break;  // checked after reading the epoch: no lost wake-up
    const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    MINIPS_CHECK(timeout_s <= 0 || waited < timeout_s,
                 "SSP gate: min clock still below " << target << " after " << waited << " s (clocks stuck)");
    timespec ts{0, 2000000};  // 2 ms: a bounded sleep also covers a publisher that died mid-publish
    Futex(&hdr_->epoch, FUTEX_WAIT, e, &ts);
    ++wakeups_;
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

void ClockBoard::Unlink() { ::unlink(("/dev/shm/" + name_).c_str()); }

}  // namespace minips
