// Cross-process clock board of the one-sided (really asynchronous) SSP / ASP tables: the GPU
// ranks of one node publish their clocks into a shared-memory segment and an SSP Get blocks until
// the slowest rank is close enough.
//
// Parity: server/util/progress_tracker.{hpp,cpp} (per-worker progress + min_clock, the unique-min
// rule :46-72) and server/consistency/ssp_model.cpp:58-85 (a Get is buffered while its clock is
// more than `staleness` ahead of min_clock). The reference keeps this state inside the server
// thread of each node and answers by message; here every rank reads the others' clocks from
// shared memory, so a gate check costs a few loads instead of a round trip.
//
// Layout: a header (magic, world) and one 64-byte line per rank (no false sharing between the
// publishers). A publish is a release store of the clock followed by a bump of a 32-bit epoch word
// and a FUTEX_WAKE on it; a waiter sleeps in FUTEX_WAIT on the epoch (shared futex: the segment is
// mapped by several processes) instead of polling, and rechecks the minimum on every wake.
#pragma once

#include <atomic>
#include <cstdint>
#include <string>
#include <vector>

namespace minips {

class ClockBoard {
 public:
  // Maps /dev/shm/<name> (created and sized by the rank that passes create=true; the others
  // attach, waiting up to `attach_timeout_s` for it to appear).
  ClockBoard(const std::string& name, int world, int rank, bool create, double attach_timeout_s = 30.0);
  ~ClockBoard();
  ClockBoard(const ClockBoard&) = delete;
  ClockBoard& operator=(const ClockBoard&) = delete;

  void Publish(int64_t clock);  // this rank's clock (release)
  int64_t Get(int rank) const;
  int64_t MinClock() const;
  std::vector<int64_t> Snapshot() const;
  // Blocks until MinClock() >= target (the SSP gate); returns the seconds waited. Throws after
  // `timeout_s` (<= 0: wait forever) -- a straggler that never comes back is a failure, not a hang.
  double WaitMinAtLeast(int64_t target, double timeout_s);
  uint64_t Wakeups() const { return wakeups_; }
  void Unlink();  // remove the segment name (the creator, at shutdown)
  const std::string& Name() const { return name_; }

 private:
  struct Slot {
    std::atomic<int64_t> clock;
    char pad[56];
  };
  struct Header {
    uint64_t magic;
    int32_t world;
    std::atomic<uint32_t> epoch;  // futex word
    char pad[48];
  };
  Header* hdr_ = nullptr;
  Slot* slots_ = nullptr;
  size_t bytes_ = 0;
  int world_, rank_;
  std::string name_;
  uint64_t wakeups_ = 0;
};

}  // namespace minips
