// Base runtime types for the MI355X parameter server runtime.
//
// Parity notes (reference = Distributed-Deep-Learning/MiniPs):
//   * Key / KVPairs            -> base/magic.hpp:8-13 (Key widened to 64 bit: a 10B-row
//                                 embedding table overflows uint32).
//   * SArray (shared, zero-copy segment, type punning) -> base/third_party/sarray.h:42-304
//   * Range                    -> base/third_party/range.h:14-29
//   * ThreadsafeQueue          -> base/threadsafe_queue.hpp:10-48 (adds timed pop)
//   * Actor                    -> base/actor_model.hpp:13-34
// Everything here is host-side C++17; device buffers live in torch tensors owned by the
// Python/HIP data plane and never pass through these containers.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <initializer_list>
#include <memory>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

namespace minips {

// Timed condition wait. libstdc++ maps a steady_clock wait_for to pthread_cond_clockwait, which
// the gcc-11 ThreadSanitizer does not intercept (the unlock/relock inside the wait is invisible ->
// false "double lock" and race reports), so sanitizer builds wait on the system clock instead.
template <class Pred>
inline bool CondWaitFor(std::condition_variable& cv, std::unique_lock<std::mutex>& lk, double seconds, Pred pred) {
#if defined(__SANITIZE_THREAD__)
  const auto deadline = std::chrono::system_clock::now() +
                        std::chrono::duration_cast<std::chrono::system_clock::duration>(
                            std::chrono::duration<double>(seconds));
  return cv.wait_until(lk, deadline, pred);
#else
  return cv.wait_for(lk, std::chrono::duration<double>(seconds), pred);
#endif
}


using Key = uint64_t;

// ---------------------------------------------------------------------------------------
// Error checking: throw (never abort) so the Python bindings surface failures as exceptions.
// ---------------------------------------------------------------------------------------
struct CheckError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define MINIPS_CHECK(cond, msg)                                                        \
  do {                                                                                 \
    if (!(cond)) {                                                                     \
      std::ostringstream _os;                                                          \
      _os << __FILE__ << ":" << __LINE__ << " check failed: " #cond " " << msg;        \
      throw ::minips::CheckError(_os.str());                                           \
    }                                                                                  \
  } while (0)

// Log sink: one line per call, thread-safe. Level 0=INFO 1=WARN 2=ERROR. GLOG_v gates
// verbose lines (the reference's GLOG_v / VLOG(1) lifecycle traces).
void LogLine(int level, const std::string& line);
int VerboseLevel();
#define MINIPS_LOG(lvl, expr)                 \
  do {                                        \
    std::ostringstream _os;                   \
    _os << expr;                              \
    ::minips::LogLine(lvl, _os.str());        \
  } while (0)
#define MINIPS_VLOG(v, expr)                                   \
  do {                                                         \
    if (::minips::VerboseLevel() >= (v)) MINIPS_LOG(0, expr);  \
  } while (0)

// ---------------------------------------------------------------------------------------
// SArray<V>: shared-ownership array with zero-copy segment() and zero-copy reinterpretation
// between element types (the message payload container).
// ---------------------------------------------------------------------------------------
template <typename V>
class SArray {
 public:
  SArray() = default;
  explicit SArray(size_t n, V init = V()) { resize(n, init); }
  SArray(std::initializer_list<V> l) { CopyFrom(l.begin(), l.size()); }
  explicit SArray(const std::vector<V>& v) { CopyFrom(v.data(), v.size()); }
  SArray(const V* data, size_t n) { CopyFrom(data, n); }

  // Zero-copy type pun: the byte size must be divisible by sizeof(V).
  template <typename W>
  SArray(const SArray<W>& other) {  // NOLINT(runtime/explicit)
    *this = other;
  }
  template <typename W>
  SArray& operator=(const SArray<W>& other) {
    size_t bytes = other.size() * sizeof(W);
    MINIPS_CHECK(bytes % sizeof(V) == 0, "cannot reinterpret " << bytes << " bytes");
    size_ = bytes / sizeof(V);
    capacity_ = other.capacity() * sizeof(W) / sizeof(V);
    ptr_ = other.ptr();
    data_ = reinterpret_cast<V*>(const_cast<W*>(other.data()));
    return *this;
  }

  void CopyFrom(const V* src, size_t n) {
    resize(n);
    if (n) std::memcpy(static_cast<void*>(data_), src, n * sizeof(V));
  }

  void reserve(size_t n) {
    if (n <= capacity_) return;
    std::shared_ptr<void> np(::operator new(n * sizeof(V)), [](void* p) { ::operator delete(p); });
    V* nd = static_cast<V*>(np.get());
    if (size_) std::memcpy(static_cast<void*>(nd), data_, size_ * sizeof(V));
    ptr_ = np;
    data_ = nd;
    capacity_ = n;
  }
  void resize(size_t n, V init = V()) {
    size_t old = size_;
    if (n > capacity_) reserve(n + 5);
    size_ = n;
    for (size_t i = old; i < n; ++i) data_[i] = init;
  }
  void push_back(const V& v) {
    if (size_ == capacity_) reserve(size_ * 2 + 5);
    data_[size_++] = v;
  }
  void append(const SArray<V>& o) {
    if (o.empty()) return;
    size_t old = size_;
    resize(size_ + o.size());
    std::memcpy(static_cast<void*>(data_ + old), o.data(), o.size() * sizeof(V));
  }
  void clear() { *this = SArray<V>(); }

  // Zero-copy slice [b, e).
  SArray<V> segment(size_t b, size_t e) const {
    MINIPS_CHECK(b <= e && e <= size_, "bad segment [" << b << "," << e << ") of " << size_);
    SArray<V> r;
    r.ptr_ = ptr_;
    r.data_ = data_ + b;
    r.size_ = e - b;
    r.capacity_ = e - b;
    return r;
  }

  V* data() const { return data_; }
  size_t size() const { return size_; }
  size_t capacity() const { return capacity_; }
  bool empty() const { return size_ == 0; }
  V* begin() { return data_; }
  V* end() { return data_ + size_; }
  const V* begin() const { return data_; }
  const V* end() const { return data_ + size_; }
  V& operator[](size_t i) { return data_[i]; }
  const V& operator[](size_t i) const { return data_[i]; }
  V& back() { return data_[size_ - 1]; }
  const std::shared_ptr<void>& ptr() const { return ptr_; }
  std::vector<V> ToVector() const { return std::vector<V>(begin(), end()); }

 private:
  std::shared_ptr<void> ptr_;
  V* data_ = nullptr;
  size_t size_ = 0;
  size_t capacity_ = 0;
};

using Keys = SArray<Key>;
using KVPairs = std::pair<SArray<Key>, SArray<double>>;

struct Range {
  uint64_t begin_ = 0, end_ = 0;
  Range() = default;
  Range(uint64_t b, uint64_t e) : begin_(b), end_(e) {}
  uint64_t begin() const { return begin_; }
  uint64_t end() const { return end_; }
  uint64_t size() const { return end_ - begin_; }
  bool operator==(const Range& o) const { return begin_ == o.begin_ && end_ == o.end_; }
};

// ---------------------------------------------------------------------------------------
// ThreadsafeQueue: mutex + condvar FIFO.
// ---------------------------------------------------------------------------------------
template <typename T>
class ThreadsafeQueue {
 public:
  // Notifies while holding the lock: a waiter that pops the element and then destroys the queue
  // (a call-scoped reply queue, Engine::InitTable) cannot do so while Push still touches it.
  void Push(T elem) {
    std::lock_guard<std::mutex> lk(mu_);
    queue_.push_back(std::move(elem));
    cond_.notify_all();
  }
  void WaitAndPop(T* elem) {
    std::unique_lock<std::mutex> lk(mu_);
    cond_.wait(lk, [this] { return !queue_.empty(); });
    *elem = std::move(queue_.front());
    queue_.pop_front();
  }
  // Returns false on timeout (the reference has no timeouts: a hung barrier hangs forever).
  bool WaitAndPopFor(T* elem, double seconds) {
    std::unique_lock<std::mutex> lk(mu_);
    if (!CondWaitFor(cond_, lk, seconds, [this] { return !queue_.empty(); }))
      return false;
    *elem = std::move(queue_.front());
    queue_.pop_front();
    return true;
  }
  bool TryPop(T* elem) {
    std::lock_guard<std::mutex> lk(mu_);
    if (queue_.empty()) return false;
    *elem = std::move(queue_.front());
    queue_.pop_front();
    return true;
  }
  size_t Size() const {
    std::lock_guard<std::mutex> lk(mu_);
    return queue_.size();
  }

 private:
  mutable std::mutex mu_;
  std::condition_variable cond_;
  std::deque<T> queue_;
};

}  // namespace minips
