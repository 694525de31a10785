#include "rccl_comm.h"

#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>

namespace minips {

// The entry points of one RCCL shared object, resolved by name (decltype of the rccl.h
// declarations keeps the signatures exact).
class RcclLib {
 public:
  explicit RcclLib(const std::string& path) {
    // the file torch already mapped: dlopen returns that same object (one RCCL per process)
    handle_ = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!handle_) throw std::runtime_error("rccl: dlopen " + path + ": " + dlerror());
#define MINIPS_RCCL_SYM(name) name = reinterpret_cast<decltype(&::name)>(Sym(#name))
    MINIPS_RCCL_SYM(ncclGetUniqueId);
    MINIPS_RCCL_SYM(ncclCommInitRank);
    MINIPS_RCCL_SYM(ncclCommDestroy);
    MINIPS_RCCL_SYM(ncclCommAbort);
    MINIPS_RCCL_SYM(ncclCommGetAsyncError);
    MINIPS_RCCL_SYM(ncclGetErrorString);
    MINIPS_RCCL_SYM(ncclGroupStart);
    MINIPS_RCCL_SYM(ncclGroupEnd);
    MINIPS_RCCL_SYM(ncclSend);
    MINIPS_RCCL_SYM(ncclRecv);
    MINIPS_RCCL_SYM(ncclReduceScatter);
    MINIPS_RCCL_SYM(ncclAllGather);
    MINIPS_RCCL_SYM(ncclAllReduce);
#undef MINIPS_RCCL_SYM
  }
  static const RcclLib* Get(const std::string& path) {
    static std::mutex mu;
    static std::map<std::string, std::unique_ptr<RcclLib>> libs;
    std::lock_guard<std::mutex> lk(mu);
    auto& l = libs[path];
    if (!l) l.reset(new RcclLib(path));
    return l.get();
  }

  decltype(&::ncclGetUniqueId) ncclGetUniqueId;
  decltype(&::ncclCommInitRank) ncclCommInitRank;
  decltype(&::ncclCommDestroy) ncclCommDestroy;
  decltype(&::ncclCommAbort) ncclCommAbort;
  decltype(&::ncclCommGetAsyncError) ncclCommGetAsyncError;
  decltype(&::ncclGetErrorString) ncclGetErrorString;
  decltype(&::ncclGroupStart) ncclGroupStart;
  decltype(&::ncclGroupEnd) ncclGroupEnd;
  decltype(&::ncclSend) ncclSend;
  decltype(&::ncclRecv) ncclRecv;
  decltype(&::ncclReduceScatter) ncclReduceScatter;
  decltype(&::ncclAllGather) ncclAllGather;
  decltype(&::ncclAllReduce) ncclAllReduce;

 private:
  void* Sym(const char* name) {
    void* p = dlsym(handle_, name);
    if (!p) throw std::runtime_error(std::string("rccl: missing symbol ") + name);
    return p;
  }
  void* handle_ = nullptr;  // never closed: communicators may outlive any one owner
};

namespace {

ncclDataType_t ToNccl(int dtype) {
  switch (dtype) {
    case RcclComm::kI8: return ncclInt8;
    case RcclComm::kI32: return ncclInt32;
    case RcclComm::kI64: return ncclInt64;
    case RcclComm::kF16: return ncclFloat16;
    case RcclComm::kBF16: return ncclBfloat16;
    case RcclComm::kF32: return ncclFloat32;
    case RcclComm::kF64: return ncclFloat64;
    default: throw std::runtime_error("rccl: dtype code " + std::to_string(dtype));
  }
}

// RAII group: ncclGroupEnd runs even when an enqueue in between throws
struct Group {
  const RcclLib* lib;
  bool open = false;
  explicit Group(const RcclLib* l) : lib(l) {}
  ncclResult_t Begin() {
    const ncclResult_t r = lib->ncclGroupStart();
    open = r == ncclSuccess;
    return r;
  }
  ncclResult_t End() {
    open = false;
    return lib->ncclGroupEnd();
  }
  ~Group() {
    if (open) (void)lib->ncclGroupEnd();
  }
};

}  // namespace

std::string RcclComm::UniqueId(const std::string& lib_path) {
  const RcclLib* lib = RcclLib::Get(lib_path);
  ncclUniqueId id;
  const ncclResult_t r = lib->ncclGetUniqueId(&id);
  if (r != ncclSuccess) throw std::runtime_error(std::string("rccl: ncclGetUniqueId: ") + lib->ncclGetErrorString(r));
  return std::string(id.internal, sizeof(id.internal));
}

namespace {
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

// One collective's entry: registers the issuing stream with the watchdog and refuses to touch an
// aborted communicator (see the abort protocol in the header).
struct RcclComm::Call {
  RcclComm* c;
  hipStream_t s;
  std::unique_lock<std::mutex> order;
  bool captured = false;  // (a stream under graph capture: no event chain into or out of the graph)
  Call(RcclComm* comm, hipStream_t stream) : c(comm), s(stream), order(comm->order_mu_) {
    c->in_call_.fetch_add(1);
    if (c->abort_req_.load()) {
      c->in_call_.fetch_sub(1);
      std::lock_guard<std::mutex> lk(c->mu_);
      throw std::runtime_error("rccl: communicator aborted (" + c->error_ + ")");
    }
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    captured = hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
    // after the previous collective, whichever stream it went to (issue order = GPU order)
    const bool chain = !captured && c->order_stream_ && c->order_stream_ != s;
    if (chain && hipStreamWaitEvent(s, c->order_ev_, 0) != hipSuccess) {
      c->in_call_.fetch_sub(1);
      throw std::runtime_error("rccl: stream wait on the previous collective failed");
    }
    std::lock_guard<std::mutex> lk(c->mu_);
    for (const Probe& p : c->streams_)
      if (p.stream == s) return;
    Probe p;
    p.stream = s;
    if (hipEventCreateWithFlags(&p.ev, hipEventDisableTiming) != hipSuccess) p.ev = nullptr;
    c->streams_.push_back(p);
  }
  ~Call() {
    if (captured) c->order_stream_ = nullptr;
    else if (c->order_ev_ && hipEventRecord(c->order_ev_, s) == hipSuccess) c->order_stream_ = s;
    c->in_call_.fetch_sub(1);
  }
};

RcclComm::RcclComm(const std::string& lib_path, const std::string& unique_id, int world, int rank, int device,
                   double timeout_s, bool teardown)
    : lib_(RcclLib::Get(lib_path)), world_(world), rank_(rank), device_(device), timeout_s_(timeout_s),
      teardown_(teardown) {
  if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("rccl: rank / world");
  ncclUniqueId id;
  if (unique_id.size() != sizeof(id.internal)) throw std::runtime_error("rccl: unique id must be 128 bytes");
  std::memcpy(id.internal, unique_id.data(), sizeof(id.internal));
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("rccl: hipSetDevice");
  Check(lib_->ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
  if (hipEventCreateWithFlags(&order_ev_, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess)
    throw std::runtime_error("rccl: hipEventCreateWithFlags");
  if (timeout_s_ > 0) wd_ = std::thread([this] { Watch(); });
}

RcclComm::~RcclComm() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    wstop_ = true;
  }
  wcv_.notify_all();
  if (wd_.joinable()) wd_.join();
  if (!aborted_.load() && comm_) (void)lib_->ncclCommDestroy(comm_);
  for (Probe& p : streams_)
    if (p.ev) (void)hipEventDestroy(p.ev);
  if (order_ev_) (void)hipEventDestroy(order_ev_);
}

void RcclComm::Watch() {
  (void)hipSetDevice(device_);
  const double period = std::min(1.0, std::max(0.01, timeout_s_ / 4));
  std::unique_lock<std::mutex> lk(mu_);
  while (!wstop_ && !aborted_.load()) {
    wcv_.wait_for(lk, std::chrono::duration<double>(period), [&] { return wstop_; });
    if (wstop_) break;
    const double t = now_s();
    std::string why;
    for (Probe& p : streams_) {
      if (!p.ev) continue;
      if (!p.pending) {  // a probe behind whatever the stream holds now
        // (never into a stream being captured into a HIP graph: the record would become a node)
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(p.stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) continue;
        if (hipEventRecord(p.ev, p.stream) == hipSuccess) {
          p.pending = true;
          p.t_rec = t;
        }
        continue;
      }
      const hipError_t q = hipEventQuery(p.ev);
      if (q == hipSuccess) {
        p.pending = false;
      } else if (q == hipErrorNotReady && t - p.t_rec > timeout_s_) {
        char buf[160];
        std::snprintf(buf, sizeof buf, "a collective of rank %d did not complete within %.0f s (stream %p)", rank_,
                      timeout_s_, (void*)p.stream);
        why = buf;
        break;
      } else if (q != hipErrorNotReady) {
        why = std::string("stream error: ") + hipGetErrorString(q);
        break;
      }
    }
    if (why.empty()) {
      lk.unlock();
      const std::string e = AsyncError();
      lk.lock();
      if (e.empty()) continue;
      why = "RCCL async error: " + e;
    }
    lk.unlock();
    Abort(why);
    if (teardown_) {
      std::fprintf(stderr, "[minips rccl watchdog] rank %d: %s -- communicator aborted, tearing the process down\n",
                   rank_, why.c_str());
      std::fflush(stderr);
      std::abort();
    }
    std::fprintf(stderr, "[minips rccl watchdog] rank %d: %s -- communicator aborted\n", rank_, why.c_str());
    return;
  }
}

void RcclComm::Check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess || r == ncclInProgress) return;
  throw std::runtime_error(std::string("rccl: ") + what + ": " + lib_->ncclGetErrorString(r));
}

void RcclComm::AllToAllV(const void* send, const std::vector<int64_t>& send_rows, void* recv,
                         const std::vector<int64_t>& recv_rows, int64_t row_bytes, hipStream_t s) {
  Call call(this, s);
  if ((int)send_rows.size() != world_ || (int)recv_rows.size() != world_ || row_bytes <= 0)
    throw std::runtime_error("rccl: all-to-all-v needs one count per rank");
  // whole 16-bit words when the rows allow it (RCCL moves elements of the given type)
  const bool b2 = row_bytes % 2 == 0;
  const ncclDataType_t t = b2 ? ncclBfloat16 : ncclInt8;
  const int64_t elem = b2 ? 2 : 1, per_row = row_bytes / elem;
  const char* sp = static_cast<const char*>(send);
  char* rp = static_cast<char*>(recv);
  Group g(lib_);
  Check(g.Begin(), "ncclGroupStart");
  int64_t so = 0, ro = 0;
  for (int p = 0; p < world_; ++p) {
    if (send_rows[p] > 0)
      Check(lib_->ncclSend(sp + so * row_bytes, (size_t)(send_rows[p] * per_row), t, p, comm_, s), "ncclSend");
    if (recv_rows[p] > 0)
      Check(lib_->ncclRecv(rp + ro * row_bytes, (size_t)(recv_rows[p] * per_row), t, p, comm_, s), "ncclRecv");
    so += send_rows[p];
    ro += recv_rows[p];
  }
  Check(g.End(), "ncclGroupEnd");
}

void RcclComm::AllToAll(const void* send, void* recv, int64_t block_bytes, hipStream_t s) {
  std::vector<int64_t> ones(world_, 1);
  AllToAllV(send, ones, recv, ones, block_bytes, s);
}

void RcclComm::ReduceScatter(const void* send, void* recv, int64_t count, int dtype, hipStream_t s) {
  Call call(this, s);
  Check(lib_->ncclReduceScatter(send, recv, (size_t)count, ToNccl(dtype), ncclSum, comm_, s), "ncclReduceScatter");
}

void RcclComm::AllGather(const void* send, void* recv, int64_t count, int dtype, hipStream_t s) {
  Call call(this, s);
  Check(lib_->ncclAllGather(send, recv, (size_t)count, ToNccl(dtype), comm_, s), "ncclAllGather");
}

void RcclComm::AllReduce(const void* send, void* recv, int64_t count, int dtype, int op, hipStream_t s) {
  Call call(this, s);
  const ncclRedOp_t o = op == 1 ? ncclMax : op == 2 ? ncclMin : ncclSum;
  Check(lib_->ncclAllReduce(send, recv, (size_t)count, ToNccl(dtype), o, comm_, s), "ncclAllReduce");
}

std::string RcclComm::AsyncError() {
  if (abort_req_.load()) {
    std::lock_guard<std::mutex> lk(mu_);
    return error_.empty() ? "aborted" : error_;
  }
  ncclResult_t e = ncclSuccess;
  const ncclResult_t r = lib_->ncclCommGetAsyncError(comm_, &e);
  if (r != ncclSuccess) return std::string("ncclCommGetAsyncError: ") + lib_->ncclGetErrorString(r);
  if (e == ncclSuccess || e == ncclInProgress) return "";
  return lib_->ncclGetErrorString(e);
}

void RcclComm::Abort(const std::string& why) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (abort_req_.load()) return;
    error_ = why;
    abort_req_.store(true);
  }
  // callers inside an enqueue normally leave within microseconds; one blocked on a dead peer does
  // not -- ncclCommAbort is the call that releases it, so the wait is bounded
  const double t0 = now_s();
  while (in_call_.load() != 0 && now_s() - t0 < 2.0) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  (void)lib_->ncclCommAbort(comm_);
  aborted_.store(true);
}

}  // namespace minips
