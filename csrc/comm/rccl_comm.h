// Native RCCL data plane of one rank (SURVEY.md §5.8 / §7.2 csrc/comm/rccl_comm): the PS message
// patterns as RCCL collectives over xGMI, enqueued straight onto the caller's HIP stream.
//
//   C1/C2 sparse Get   all-to-all of per-owner counts, all-to-all-v of keys and of rows
//   C3    sparse Add   all-to-all-v of gradient rows into the owner shards
//   C1/C3 dense        reduce-scatter of gradients / all-gather of parameters (equal shards)
//
// Parity: the reference's Get / Add hops are native too -- KVClientTable::Get_/Add_ slice and send
// per server (worker/kv_client_table.hpp:168-195), the Sender thread pops and sends
// (comm/sender.cpp:7-30), Mailbox::Send frames each message (comm/mailbox.cpp:231-308). Here one
// rank's whole exchange is ONE grouped RCCL launch (ncclGroupStart / per-peer ncclSend+ncclRecv /
// ncclGroupEnd) issued from C++: no c10d work object, no per-call stream-sync events, no Python
// (c10d all_to_all_single with splits cost 23.6 us of host time per call, profiles/r5/host_issue.txt).
//
// The library is the RCCL instance torch already loaded (its path is passed in and dlopen'ed, so
// the process holds ONE RCCL); the communicator is our own (ncclCommInitRank from a unique id that
// rank 0 creates and the ranks exchange over the c10d store), separate from torch's process group.
// Ordering: every rank issues this communicator's collectives in the same program order (the
// contract of minips_amd/ps/comm.py), so the n-th launch matches on every rank whatever stream
// issues it.
//
// Failure detection (what torch's ProcessGroupNCCL watchdog does for its own communicator): a
// watchdog thread records a probe event on every stream that issued a collective, every
// timeout / 4 (<= 1 s), and expects it to complete within `timeout_s`. A probe that does not --
// a collective waiting for a dead or stuck peer -- aborts the communicator (ncclCommAbort: the
// spinning kernels exit), so the rank fails instead of hanging: with `teardown` the process ends
// (TORCH_NCCL_ASYNC_ERROR_HANDLING=1, the default of init_distributed), otherwise the next call
// raises (=2, the in-place rollback of minips_amd/train.py catches it as a comm failure).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace minips {

class RcclLib;  // the dlopen'ed entry points

class RcclComm {
 public:
  // dtype codes of the Python side (minips_amd/ps/comm.py _RCCL_DTYPES)
  enum DType { kI8 = 0, kI32 = 1, kI64 = 2, kF16 = 3, kBF16 = 4, kF32 = 5, kF64 = 6 };

  // A fresh unique id (rank 0), as 128 raw bytes.
  static std::string UniqueId(const std::string& lib_path);

  RcclComm(const std::string& lib_path, const std::string& unique_id, int world, int rank, int device,
           double timeout_s = 60.0, bool teardown = false);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  int world() const { return world_; }
  int rank() const { return rank_; }

  // Rows of `row_bytes` bytes: send[sum(send_rows[:p]) ...] to peer p, recv into
  // recv[sum(recv_rows[:p]) ...] from peer p; one grouped launch (empty messages skipped).
  void AllToAllV(const void* send, const std::vector<int64_t>& send_rows, void* recv,
                 const std::vector<int64_t>& recv_rows, int64_t row_bytes, hipStream_t s);
  // Equal blocks of `block_bytes` per peer (the count exchange).
  void AllToAll(const void* send, void* recv, int64_t block_bytes, hipStream_t s);
  // recv[count] = sum over ranks of send[rank * count, (rank + 1) * count)
  void ReduceScatter(const void* send, void* recv, int64_t count, int dtype, hipStream_t s);
  // recv[world * count] = every rank's send[count], in rank order
  void AllGather(const void* send, void* recv, int64_t count, int dtype, hipStream_t s);
  // op: 0 sum, 1 max, 2 min
  void AllReduce(const void* send, void* recv, int64_t count, int dtype, int op, hipStream_t s);

  // Failure handling: an asynchronous RCCL error ("" when none), and abort (every pending and
  // later call on this communicator fails at once; a peer's loss must not hang the rank).
  std::string AsyncError();
  void Abort(const std::string& why = "aborted by the caller");
  bool aborted() const { return aborted_.load(); }

 private:
  struct Call;  // entry guard of one collective (stream registration, abort check)
  void Check(ncclResult_t r, const char* what);
  void Watch();
  const RcclLib* lib_;
  ncclComm_t comm_ = nullptr;
  int world_, rank_, device_;
  double timeout_s_;
  bool teardown_;
  // abort protocol (seq_cst Dekker pair): a caller bumps in_call_ then reads abort_req_; the
  // watchdog sets abort_req_ then waits (bounded) for in_call_ == 0 before ncclCommAbort
  std::atomic<int> in_call_{0};
  std::atomic<bool> abort_req_{false}, aborted_{false};
  std::mutex mu_;  // streams_, error_
  std::string error_;
  struct Probe {
    hipStream_t stream;
    hipEvent_t ev = nullptr;
    bool pending = false;
    double t_rec = 0;
  };
  std::vector<Probe> streams_;
  // issue order across streams: RCCL itself lets a collective enqueued on another stream run ahead
  // of an earlier one (measured: tests/test_rccl_gpu.py), so each collective's stream first waits
  // for the previous collective's completion event -- one GPU order, the issue order, as
  // ProcessGroupNCCL's single internal stream gives (the data plane's deadlock-freedom argument,
  // minips_amd/ps/comm.py). order_mu_ is held across a whole call (one issuing thread at a time).
  std::mutex order_mu_;
  hipEvent_t order_ev_ = nullptr;
  hipStream_t order_stream_ = nullptr;
  std::thread wd_;
  std::condition_variable wcv_;
  bool wstop_ = false;
};

}  // namespace minips
