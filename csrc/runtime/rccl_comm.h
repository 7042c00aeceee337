// RCCL communicator owned by the framework (one per process / GPU), used for the DDP gradient
// all-reduce and the initial parameter broadcast on a dedicated HIP stream.
//
// Replaces the reference's implicit ProcessGroupNCCL (mnist_ddp.py:33-37, :173).  Symbols are
// resolved at run time from the RCCL that PyTorch already loaded (torch/lib/librccl.so), so the
// process holds exactly one RCCL and one HIP runtime; the ncclUniqueId is exchanged by the caller
// through the torch.distributed TCPStore (env:// rendezvous).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>

namespace mnist {

class RcclComm {
 public:
  static constexpr int kUniqueIdBytes = 128;
  static bool available();
  static std::string version();
  static std::vector<uint8_t> unique_id();

  // Non-blocking communicator where the RCCL exports ncclCommInitRankConfig / ncclCommAbort (the
  // init is polled here and aborted after init_timeout_s), else a blocking ncclCommInitRank.
  // wait = false (non-blocking communicator only): return as soon as the init is under way in RCCL's
  // own thread; the caller polls init_status() and may abort() it at any time (distributed.py
  // PendingRcclComm: the init never holds up the trainer, and a failed or unneeded one is dropped)
  RcclComm(const std::vector<uint8_t>& uid, int world_size, int rank, int device, double init_timeout_s = 600.0,
           bool wait = true);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  // in-place sum all-reduce of fp32 (dtype 0) or bf16 (dtype 1) elements on `stream`
  void allreduce_sum(void* buf, int64_t count, int dtype, hipStream_t stream);
  void broadcast(void* buf, int64_t count, int dtype, int root, hipStream_t stream);
  // ncclCommAbort: collectives stuck on the device return (RCCL's abort flag), the communicator is
  // unusable afterwards (calls throw); idempotent
  void abort();
  bool aborted() const { return aborted_; }
  bool nonblocking() const { return nonblocking_; }
  int async_error() const;       // ncclCommGetAsyncError (0 = ncclSuccess, 7 = in progress)
  // init progress of a wait = false communicator: 0 ready, 7 (ncclInProgress) still running, any other
  // value the RCCL error code (error_string); -1 after abort()
  int init_status() const;
  static std::string error_string(int code);
  int world_size() const { return world_; }
  int rank() const { return rank_; }

 private:
  // a call's result: ncclInProgress (non-blocking communicator) is polled to completion first
  void finish(int r, const char* what, double timeout_s = 300.0);
  void live(const char* what) const;
  void* comm_ = nullptr;
  int world_, rank_;
  bool nonblocking_ = false, aborted_ = false;
};

// roctx ranges (no-ops when roctx is not loaded)
void roctx_push(const char* name);
void roctx_pop();

}  // namespace mnist
