// Native DDP gradient reducer for the module-level path (reference mnist_ddp.py:173 + the c10d
// Reducer that torch DDP drives from autograd hooks).
//
// Python registers one post-accumulate-grad hook per parameter; each hook calls mark_ready()
// with the gradient's device pointer.  The reducer copies the gradient into its flat fp32 bucket
// pre-scaled by 1/world_size on the autograd (compute) stream; when the last parameter of a
// bucket arrives it records an event, makes its own high-priority comm stream wait on it and
// enqueues the RCCL all-reduce there, so the 4.7 MB fc bucket is on the wire while autograd is
// still computing the conv gradients.  finalize() (queued on the autograd engine) joins the comm
// stream into the compute stream and copies the averaged buckets back into every .grad.
// Buckets are always launched in index order, the same on every rank (RCCL requires it).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <vector>

#include "rccl_comm.h"

namespace mnist {

class BucketReducer {
 public:
  // bucket_numels[b] = element counts of the bucket's parameters, in ready (slot) order
  BucketReducer(const std::vector<std::vector<int64_t>>& bucket_numels, int world_size,
                std::shared_ptr<RcclComm> comm);
  ~BucketReducer();
  BucketReducer(const BucketReducer&) = delete;
  BucketReducer& operator=(const BucketReducer&) = delete;

  void prepare();   // start of an iteration: nothing pending, nothing launched
  // the gradient of (bucket b, slot) is final on `stream`; grad == nullptr means "no gradient"
  // (zeros are reduced); grad_out is where finalize() writes the averaged gradient back
  void mark_ready(int b, int slot, const float* grad, float* grad_out, hipStream_t stream);
  void finalize(hipStream_t stream);
  int num_buckets() const { return (int)buckets_.size(); }
  int64_t bucket_numel(int b) const { return buckets_.at(b).numel; }
  uintptr_t bucket_ptr(int b) const { return reinterpret_cast<uintptr_t>(buckets_.at(b).buf); }
  int64_t launches() const { return launches_; }

 private:
  struct Bucket {
    float* buf = nullptr;
    int64_t numel = 0;
    std::vector<int64_t> offs, numels;
    std::vector<float*> outs;
    std::vector<char> seen;
    int pending = 0;
    bool launched = false;
    hipEvent_t ready = nullptr, done = nullptr;
  };
  void launch(int b, hipStream_t stream);

  std::vector<Bucket> buckets_;
  int world_;
  std::shared_ptr<RcclComm> comm_;
  hipStream_t comm_stream_ = nullptr;
  int next_launch_ = 0;
  int64_t launches_ = 0;
};

}  // namespace mnist
