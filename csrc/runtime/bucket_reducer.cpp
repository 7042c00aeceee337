#include "bucket_reducer.h"

#include <algorithm>
#include <stdexcept>
#include <string>

#include "../include/kernels.h"

namespace mnist {

namespace {
void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

BucketReducer::BucketReducer(const std::vector<std::vector<int64_t>>& bucket_numels, int world_size,
                             std::shared_ptr<RcclComm> comm)
    : world_(world_size), comm_(std::move(comm)) {
  if (world_ < 1) throw std::runtime_error("BucketReducer: world_size must be >= 1");
  int lo = 0, hi = 0;
  hip_ok(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
  hip_ok(hipStreamCreateWithPriority(&comm_stream_, hipStreamNonBlocking, hi), "hipStreamCreateWithPriority");
  buckets_.resize(bucket_numels.size());
  for (size_t b = 0; b < bucket_numels.size(); ++b) {
    Bucket& k = buckets_[b];
    int64_t off = 0;
    for (int64_t n : bucket_numels[b]) {
      k.offs.push_back(off);
      k.numels.push_back(n);
      off += (n + 3) / 4 * 4;   // 16-B aligned views: the copy kernel runs float4-wide
    }
    k.numel = off;
    k.outs.assign(k.numels.size(), nullptr);
    k.seen.assign(k.numels.size(), 0);
    hip_ok(hipMalloc(&k.buf, (size_t)(off > 0 ? off : 1) * sizeof(float)), "hipMalloc(bucket)");
    launch_fill(k.buf, (int64_t)(off > 0 ? off : 1) * (int64_t)sizeof(float), 0, nullptr);
    hip_ok(hipStreamSynchronize(nullptr), "fill(bucket)");
    hip_ok(hipEventCreateWithFlags(&k.ready, hipEventDisableTiming), "hipEventCreate");
    hip_ok(hipEventCreateWithFlags(&k.done, hipEventDisableTiming), "hipEventCreate");
  }
  prepare();
}

BucketReducer::~BucketReducer() {
  if (comm_stream_) hipStreamSynchronize(comm_stream_);
  for (auto& k : buckets_) {
    if (k.ready) hipEventDestroy(k.ready);
    if (k.done) hipEventDestroy(k.done);
    if (k.buf) hipFree(k.buf);
  }
  if (comm_stream_) hipStreamDestroy(comm_stream_);
}

void BucketReducer::prepare() {
  for (auto& k : buckets_) {
    k.pending = (int)k.numels.size();
    k.launched = false;
    std::fill(k.seen.begin(), k.seen.end(), 0);
  }
  next_launch_ = 0;
}

void BucketReducer::launch(int b, hipStream_t stream) {
  // all-reduces leave in bucket order on every rank: a bucket that completes early waits for
  // its predecessors (they are launched from here as soon as they complete)
  (void)b;
  while (next_launch_ < (int)buckets_.size() && buckets_[next_launch_].pending == 0 &&
         !buckets_[next_launch_].launched) {
    Bucket& n = buckets_[next_launch_];
    hip_ok(hipEventRecord(n.ready, stream), "hipEventRecord");
    hip_ok(hipStreamWaitEvent(comm_stream_, n.ready, 0), "hipStreamWaitEvent");
    if (comm_) comm_->allreduce_sum(n.buf, n.numel, 0, comm_stream_);
    hip_ok(hipEventRecord(n.done, comm_stream_), "hipEventRecord");
    n.launched = true;
    ++launches_;
    ++next_launch_;
  }
}

void BucketReducer::mark_ready(int b, int slot, const float* grad, float* grad_out, hipStream_t stream) {
  if (b < 0 || b >= (int)buckets_.size()) throw std::runtime_error("BucketReducer: bad bucket");
  Bucket& k = buckets_[b];
  if (slot < 0 || slot >= (int)k.numels.size()) throw std::runtime_error("BucketReducer: bad slot");
  if (k.seen[slot]) throw std::runtime_error("BucketReducer: parameter marked ready twice in one iteration");
  k.seen[slot] = 1;
  float* view = k.buf + k.offs[slot];
  if (grad) launch_scale_copy(view, grad, k.numels[slot], 1.0f / (float)world_, stream);
  else launch_fill(view, (int64_t)k.numels[slot] * (int64_t)sizeof(float), 0, stream);
  hip_ok(hipGetLastError(), "scale_copy launch");
  k.outs[slot] = grad_out;
  if (--k.pending == 0) launch(b, stream);
}

void BucketReducer::finalize(hipStream_t stream) {
  for (size_t b = 0; b < buckets_.size(); ++b) {   // parameters that produced no gradient: zeros
    Bucket& k = buckets_[b];
    for (size_t s = 0; s < k.numels.size(); ++s)
      if (!k.seen[s]) mark_ready((int)b, (int)s, nullptr, nullptr, stream);
  }
  for (auto& k : buckets_) {
    if (!k.launched) throw std::runtime_error("BucketReducer: bucket never launched");
    hip_ok(hipStreamWaitEvent(stream, k.done, 0), "hipStreamWaitEvent");
    for (size_t s = 0; s < k.numels.size(); ++s)
      if (k.outs[s])
        hip_ok(hipMemcpyAsync(k.outs[s], k.buf + k.offs[s], k.numels[s] * sizeof(float), hipMemcpyDeviceToDevice,
                              stream), "hipMemcpyAsync");
  }
  prepare();
}

}  // namespace mnist
