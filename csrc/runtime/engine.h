// Native training/eval step engine for the MNIST CNN on one MI355X.
//
// This is the hot loop of reference mnist_ddp.py:65-86 (train) and :89-105 (test) re-designed
// for the GPU: the dataset is HBM resident, every step is a fixed sequence of 8 hand-written
// kernels (no host work, no sync), DDP gradient averaging is an RCCL all-reduce per gradient
// bucket on a second stream overlapped with the remaining backward kernels, and whole chunks of
// steps are captured once into a hipGraph and replayed (launch overhead amortised to ~0).
//
// Per training step: three streams whose cross-stream events become parallel branches of the
// captured graph (compute C, wgrad W, comm/optimizer M):
//   C: trunk_fwd -> fc1_fwd -> head_train -> fc_bwd -ev_fc-> conv2_dgrad -(wait ev_w)-> reduce -ev_conv->
//   W:                                          wait ev_fc: conv2_wgrad -ev_w->
//   M:                                          wait ev_fc: [allreduce(fc bucket)] -> adadelta(fc)
//                                               wait ev_conv: [allreduce(conv bucket)] -> adadelta(conv, step++) -ev_done-> C
// The fc-bucket all-reduce + its Adadelta update (98.4 % of parameters) overlap the whole conv
// backward; conv2 wgrad overlaps conv2 dgrad.  With world_size == 1 the all-reduces are skipped.
#pragma once
#include <stdlib.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <string>
#include <utility>
#include <vector>

#include "../include/kernels.h"
#include "rccl_comm.h"
#include "xgmi_comm.h"

namespace mnist {

struct EngineBuffers {
  // model / optimizer state (allocated by the Python side so parameters are torch tensors)
  float* param = nullptr;       // flat fp32 [PARAM_TOTAL]
  float* grad = nullptr;        // flat fp32 [PARAM_TOTAL] (= DDP bucket storage)
  float* square_avg = nullptr;
  float* acc_delta = nullptr;
  float* lr = nullptr;          // device scalar
  uint16_t* w2f = nullptr;
  uint16_t* w2d = nullptr;
  uint16_t* w1 = nullptr;
  uint16_t* w1t = nullptr;
  StepState* state = nullptr;
  float* loss_log = nullptr;    // [max steps per epoch]
  // datasets (HBM resident)
  const uint8_t* train_u8 = nullptr;
  const int32_t* train_labels = nullptr;
  const int32_t* train_idx = nullptr;   // [steps * B] this rank's epoch order
  uint8_t* epoch_u8 = nullptr;          // optional [steps * B][784] pre-gathered rows (gather_rows)
  int32_t* epoch_labels = nullptr;      // optional [steps * B]
  const uint8_t* test_u8 = nullptr;
  const int32_t* test_labels = nullptr;
  const int32_t* test_idx = nullptr;    // [N_test]
  float* test_loss_rows = nullptr;      // [N_test]
  int32_t* test_correct = nullptr;      // [N_test]
};

class Engine {
 public:
  Engine(const EngineBuffers& buf, int max_batch, int max_test_batch, hipStream_t compute,
         hipStream_t comm, int world_size, float rho, float eps, float weight_decay);
  ~Engine();

  void attach_comm(std::shared_ptr<RcclComm> comm);   // enables the overlapped DDP path
  // optional second communicator for the fc bucket (opt-in, MNIST_AMD_RCCL_COMMS=2): its all-reduce
  // may then overlap the conv bucket's on the first.  Concurrent collectives on two communicators are
  // deadlock-prone in NCCL/RCCL, so by default schedule 3 runs both buckets on ONE communicator,
  // ordered fc -> conv by a device counter (see enqueue_step)
  void attach_comm2(std::shared_ptr<RcclComm> comm);
  // direct xGMI all-reduce (channels XGMI_CH_CONV / XGMI_CH_FC over x->in() -> x->out()) in place
  // of the RCCL all-reduces of schedule 3; while attached the gradient producers write x->in()
  // instead of buf.grad; RCCL stays attached for the parameter broadcast
  void attach_xgmi(std::shared_ptr<XgmiComm> x);
  static constexpr int XGMI_CH_CONV = 0, XGMI_CH_FC = 1, XGMI_CH_CONV2 = 2;
  // xGMI fused schedule, conv bucket split (needs a 3-channel communicator and a third stream that
  // passes probe_stream_handoff): conv2.weight/bias (98 % of the conv bucket, final after
  // conv2_wgrad) are reduced, exchanged and updated on `conv2_stream` while conv2_dgrad runs; only
  // conv1's 320 values follow dgrad on the critical path (and that launch holds its completion until
  // the conv2 update is published, so the next trunk_fwd reads the new conv2 weights)
  void set_conv_split(bool on, uintptr_t conv2_stream);
  // xGMI: fold the Adadelta steps into the all-reduce kernels (fc: gather phase; conv: slab reduce
  // + one-shot + update in one launch).  Off = separate reduce / all-reduce / update launches.
  void set_xgmi_fuse_update(bool on) { xgmi_fuse_update_ = on; }
  void set_bucket_split(bool two_buckets) { two_buckets_ = two_buckets; }
  void set_concurrent(bool on);      // multi-stream single-GPU graph (creates the wgrad stream)
  // DDP schedule: 0 = conv backward on the forked branch, conv bucket + update on the comm stream;
  // 1 = only the fc bucket all-reduce + fc update fork off, everything else stays on compute;
  // 2 (needs attach_comm2) = as 1, but the fc branch is joined just before the next step's fc1,
  //   so it overlaps the conv backward, the conv bucket, the conv update AND the next trunk_fwd;
  // 3 = as 2, but the per-step fork / join are device-counter hand-offs (one-WG signal / wait
  //   kernels) instead of captured cross-queue edges; only each chunk's first fork and last join
  //   are graph edges.  Needs only attach_comm (or the xGMI comm): with one RCCL communicator the
  //   conv all-reduce waits on a counter for the fc all-reduce of the same step
  void set_dist_schedule(int s) { dist_sched_ = s; }
  // Schedule 3 spins on one stream until the other signals; that is only deadlock-free when the
  // compute and comm streams sit on different hardware queues (HIP shares queues beyond
  // GPU_MAX_HW_QUEUES).  Each stream waits (spin kernel, `timeout_s`) for a signal enqueued on the
  // other afterwards; true if both hand-offs completed.  Eager, no graph; call before training.
  bool probe_stream_handoff(double timeout_s);
  bool probe_stream_pair(hipStream_t x, hipStream_t y, double timeout_s);
  // single GPU: fold the fc Adadelta step into fc_bwd (FcUpdate; bitwise equal either way, off by
  // default: measured 87.2 vs 85.9 us/step at B = 200)
  void set_fuse_fc_update(bool on) { fuse_fc_update_ = on; }
  // single GPU: run the fc Adadelta step on the comm stream, overlapped with the conv backward, with
  // the schedule-3 device-counter hand-offs (needs probe_stream_handoff() to pass)
  void set_overlap_fc_update(bool on) { overlap_fc_update_ = on; }
  // single-GPU overlap schedule: the conv2 slab reduce + conv2 update ride in the dgrad launch
  // (launch_conv_dgrad_update, w2d ping-pong); only the conv1 part stays in the step tail
  void set_dgrad_update(bool on) { dgrad_update_ = on; }
  // schedule-3 chunks as two graphs (side chain + compute chain) launched concurrently from two host
  // threads (default on; see capture_train_split).  Off: one multi-stream graph per chunk.
  void set_side_first(bool on) { side_first_ = on; }
  // single-GPU overlap schedule: conv2's slab reduce + update on the comm stream under conv2_dgrad
  void set_side_conv2(bool on) { side_conv2_ = on; }


  // --- training
  void begin_epoch(uint64_t seed, uint64_t rng_base, int step0, int flags);   // 24-byte H2D, eager
  // enqueue n steps eagerly; `stride` = full batch size (row offset of step s is s*stride)
  void train_steps(int n, int batch, int stride);
  int capture_train(int n, int batch, int stride);   // capture n steps into a graph, returns id
  // profiling window: n eager steps, each phase (fwd, fc bwd, conv wgrad, fc all-reduce + update,
  // conv dgrad, conv all-reduce + update) inside its own roctx range and drained before the range
  // closes, so rocprofv3 --marker-trace attributes device time per phase (serialised: the DDP
  // overlap is given up inside the window; results are bitwise those of the graph path)
  void profile_steps(int n, int batch, int stride);
  void replay(int graph_id);
  // device-side DataLoader: pre-gather epoch rows [start, start+n) (needs epoch_u8/epoch_labels);
  // the step kernels then read the batch directly instead of through the index vector
  void gather_rows(int64_t start, int64_t n);
  // --- eval (SequentialSampler over the test set, `n_batches` of `batch`, last may be short)
  void eval(int n_total, int batch);
  int capture_eval(int n_total, int batch);
  // --- misc
  void refresh_shadows();
  void broadcast_params(int root);                   // DDP construction: rank-0 params to all
  void synchronize();                                // all streams, then check_errors()
  void sync_streams();                               // all streams, no error-flag read-back
  // device error flags: (schedule-3 hand-off timeout, xGMI error code); a 4-byte D2H each, call
  // after the work of interest has completed (e.g. once per epoch)
  std::pair<int, int> errors() const;
  void check_errors() const;                         // throws with a decoded message
  static std::string describe_xgmi_error(int code);
  int64_t workspace_bytes() const { return ws_bytes_; }

  // single-op entry points used by the numerics tests / module API
  const EngineBuffers& buffers() const { return buf_; }

 private:
  void enqueue_step(int batch, bool last);
  bool uses_side_streams() const;
  int capture_train_split(int n, int batch);
  void reset_host_state();
  void side_worker();
  void enqueue_eval(int n_total, int batch);
  void alloc_workspace();

  EngineBuffers buf_;
  int max_batch_, max_test_batch_;
  hipStream_t compute_, comm_stream_;
  int world_;
  float rho_, eps_, wd_;
  bool two_buckets_ = true;
  int idx_stride_ = 0;
  bool concurrent_ = false;
  int dist_sched_ = 1;
  std::shared_ptr<RcclComm> comm_, comm2_;
  std::shared_ptr<XgmiComm> xgmi_;
  float* grad_own_ = nullptr;       // buf_.grad as given (restored when the xGMI comm is detached)
  bool xgmi_fuse_update_ = true;
  bool side_pending_ = false;       // schedule 2/3: the previous step's fc branch is not joined yet
  bool side_forked_ = false;        // schedule 3: comm stream already ordered after this chunk's start
  int* sync_ = nullptr;             // [0] fc grads ready count, [1] fc update done count, [2] error,
                                    // [3]/[4] conv split, [8..11] probes, [16..31] / [32..47] fc1+head
                                    // tile counters (FC1_HEAD_MAX_TILES each),
                                    // [12] fc all-reduce done (1 comm)
  bool fuse_fc_update_ = false;
  bool overlap_fc_update_ = false;
  bool dgrad_update_ = true;
  bool side_first_ = true;
  bool side_conv2_ = false;
  bool enq_main_ = true, enq_side_ = true;   // two-pass capture: which streams enqueue_step feeds
  bool enq_side2_ = true;                     // split capture: the third (conv2) stream's pass
  bool skip_join_ = false;                    // split capture: the chunk-end join is a replay event
  std::vector<hipGraphExec_t> side_graphs_;   // per graph id: its side-chain graph (split capture) or null
  std::vector<hipGraphExec_t> side2_graphs_;  // per graph id: its conv2-stream graph (third-stream split) or null
  hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr, ev_join2_ = nullptr;
  std::thread side_thread_;                   // launches side graphs concurrently with the compute graph
  std::mutex side_mu_;
  std::condition_variable side_cv_;
  hipGraphExec_t side_job_ = nullptr, side2_job_ = nullptr;
  bool side_done_ = false, side_stop_ = false;
  hipError_t side_err_ = hipSuccess;
  bool conv_split_ = false;
  hipStream_t conv2_stream_ = nullptr;   // owned by the caller (torch stream)
  hipEvent_t ev_c2_ = nullptr;
  bool trace_ = false;              // profile_steps: roctx range + drain per phase
  void phase_begin(const char* name);
  void phase_end();
  uint16_t* w1t_alt_ = nullptr;     // second transposed fc1 shadow (fused fc update ping-pong)
  bool w1t_in_alt_ = false;         // enqueue-time: the current w1t lives in w1t_alt_
  float* c1red_ = nullptr;          // conv1 partial group sums (large batches)
  // MNIST_AMD_C1_PREREDUCE=0 turns the large-batch conv1 pre-reduce off (A/B, numerics checks)
  bool c1_prereduce_ = [] { const char* e = getenv("MNIST_AMD_C1_PREREDUCE"); return !(e && e[0] == '0'); }();
  uint16_t* w2d_alt_ = nullptr;     // second dgrad-layout conv2 shadow (conv split / dgrad_update ping-pong)
  bool w2d_in_alt_ = false;
  hipEvent_t ev_fc_ = nullptr, ev_conv_ = nullptr, ev_done_ = nullptr, ev_w_ = nullptr;
  hipStream_t wgrad_stream_ = nullptr;
  // workspace
  int64_t ws_bytes_ = 0;
  void* ws_ = nullptr;
  uint16_t *a1_, *p_, *dz1_, *h_bf_, *dl_bf_;
  uint8_t* dyc_;                     // compact un-pooled gradient records (DYC_REC per pooled position)
  uint8_t* pmask_;
  float *z1part_, *loss_rows_, *c1part_, *w2part_, *fcpart_;
  std::vector<hipGraphExec_t> graphs_;
  std::vector<hipGraph_t> graph_defs_;
};

}  // namespace mnist
