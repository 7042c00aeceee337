// Native training/eval step engine for the MNIST CNN on one MI355X.
//
// This is the hot loop of reference mnist_ddp.py:65-86 (train) and :89-105 (test) re-designed
// for the GPU: the dataset is HBM resident, every step is a fixed sequence of hand-written kernels
// (no host work, no sync), and whole chunks of steps are captured once into hipGraphs and replayed.
//
// Schedules (set_schedule; C = compute stream, M = comm stream, [k] = device counter sync_[k]):
//   SERIAL   (single GPU, fallback)  C: trunk, fc1, head, fc_bwd, wgrad, dgrad, reduce+update(all)
//   OVERLAP  (single GPU, default)   C: trunk(hold [1]>=[0]), fc1, head, fc_bwd, wgrad(+[0]),
//                                       dgrad(+[4]), conv1 reduce+update(hold [3]>=[4])
//                                    M: (+[3] of the previous step) wait [0]: fc update (hold [4]>=[3]+1),
//                                       conv2 reduce+update (+[1] at start); chunk end: +[3]
//   RCCL     (DDP over RCCL)         C: trunk(hold [1]>=[0]), fc1, head, fc_bwd -ev_fc-> wgrad(+[0]),
//                                       dgrad, conv reduce, (wait ev_done) all-reduce(conv), update(conv)
//                                    M: (wait ev_fc) all-reduce(fc) -ev_done->, update(fc), +[1]
//                                    one communicator, collectives issued and run in step order fc ->
//                                    conv (graph edges); the fc update is ordered by the counters
//                                    (set_rccl_handoff; off: update(fc) before ev_done): one graph per chunk
//   XGMI     (DDP over the direct xGMI kernels) the OVERLAP structure with the all-reduces fused in:
//                                    M: fc all-reduce+update (xgmi_fc_fused), conv2 reduce+all-reduce+
//                                    update; C: conv1 reduce+all-reduce+update (fuse off: separate
//                                    all-reduce / update launches, conv bucket after dgrad on C)
// OVERLAP and XGMI chunks are captured as two graphs (M chain, C chain) launched concurrently from two
// host threads (capture_train_split); a chunk's first fork and last join are replay events.
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
  // fp32: the --dtype fp32 step (f32_net.hip: f32-input MFMA GEMMs, fp32 activations); SERIAL
  // (single GPU), RCCL (one all-reduce of the whole gradient before the update) or XGMI (one two-shot
  // xGMI all-reduce of the whole gradient with the update fused) schedules, all on the compute stream
  Engine(const EngineBuffers& buf, int max_batch, int max_test_batch, hipStream_t compute,
         hipStream_t comm, int world_size, float rho, float eps, float weight_decay, bool fp32 = false);
  ~Engine();

  enum Schedule : int { SERIAL = 0, OVERLAP = 1, RCCL = 2, XGMI = 3 };
  void attach_comm(std::shared_ptr<RcclComm> comm);   // RCCL schedule transport (+ parameter broadcast)
  // direct xGMI all-reduce (channels XGMI_CH_CONV / XGMI_CH_FC / XGMI_CH_CONV2 over x->in() -> x->out());
  // while attached the gradient producers write x->in() instead of buf.grad
  void attach_xgmi(std::shared_ptr<XgmiComm> x);
  static constexpr int XGMI_CH_CONV = 0, XGMI_CH_FC = 1, XGMI_CH_CONV2 = 2;
  // xGMI: fold the Adadelta steps into the all-reduce kernels (fc: gather phase; conv2 on the comm
  // stream and conv1 on compute: slab reduce + one-shot + update in one launch each).  Off = separate
  // reduce / all-reduce / update launches (the A/B oracle of the fused kernels' bits).
  void set_xgmi_fuse_update(bool on) { xgmi_fuse_update_ = on; }
  void set_bucket_split(bool two_buckets) { two_buckets_ = two_buckets; }   // RCCL: 2 buckets or 1
  // RCCL two-bucket schedule: the fc update after the join, ordered by device-counter holds (needs
  // the compute / comm streams on distinct hardware queues: probe_stream_handoff); off = the update
  // before the join (graph edges only)
  void set_rccl_handoff(bool on) { rccl_handoff_ = on; }
  // side schedules: fc_bwd's weight-gradient roles on the comm stream (default on): role A alone for
  // B > 1024 (lean kernel ahead of the split reduce), roles C + A for B <= 1024 in the chained OVERLAP /
  // XGMI schedules (released by fc_bwd's start)
  void set_fc_dw1_side(bool on) { fc_dw1_side_ = on; }
  bool fc_dw1_side() const { return fc_dw1_side_; }
  // test hook: the second w1t copy (fc update beside fc_bwd role B); off reintroduces the race it fixes
  void set_w1t_pingpong(bool on) { w1t_pingpong_ = on; }
  bool w1t_pingpong() const { return w1t_pingpong_; }
  // single-GPU OVERLAP step tail: conv1's reduce + update on 80 one-wave workgroups (1) or as the 20
  // conv1 parts of the 256-thread reduce launch (0); bitwise equal (A/B hook)
  void set_c1_lanes(bool on) { c1_lanes_ = on; }
  bool c1_lanes() const { return c1_lanes_; }
  // Selects the schedule (checks its transport is attached), waits for all streams and zeroes the
  // hand-off counters and their error flag, so a schedule never inherits another's counts (e.g. an
  // aborted validation).  Detaching the xgmi communicator of the XGMI schedule unsets the schedule.
  void set_schedule(int s);
  int schedule() const { return sched_; }
  void reset_counters();
  // OVERLAP / XGMI spin on one stream until the other signals; that is only deadlock-free when the
  // compute and comm streams sit on different hardware queues (HIP shares queues beyond
  // GPU_MAX_HW_QUEUES).  Each stream waits (spin kernel, `timeout_s`) for a signal enqueued on the
  // other afterwards; true if both hand-offs completed.  Eager, no graph; call before training.
  bool probe_stream_handoff(double timeout_s);
  // fault injection (tests): hold the compute stream (a spinning one-workgroup kernel, `timeout_s`)
  // until fault_release, launched on another stream, lets it go
  void fault_hold(double timeout_s);
  void fault_release(hipStream_t s);

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
  // device error flags: (stream hand-off timeout, xGMI error code); a 4-byte D2H each, call
  // after the work of interest has completed (e.g. once per epoch)
  std::pair<int, int> errors() const;
  void check_errors() const;                         // throws with a decoded message
  static std::string describe_xgmi_error(int code);
  int64_t workspace_bytes() const { return ws_bytes_; }
  bool fp32() const { return f32_; }

  // single-op entry points used by the numerics tests / module API
  const EngineBuffers& buffers() const { return buf_; }

 private:
  void enqueue_step(int batch, bool last);
  void enqueue_step_f32(int batch, bool last);
  F32Step f32_args() const;
  bool side_schedule() const { return sched_ == OVERLAP || sched_ == XGMI; }
  bool probe_stream_pair(hipStream_t x, hipStream_t y, double timeout_s);
  int capture_train_split(int n, int batch);
  void reset_host_state();
  void side_worker(int k);
  void enqueue_eval(int n_total, int batch);
  void alloc_workspace();
  void alloc_workspace_f32();

  EngineBuffers buf_;
  int max_batch_, max_test_batch_;
  hipStream_t compute_, comm_stream_;
  int world_;
  float rho_, eps_, wd_;
  bool two_buckets_ = true;
  bool rccl_handoff_ = false;
  bool fc_dw1_side_ = true;
  bool w1t_pingpong_ = true;
  bool c1_lanes_ = true;
  int idx_stride_ = 0;
  int sched_ = SERIAL;
  std::shared_ptr<RcclComm> comm_;
  std::shared_ptr<XgmiComm> xgmi_;
  float* grad_own_ = nullptr;       // buf_.grad as given (restored when the xGMI comm is detached)
  bool xgmi_fuse_update_ = true;
  bool side_pending_ = false;       // the previous step's fc update is not joined yet
  bool side_forked_ = false;        // comm stream already ordered after this chunk's start
  bool comm_sig3_pending_ = false;  // OVERLAP chain: the last conv2 update's [3] signal is owed
  int* sync_ = nullptr;             // [0] wgrad starts (fc grads final), [1] fc updates done, [2] error,
                                    // [3] conv2 updates done, [4] dgrad starts, [5] fc_bwd starts,
                                    // [8..11] probe scratch,
                                    // [12..15] fault-injection hold
  // split capture: which stream's pass enqueue_step feeds (main = compute, side = comm)
  bool enq_main_ = true, enq_side_ = true;
  bool skip_join_ = false;                    // split capture: the chunk-end join is a replay event
  std::vector<hipGraphExec_t> side_graphs_;   // per graph id: its side-chain graph (split capture) or null
  hipEvent_t ev_fork_ = nullptr;
  // side-graph launcher: the comm stream's graph on its own host thread, concurrently with the compute
  // graph's launch on the calling thread
  struct SideLauncher {
    std::thread thread;
    std::mutex mu;
    std::condition_variable cv;
    hipGraphExec_t job = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t join = nullptr;                // recorded on `stream` after the graph (chunk-end join)
    bool done = false, stop = false;
    hipError_t err = hipSuccess;
  };
  SideLauncher side_[1];
  void side_start(int k, hipGraphExec_t g, hipStream_t s);
  hipError_t side_wait(int k);
  bool trace_ = false;              // profile_steps: roctx range + drain per phase
  void phase_begin(const char* name);
  void phase_end();
  float* c1red_ = nullptr;          // conv1 partial group sums (large batches)
  uint16_t* w2d_alt_ = nullptr;     // second dgrad-layout conv2 shadow (conv2 update on the comm stream)
  bool w2d_in_alt_ = false;         // enqueue-time: the current w2d lives in w2d_alt_
  uint16_t* w1t_alt_ = nullptr;     // second transposed fc1 shadow (side fc weight gradients: the fc
                                    // update of step k runs beside fc_bwd role B, which reads w1t)
  bool w1t_in_alt_ = false;         // enqueue-time: the current w1t lives in w1t_alt_
  hipEvent_t ev_fc_ = nullptr, ev_done_ = nullptr;
  // workspace
  int64_t ws_bytes_ = 0;
  void* ws_ = nullptr;
  uint16_t *a1_, *p_, *dz1_, *h_bf_, *dl_bf_;
  uint8_t* dyc_;                     // compact un-pooled gradient records (DYC_REC per pooled position)
  uint8_t* pmask_;
  float *z1part_, *loss_rows_, *c1part_, *w2part_, *fcpart_;
  // fp32 mode workspace (F32Step's buffers)
  bool f32_ = false;
  void* ws32_ = nullptr;
  F32Step f32ws_{};
  std::vector<hipGraphExec_t> graphs_;
  std::vector<hipGraph_t> graph_defs_;
};

}  // namespace mnist
