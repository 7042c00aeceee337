#include "engine.h"
#include "host_logic.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace mnist {

#define HIP_OK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess)                                                                  \
      throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_));           \
  } while (0)

namespace {
inline int round_up(int x, int m) { return (x + m - 1) / m * m; }
}  // namespace

Engine::Engine(const EngineBuffers& buf, int max_batch, int max_test_batch, hipStream_t compute,
               hipStream_t comm, int world_size, float rho, float eps, float weight_decay, bool fp32)
    : buf_(buf), max_batch_(max_batch), max_test_batch_(max_test_batch), compute_(compute),
      comm_stream_(comm), world_(world_size), rho_(rho), eps_(eps), wd_(weight_decay), f32_(fp32) {
  if (max_batch < 1 || max_test_batch < 0) throw std::runtime_error("bad batch sizes");
  HIP_OK(hipEventCreateWithFlags(&ev_fc_, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&ev_done_, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming));
  for (SideLauncher& l : side_) HIP_OK(hipEventCreateWithFlags(&l.join, hipEventDisableTiming));
  alloc_workspace();
  if (f32_) alloc_workspace_f32();
}

Engine::~Engine() {
  for (SideLauncher& l : side_) {
    if (l.thread.joinable()) {
      {
        std::lock_guard<std::mutex> lk(l.mu);
        l.stop = true;
      }
      l.cv.notify_all();
      l.thread.join();
    }
    if (l.join) hipEventDestroy(l.join);
  }
  for (auto g : side_graphs_)
    if (g) hipGraphExecDestroy(g);
  for (auto g : graphs_) hipGraphExecDestroy(g);
  for (auto g : graph_defs_) hipGraphDestroy(g);
  for (hipEvent_t e : {ev_fc_, ev_done_, ev_fork_})
    if (e) hipEventDestroy(e);
  if (ws_) hipFree(ws_);
  if (ws32_) hipFree(ws32_);
}

void Engine::alloc_workspace() {
  const WorkspaceLayout L =
      compute_workspace_layout(max_batch_, max_test_batch_, conv_wgrad_groups(max_batch_), fc_bwd_splits(max_batch_));
  ws_bytes_ = L.total;
  HIP_OK(hipMalloc(&ws_, ws_bytes_));
  launch_fill(ws_, ws_bytes_, 0, nullptr);   // padding rows of p etc. must be finite
  HIP_OK(hipStreamSynchronize(nullptr));
  char* base = static_cast<char*>(ws_);
  a1_ = reinterpret_cast<uint16_t*>(base + L.a1);
  p_ = reinterpret_cast<uint16_t*>(base + L.p);
  pmask_ = reinterpret_cast<uint8_t*>(base + L.pmask);
  z1part_ = reinterpret_cast<float*>(base + L.z1part);
  loss_rows_ = reinterpret_cast<float*>(base + L.loss_rows);
  dz1_ = reinterpret_cast<uint16_t*>(base + L.dz1);
  h_bf_ = reinterpret_cast<uint16_t*>(base + L.h_bf);
  dl_bf_ = reinterpret_cast<uint16_t*>(base + L.dl_bf);
  dyc_ = reinterpret_cast<uint8_t*>(base + L.dyc);
  c1part_ = reinterpret_cast<float*>(base + L.c1part);
  w2part_ = reinterpret_cast<float*>(base + L.w2part);
  fcpart_ = reinterpret_cast<float*>(base + L.fcpart);
  sync_ = reinterpret_cast<int*>(base + L.sync);
  w2d_alt_ = reinterpret_cast<uint16_t*>(base + L.w2d_alt);
  c1red_ = reinterpret_cast<float*>(base + L.c1red);
  w1t_alt_ = reinterpret_cast<uint16_t*>(base + L.w1t_alt);
}

void Engine::alloc_workspace_f32() {
  const int64_t M = max_batch_, Ma = max_batch_ > max_test_batch_ ? max_batch_ : max_test_batch_;
  // fc1 split-K partials: 36 splits up to 1024 rows, 9 beyond (f32_fc1_splits), for any batch <= Ma
  const int64_t z1rows = std::max<int64_t>(36 * std::min<int64_t>(Ma, 1024), 9 * Ma);
  int64_t off = 0;
  auto carve = [&](int64_t bytes) { int64_t o = off; off += ws_align256(bytes); return o; };
  const int64_t o_w2f = carve(9 * C1 * C2 * 4), o_w2b = carve(9 * C1 * C2 * 4), o_w1p = carve((int64_t)NH * NFLAT * 4);
  const int64_t o_a1 = carve(Ma * H1 * H1 * C1 * 4), o_y2 = carve(Ma * H2 * H2 * C2 * 4);
  const int64_t o_p = carve(Ma * NFLAT * 4), o_pm = carve(Ma * NFLAT), o_z1 = carve(z1rows * NH * 4);
  const int64_t o_h = carve(M * NH * 4), o_dz1 = carve(M * NH * 4), o_dl = carve(M * 16 * 4);
  const int64_t o_loss = carve(M * 4);
  const int64_t o_c2 = carve((int64_t)F32_MAX_SPLITS * C2 * (9 * C1 + 1) * 4);
  const int64_t o_c1 = carve((int64_t)F32_C1W_BLOCKS * C1 * 10 * 4);
  const int64_t o_dx1 = carve(M * H1 * H1 * C1 * 4);
  HIP_OK(hipMalloc(&ws32_, off));
  launch_fill(ws32_, off, 0, nullptr);
  HIP_OK(hipStreamSynchronize(nullptr));
  ws_bytes_ += off;
  char* b = static_cast<char*>(ws32_);
  F32Step& w = f32ws_;
  w.w2fwd = reinterpret_cast<float*>(b + o_w2f);
  w.w2bwd = reinterpret_cast<float*>(b + o_w2b);
  w.w1p = reinterpret_cast<float*>(b + o_w1p);
  w.a1 = reinterpret_cast<float*>(b + o_a1);
  w.dx1 = reinterpret_cast<float*>(b + o_dx1);
  w.y2 = reinterpret_cast<float*>(b + o_y2);
  w.p = reinterpret_cast<float*>(b + o_p);
  w.pm = reinterpret_cast<uint8_t*>(b + o_pm);
  w.z1part = reinterpret_cast<float*>(b + o_z1);
  w.h = reinterpret_cast<float*>(b + o_h);
  w.dz1 = reinterpret_cast<float*>(b + o_dz1);
  w.dl = reinterpret_cast<float*>(b + o_dl);
  w.loss_rows = reinterpret_cast<float*>(b + o_loss);
  w.c2part = reinterpret_cast<float*>(b + o_c2);
  w.c1part = reinterpret_cast<float*>(b + o_c1);
}

F32Step Engine::f32_args() const {
  F32Step a = f32ws_;
  a.param = buf_.param;
  a.grad = buf_.grad;
  a.loss_log = buf_.loss_log;
  return a;
}

void Engine::attach_comm(std::shared_ptr<RcclComm> comm) {
  if (comm && comm->world_size() != world_) throw std::runtime_error("comm world size mismatch");
  comm_ = std::move(comm);
}

void Engine::attach_xgmi(std::shared_ptr<XgmiComm> x) {
  if (x && x->world_size() != world_) throw std::runtime_error("xgmi world size mismatch");
  if (x && x->world_size() > 1 && !x->connected()) throw std::runtime_error("xgmi communicator not connected");
  if (x && x->numel() != PARAM_TOTAL) throw std::runtime_error("xgmi communicator must cover the flat gradient");
  if (x && x->channels() <= XGMI_CH_CONV2) throw std::runtime_error("xgmi communicator needs 3 channels");
  if (!x && sched_ == XGMI) {           // no schedule until set_schedule (enqueue refuses SERIAL at world > 1)
    sync_streams();
    sched_ = SERIAL;
  }
  if (!grad_own_) grad_own_ = buf_.grad;
  // the gradient producers write straight into the communicator's (IPC-exported) input buffer
  buf_.grad = x ? x->in() : grad_own_;
  xgmi_ = std::move(x);
}

void Engine::set_schedule(int s) {
  if (s == SERIAL || s == OVERLAP) {
    if (world_ != 1 || comm_ || xgmi_)
      throw std::runtime_error("engine: the single-GPU schedules need world size 1 and no transport attached");
  } else if (s == RCCL) {
    if (!comm_) throw std::runtime_error("engine: the RCCL schedule needs an RCCL communicator");
    if (xgmi_) throw std::runtime_error("engine: detach the xgmi communicator before selecting RCCL");
  } else if (s == XGMI) {
    if (!xgmi_) throw std::runtime_error("engine: the XGMI schedule needs an xgmi communicator");
  } else {
    throw std::runtime_error("engine: unknown schedule " + std::to_string(s));
  }
  sched_ = s;
  reset_counters();
}

void Engine::reset_counters() {
  // the hand-off counters only move in matched pairs inside a completed chunk; after a schedule
  // change or an aborted chunk they restart from zero, and so does the hand-off error flag [2]
  // (callers read it with check_errors before they get here)
  sync_streams();
  launch_fill(sync_ + 0, 6 * sizeof(int), 0, compute_);
  HIP_OK(hipStreamSynchronize(compute_));
  reset_host_state();
}

void Engine::begin_epoch(uint64_t seed, uint64_t rng_base, int step0, int flags) {
  // 24 bytes as kernel arguments, ordered on the compute stream (never inside a captured graph):
  // no host sync, so the next epoch is enqueued while the previous one still runs
  launch_set_state(buf_.state, StepState{step0, flags, seed, rng_base}, compute_);
}

void Engine::phase_begin(const char* name) {
  if (trace_) roctx_push(name);
}

void Engine::phase_end() {
  if (!trace_) return;
  HIP_OK(hipStreamSynchronize(compute_));
  HIP_OK(hipStreamSynchronize(comm_stream_));
  roctx_pop();
}

void Engine::profile_steps(int n, int batch, int stride) {
  if (batch < 1 || batch > max_batch_) throw std::runtime_error("batch exceeds engine capacity");
  idx_stride_ = stride;
  trace_ = true;
  try {
    for (int i = 0; i < n; ++i) {
      roctx_push("train_step");
      enqueue_step(batch, i == n - 1);
      HIP_OK(hipStreamSynchronize(compute_));
      roctx_pop();
    }
  } catch (...) {
    trace_ = false;
    throw;
  }
  trace_ = false;
  HIP_OK(hipGetLastError());
}

void Engine::enqueue_step(int batch, bool last) {
  // the head scales by 1/(B*world): without a transport every rank would train alone on a gradient
  // world times too small
  if (world_ > 1 && sched_ != RCCL && sched_ != XGMI)
    throw std::runtime_error("engine: world size > 1 needs the RCCL or XGMI schedule");
  if (f32_) {
    enqueue_step_f32(batch, last);
    return;
  }
  const int B = batch, Bp = round_up(B, 32);
  const int stride = idx_stride_;
  float* P = buf_.param;
  // DDP averaging: each rank's head scales the loss gradient by 1/(world*B) and the all-reduce sums,
  // so every row's bf16 gradient operands (dz1, dl) are bitwise those of the world-1 run on the
  // world*B batch (scaling by 1/B and then by 1/world rounds the fp32 constant differently and flips
  // bf16 ties: a systematic ~7e-6 gradient offset, tools/ddp_equivalence.py)
  const float gscale = kDdpEpilogueScale;
  // split capture (capture_train_split): M = enqueue the compute-stream work, S = the comm stream's
  const bool M = enq_main_, S = enq_side_;
  const bool side = side_schedule();
  const bool xg = sched_ == XGMI;

  // pre-gathered epoch rows when available (one load level less on every step's critical path)
  const bool pre = buf_.epoch_u8 != nullptr;
  const uint8_t* data = pre ? buf_.epoch_u8 : buf_.train_u8;
  const int32_t* idxp = pre ? nullptr : buf_.train_idx;
  const int32_t* labels = pre ? buf_.epoch_labels : buf_.train_labels;
  TrunkFwdArgs tf{data, idxp, stride, buf_.state, P + OFF_CONV1_W, P + OFF_CONV1_B,
                  buf_.w2f, P + OFF_CONV2_B, a1_, p_, pmask_, nullptr};
  if (side && !side_forked_) {         // once per chunk: order the comm stream after the chunk start
    HIP_OK(hipEventRecord(ev_fc_, compute_));
    HIP_OK(hipStreamWaitEvent(comm_stream_, ev_fc_, 0));
    side_forked_ = true;
  }
  // the previous step's fc update (comm stream) must be done before fc1_fwd reads w1: trunk_fwd
  // holds its completion for it (device counters, no extra launch)
  if ((side || sched_ == RCCL) && side_pending_) {
    tf.wait_a = sync_ + 1;
    tf.wait_b = sync_ + 0;
    tf.wait_err = sync_ + 2;
  }
  side_pending_ = false;
  phase_begin("fwd");
  if (M) launch_trunk_fwd(tf, B, true, compute_);
  if (M) launch_fc1_fwd(p_, buf_.w1, z1part_, B, compute_);
  HeadArgs ha{};
  ha.z1part = z1part_; ha.b_fc1 = P + OFF_FC1_B; ha.w_fc2 = P + OFF_FC2_W; ha.b_fc2 = P + OFF_FC2_B;
  ha.labels = labels; ha.idx = idxp; ha.idx_step_stride = stride;
  ha.state = buf_.state; ha.inv_batch = ddp_head_inv_batch(B, world_);
  ha.loss_rows = loss_rows_; ha.dz1 = dz1_; ha.h_bf = h_bf_; ha.dl_bf = dl_bf_;
  if (M) launch_head_train(ha, B, Bp, compute_);
  phase_end();
  FcBwdArgs fb{dz1_, p_, pmask_, buf_.w1t, h_bf_, dl_bf_, loss_rows_, buf_.state,
               buf_.grad, dyc_, buf_.loss_log, gscale, 1.0f / (float)B, fcpart_};
  // B > 1024: the fc split partials are summed on the comm stream, ahead of the fc update /
  // all-reduce that consumes them, instead of on the compute chain (SERIAL / one-bucket RCCL: here)
  const bool fc_reduce_side = fc_bwd_splits(B) > 1 && (side || (sched_ == RCCL && two_buckets_));
  // ... and the fc1 weight gradient itself (fc_bwd role A: 145 workgroups per 1024-row split streaming
  // p from HBM) leaves the compute chain for the comm stream, ahead of that reduce, where it runs
  // beside conv2_wgrad / conv2_dgrad.  The next step cannot overwrite p / dz1 before it is done: the
  // comm stream's later launches (fc update, conv2 update) gate the next trunk_fwd / fc1_fwd.
  const bool dw1_side = fc_reduce_side && fc_dw1_side_;
  // OVERLAP / XGMI chain, B <= 1024: both fc weight gradients (roles C + A, 146 workgroups) leave the
  // compute launch for the comm stream, released by fc_bwd's start (counter [5]: head_train done)
  // instead of by wgrad's start, so the fc update (or fc all-reduce + update) that follows them
  // starts ~wgrad's length earlier and the comm chain - conv2's reduce + update at its end gates the
  // next trunk_fwd - finishes earlier.  The compute chain keeps role B (dy records) only.
  const bool fcw_side = side && !trace_ && (!xg || xgmi_fuse_update_) && fc_bwd_splits(B) == 1 &&
                        fc_dw1_side_;
  // [5] counts fc_bwd starts in every schedule that counts wgrad starts in [0] (lockstep with [1])
  if (side || (sched_ == RCCL && two_buckets_)) fb.signal_ctr = sync_ + 5;
  const int roles = fcw_side ? FCB_ROLE_B : dw1_side ? (FCB_ROLE_C | FCB_ROLE_B) : FCB_ROLES_ALL;
  // ... so that fc update runs beside role B, which reads w1t: role B reads this step's copy while the
  // update writes the other (ping-pong like w2d below; every element is rewritten each step)
  uint16_t* const w1t_cur = w1t_in_alt_ ? w1t_alt_ : buf_.w1t;
  // (w1t_pingpong_ off: test hook only - the update overwrites the copy role B reads, the race the
  // ping-pong exists for; docs/DEBUGGING.md "race-window widening")
  const bool w1t_pp = fcw_side && w1t_pingpong_;
  uint16_t* const w1t_next = w1t_pp ? (w1t_in_alt_ ? buf_.w1t : w1t_alt_) : w1t_cur;
  fb.w1t = w1t_cur;
  phase_begin("bwd_fc");
  if (M) launch_fc_bwd(fb, B, Bp, compute_, !fc_reduce_side, roles);
  phase_end();

  AdadeltaArgs ad{P, buf_.grad, buf_.square_avg, buf_.acc_delta, buf_.lr, rho_, eps_, wd_,
                  buf_.w2f, buf_.w2d, buf_.w1, w1t_next, nullptr};
  ad.wt = B <= WT_MAX_B;                          // write-through stores at small batches (store16)
  if (w1t_pp) w1t_in_alt_ = !w1t_in_alt_;
  ConvBwdArgs cb{dyc_, a1_, buf_.w2d, P + OFF_CONV1_W, P + OFF_CONV1_B, data,
                 idxp, stride, buf_.state, c1part_, w2part_, buf_.grad, gscale,
                 conv_wgrad_groups(B), nullptr};
  cb.c1_rows = conv_dgrad_c1_rows(B);
  if (cb.c1_rows > C1_PRE_MIN_SLABS) cb.c1red = c1red_;   // large batch: conv1 partials pre-reduced
  cb.dgrad_full_grid = sched_ == OVERLAP || sched_ == SERIAL ? 0 : 1;
  AdadeltaArgs adc = ad;
  adc.state_inc = buf_.state;   // last kernel of the step advances the device step counter

  if (sched_ == SERIAL) {
    phase_begin("bwd_conv_wgrad");
    launch_conv_wgrad(cb, B, compute_);
    phase_end();
    phase_begin("bwd_conv_dgrad");
    launch_conv_dgrad(cb, B, compute_);
    phase_end();
    phase_begin("grad_reduce+update");          // conv slab reduce + the whole Adadelta update
    launch_adadelta_reduce(adc, cb, B, compute_);
    phase_end();
    return;
  }

  if (sched_ == RCCL) {
    if (!two_buckets_) {                        // one bucket: one all-reduce after the whole backward
      launch_conv_wgrad(cb, B, compute_);
      launch_conv_dgrad(cb, B, compute_);
      launch_conv_grad_reduce(cb, B, compute_);
      comm_->allreduce_sum(buf_.grad, PARAM_TOTAL, 0, compute_);
      launch_adadelta(adc, ADA_ALL, compute_);
      return;
    }
    // the fc bucket (98.4 % of the bytes) forks onto the comm stream as soon as fc_bwd is done and
    // overlaps the conv backward; the conv bucket follows on compute after the join, so the one
    // communicator sees fc, conv in the same order on every rank and never two collectives at once.
    // The join waits for the fc all-reduce (and conv2's slab reduce, below) only: the fc update runs
    // after them on the comm stream (144 workgroups, beside the conv tail) and is ordered before the
    // next step's fc1_fwd by trunk_fwd's completion hold on device counters ([0] wgrad starts, [1] fc
    // updates done), as in OVERLAP - at world > 1 the update is not on the path to the conv all-reduce.
    // (capture order matters: the graph executor keeps a fork's first-captured child on the
    // launching queue, so conv2 wgrad is enqueued before the comm branch)
    HIP_OK(hipEventRecord(ev_fc_, compute_));
    ConvBwdArgs cbs = cb;
    cbs.signal_ctr = sync_ + 0;                   // wgrad's start: this step's fc grads are final
    phase_begin("bwd_conv_wgrad");
    launch_conv_wgrad(cbs, B, compute_);
    phase_end();
    phase_begin("allreduce_fc+update");
    HIP_OK(hipStreamWaitEvent(comm_stream_, ev_fc_, 0));
    if (dw1_side) launch_fc_bwd_dw1(fb, B, Bp, comm_stream_);
    if (fc_reduce_side) launch_fc_grad_reduce(fb, B, comm_stream_);
    comm_->allreduce_sum(buf_.grad + OFF_FC1_W, OFF_CONV1_W - OFF_FC1_W, 0, comm_stream_);
    // hand-offs (distinct queues): conv2's slab reduce (289 of the conv bucket's 309 reduce
    // workgroups) follows the fc all-reduce on the comm stream, released by dgrad's start (wgrad,
    // which writes the slabs, is done) and running under dgrad; the join waits for it, so the step
    // tail keeps only conv1's 20 reduce workgroups before the conv all-reduce.  The fc update comes
    // after it (world 1, 600 steps: 82.5-82.6 -> 75.3 us/step; the update before it, so that the
    // join also waits for the update: 86.7; profiles/r5/ddp_world1/rccl_conv2_reduce_side.txt)
    const bool c2r = rccl_handoff_ && !trace_;
    if (c2r) {
      launch_stream_wait(sync_ + 4, sync_ + 3, 1, sync_ + 2, comm_stream_);
      launch_conv_grad_reduce_parts(cb, B, 0, RED_W2_PARTS, comm_stream_);
      launch_stream_signal(sync_ + 3, comm_stream_);
    }
    if (rccl_handoff_) {
      HIP_OK(hipEventRecord(ev_done_, comm_stream_));
      launch_adadelta(ad, ADA_FC, comm_stream_, ADA_FC_LEAN_GRID);
      launch_stream_signal(sync_ + 1, comm_stream_);  // fc update of this step done
      side_pending_ = true;
    } else {                                      // streams share a hardware queue: no counter holds
      launch_adadelta(ad, ADA_FC, comm_stream_);
      HIP_OK(hipEventRecord(ev_done_, comm_stream_));
    }
    phase_end();
    phase_begin("bwd_conv_dgrad");
    ConvBwdArgs cbd = cb;
    if (c2r) cbd.signal_ctr = sync_ + 4;        // dgrad's start releases conv2's reduce on the comm stream
    launch_conv_dgrad(cbd, B, compute_);
    phase_end();
    phase_begin("allreduce_conv+update");
    if (c2r)
      launch_conv_grad_reduce_parts(cb, B, RED_W2_PARTS, RED_ALL_PARTS, compute_);
    else
      launch_conv_grad_reduce(cb, B, compute_);
    HIP_OK(hipStreamWaitEvent(compute_, ev_done_, 0));
    comm_->allreduce_sum(buf_.grad + OFF_CONV1_W, PARAM_TOTAL - OFF_CONV1_W, 0, compute_);
    launch_adadelta(adc, ADA_CONV, compute_);
    phase_end();
    if (last && rccl_handoff_) {                  // chunk end: the comm stream joins (fc update done)
      HIP_OK(hipEventRecord(ev_done_, comm_stream_));
      HIP_OK(hipStreamWaitEvent(compute_, ev_done_, 0));
      side_pending_ = false;
    }
    return;
  }

  // ---- OVERLAP / XGMI: device-counter hand-offs between the compute and comm streams
  if (xg) ad.grad = adc.grad = xgmi_->out();    // the update reads the all-reduced gradients
  ConvBwdArgs cbs = cb;
  cbs.signal_ctr = sync_ + 0;                     // wgrad's start: fc grads of this step are final
  phase_begin("bwd_conv_wgrad");
  if (M) launch_conv_wgrad(cbs, B, compute_);
  phase_end();
  // OVERLAP (not in the traced profiling window, whose phase syncs would deadlock a hold): the comm
  // chain's hand-offs ride on its update kernels - the fc update holds its completion until dgrad
  // has started, conv2's reduce + update signals "fc update done" [1] at its start, and its own
  // "conv2 update done" [3] is signalled by the next step's first comm launch, which then waits for
  // that step's wgrad: one small launch per step instead of two waits and two signals
  // XGMI (fused kernels) runs the same chain: the fc all-reduce + update holds its completion, the
  // conv2 reduce + all-reduce + update signals [1] at its start (world-1 timeline: two hand-off launches
  // a step fewer, conv2's part no longer queued behind them)
  const bool chain = !trace_ && (!xg || xgmi_fuse_update_);
  phase_begin("allreduce_fc+update");
  if (S) {
    int* const rel = fcw_side ? sync_ + 5 : sync_ + 0;   // fc_bwd's start / wgrad's start
    if (chain && comm_sig3_pending_)
      launch_stream_signal_wait(sync_ + 3, rel, sync_ + 1, 1, sync_ + 2, comm_stream_);
    else
      launch_stream_wait(rel, sync_ + 1, 1, sync_ + 2, comm_stream_);
    comm_sig3_pending_ = false;
    FcBwdArgs fw = fb;
    fw.signal_ctr = nullptr;
    if (fcw_side && xg) launch_fc_bwd(fw, B, Bp, comm_stream_, true, FCB_ROLE_C | FCB_ROLE_A);
    if (dw1_side) launch_fc_bwd_dw1(fb, B, Bp, comm_stream_);
    if (fc_reduce_side) launch_fc_grad_reduce(fb, B, comm_stream_);
    if (!xg) {
      AdadeltaArgs af = ad;
      if (chain) {                              // completes once this step's dgrad has started
        af.hold_a = sync_ + 4;
        af.hold_b = sync_ + 3;
        af.hold_delta = 1;
        af.hold_err = sync_ + 2;
      }
      // 144 workgroups instead of 577: the update has ~15 us of slack before the next step's trunk
      // ends, and fewer co-resident waves leave wgrad / dgrad more of the CUs (600 steps, two boxes:
      // 65.9 -> 65.2, 65.0-65.7 -> 64.4-64.9 us/step; 96 / 64 workgroups: 67.6 / 74-75)
      // Side weight gradients: the update is fused into their 146 workgroups (one launch).
      if (fcw_side)
        launch_fc_wgrad_update(fw, af, B, Bp, comm_stream_);
      else
        launch_adadelta(af, ADA_FC, comm_stream_, ADA_FC_LEAN_GRID);
    } else if (xgmi_fuse_update_) {             // fc bucket all-reduce with the fc Adadelta step fused
      AdadeltaArgs af = ad;
      if (chain) {                              // completes once this step's dgrad has started
        af.hold_a = sync_ + 4;
        af.hold_b = sync_ + 3;
        af.hold_delta = 1;
        af.hold_err = sync_ + 2;
      }
      xgmi_->allreduce_fc_fused(XGMI_CH_FC, comm_stream_, af);
    } else {
      xgmi_->allreduce(XGMI_CH_FC, OFF_FC1_W, OFF_CONV1_W - OFF_FC1_W, comm_stream_);
      launch_adadelta(ad, ADA_FC, comm_stream_);
    }
    if (!chain) launch_stream_signal(sync_ + 1, comm_stream_);   // fc update of this step done
  }
  phase_end();
  side_pending_ = true;
  if (xg && !xgmi_fuse_update_) {
    // separate launches (reference for the fused kernels' bits): the conv bucket after dgrad
    phase_begin("bwd_conv_dgrad");
    if (M) launch_conv_dgrad(cb, B, compute_);
    phase_end();
    phase_begin("allreduce_conv+update");
    if (M) {
      launch_conv_grad_reduce(cb, B, compute_);
      xgmi_->allreduce(XGMI_CH_CONV, OFF_CONV1_W, PARAM_TOTAL - OFF_CONV1_W, compute_);
      launch_adadelta(adc, ADA_CONV, compute_);
    }
    phase_end();
  } else {
    // conv2's slab reduce (+ exchange) + update on the comm stream after the fc update, released by
    // dgrad's start (= wgrad done, counter [4]) and running under conv2_dgrad, which reads this step's
    // w2d while the update writes the other copy (ping-pong, host-tracked and static within a
    // captured chunk; a chunk that ends on the alternate copy copies it back); counter [3] = conv2
    // updates published.  Only conv1's part (20 reduce workgroups) stays on the compute stream, and
    // that launch holds its completion until [3] catches up, so the next trunk_fwd reads the new
    // conv2 weights.
    uint16_t* w2d_cur = w2d_in_alt_ ? w2d_alt_ : buf_.w2d;
    AdadeltaArgs u2 = adc;
    u2.state_inc = nullptr;
    u2.w2d = w2d_in_alt_ ? buf_.w2d : w2d_alt_;
    cb.w2d = w2d_cur;
    hipStream_t s2 = comm_stream_;
    if (S) {
      if (!chain) launch_stream_wait(sync_ + 4, sync_ + 3, 1, sync_ + 2, s2);
      if (chain) u2.signal_start = sync_ + 1;     // the fc update (previous launch) is done
      if (xg) {
        XgmiConvPart p2;
        p2.lo = 0;
        p2.hi = RED_W2_PARTS;
        xgmi_->conv_reduce_fused(XGMI_CH_CONV2, cb, B, comm_stream_, u2, p2);
      } else {
        launch_adadelta_reduce_parts(u2, cb, B, 0, RED_W2_PARTS, s2);
      }
      if (chain && !last)
        comm_sig3_pending_ = true;                // signalled by the next step's first comm launch
      else
        launch_stream_signal(sync_ + 3, s2);
    }
    ConvBwdArgs cbd = cb;
    cbd.signal_ctr = sync_ + 4;
    phase_begin("bwd_conv_dgrad");
    if (M) launch_conv_dgrad(cbd, B, compute_);
    phase_end();
    phase_begin("allreduce_conv1+update");
    if (M && xg) {
      XgmiConvPart p1;
      p1.lo = RED_W2_PARTS;
      p1.hi = RED_ALL_PARTS;
      p1.wait_a = sync_ + 3;
      p1.wait_b = sync_ + 4;
      p1.wait_err = sync_ + 2;
      xgmi_->conv_reduce_fused(XGMI_CH_CONV, cb, B, compute_, adc, p1);
    } else if (M) {
      AdadeltaArgs u1 = adc;
      u1.hold_a = sync_ + 3;
      u1.hold_b = sync_ + 4;
      u1.hold_err = sync_ + 2;
      if (c1_lanes_)
        launch_adadelta_c1(u1, cb, B, compute_);
      else
        launch_adadelta_reduce_parts(u1, cb, B, RED_W2_PARTS, RED_ALL_PARTS, compute_);
    }
    phase_end();
    w2d_in_alt_ = !w2d_in_alt_;
    if (last && w1t_in_alt_) {                  // after the conv1 part: the fc update is published
      if (M)
        HIP_OK(hipMemcpyAsync(buf_.w1t, w1t_alt_, (size_t)NFLAT * NH * sizeof(uint16_t), hipMemcpyDeviceToDevice,
                              compute_));
      w1t_in_alt_ = false;
    }
    if (last && w2d_in_alt_) {
      if (M)
        HIP_OK(hipMemcpyAsync(buf_.w2d, w2d_alt_, (size_t)9 * C1 * C2 * sizeof(uint16_t), hipMemcpyDeviceToDevice,
                              compute_));
      w2d_in_alt_ = false;
    }
  }
  if (last) {                                              // chunk end: one real join edge
    if (M && !skip_join_) {
      HIP_OK(hipEventRecord(ev_done_, comm_stream_));
      HIP_OK(hipStreamWaitEvent(compute_, ev_done_, 0));
    }
    side_pending_ = false;
    side_forked_ = false;
  }
}

// fp32 step: forward, every gradient, (RCCL: one all-reduce of the whole flat gradient on the
// compute stream), the whole Adadelta update (which advances the device step counter) - SERIAL / RCCL.
// OVERLAP (single GPU): the fc update (98 % of the parameters) runs on the comm stream beside the
// conv backward once the fc gradients are final; the next step's first kernel waits for it.
//   C: (wait [1] >= [0]) forward, fc2 / fc1-bias grads, +[0], fc1 input grad, +[4], conv2 input grad
//      + conv1 weight grad, wait [3] >= [4], conv reduce, conv update (+step)
//   M: wait [0] >= [1]+1, fc1 weight grad, fc update, +[1], wait [4] >= [3]+1, conv2 weight grad, +[3]
// XGMI (world > 1) runs the same two chains with each update replaced by its bucket's all-reduce with
// the Adadelta step fused: the fc bucket (two-shot) on the comm stream beside the conv backward, the
// conv bucket (one-shot) at the step tail (different channels, so the two never share flags)
void Engine::enqueue_step_f32(int batch, bool last) {
  // RCCL with hand-offs: the same chains in one graph, the fc bucket's all-reduce ahead of the fc
  // update on the comm stream, the conv bucket's after compute's wait for [3] (which follows the fc
  // all-reduce on the comm stream: the communicator never has two collectives in flight, fc first)
  const bool rc = sched_ == RCCL && rccl_handoff_ && two_buckets_ && !trace_;
  if (sched_ == OVERLAP || sched_ == XGMI || rc) {
    const bool xg = sched_ == XGMI;
    const bool M = enq_main_, S = enq_side_;
    if (!side_forked_) {
      HIP_OK(hipEventRecord(ev_fc_, compute_));
      HIP_OK(hipStreamWaitEvent(comm_stream_, ev_fc_, 0));
      side_forked_ = true;
    }
    const bool pre = buf_.epoch_u8 != nullptr;
    F32Step a = f32_args();
    a.data_u8 = pre ? buf_.epoch_u8 : buf_.train_u8;
    a.idx = pre ? nullptr : buf_.train_idx;
    a.idx_step_stride = idx_stride_;
    a.labels = pre ? buf_.epoch_labels : buf_.train_labels;
    a.state = buf_.state;
    a.inv_batch = ddp_head_inv_batch(batch, world_);
    AdadeltaArgs ad{buf_.param, buf_.grad, buf_.square_avg, buf_.acc_delta, buf_.lr, rho_, eps_, wd_,
                    buf_.w2f, buf_.w2d, buf_.w1, buf_.w1t, nullptr};
    // ... and the conv2 weight gradient (reads dy2 + a1) on the comm stream beside the conv2 input
    // gradient + conv1 weight gradient: [4] counts fc1 input gradients (dy2) done, [3] conv2 weight
    // gradients done (the bf16 schedules' dgrad / conv2 counters, unused by the fp32 step)
    if (M) {
      if (side_pending_) launch_stream_wait(sync_ + 1, sync_ + 0, 0, sync_ + 2, compute_);
      launch_f32_forward(a, batch, true, compute_);
      launch_f32_fc_small(a, batch, compute_);
      launch_stream_signal(sync_ + 0, compute_);
      launch_f32_fc1x(a, batch, compute_);
      launch_stream_signal(sync_ + 4, compute_);
      launch_f32_conv2x_conv1w(a, batch, compute_);
      launch_stream_wait(sync_ + 3, sync_ + 4, 0, sync_ + 2, compute_);
      launch_f32_conv_reduce(a, batch, compute_);
    }
    // the conv bucket's tail (all-reduce + update, compute stream).  RCCL runs one communicator's
    // collectives in ISSUE order, even across streams, so with RCCL the conv all-reduce is enqueued
    // after the comm chain's fc all-reduce: compute reaches it only after [3] >= [4], which the comm
    // chain signals after the fc all-reduce - issued the other way round, the fc all-reduce would queue
    // behind a conv all-reduce that waits for it (a cycle broken only by the 60 s hand-off timeout)
    auto conv_tail = [&] {
      AdadeltaArgs ac = ad;
      ac.state_inc = buf_.state;
      if (xg) {
        ac.grad = xgmi_->out();
        xgmi_->allreduce(XGMI_CH_CONV, OFF_CONV1_W, PARAM_TOTAL - OFF_CONV1_W, compute_, &ac);
      } else {
        if (rc) comm_->allreduce_sum(buf_.grad + OFF_CONV1_W, PARAM_TOTAL - OFF_CONV1_W, 0, compute_);
        launch_adadelta(ac, ADA_CONV, compute_);
      }
    };
    if (M && !rc) conv_tail();
    if (S) {
      launch_stream_wait(sync_ + 0, sync_ + 1, 1, sync_ + 2, comm_stream_);
      launch_f32_fc1w(a, batch, comm_stream_);
      if (xg) {
        AdadeltaArgs af = ad;
        af.grad = xgmi_->out();
        xgmi_->allreduce(XGMI_CH_FC, OFF_FC1_W, OFF_CONV1_W - OFF_FC1_W, comm_stream_, &af);
      } else {
        if (rc) comm_->allreduce_sum(buf_.grad + OFF_FC1_W, OFF_CONV1_W - OFF_FC1_W, 0, comm_stream_);
        launch_adadelta(ad, ADA_FC, comm_stream_);
      }
      launch_stream_signal(sync_ + 1, comm_stream_);
      launch_stream_wait(sync_ + 4, sync_ + 3, 1, sync_ + 2, comm_stream_);
      launch_f32_conv2w(a, batch, comm_stream_);
      launch_stream_signal(sync_ + 3, comm_stream_);
    }
    if (M && rc) conv_tail();
    side_pending_ = true;
    if (last) {
      if (M && !skip_join_) {
        HIP_OK(hipEventRecord(ev_done_, comm_stream_));
        HIP_OK(hipStreamWaitEvent(compute_, ev_done_, 0));
      }
      side_pending_ = false;
      side_forked_ = false;
    }
    return;
  }
  const bool pre = buf_.epoch_u8 != nullptr;
  F32Step a = f32_args();
  a.data_u8 = pre ? buf_.epoch_u8 : buf_.train_u8;
  a.idx = pre ? nullptr : buf_.train_idx;
  a.idx_step_stride = idx_stride_;
  a.labels = pre ? buf_.epoch_labels : buf_.train_labels;
  a.state = buf_.state;
  a.inv_batch = ddp_head_inv_batch(batch, world_);
  phase_begin("fwd");
  launch_f32_forward(a, batch, true, compute_);
  phase_end();
  phase_begin("bwd");
  launch_f32_backward(a, batch, compute_);
  phase_end();
  phase_begin("allreduce+update");
  AdadeltaArgs ad{buf_.param, buf_.grad, buf_.square_avg, buf_.acc_delta, buf_.lr, rho_, eps_, wd_,
                  buf_.w2f, buf_.w2d, buf_.w1, buf_.w1t, buf_.state};
  if (sched_ == RCCL) comm_->allreduce_sum(buf_.grad, PARAM_TOTAL, 0, compute_);
  launch_adadelta(ad, ADA_ALL, compute_);
  phase_end();
}

void Engine::train_steps(int n, int batch, int stride) {
  if (batch < 1 || batch > max_batch_) throw std::runtime_error("batch exceeds engine capacity");
  idx_stride_ = stride;
  for (int i = 0; i < n; ++i) enqueue_step(batch, i == n - 1);
  HIP_OK(hipGetLastError());
}

int Engine::capture_train(int n, int batch, int stride) {
  if (batch < 1 || batch > max_batch_) throw std::runtime_error("batch exceeds engine capacity");
  idx_stride_ = stride;
  if (side_schedule()) return capture_train_split(n, batch);
  // SERIAL / RCCL: one graph, steps in order (RCCL: the communicator's collectives are captured in
  // the order every rank issues them - fc, conv, fc, ... - so RCCL's own ordering of one
  // communicator's kernels across streams can never chain a collective behind a later step's)
  hipGraph_t g = nullptr;
  HIP_OK(hipStreamBeginCapture(compute_, hipStreamCaptureModeRelaxed));
  try {
    for (int i = 0; i < n; ++i) enqueue_step(batch, i == n - 1);
  } catch (...) {
    reset_host_state();
    hipStreamEndCapture(compute_, &g);
    if (g) hipGraphDestroy(g);
    throw;
  }
  HIP_OK(hipStreamEndCapture(compute_, &g));
  hipGraphExec_t ex = nullptr;
  HIP_OK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  // (no hipGraphUpload: on this ROCm 7 runtime it segfaults right after instantiate - measured on
  // the box; first-replay costs are taken by an untimed warm replay instead, FusedTrainer.warm_graphs)
  graph_defs_.push_back(g);
  graphs_.push_back(ex);
  side_graphs_.push_back(nullptr);
  return (int)graphs_.size() - 1;
}

void Engine::reset_host_state() {
  comm_sig3_pending_ = false;
  enq_main_ = enq_side_ = true;
  skip_join_ = false;
  side_pending_ = false;
  side_forked_ = false;
  w2d_in_alt_ = false;
  w1t_in_alt_ = false;
}

// OVERLAP / XGMI chunks as TWO graphs: the side chain (comm stream: per step counter waits, the fc
// update or all-reduce, the conv2 part, counter signals) and the compute chain, captured in two
// passes over the same steps (host state - the w2d ping-pong, the pending hand-off - replayed
// identically) and launched concurrently from two host threads (replay()).  One multi-stream graph
// submitted its side branch only after the whole compute branch (~3.6 us of host time per node), so
// after every host sync the second step's trunk_fwd sat ~0.45 ms (20-step chunk) on the device
// counter the side chain had not yet reached the queue to signal: the driver's 20-step bench window
// read 93-97 us/step against 73.5 steady state.  The fork (chunk start -> comm stream) and the join
// (comm stream -> compute) become two events at replay.
int Engine::capture_train_split(int n, int batch) {
  const bool sp = side_pending_, w2 = w2d_in_alt_, w1 = w1t_in_alt_;
  hipGraph_t gs = nullptr, gm = nullptr;
  auto pass = [&](hipStream_t s, bool m, bool side, hipGraph_t* out) {
    side_pending_ = sp;
    w2d_in_alt_ = w2;
    w1t_in_alt_ = w1;
    comm_sig3_pending_ = false;
    side_forked_ = true;                   // forks / joins are events at replay, not captured edges
    enq_main_ = m;
    enq_side_ = side;
    skip_join_ = true;
    HIP_OK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    for (int i = 0; i < n; ++i) enqueue_step(batch, i == n - 1);
    HIP_OK(hipStreamEndCapture(s, out));
  };
  try {
    pass(comm_stream_, false, true, &gs);
    pass(compute_, true, false, &gm);
    enq_main_ = enq_side_ = true;
    skip_join_ = false;
  } catch (...) {
    reset_host_state();
    hipStreamCaptureStatus st;
    for (hipStream_t s : {comm_stream_, compute_}) {
      hipGraph_t junk = nullptr;
      if (s && hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusActive)
        hipStreamEndCapture(s, &junk);
      if (junk) hipGraphDestroy(junk);
    }
    for (hipGraph_t g : {gs, gm})
      if (g) hipGraphDestroy(g);
    throw;
  }
  hipGraphExec_t xs = nullptr, xm = nullptr;
  HIP_OK(hipGraphInstantiate(&xs, gs, nullptr, nullptr, 0));
  HIP_OK(hipGraphInstantiate(&xm, gm, nullptr, nullptr, 0));
  graph_defs_.push_back(gs);
  graph_defs_.push_back(gm);
  graphs_.push_back(xm);
  side_graphs_.push_back(xs);
  return (int)graphs_.size() - 1;
}

// --- side-graph launcher thread: hipGraphLaunch(side, comm stream) + the join event, concurrently
// with the compute graph's launch on the calling thread (measured 20-step window, single GPU: 75.8
// vs 78.9 us/step launching both from the calling thread)
void Engine::side_worker(int k) {
  SideLauncher& l = side_[k];
  std::unique_lock<std::mutex> lk(l.mu);
  for (;;) {
    l.cv.wait(lk, [&l] { return l.stop || l.job != nullptr; });
    if (l.stop) return;
    hipGraphExec_t job = l.job;
    hipStream_t s = l.stream;
    lk.unlock();
    hipError_t e = hipGraphLaunch(job, s);
    if (e == hipSuccess) e = hipEventRecord(l.join, s);
    lk.lock();
    l.err = e;
    l.job = nullptr;
    l.done = true;
    l.cv.notify_all();
  }
}

void Engine::side_start(int k, hipGraphExec_t g, hipStream_t s) {
  SideLauncher& l = side_[k];
  {
    std::lock_guard<std::mutex> lk(l.mu);
    if (!l.thread.joinable()) l.thread = std::thread(&Engine::side_worker, this, k);
    l.job = g;
    l.stream = s;
    l.done = false;
  }
  l.cv.notify_all();
}

hipError_t Engine::side_wait(int k) {
  SideLauncher& l = side_[k];
  std::unique_lock<std::mutex> lk(l.mu);
  l.cv.wait(lk, [&l] { return l.done; });
  return l.err;
}

void Engine::gather_rows(int64_t start, int64_t n) {
  if (!buf_.epoch_u8 || !buf_.epoch_labels) throw std::runtime_error("gather_rows: no epoch buffers");
  launch_gather_rows(buf_.train_u8, buf_.train_labels, buf_.train_idx, start, n, buf_.epoch_u8, buf_.epoch_labels,
                     compute_);
  HIP_OK(hipGetLastError());
}

void Engine::replay(int id) {
  if (id < 0 || id >= (int)graphs_.size()) throw std::runtime_error("bad graph id");
  hipGraphExec_t side = side_graphs_[id];
  if (!side) {
    HIP_OK(hipGraphLaunch(graphs_[id], compute_));
    return;
  }
  HIP_OK(hipEventRecord(ev_fork_, compute_));          // side chain ordered after earlier compute work
  HIP_OK(hipStreamWaitEvent(comm_stream_, ev_fork_, 0));
  side_start(0, side, comm_stream_);
  const hipError_t em = hipGraphLaunch(graphs_[id], compute_);
  const hipError_t es = side_wait(0);
  HIP_OK(em);
  HIP_OK(es);
  HIP_OK(hipStreamWaitEvent(compute_, side_[0].join, 0));   // chunk end: compute joins the side chain
}

void Engine::enqueue_eval(int n_total, int batch) {
  const float* P = buf_.param;
  for (int s = 0; s < n_total; s += batch) {
    const int B = (n_total - s) < batch ? (n_total - s) : batch;
    if (f32_) {
      F32Step a = f32_args();
      a.data_u8 = buf_.test_u8;
      a.idx = buf_.test_idx + s;
      a.idx_step_stride = 0;
      a.labels = buf_.test_labels;
      a.state = nullptr;
      a.loss_rows = buf_.test_loss_rows + s;
      a.correct = buf_.test_correct + s;
      launch_f32_forward(a, B, false, compute_);
      continue;
    }
    TrunkFwdArgs tf{buf_.test_u8, buf_.test_idx + s, 0, nullptr, P + OFF_CONV1_W, P + OFF_CONV1_B,
                    buf_.w2f, P + OFF_CONV2_B, nullptr, p_, nullptr, nullptr};
    launch_trunk_fwd(tf, B, false, compute_);
    launch_fc1_fwd(p_, buf_.w1, z1part_, B, compute_);
    HeadArgs ha{};
    ha.z1part = z1part_; ha.b_fc1 = P + OFF_FC1_B; ha.w_fc2 = P + OFF_FC2_W; ha.b_fc2 = P + OFF_FC2_B;
    ha.labels = buf_.test_labels; ha.idx = buf_.test_idx + s; ha.idx_step_stride = 0;
    ha.loss_rows = buf_.test_loss_rows + s; ha.correct_out = buf_.test_correct + s;
    launch_head_eval(ha, B, compute_);
  }
}

void Engine::eval(int n_total, int batch) {
  if (batch < 1 || batch > max_test_batch_) throw std::runtime_error("test batch exceeds engine capacity");
  enqueue_eval(n_total, batch);
  HIP_OK(hipGetLastError());
}

int Engine::capture_eval(int n_total, int batch) {
  if (batch < 1 || batch > max_test_batch_) throw std::runtime_error("test batch exceeds engine capacity");
  hipGraph_t g = nullptr;
  HIP_OK(hipStreamBeginCapture(compute_, hipStreamCaptureModeRelaxed));
  enqueue_eval(n_total, batch);
  HIP_OK(hipStreamEndCapture(compute_, &g));
  hipGraphExec_t ex = nullptr;
  HIP_OK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  // (no hipGraphUpload: on this ROCm 7 runtime it segfaults right after instantiate - measured on
  // the box; first-replay costs are taken by an untimed warm replay instead, FusedTrainer.warm_graphs)
  graph_defs_.push_back(g);
  graphs_.push_back(ex);
  side_graphs_.push_back(nullptr);
  return (int)graphs_.size() - 1;
}

void Engine::refresh_shadows() {
  AdadeltaArgs ad{buf_.param, buf_.grad, buf_.square_avg, buf_.acc_delta, buf_.lr, rho_, eps_, wd_,
                  buf_.w2f, buf_.w2d, buf_.w1, buf_.w1t, nullptr};
  launch_refresh_shadows(ad, compute_);
  HIP_OK(hipGetLastError());
}

void Engine::broadcast_params(int root) {
  if (!comm_) throw std::runtime_error("no communicator attached");
  comm_->broadcast(buf_.param, PARAM_TOTAL, 0, root, compute_);
  refresh_shadows();
}

bool Engine::probe_stream_pair(hipStream_t x, hipStream_t y, double timeout_s) {
  // scratch counters sync_[8..11]: [8] a, [9] b, [10] zero, [11] error
  launch_fill(sync_ + 8, 4 * sizeof(int), 0, x);
  HIP_OK(hipStreamSynchronize(x));
  launch_stream_wait(sync_ + 8, sync_ + 10, 1, sync_ + 11, x, timeout_s);   // x waits ...
  launch_stream_signal(sync_ + 8, y);                                        // ... for y
  launch_stream_wait(sync_ + 9, sync_ + 10, 1, sync_ + 11, y, timeout_s);   // y waits ...
  launch_stream_signal(sync_ + 9, x);                                        // ... for x
  HIP_OK(hipStreamSynchronize(x));
  HIP_OK(hipStreamSynchronize(y));
  int err = 0;
  HIP_OK(hipMemcpy(&err, sync_ + 11, sizeof(int), hipMemcpyDeviceToHost));
  return err == 0;
}

bool Engine::probe_stream_handoff(double timeout_s) { return probe_stream_pair(compute_, comm_stream_, timeout_s); }

// fault injection (tests): the compute stream spins until fault_release (scratch counters
// [12] released, [13] zero, [14] the hold's own timeout flag - never the engine's error flag [2])
void Engine::fault_hold(double timeout_s) {
  launch_fill(sync_ + 12, 4 * sizeof(int), 0, compute_);
  launch_stream_wait(sync_ + 12, sync_ + 13, 1, sync_ + 14, compute_, timeout_s);
  HIP_OK(hipGetLastError());
}

void Engine::fault_release(hipStream_t s) {
  launch_stream_signal(sync_ + 12, s);
  HIP_OK(hipGetLastError());
}

std::pair<int, int> Engine::errors() const {
  int err = 0;
  HIP_OK(hipMemcpy(&err, sync_ + 2, sizeof(int), hipMemcpyDeviceToHost));
  return {err, xgmi_ ? xgmi_->error() : 0};
}

std::string Engine::describe_xgmi_error(int code) {
  static const char* names[] = {"?", "two-shot all-reduce", "one-shot all-reduce", "fused fc all-reduce+Adadelta",
                                "fused conv reduce+all-reduce+Adadelta"};
  const int kid = (code >> 24) & 0xff;
  return std::string(names[kid >= 1 && kid <= 4 ? kid : 0]) + " kernel, stage " + std::to_string((code >> 16) & 0xf) +
         ", waiting for peer rank " + std::to_string((code >> 12) & 0xf) + ", workgroup " + std::to_string(code & 0xfff);
}

void Engine::check_errors() const {
  const auto e = errors();
  if (e.first) throw std::runtime_error("engine: a stream hand-off timed out (results invalid)");
  if (e.second)
    throw std::runtime_error("engine: an xGMI all-reduce stage timed out (results invalid): " +
                             describe_xgmi_error(e.second));
}

void Engine::sync_streams() {
  HIP_OK(hipStreamSynchronize(compute_));
  HIP_OK(hipStreamSynchronize(comm_stream_));
}

void Engine::synchronize() {
  sync_streams();
  check_errors();
}

}  // namespace mnist
