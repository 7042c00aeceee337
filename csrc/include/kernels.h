// Host-visible launch interface of the hand-written gfx950 kernels.  Every launcher only
// enqueues on the given stream (no allocation, no sync) so the sequences are graph-capturable.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "mnist_common.h"

namespace mnist {

// write-through (sc1) stores for batches up to this size (device_utils.h store16)
constexpr int WT_MAX_B = 1024;

// ---------------- forward ----------------
struct TrunkFwdArgs {
  const uint8_t* data_u8;     // [N][784] raw dataset, HBM resident
  const int32_t* idx;         // epoch index vector; row b of step s = idx[s*idx_step_stride + b]
  int64_t idx_step_stride;    // = batch size for the training stream, 0 for a fixed batch
  const StepState* state;     // step counter + dropout RNG (may be null in eval)
  const float* w1c;           // conv1.weight fp32 [32][9]
  const float* b1c;           // conv1.bias   fp32 [32]
  const uint16_t* w2f;        // conv2 weight bf16 [64][9][32]
  const float* b2c;           // conv2.bias   fp32 [64]
  uint16_t* a1_out;           // bf16 [B][26][26][32]  (train only)
  uint16_t* p_out;            // bf16 [B][9216]
  uint8_t* pmask_out;         // u8   [B][9216]        (train only)
  const float* xin;           // optional fp32 [B][784] already-normalised input (module API);
                              // when set, data_u8/idx are ignored
  const int* wait_a;          // optional (schedule 3): completion held until *wait_a >= *wait_b
  const int* wait_b;
  int* wait_err;
};
void launch_trunk_fwd(const TrunkFwdArgs& a, int B, bool train, hipStream_t s);
constexpr int TRUNK_IMG_MAX_B = 256;      // B <= this: one workgroup per image (every image has a CU)
int trunk_strips_per_wg(int B);           // 3 (whole image per workgroup) or 1 (one strip)

// fc1 split-K partial GEMM: z1part[s][b][o] = sum_{i in chunk s} p[b][i] * w1[o][i]
constexpr int FC1_KSPLIT = 32;            // small batches: 16-row tiles, fragments straight from HBM/L2
constexpr int FC1_KSPLIT_BIG = 4;         // B >= FC1_BIG_MIN_B: 64x128 LDS-staged tiles, K/4 each
constexpr int FC1_BIG_MIN_B = 512;
__host__ __device__ inline int fc1_ksplit(int B) { return B >= FC1_BIG_MIN_B ? FC1_KSPLIT_BIG : FC1_KSPLIT; }
void launch_fc1_fwd(const uint16_t* p, const uint16_t* w1, float* z1part, int B, hipStream_t s);

// Head: reduce fc1 partials + bias -> ReLU -> dropout(0.5) -> fc2 -> log_softmax (+ NLL + backward)
struct HeadArgs {
  const float* z1part;        // [fc1_ksplit(B)][B][128]
  const float* b_fc1;         // [128]
  const float* w_fc2;         // [10][128] fp32
  const float* b_fc2;         // [10]
  const int32_t* labels;      // train: dataset labels [N] gathered through idx; eval: same
  const int32_t* idx;
  int64_t idx_step_stride;
  const StepState* state;
  float inv_batch;            // 1/B (nll mean)
  // outputs (train)
  float* loss_rows;           // [B] per-row NLL
  uint16_t* dz1;              // bf16 [Bp][128] grad wrt fc1 pre-activation (rows >= B zeroed)
  uint16_t* h_bf;             // bf16 [Bp][128] fc1 activations after ReLU+dropout (rows >= B zeroed)
  uint16_t* dl_bf;            // bf16 [Bp][16]  d loss / d logits (cols >= 10, rows >= B zeroed)
  // outputs (eval)
  float* logp_out;            // optional [B][10]
  int32_t* correct_out;       // [B] 1 if argmax == label
  const float* dlogp;         // module API backward: upstream grad wrt log-probs [B][10] (replaces NLL)
};
void launch_head_train(const HeadArgs& a, int B, int Bp, hipStream_t s);
void launch_head_eval(const HeadArgs& a, int B, hipStream_t s);
// module API forward: log-probs with (train) or without (eval) dropout-2
void launch_head_fwd(const HeadArgs& a, int B, bool train, hipStream_t s);

// ---------------- backward ----------------
// Compact gradient wrt the conv2 output (the max-pool backward input): one record per (image,
// pooled position) = 64 bf16 pooled gradients (already dropout-scaled, ReLU-masked) followed by the
// 64 argmax codes (2x2 window position, 0..3) as bit planes: per 8-channel chunk c8 two bytes at
// DYC_ROUTE + 2 c8, bit i of the first = bit 0 of channel 8 c8 + i's code, of the second = bit 1
// (16 B of codes instead of 64: 144-B records, 25 % fewer record bytes written by fc_bwd and read by
// the conv backward).  Dense dy[y][x][c] = (code == 2(y&1)+(x&1)) ? g : 0.
constexpr int DYC_REC = 144, DYC_ROUTE = 128;
constexpr int64_t DYC_BYTES_PER_IMAGE = (int64_t)NPOOL * DYC_REC;   // 20736

struct FcBwdArgs {
  const uint16_t* dz1;        // bf16 [Bp][128]
  const uint16_t* p;          // bf16 [Bp][9216] (rows >= B are masked)
  const uint8_t* pmask;       // [B][9216]
  const uint16_t* w1t;        // bf16 [9216][128] (read by role B)
  const uint16_t* h_bf;       // bf16 [Bp][128]
  const uint16_t* dl_bf;      // bf16 [Bp][16]
  const float* loss_rows;     // [B]
  const StepState* state;
  float* grad;                // flat fp32 grad buffer (writes fc1.w, fc1.b, fc2.w, fc2.b)
  uint8_t* dyc;               // compact grad wrt conv2 output: [B][144] records (see DYC_REC)
  float* loss_log;            // [steps] mean loss per step (indexed by state->step)
  float grad_scale;           // extra gradient scale applied in the epilogue.  The engine passes 1.0: its
                              // DDP averaging lives in the head (inv_batch = 1/(B*world)); only a caller
                              // that leaves inv_batch at 1/B would pass 1/world_size here
  float inv_batch;
  float* part;                // B > FC_BWD_SPLIT_ROWS: [fc_bwd_splits(B)][FCB_PART_STRIDE] partial fc grads
  int* signal_ctr;            // optional: the launch's first workgroup adds 1 at its start (schedule-3 hand-off)
};
// Large batches split the batch (= K of the fc weight gradients) over fc_bwd_splits(B) groups of
// workgroups writing fp32 partials that fc_grad_reduce sums in fixed order; B <= 1024 writes the
// gradients directly.  Role B processes FCB_MR(B) 16-row tiles per workgroup (w1 slice kept in VGPRs).
constexpr int FC_BWD_SPLIT_ROWS = 1024;
__host__ __device__ inline int fc_bwd_splits(int B) { return (B + FC_BWD_SPLIT_ROWS - 1) / FC_BWD_SPLIT_ROWS; }
__host__ __device__ inline int fcb_mr(int B) { return B >= 2048 ? 8 : B >= 128 ? 2 : 1; }   // role-B row tiles per workgroup (B = 200: 2 measured 73.1-73.2 vs 74.1-74.6 us/step)
// partial layout per split: fc1.w [128][9216], fc1.b [128], fc2.w [10][128], fc2.b [10], loss sum, pad
constexpr int64_t FCB_PART_W1 = 0, FCB_PART_B1 = 128 * 9216, FCB_PART_W2 = FCB_PART_B1 + 128,
                  FCB_PART_B2 = FCB_PART_W2 + 1280, FCB_PART_LOSS = FCB_PART_B2 + 10,
                  FCB_PART_STRIDE = (FCB_PART_LOSS + 1 + 63) / 64 * 64;
// reduce = false (B > 1024): the split partials are left for launch_fc_grad_reduce, which the
// engine runs on the comm stream ahead of the fc all-reduce / update (off the compute chain)
// fc_bwd workgroup roles (fc_head.hip): C = fc2 weight / bias gradient + loss, A = fc1 weight / bias
// gradient, B = gradient into the conv trunk (compact dy records)
constexpr int FCB_ROLE_C = 1, FCB_ROLE_A = 2, FCB_ROLE_B = 4, FCB_ROLES_ALL = 7;
void launch_fc_bwd(const FcBwdArgs& a, int B, int Bp, hipStream_t s, bool reduce = true, int roles = FCB_ROLES_ALL);
struct AdadeltaArgs;
// roles C + A with the fc Adadelta step fused (one split; single-GPU OVERLAP chain)
void launch_fc_wgrad_update(const FcBwdArgs& a, const AdadeltaArgs& u, int B, int Bp, hipStream_t s);
// role A (fc1 weight gradient split partials) alone, for B > 1024 with reduce = false / with_a = false
void launch_fc_bwd_dw1(const FcBwdArgs& a, int B, int Bp, hipStream_t s);
void launch_fc_grad_reduce(const FcBwdArgs& a, int B, hipStream_t s);   // no-op for B <= 1024
void launch_fc_bwd_role(const FcBwdArgs& a, int B, int Bp, int role, hipStream_t s);   // profiling aid

struct ConvBwdArgs {
  const uint8_t* dyc;         // compact un-pooled gradient (written by fc_bwd role B)
  const uint16_t* a1;         // bf16 [B][26][26][32]
  const uint16_t* w2d;        // bf16 [9][32][64]
  const float* w1c;           // conv1 fp32 [32][9]
  const float* b1c;           // [32]
  const uint8_t* data_u8;
  const int32_t* idx;
  int64_t idx_step_stride;
  const StepState* state;
  float* c1part;              // [4*B][320] conv1 wgrad(288)+bias(32) partials (dgrad kernel)
  float* w2part;              // [G][18432 + 64] conv2 wgrad + bias partials
  float* grad;                // flat fp32 grad buffer (conv params written by the reduce kernel)
  float grad_scale;           // as FcBwdArgs::grad_scale: 1.0 from the engine (averaging in the head)
  int wgrad_groups;           // G
  const float* xin;           // optional fp32 [B][784] input (module API), replaces data_u8/idx
  int* signal_ctr;            // optional: conv2_wgrad / conv2_dgrad add 1 at kernel start (schedule-3 hand-offs)
  // optional [C1_PRE_SLABS][320]: when set, launch_conv_dgrad pre-reduces the 4B conv1
  // partials into C1_PRE_SLABS fixed-order group sums and the conv reduce reads those (large B:
  // 20 reduce workgroups walking 4B slabs is a dependent-load chain, 81 us at B = 8192)
  float* c1red;
  int c1_rows;                // conv1 partial rows the dgrad launch writes: conv_dgrad_c1_rows(B)
  int dgrad_full_grid;        // 1: persistent dgrad on 2 x CUs workgroups; 0: the equal-count grid
};
// 4B: 4 strips of 7 rows per image, items of the persistent dgrad (2 workgroups per CU)
int conv_dgrad_c1_rows(int B);
// test / tuning hooks (host globals, read at enqueue): persistent dgrad grid (0 = 2 x CUs) and the
// wgrad form (-1 = by batch, 0 = lean lockstep halves, 1 = staggered halves)
void set_dgrad_grid(int n);
void set_wgrad_form(int f);
constexpr int C1_PRE_SLABS = 256;
constexpr int C1_PRE_MIN_SLABS = 1024;    // engine: pre-reduce when c1_rows exceeds this
int conv_wgrad_groups(int B);
void launch_conv_bwd(const ConvBwdArgs& a, int B, hipStream_t s);      // dgrad(+conv1 wgrad) and wgrad
void launch_conv_dgrad(const ConvBwdArgs& a, int B, hipStream_t s);    // conv2 dgrad + conv1 wgrad partials
void launch_conv_wgrad(const ConvBwdArgs& a, int B, hipStream_t s);    // conv2 wgrad + bias partials
void launch_conv_grad_reduce(const ConvBwdArgs& a, int B, hipStream_t s);
// reduce blocks [lo, hi) only (RED_W2_PARTS conv2 blocks, then the conv1 ones: see RED_ALL_PARTS)
void launch_conv_grad_reduce_parts(const ConvBwdArgs& a, int B, int lo, int hi, hipStream_t s);

// ---------------- optimizer ----------------
struct AdadeltaArgs {
  float* param;               // flat fp32
  const float* grad;
  float* square_avg;
  float* acc_delta;
  const float* lr;            // device scalar (StepLR writes it once per epoch)
  float rho, eps, weight_decay;
  uint16_t* w2f;              // bf16 shadows refreshed in the same pass
  uint16_t* w2d;
  uint16_t* w1;
  uint16_t* w1t;
  StepState* state_inc;       // if non-null, block 0 advances state->step (end-of-step marker)
  // optional completion hold (adadelta_reduce_kernel): the launch completes only once
  // *hold_a >= *hold_b (read when its last workgroup gets there); timeout -> *hold_err = 1
  const int* hold_a;
  const int* hold_b;
  int* hold_err;
  int wt;                     // write-through parameter / state / shadow stores (engine: B <= WT_MAX_B)
  int hold_delta;             // hold until *hold_a >= *hold_b + hold_delta (adadelta_kernel; the
                              // reduce kernel holds with delta 0)
  int* signal_start;          // optional: the first workgroup adds 1 at kernel start (the previous
                              // kernel on the stream has completed: a hand-off without a launch)
};
enum AdadeltaRegion { ADA_ALL = 0, ADA_FC = 1, ADA_CONV = 2 };
// grid > 0 (ADA_FC only): that many workgroups walk the 577 fc tiles grid-stride (ADA_FC_LEAN_GRID:
// the single-GPU overlapped update, which runs beside wgrad / dgrad with slack to spare)
constexpr int ADA_FC_LEAN_GRID = 144;
void launch_adadelta(const AdadeltaArgs& a, int region, hipStream_t s, int grid = 0);
// conv gradient slab reduce + the whole Adadelta update in one launch (serial single-GPU step tail)
void launch_adadelta_reduce(const AdadeltaArgs& a, const ConvBwdArgs& c, int B, hipStream_t s);
// conv-only form restricted to reduce parts [lo, hi) (conv_grad_reduce.h partition)
void launch_adadelta_reduce_parts(const AdadeltaArgs& a, const ConvBwdArgs& c, int B, int lo, int hi, hipStream_t s);
// the conv1 parts [RED_W2_PARTS, RED_ALL_PARTS) of that launch, bitwise equal, on 80 one-wave workgroups
// (one float4 column each, the slice tree on cross-lane moves)
void launch_adadelta_c1(const AdadeltaArgs& a, const ConvBwdArgs& c, int B, hipStream_t s);
// Refresh bf16 shadows from fp32 params without an update (after load_state_dict / broadcast).
void launch_refresh_shadows(const AdadeltaArgs& a, hipStream_t s);

// misc
void launch_set_step(StepState* st, int step, hipStream_t s);
void launch_set_state(StepState* st, const StepState& v, hipStream_t s);
// epoch pre-gather: dst rows [start, start+n) = src rows idx[start..start+n) (+ labels)
// synthetic data generator v3 (csrc/kernels/datagen.hip): render n images [n, 784] from a host plan
// (n x 96-B synth::Sample records, csrc/data/synth_render.h) and the zero-bordered templates
void launch_synth_render(const void* plan, const float* templates, int64_t n, uint8_t* out, hipStream_t s);
void launch_gather_rows(const uint8_t* src_u8, const int32_t* src_labels, const int32_t* idx, int64_t start,
                        int64_t n, uint8_t* dst_u8, int32_t* dst_labels, hipStream_t s);
// device-counter stream hand-offs (engine DDP schedule 3)
void launch_stream_signal(int* ctr, hipStream_t s);
// byte fill of [p, p + bytes) on `s` (hipMemset's job without the runtime's blit kernels)
void launch_fill(void* p, int64_t bytes, int value, hipStream_t s);
void launch_stream_wait(const int* a, const int* b, int delta, int* err, hipStream_t s, double timeout_s = 60.0);
// signal then wait in one launch (*sig += 1; wait *a >= *b + delta)
void launch_stream_signal_wait(int* sig, const int* a, const int* b, int delta, int* err, hipStream_t s,
                               double timeout_s = 60.0);
// dst[i] = src[i] * s (DDP bucket copy-in with the 1/world_size pre-division)
void launch_scale_copy(float* dst, const float* src, int64_t n, float s, hipStream_t stream);

// code-object preload, one per kernel translation unit (hipFuncGetAttributes on one of its kernels)
void preload_trunk();
void preload_fc_head();
void preload_conv_bwd();
void preload_adadelta();
void preload_comm();
void preload_xgmi();
void preload_f32();

// ---------------- fp32 step (--dtype fp32; f32_net.hip): f32-input MFMA GEMMs + VALU kernels
struct F32Step {
  // batch source: pre-gathered rows (idx = null, row = step * idx_step_stride + b) or dataset rows
  // through the index vector; eval: the test split, idx = test_idx + first row, stride 0
  const uint8_t* data_u8;
  const int32_t* idx;
  int64_t idx_step_stride;
  const int32_t* labels;
  const StepState* state;     // null in eval (step 0, no dropout)
  const float* param;         // flat fp32 parameters
  float* grad;                // flat fp32 gradient (every parameter written each step)
  float* loss_log;            // [steps] mean loss per step (train)
  float inv_batch;            // 1 / (B * world): DDP averaging folded into the loss gradient
  // workspace (fp32 unless noted)
  float* w2fwd;               // [9][32][64] conv2 weight, forward B operand
  float* w2bwd;               // [9][64][32] conv2 weight, input-gradient B operand
  float* w1p;                 // [128][144][64] fc1 weight with its input index position-major
                              // (pooled position, channel): the fc1 input-gradient B operand
  float* a1;                  // [B][26][26][32] ReLU(conv1)
  float* dx1;                 // [B][26][26][32] the conv1 pre-activation gradient (its own buffer, so
                              // the conv2 weight gradient - which reads a1 - can run beside it)
  float* y2;                  // [B][24][24][64] conv2 pre-activation; then its gradient
  float* p;                   // [B][9216] pooled + dropout, torch flatten order
  uint8_t* pm;                // [B][9216] argmax (bits 0-1), dropout keep (2), pooled > 0 (3)
  float* z1part;              // [f32_fc1_splits(B)][B][128]
  float* h;                   // [B][128] fc1 activations after ReLU + dropout
  float* dz1;                 // [B][128] gradient wrt the fc1 pre-activation
  float* dl;                  // [B][16] gradient wrt the logits
  float* loss_rows;           // [B] per-row NLL (train and eval)
  int32_t* correct;           // eval: [B] argmax == label
  float* c2part;              // [f32_conv2w_splits(B)][64][289] conv2 weight + bias partials
  float* c1part;              // [F32_C1W_BLOCKS][32][10] conv1 weight + bias partials
};
constexpr int F32_MAX_SPLITS = 128;
constexpr int F32_C1W_BLOCKS = 1024;         // conv1 weight-gradient workgroups (= partial slabs)
int f32_fc1_splits(int B);
int f32_conv2w_splits(int B);
int f32_conv1w_splits(int B);
// prep + conv1 + conv2 + pool (+dropout) + fc1 + head (train: loss + logit / dz1 gradients; eval:
// per-row NLL + hits)
void launch_f32_forward(const F32Step& a, int B, bool train, hipStream_t s);
// fc2 / fc1-bias grads + loss log, fc1 weight grad, fc1 input grad (+ unpool), conv2 weight grad,
// conv2 input grad (+ conv1 ReLU), conv1 weight grad, split-K reduce: every gradient of the step
void launch_f32_backward(const F32Step& a, int B, hipStream_t s);
void launch_f32_backward_fc(const F32Step& a, int B, hipStream_t s);     // = the first half of it:
void launch_f32_fc_small(const F32Step& a, int B, hipStream_t s);   // fc2 weight / bias, fc1 bias, loss log
void launch_f32_fc1w(const F32Step& a, int B, hipStream_t s);       // fc1 weight (reads dz1 + p)
void launch_f32_backward_conv(const F32Step& a, int B, hipStream_t s);   // = the second half
// ... which is, in order: fc1 input gradient (dy2), conv2 weight gradient (reads dy2 + a1), conv2
// input gradient + conv1 weight gradient (dy2 -> dx1), split-K reduce (both partial sets).  The
// OVERLAP schedule runs the weight gradient on the comm stream beside the input-gradient part.
void launch_f32_fc1x(const F32Step& a, int B, hipStream_t s);
void launch_f32_conv2w(const F32Step& a, int B, hipStream_t s);
void launch_f32_conv2x_conv1w(const F32Step& a, int B, hipStream_t s);
void launch_f32_conv_reduce(const F32Step& a, int B, hipStream_t s);

// direct xGMI all-reduce (reduce-scatter + all-gather over IPC-mapped peer buckets; xgmi_allreduce.hip)
constexpr int XGMI_MAX_RANKS = 8;          // one node
constexpr int XGMI_MAX_WG = 512;           // flag slots per (stage, rank)
constexpr int XGMI_FLAG_INTS = 2 * XGMI_MAX_RANKS * XGMI_MAX_WG;   // [stage][src rank][wg]
struct XgmiArgs {
  const float* in[XGMI_MAX_RANKS];   // every rank's input bucket (peer mappings; own = local)
  float* out[XGMI_MAX_RANKS];        // every rank's output bucket
  int* flags[XGMI_MAX_RANKS];        // every rank's flag block of this channel
  float* stage[XGMI_MAX_RANKS];      // one-shot: every rank's staging block of this channel (2 slots)
  int64_t slot_floats;               // one-shot: floats per staging slot
  int* ctr;                          // local per-WG call counters [XGMI_MAX_WG]
  int* err;                          // local error flag (timeout)
  int world, rank;
  int64_t nvec;                      // bucket length in float4s
  const uint64_t* timeout_ticks;     // device: stage-wait timeout, s_memrealtime ticks (100 MHz)
  // optional fused Adadelta (conv bucket): with fuse_ada, phase 2 applies the update to every element
  // it gathers (flat index ada_base + bucket index; grad = the reduced values), refreshes the conv2
  // bf16 shadows and advances ada.state_inc->step - the bucket's separate update launch disappears
  int fuse_ada;
  int64_t ada_base;
  AdadeltaArgs ada;
  int max_wg;                        // residency cap on the launch grid (XgmiGrids; every rank the same)
  int release;                       // system-scope release fence before each stage flag store
  int acquire;                       // system-scope acquire after each matched stage poll (opt-in)
};
// Every xGMI kernel's workgroup b spins until workgroup b of every peer arrives, so the workgroups
// that can be spinning at the same moment - on one GPU: the fc-bucket kernel on the comm stream and
// the conv-bucket kernel on the compute stream, times the ranks that share the GPU - must all be
// resident at once.  The kernels loop over their index sets (any grid >= a small minimum works) and
// the grids are sized from the occupancy API: co_ranks * sum(grid_k / (occupancy_k * CUs)) <= budget
// for each pair that runs concurrently.  Kernel ids in the error code (XgmiComm::error):
enum XgmiKernelId { XGMI_K_TWOSHOT = 1, XGMI_K_ONESHOT = 2, XGMI_K_FC_FUSED = 3, XGMI_K_CONV_FUSED = 4 };
struct XgmiGrids {
  int fc_fused, conv_fused;          // fused schedule: fc (comm stream) || conv (compute stream)
  int twoshot, oneshot;              // separate launches: two-shot fc || one-shot conv (caps)
  int cap_fc_fused, cap_conv_fused, cap_twoshot, cap_oneshot;   // resident WGs per GPU (occupancy x CUs)
  double load_fused, load_separate;  // co_ranks * sum(grid / cap) of each concurrent pair
};
// Throws std::runtime_error when even the minimum grids cannot be co-resident (caller falls back).
XgmiGrids xgmi_plan_grids(int world, int co_ranks, int64_t oneshot_max_floats, double budget);
constexpr int XGMI_CONV_VB_MAX = 8;        // conv fused: virtual reduce blocks per workgroup (grid >= 39)
int xgmi_workgroups(int64_t nvec, int world, bool fuse_ada);
void launch_xgmi_allreduce(const XgmiArgs& a, hipStream_t s);
// small buckets: one-shot variant - copy-in to a staging slot (alternating by call parity), ONE
// stage hand-off, every rank sums all ranks' slots itself (same rank order -> same bits as above)
void launch_xgmi_allreduce_oneshot(const XgmiArgs& a, hipStream_t s);
// the engine's fc bucket [0, OFF_CONV1_W) with the fc Adadelta step + w1/w1t shadows fused (two-shot,
// 64x32 fc1.weight tiles as the unit of work; needs a.ada and a.nvec == OFF_CONV1_W / 4)
int xgmi_fc_fused_workgroups(int world);
void launch_xgmi_fc_fused(const XgmiArgs& a, hipStream_t s);
// the engine's conv bucket [OFF_CONV1_W, PARAM_TOTAL): conv gradient slab reduce (conv_grad_reduce's
// partition and order) + one-shot all-reduce through the staging slots + Adadelta + conv2 shadows,
// one launch (needs a.ada; a.nvec == (PARAM_TOTAL - OFF_CONV1_W) / 4; c.grad is not written)
// `part` selects reduce blocks [lo, hi) of conv_grad_reduce's partition (RED_W2_WGS = 289 conv2
// blocks, then 20 conv1 blocks); the conv bucket split runs conv2 right after conv2_wgrad on the comm
// stream and conv1 after conv2_dgrad, whose launch holds its completion until *wait_a >= *wait_b.
constexpr int RED_W2_PARTS = 289, RED_ALL_PARTS = 309;   // = conv_grad_reduce.h RED_W2_WGS / RED_WGS
struct XgmiConvPart {
  int lo = 0, hi = RED_ALL_PARTS;
  const int* wait_a = nullptr;
  const int* wait_b = nullptr;
  int* wait_err = nullptr;
};
void launch_xgmi_conv_reduce_fused(const XgmiArgs& a, const ConvBwdArgs& c, int B, hipStream_t s,
                                   const XgmiConvPart& part = XgmiConvPart{});

}  // namespace mnist
