// Fused conv trunk forward: gather+normalise -> conv1+bias+ReLU -> conv2 (MFMA implicit GEMM)
// -> +bias -> ReLU -> maxpool 2x2 -> dropout(0.25) -> flatten.
//
// Replaces reference mnist_ddp.py:49-56 (conv1, relu, conv2, relu, max_pool2d, dropout1, flatten)
// plus the DataLoader's ToTensor/Normalize (mnist_ddp.py:153-156) and the H2D copy (:68).
//
// One workgroup = NS strips of 8 conv2-output rows of one image (3 strips per image; NS = 1 with
// 4 waves, or NS = 3 = the whole image with 12 waves, chosen by batch size: trunk_strips_per_wg).
//   * the input rows are gathered from the HBM-resident uint8 dataset by index and normalised;
//   * conv1 (K=9, too small for MFMA) runs on the VALU in fp32 straight into an NHWC bf16 LDS tile;
//   * conv2 is an implicit GEMM on v_mfma_f32_16x16x32_bf16: M = 192 pixels per strip, N = 64,
//     K = 9 taps x 32 channels; one 32-deep k-step is exactly one tap, so every A fragment is one
//     16-byte LDS read of 8 contiguous channels at (pixel + tap offset);
//   * the M index is ordered pool-window-major (m = 4*window + q), so each lane's 4 accumulator
//     registers hold one whole 2x2 window: max-pool + argmax happen in registers;
//   * dropout uses Philox-4x32-10 keyed by (seed, per-step offset, element index / 16) with one
//     random byte per element, so the mask is a pure function of (step, position) and identical
//     across launch geometries and graph replays.
#include "../include/device_utils.h"
#include "../include/kernels.h"
#include "../include/timeline.h"

namespace mnist {

// Phase timing (tools/phase_timing.hip compiles this file with MNIST_PHASE_TIMING): thread 0 of
// every workgroup records s_memtime at each phase boundary.
#ifdef MNIST_PHASE_TIMING
// PHASE_MARK_BY(t, i): the same by thread t (tools/exp/trunk_pipe_exp.hip marks a second role).
constexpr int kPhaseMaxWG = 4096, kPhaseSlots = 16;
__device__ uint64_t g_phase_times[kPhaseMaxWG * kPhaseSlots];
#define PHASE_MARK_BY(t, i)                                                                    \
  if (threadIdx.x == (t) && blockIdx.y * gridDim.x + blockIdx.x < kPhaseMaxWG)                 \
    g_phase_times[(blockIdx.y * gridDim.x + blockIdx.x) * kPhaseSlots + (i)] = __builtin_amdgcn_s_memtime();
#define PHASE_MARK(i) PHASE_MARK_BY(0, i)
#else
#define PHASE_MARK_BY(t, i)
#define PHASE_MARK(i)
#endif

namespace {
constexpr int STRIP = 8;                      // conv2 output rows per strip (3 strips per image)
constexpr int WIN = (STRIP / 2) * HP;         // 48 pool windows per strip

// One workgroup = NS strips of one image (NS = 1: 4 waves, grid 3 x B; NS = 3: 12 waves, grid B).
// NS = 3 stages the conv2 weights (36.9 KB) once per image instead of once per strip and computes
// the 26 a1 rows once (strips recompute 2 halo rows); it is the faster form while every image
// gets a CU of its own (B <= 256), NS = 1 (three workgroups per CU) beyond.
//
// LDS carve (bytes, 16-aligned), time-shared so NS = 1 fits three workgroups per CU (160 KiB):
//   [0, A1S)           a1 tile (bf16 NHWC, swizzled)          -> after the MFMA loop: pool staging
//   [W2S_OFF, +36864)  conv2 weights: the EARLY chunks of every thread are stored in phase 0, the
//                      input rows + conv1 weights live where the parked chunks go until conv1 has
//                      consumed them, then the parked chunks are stored from VGPRs (phase 1b)
//                      -> later: flags
template <int NS>
struct TrunkCfg {
  static constexpr int THREADS = 256 * NS;
  static constexpr int ROWS2 = STRIP * NS;                    // conv2 output rows
  static constexpr int A1_ROWS = ROWS2 + 2, X_ROWS = ROWS2 + 4;
  static constexpr int A1S_BYTES = A1_ROWS * H1 * C1 * 2;     // 16640 | 43264
  static constexpr int W2S_OFF = A1S_BYTES, W2S_BYTES = C2 * 9 * C1 * 2;
  static constexpr int CHUNKS = W2S_BYTES / 16 / THREADS;     // 16-B weight chunks per thread: 9 | 3
  static constexpr int EARLY = NS == 1 ? 7 : 2;               // stored in phase 0, rest parked
  static constexpr int XS_OFF = W2S_OFF + EARLY * THREADS * 16, XS_BYTES = X_ROWS * IMG * 4;
  // conv1 weights + bias (320 floats) staged once per workgroup, past the input rows (also in the
  // parked-chunk region, consumed at the start of phase 1)
  static constexpr int W1S_OFF = XS_OFF + XS_BYTES, W1S_BYTES = (C1 * 9 + C1) * 4;
  static constexpr int WIN_LD = WIN * NS + 4;                 // [channel][window] row: 52 | 148 =
                                                              // 20 mod 32 words -> conflict-free rows
  static constexpr int POOL_OFF = 0, POOL_BYTES = C2 * WIN_LD * 4;
  static constexpr int FLAG_OFF = W2S_OFF, FLAG_BYTES = C2 * WIN_LD;
  // the workgroup's pmask words ([pooled position / 4][channel] uint32, a contiguous 3 KB per strip
  // of the global layout) staged past the flags, then stored as whole 16-B lanes
  static constexpr int PM_OFF = (FLAG_OFF + FLAG_BYTES + 15) / 16 * 16, PM_BYTES = NS * (WIN / 4) * C2 * 4;
  static constexpr int LDS = W2S_OFF + W2S_BYTES;             // 53504 | 80128
  static constexpr int C1_PIX = THREADS / 4;                  // conv1 pixels per pass (4 chunks each)
  static constexpr int C1_ITERS = (A1_ROWS * H1 + C1_PIX - 1) / C1_PIX;   // 5 | 4
  static_assert(CHUNKS * THREADS * 16 == W2S_BYTES, "weight chunking");
  static_assert(XS_OFF + XS_BYTES <= LDS, "input rows alias the parked weight chunks");
  static_assert(W1S_OFF % 16 == 0 && W1S_OFF + W1S_BYTES <= LDS, "conv1 weights alias the parked chunks");
  static_assert(POOL_BYTES <= A1S_BYTES && PM_OFF + PM_BYTES <= LDS, "epilogue staging aliasing");
  static_assert(NS != 1 || 3 * LDS <= 160 * 1024, "three strip workgroups per CU");
};

// 16-byte-chunk XOR swizzles (4 chunks of 8 channels per 64-byte row) against ds_read_b128 bank
// conflicts.  a1: keyed by the pixel's column, which makes the conv2 A-fragment reads (2 rows x 8
// columns of pixels per 16-lane group) conflict-free (tools/lds_banks.py: 4 LDS cycles per
// wave-instruction vs 8 unswizzled) while each conv1 store stays 64 contiguous bytes per pixel.
// w2: rows indexed by (channel, tap).
__device__ __forceinline__ int swz_a1(int col) { return col & 3; }
__device__ __forceinline__ int swz_w2(int n) { return (4 - ((n >> 2) & 3)) & 3; }
}  // namespace

// input-row source: pre-gathered epoch rows, rows by index, or fp32 module input (a template
// parameter so phase 0 has no load under a branch: such a load ends in vmcnt(0) at the join)
enum TrunkX { TX_PRE = 0, TX_IDX = 1, TX_XIN = 2 };

template <bool TRAIN, int NS, int XM>
__global__ __launch_bounds__(256 * NS, NS == 1 ? 3 : 1) void trunk_fwd_kernel(TrunkFwdArgs a) {
  TL_SCOPE(TL_TRUNK);
  RW_ENTRY();
  using K = TrunkCfg<NS>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[K::LDS];
  float* xs = reinterpret_cast<float*>(smem + K::XS_OFF);
  float* w1s = reinterpret_cast<float*>(smem + K::W1S_OFF);
  uint16_t* a1s = reinterpret_cast<uint16_t*>(smem);
  uint16_t* w2s = reinterpret_cast<uint16_t*>(smem + K::W2S_OFF);
  float* pool_s = reinterpret_cast<float*>(smem + K::POOL_OFF);
  uint8_t* flag_s = smem + K::FLAG_OFF;

  const int tid = threadIdx.x;
  const int strip0 = blockIdx.x * NS;   // first strip of this workgroup
  const int b = blockIdx.y;             // row in batch
  // the whole step state read once at entry (phase 4's dropout key would otherwise be re-loaded
  // after the phase-1 global stores, two dependent round trips at the tail)
  const StepState* st = a.state ? a.state : &g_zero_state;   // unconditional state loads
  const int step = st->step, st_flags = st->flags;
  const uint64_t st_seed = st->seed, st_rng_base = st->rng_base;
  PHASE_MARK(0);

  // ---- phase 0: issue every global load first (input rows, conv2 weights, conv1 weights, conv2
  // bias) - all unconditional, so the waits count exactly - then fill LDS: conv2 weights swizzled,
  // input rows normalised to fp32 by IEEE arithmetic (bitwise the table; a table lookup would be a
  // dependent load per pixel).
  const int c = tid & 3;                         // conv1: fixed 8-channel chunk per thread
  float bias2[4];
  constexpr int PARKED = K::CHUNKS - K::EARLY;
  static_assert(PARKED == 1 || PARKED == 2, "parked chunk count");
  uint4 wp0, wp1 = {0u, 0u, 0u, 0u};            // conv2-weight chunks held in VGPRs until phase 1b
                                                 // (named scalars: an array here lands in scratch)
  {
    const uint4* src = reinterpret_cast<const uint4*>(a.w2f);
    uint4 wv[K::EARLY];
#pragma unroll
    for (int i = 0; i < K::EARLY; ++i) wv[i] = src[tid + K::THREADS * i];
    wp0 = src[tid + K::THREADS * K::EARLY];
    if constexpr (PARKED == 2) wp1 = src[tid + K::THREADS * (K::EARLY + 1)];
    // conv1 weights [32][9] (72 float4) + bias (8 float4): 80 threads fetch them once per workgroup
    // (per-thread copies were 18 float4 loads x 768 threads of L1 traffic)
    const float4 w1v = tid < 72 ? reinterpret_cast<const float4*>(a.w1c)[tid]
                                : reinterpret_cast<const float4*>(a.b1c)[tid < 80 ? tid - 72 : 0];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) bias2[nt] = a.b2c[nt * 16 + (tid & 15)];
    // input rows: pixel e = tid + THREADS*j, one coalesced byte (or float) load each
    constexpr int NX = K::X_ROWS * IMG;
    constexpr int XJ = (NX + K::THREADS - 1) / K::THREADS;   // 2
    const int64_t xoff = (int64_t)strip0 * STRIP * IMG;
    float xv[XJ];
    if constexpr (XM == TX_XIN) {
#pragma unroll
      for (int j = 0; j < XJ; ++j) {
        const int e = tid + K::THREADS * j;
        xv[j] = a.xin[(int64_t)b * (IMG * IMG) + xoff + (e < NX ? e : 0)];
      }
    } else {
      const int64_t row = (int64_t)step * a.idx_step_stride + b;
      const int64_t img = (XM == TX_IDX) ? (int64_t)a.idx[row] : row;
      const uint8_t* src8 = a.data_u8 + img * (IMG * IMG) + xoff;
#pragma unroll
      for (int j = 0; j < XJ; ++j) {
        const int e = tid + K::THREADS * j;
        xv[j] = __builtin_bit_cast(float, (uint32_t)src8[e < NX ? e : 0]);
      }
    }
#pragma unroll
    for (int i = 0; i < K::EARLY; ++i) {         // swizzle only permutes chunks inside a 64-B row
      const int ch = tid + K::THREADS * i;
      const int row = ch >> 2, kc = ch & 3;      // row = n*9 + tap
      *reinterpret_cast<uint4*>(w2s + row * 32 + ((kc ^ swz_w2(row / 9)) * 8)) = wv[i];
    }
    if (tid < 80) {                              // pair-interleaved: [chunk c][pair jp][tap t | bias][2]
      const float fv[4] = {w1v.x, w1v.y, w1v.z, w1v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int f = 4 * tid + e;                 // w1c[ch][t] (f < 288) or b1c[ch]
        const int ch = f < C1 * 9 ? f / 9 : f - C1 * 9, t = f < C1 * 9 ? f - 9 * (f / 9) : 9;
        w1s[(((ch >> 3) * 4 + ((ch & 7) >> 1)) * 10 + t) * 2 + (ch & 1)] = fv[e];
      }
    }
#pragma unroll
    for (int j = 0; j < XJ; ++j) {
      const int e = tid + K::THREADS * j;
      if (e < NX) xs[e] = (XM == TX_XIN) ? xv[j] : normalize_u8_alu(__builtin_bit_cast(uint32_t, xv[j]));
    }
  }
  __syncthreads();
  PHASE_MARK(1);

  // ---- phase 1: conv1 + bias + ReLU (fp32 VALU) -> a1 tile (bf16 NHWC, swizzled) [+ HBM copy].
  // Channel pairs on v_pk_fma_f32 (the input pixel broadcast to both halves): per channel the same
  // fma chain as conv1_preact (bias, then taps in row-major order), so bitwise the scalar result.
  float2v wp[4][9], bp[4];
  {
    const float2v* wl = reinterpret_cast<const float2v*>(w1s) + c * 40;
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
#pragma unroll
      for (int t = 0; t < 9; ++t) wp[jp][t] = wl[jp * 10 + t];
      bp[jp] = wl[jp * 10 + 9];
    }
  }
#pragma unroll
  for (int i = 0; i < K::C1_ITERS; ++i) {
    const int pidx = (tid >> 2) + K::C1_PIX * i;
    if (pidx < K::A1_ROWS * H1) {
      const int r = pidx / H1, col = pidx - r * H1;
      const float* xp = xs + r * IMG + col;
      float xv[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) xv[t] = xp[(t / 3) * IMG + t % 3];
      float o[8];
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        float2v acc = bp[jp];
#pragma unroll
        for (int t = 0; t < 9; ++t) acc = __builtin_elementwise_fma(float2v{xv[t], xv[t]}, wp[jp][t], acc);
        o[2 * jp] = fmaxf(acc.x, 0.0f);
        o[2 * jp + 1] = fmaxf(acc.y, 0.0f);
      }
      uint4 v;
      v.x = pack2bf(o[0], o[1]); v.y = pack2bf(o[2], o[3]);
      v.z = pack2bf(o[4], o[5]); v.w = pack2bf(o[6], o[7]);
      *reinterpret_cast<uint4*>(a1s + pidx * 32 + ((c ^ swz_a1(col)) * 8)) = v;
      if (TRAIN && (r < K::ROWS2 || strip0 + NS == 3)) {   // halo rows are written by their owner strip
        const int grow = strip0 * STRIP + r;
        // write-through: the a1 copy is read by the backward kernels only (no dirty L2 lines for
        // the kernel-end release to write back)
        store16((int)gridDim.y <= WT_MAX_B, a.a1_out, ((((int64_t)b * H1 + grow) * H1 + col) * C1 + c * 8) * 2, v);
      }
    }
  }
  __syncthreads();
  PHASE_MARK(2);

  // ---- phase 1b: the parked conv2-weight chunks (swizzled) over the consumed input rows
#pragma unroll
  for (int i = 0; i < PARKED; ++i) {
    const int ch = tid + K::THREADS * (K::EARLY + i);
    const int row = ch >> 2, kc = ch & 3;
    *reinterpret_cast<uint4*>(w2s + row * 32 + ((kc ^ swz_w2(row / 9)) * 8)) = i ? wp1 : wp0;
  }
  __syncthreads();
  PHASE_MARK(3);

  // ---- phase 2: conv2 implicit GEMM on MFMA.  Wave w works on strip w/4 of the workgroup and owns
  // its M-tiles 3(w%4)..+2 (16 pixels = 4 pool windows each) x all 4 N-tiles (64 channels);
  // K loop = 9 taps of 32 channels.
  const int wave = tid >> 6, lane = tid & 63;
  const int sl = NS == 1 ? 0 : wave >> 2, wl = wave & 3;   // strip within the workgroup, wave in strip
  const int m = lane & 15, kg = lane >> 4;
  int pix_base[3], col_base[3];
#pragma unroll
  for (int mt = 0; mt < 3; ++mt) {
    const int win = 4 * (3 * wl + mt) + (m >> 2), q = m & 3;
    const int pr = win / HP + (STRIP / 2) * sl, pc = win % HP;
    col_base[mt] = 2 * pc + (q & 1);
    pix_base[mt] = (2 * pr + (q >> 1)) * H1 + col_base[mt];
  }
  floatx4 acc[3][4];
#pragma unroll
  for (int mt = 0; mt < 3; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = floatx4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int toff = (t / 3) * H1 + (t % 3);
    bf16x8 A[3], Bf[4];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) {
      const int pix = pix_base[mt] + toff;
      A[mt] = ld16(a1s + pix * 32 + ((kg ^ swz_a1(col_base[mt] + t % 3)) * 8));
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int n = nt * 16 + m;
      Bf[nt] = ld16(w2s + (n * 9 + t) * 32 + ((kg ^ swz_w2(n)) * 8));
    }
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = mfma16x16x32(A[mt], Bf[nt], acc[mt][nt]);
  }

  __syncthreads();   // a1 tile and conv2 weights are consumed: their regions become the staging
  PHASE_MARK(4);
  // ---- phase 3: bias + ReLU + 2x2 max-pool (in registers) -> LDS staging [channel][window]
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int n = nt * 16 + m;
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) {
      const int win = WIN * sl + 4 * (3 * wl + mt) + kg;
      float best = fmaxf(acc[mt][nt][0] + bias2[nt], 0.0f);
      int arg = 0;
#pragma unroll
      for (int r = 1; r < 4; ++r) {
        const float v = fmaxf(acc[mt][nt][r] + bias2[nt], 0.0f);
        if (v > best) { best = v; arg = r; }   // first max wins, as torch max_pool2d
      }
      pool_s[n * K::WIN_LD + win] = best;
      flag_s[n * K::WIN_LD + win] = (uint8_t)(arg | ((best > 0.0f) ? 8 : 0));
    }
  }
  __syncthreads();
  PHASE_MARK(5);

  // ---- phase 4: dropout + coalesced stores.  One thread = 16 contiguous flat elements of one
  // channel = exactly one Philox block (3 per channel-strip).
  const uint64_t seed = st_seed;
  const uint64_t off = st_rng_base + 2ull * (uint64_t)step;
  const bool drop = TRAIN && !(st_flags & STEP_FLAG_NO_DROPOUT);
  if (tid < C2 * 3 * NS) {
    const int n = tid / (3 * NS), j16 = (tid - n * 3 * NS) * 16;
    const int flat = n * NPOOL + strip0 * WIN + j16;
    const float* ps = pool_s + n * K::WIN_LD + j16;
    float o[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 pv = *reinterpret_cast<const float4*>(ps + 4 * q);
      o[4 * q] = pv.x; o[4 * q + 1] = pv.y; o[4 * q + 2] = pv.z; o[4 * q + 3] = pv.w;
    }
    if (TRAIN) {
      const uint4 fl = *reinterpret_cast<const uint4*>(flag_s + n * K::WIN_LD + j16);
      u32x4 rw = {0u, 0u, 0u, 0u};
      if (drop) rw = dropout_block(seed, off, ((uint64_t)b * NFLAT + flat) >> 4);
      uint32_t mk[4] = {fl.x, fl.y, fl.z, fl.w};
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const bool keep = dropout_byte(rw, k) < KEEP1_THR8;
        o[k] = keep ? (drop ? o[k] * (1.0f / KEEP1) : o[k]) : 0.0f;
        if (keep) mk[k >> 2] |= 4u << (8 * (k & 3));
      }
      // pmask layout [b][pooled position / 4][channel][4] (mnist_common.h): fc_bwd role B reads one
      // contiguous 256-B run per row and 4-position group instead of 4 bytes per 144-B stride.
      // Staged in LDS (this thread's words are 256 B apart), stored below as 16-B lanes.
      uint32_t* pm_s = reinterpret_cast<uint32_t*>(smem + K::PM_OFF);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) pm_s[((j16 >> 2) + q4) * C2 + n] = mk[q4];
    }
    uint4 s0, s1;
    s0.x = pack2bf(o[0], o[1]);   s0.y = pack2bf(o[2], o[3]);
    s0.z = pack2bf(o[4], o[5]);   s0.w = pack2bf(o[6], o[7]);
    s1.x = pack2bf(o[8], o[9]);   s1.y = pack2bf(o[10], o[11]);
    s1.z = pack2bf(o[12], o[13]); s1.w = pack2bf(o[14], o[15]);
    const int64_t pb = ((int64_t)b * NFLAT + flat) * 2;           // write-through (read by later kernels)
    store16((int)gridDim.y <= WT_MAX_B, a.p_out, pb, s0);
    store16((int)gridDim.y <= WT_MAX_B, a.p_out, pb + 16, s1);
  }
  if (TRAIN) {
    // the workgroup's pmask region: NS x 3 KB contiguous from position group strip0 * WIN / 4
    // (write-through at small batches, as p_out; one 16-B lane per thread)
    lds_barrier();
    if (tid < K::PM_BYTES / 16)
      store16((int)gridDim.y <= WT_MAX_B, a.pmask_out, (int64_t)b * NFLAT + strip0 * (WIN / 4) * C2 * 4 + tid * 16,
              reinterpret_cast<const uint4*>(smem + K::PM_OFF)[tid]);
  }
  PHASE_MARK(6);
  // DDP schedule 3: the kernel completes only once the comm stream's fc update of the previous step
  // is done (*wait_a >= *wait_b), so fc1_fwd - which reads the updated fc weights - can follow with
  // no separate wait launch; one lane of the last workgroup spins while the others drain.
  if (a.wait_a && blockIdx.x == gridDim.x - 1 && b == (int)gridDim.y - 1 && tid == 0)
    spin_until_geq(a.wait_a, __hip_atomic_load(a.wait_b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                   a.wait_err);
}

int trunk_strips_per_wg(int B) { return B <= TRUNK_IMG_MAX_B ? 3 : 1; }

template <bool TRAIN, int NS>
static void launch_trunk(const TrunkFwdArgs& a, dim3 grid, hipStream_t s) {
  if (a.xin)
    hipLaunchKernelGGL((trunk_fwd_kernel<TRAIN, NS, TX_XIN>), grid, dim3(256 * NS), 0, s, a);
  else if (a.idx)
    hipLaunchKernelGGL((trunk_fwd_kernel<TRAIN, NS, TX_IDX>), grid, dim3(256 * NS), 0, s, a);
  else
    hipLaunchKernelGGL((trunk_fwd_kernel<TRAIN, NS, TX_PRE>), grid, dim3(256 * NS), 0, s, a);
}

void launch_trunk_fwd(const TrunkFwdArgs& a, int B, bool train, hipStream_t s) {
  if (trunk_strips_per_wg(B) == 3) {
    if (train) launch_trunk<true, 3>(a, dim3(1, B), s);
    else launch_trunk<false, 3>(a, dim3(1, B), s);
  } else {
    if (train) launch_trunk<true, 1>(a, dim3(3, B), s);
    else launch_trunk<false, 1>(a, dim3(3, B), s);
  }
}

TL_DEFINE_HOST(trunk)

// load this translation unit's gfx950 code object now (startup prewarm thread) instead of at its
// first launch inside the timed run
void preload_trunk() {
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&(trunk_fwd_kernel<true, 3, TX_PRE>)));
}

}  // namespace mnist
