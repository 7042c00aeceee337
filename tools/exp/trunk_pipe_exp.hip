// EXPERIMENT (round 6, measured and not adopted; not part of the built extension): a pipelined
// form of the whole-image trunk_fwd (B <= 256), bitwise the classic kernel's outputs, with its own
// harness - bitwise check against the product kernel, event timing of both, and the per-stage
// s_memtime breakdown of the pipelined one.  Results and reading: docs/PERF_NOTES.md round 6
// ("B = 200 trunk: a wave-specialised pipeline") and profiles/r6/ab/trunk_pipe/.
//
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize -Icsrc/include \
//          [-DPIPE_MFMA_WAVES=8] [-DTRUNK_PIPE_PRIO=n] [-DTRUNK_PIPE_VPRIO=n] \
//          tools/exp/trunk_pipe_exp.hip -o tools/exp/trunk_pipe_exp
// run:   tools/exp/trunk_pipe_exp [B = 200]
#define MNIST_PHASE_TIMING 1
#include "../../csrc/kernels/trunk_fwd.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace mnist {

// Pipelined whole-image form (B <= TRUNK_IMG_MAX_B, one 12-wave workgroup per image and per CU).
// The classic form runs every phase on all 12 waves between barriers - conv1 VALU, then conv2 MFMA,
// then the pool epilogue - so the matrix pipe idles through the vector phases and the other way
// round.  Here waves 0-3 (one per SIMD) run conv2's MFMA + pool epilogue strip after strip while
// waves 4-11 compute the next strip's conv1 rows and then the finished strips' dropout + stores:
//
//   stage   waves 0-3 (MFMA)            waves 4-11 (VALU)
//   S1      conv1 rows 0-9 (all 12 waves: strip 0's input)
//   S2      conv2 + pool, strip 0       conv1 rows 10-17
//   S3      conv2 + pool, strip 1       conv1 rows 18-25
//   S4      conv2 + pool, strip 2       dropout + stores, strips 0 and 1
//   S5      dropout + stores, strip 2; pmask stores
//
// One barrier between stages; a wave's role is wave-uniform, and both roles pass the same number of
// barriers.  Nothing is aliased in LDS (141 KB: one workgroup per CU anyway).  Per element the same
// arithmetic in the same order as the classic kernel: the outputs are bitwise the same.
#ifndef PIPE_MFMA_WAVES
#define PIPE_MFMA_WAVES 4                // 4: one MFMA wave per SIMD (all 4 N-tiles), 8: two (2 each)
#endif
namespace {
struct PipeCfg {
  static constexpr int THREADS = 768;
  static constexpr int A1_ROWS = 3 * STRIP + 2;                           // 26
  static constexpr int A1S_BYTES = A1_ROWS * H1 * C1 * 2;                // 43264
  static constexpr int W2S_OFF = A1S_BYTES, W2S_BYTES = C2 * 9 * C1 * 2;  // 36864
  static constexpr int CHUNKS = W2S_BYTES / 16 / THREADS;                 // 3
  static constexpr int X_ROWS = A1_ROWS + 2;                              // 28
  static constexpr int XS_OFF = W2S_OFF + W2S_BYTES, XS_BYTES = X_ROWS * IMG * 4;
  static constexpr int W1S_OFF = XS_OFF + XS_BYTES, W1S_BYTES = (C1 * 9 + C1) * 4;
  static constexpr int WIN_LD = 3 * WIN + 4;                              // 148
  static constexpr int POOL_OFF = W1S_OFF + W1S_BYTES, POOL_BYTES = C2 * WIN_LD * 4;
  static constexpr int FLAG_OFF = POOL_OFF + POOL_BYTES, FLAG_BYTES = C2 * WIN_LD;
  static constexpr int PM_OFF = (FLAG_OFF + FLAG_BYTES + 15) / 16 * 16, PM_BYTES = 3 * (WIN / 4) * C2 * 4;
  static constexpr int LDS = PM_OFF + PM_BYTES;                           // 141120
  static_assert(CHUNKS * THREADS * 16 == W2S_BYTES, "weight chunking");
  static_assert(W1S_OFF % 16 == 0 && POOL_OFF % 16 == 0, "alignment");
  static_assert(LDS <= 160 * 1024, "one workgroup per CU");
};

// conv1 + bias + ReLU of the items (pixel, chunk c) of pixels [P0, P1): thread t of N takes pixels
// P0 + t/4, P0 + t/4 + N/4, ... with its fixed chunk c = t & 3 (the chunk its weights are for); a
// compile-time trip count, unrolled, so the items' independent fma chains interleave.  Per channel
// the classic kernel's fma chain (bias, then taps in row-major order).
template <bool TRAIN, int P0, int P1, int N>
__device__ __forceinline__ void pipe_conv1_rows(int t, const float* xs, const float2v (&wp)[4][9],
                                                const float2v (&bp)[4], uint16_t* a1s, uint16_t* a1_out, int b,
                                                bool wt) {
  const int c = t & 3;
  constexpr int ITERS = (P1 - P0 + N / 4 - 1) / (N / 4);
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int pidx = P0 + (t >> 2) + (N / 4) * i;
    if (pidx >= P1) break;
    const int r = pidx / H1, col = pidx - r * H1;
    const float* xp = xs + r * IMG + col;
    float xv[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) xv[k] = xp[(k / 3) * IMG + k % 3];
    float o[8];
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      float2v acc = bp[jp];
#pragma unroll
      for (int k = 0; k < 9; ++k) acc = __builtin_elementwise_fma(float2v{xv[k], xv[k]}, wp[jp][k], acc);
      o[2 * jp] = fmaxf(acc.x, 0.0f);
      o[2 * jp + 1] = fmaxf(acc.y, 0.0f);
    }
    uint4 v;
    v.x = pack2bf(o[0], o[1]); v.y = pack2bf(o[2], o[3]);
    v.z = pack2bf(o[4], o[5]); v.w = pack2bf(o[6], o[7]);
    *reinterpret_cast<uint4*>(a1s + pidx * 32 + ((c ^ swz_a1(col)) * 8)) = v;
    if (TRAIN) store16(wt, a1_out, ((((int64_t)b * H1 + r) * H1 + col) * C1 + c * 8) * 2, v);
  }
}

// conv2 implicit GEMM of strip s for MFMA wave wl (its M-tiles 3wl..3wl+2 x N-tiles nt0..nt0+NTW-1),
// then bias + ReLU + 2x2 max-pool into the [channel][window] staging: the classic kernel's wave
// 4s + wl (NTW = 4), or half of it (NTW = 2, two MFMA waves per SIMD).  Each accumulator sees the
// same 9 MFMAs in the same order either way.
template <int NTW>
__device__ __forceinline__ void pipe_mfma_pool(int s, int wl, int nt0, int lane, const uint16_t* a1s,
                                               const uint16_t* w2s, const float (&bias2)[4], float* pool_s,
                                               uint8_t* flag_s) {
  using K = PipeCfg;
  const int m = lane & 15, kg = lane >> 4;
  int pix_base[3], col_base[3];
#pragma unroll
  for (int mt = 0; mt < 3; ++mt) {
    const int win = 4 * (3 * wl + mt) + (m >> 2), q = m & 3;
    const int pr = win / HP + (STRIP / 2) * s, pc = win % HP;
    col_base[mt] = 2 * pc + (q & 1);
    pix_base[mt] = (2 * pr + (q >> 1)) * H1 + col_base[mt];
  }
  floatx4 acc[3][NTW];
#pragma unroll
  for (int mt = 0; mt < 3; ++mt)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // one wave per SIMD runs this loop: the next tap's fragments are loaded while the current tap's
  // 12 MFMAs issue (no partner wave hides the LDS latency here)
  bf16x8 A[2][3], Bf[2][NTW];
  auto frags = [&](int t, int buf) {
    const int toff = (t / 3) * H1 + (t % 3);
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) {
      const int pix = pix_base[mt] + toff;
      A[buf][mt] = ld16(a1s + pix * 32 + ((kg ^ swz_a1(col_base[mt] + t % 3)) * 8));
    }
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n = (nt0 + j) * 16 + m;
      Bf[buf][j] = ld16(w2s + (n * 9 + t) * 32 + ((kg ^ swz_w2(n)) * 8));
    }
  };
  frags(0, 0);
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int cur = t & 1;
    if (t + 1 < 9) frags(t + 1, cur ^ 1);
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[mt][j] = mfma16x16x32(A[cur][mt], Bf[cur][j], acc[mt][j]);
  }
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = nt0 + j, n = nt * 16 + m;
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) {
      const int win = WIN * s + 4 * (3 * wl + mt) + kg;
      float best = fmaxf(acc[mt][j][0] + bias2[nt], 0.0f);
      int arg = 0;
#pragma unroll
      for (int r = 1; r < 4; ++r) {
        const float v = fmaxf(acc[mt][j][r] + bias2[nt], 0.0f);
        if (v > best) { best = v; arg = r; }   // first max wins, as torch max_pool2d
      }
      pool_s[n * K::WIN_LD + win] = best;
      flag_s[n * K::WIN_LD + win] = (uint8_t)(arg | ((best > 0.0f) ? 8 : 0));
    }
  }
}

// dropout + coalesced stores of strip s: thread t (< 192) = 16 contiguous flat elements of channel
// t / 3 (one Philox block), as the classic kernel's thread 9 * (t / 3) + 3 * s + t % 3
template <bool TRAIN>
__device__ __forceinline__ void pipe_dropout(int s, int t, const TrunkFwdArgs& a, int b, const float* pool_s,
                                             const uint8_t* flag_s, uint32_t* pm_s, uint64_t seed, uint64_t off,
                                             bool drop, bool wt) {
  using K = PipeCfg;
  const int n = t / 3, j16 = WIN * s + (t - 3 * n) * 16;
  const int flat = n * NPOOL + j16;
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
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) pm_s[((j16 >> 2) + q4) * C2 + n] = mk[q4];
  }
  uint4 s0, s1;
  s0.x = pack2bf(o[0], o[1]);   s0.y = pack2bf(o[2], o[3]);
  s0.z = pack2bf(o[4], o[5]);   s0.w = pack2bf(o[6], o[7]);
  s1.x = pack2bf(o[8], o[9]);   s1.y = pack2bf(o[10], o[11]);
  s1.z = pack2bf(o[12], o[13]); s1.w = pack2bf(o[14], o[15]);
  const int64_t pb = ((int64_t)b * NFLAT + flat) * 2;
  store16(wt, a.p_out, pb, s0);
  store16(wt, a.p_out, pb + 16, s1);
}
}  // namespace

template <bool TRAIN, int XM>
__global__ __launch_bounds__(768, 1) void trunk_fwd_pipe_kernel(TrunkFwdArgs a) {
  TL_SCOPE(TL_TRUNK);
  RW_ENTRY();
  using K = PipeCfg;
  __shared__ __attribute__((aligned(16))) unsigned char smem[K::LDS];
  float* xs = reinterpret_cast<float*>(smem + K::XS_OFF);
  float* w1s = reinterpret_cast<float*>(smem + K::W1S_OFF);
  uint16_t* a1s = reinterpret_cast<uint16_t*>(smem);
  uint16_t* w2s = reinterpret_cast<uint16_t*>(smem + K::W2S_OFF);
  float* pool_s = reinterpret_cast<float*>(smem + K::POOL_OFF);
  uint8_t* flag_s = smem + K::FLAG_OFF;
  uint32_t* pm_s = reinterpret_cast<uint32_t*>(smem + K::PM_OFF);

  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  const StepState* st = a.state ? a.state : &g_zero_state;
  const int step = st->step, st_flags = st->flags;
  const uint64_t st_seed = st->seed, st_rng_base = st->rng_base;
  const bool wt = (int)gridDim.y <= WT_MAX_B;
  PHASE_MARK(0);

  // ---- S0: every global load first (all unconditional), then LDS: conv2 weights (all chunks,
  // swizzled), conv1 weights pair-interleaved, input rows normalised
  float bias2[4];
  {
    const uint4* src = reinterpret_cast<const uint4*>(a.w2f);
    uint4 wv[K::CHUNKS];
#pragma unroll
    for (int i = 0; i < K::CHUNKS; ++i) wv[i] = src[tid + K::THREADS * i];
    const float4 w1v = tid < 72 ? reinterpret_cast<const float4*>(a.w1c)[tid]
                                : reinterpret_cast<const float4*>(a.b1c)[tid < 80 ? tid - 72 : 0];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) bias2[nt] = a.b2c[nt * 16 + (tid & 15)];
    constexpr int NX = K::X_ROWS * IMG;
    constexpr int XJ = (NX + K::THREADS - 1) / K::THREADS;   // 2
    float xv[XJ];
    if constexpr (XM == TX_XIN) {
#pragma unroll
      for (int j = 0; j < XJ; ++j) {
        const int e = tid + K::THREADS * j;
        xv[j] = a.xin[(int64_t)b * (IMG * IMG) + (e < NX ? e : 0)];
      }
    } else {
      const int64_t row = (int64_t)step * a.idx_step_stride + b;
      const int64_t img = (XM == TX_IDX) ? (int64_t)a.idx[row] : row;
      const uint8_t* src8 = a.data_u8 + img * (IMG * IMG);
#pragma unroll
      for (int j = 0; j < XJ; ++j) {
        const int e = tid + K::THREADS * j;
        xv[j] = __builtin_bit_cast(float, (uint32_t)src8[e < NX ? e : 0]);
      }
    }
#pragma unroll
    for (int i = 0; i < K::CHUNKS; ++i) {
      const int ch = tid + K::THREADS * i;
      const int row = ch >> 2, kc = ch & 3;
      *reinterpret_cast<uint4*>(w2s + row * 32 + ((kc ^ swz_w2(row / 9)) * 8)) = wv[i];
    }
    if (tid < 80) {
      const float fv[4] = {w1v.x, w1v.y, w1v.z, w1v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int f = 4 * tid + e;
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

  float2v wp[4][9], bp[4];
  {
    const float2v* wl = reinterpret_cast<const float2v*>(w1s) + (tid & 3) * 40;
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
#pragma unroll
      for (int t = 0; t < 9; ++t) wp[jp][t] = wl[jp * 10 + t];
      bp[jp] = wl[jp * 10 + 9];
    }
  }
  // ---- S1: conv1 rows 0-9 (strip 0's input) on all 12 waves
  pipe_conv1_rows<TRAIN, 0, (STRIP + 2) * H1, K::THREADS>(tid, xs, wp, bp, a1s, a.a1_out, b, wt);
  __syncthreads();
  PHASE_MARK(2);

  const uint64_t seed = st_seed;
  const uint64_t off = st_rng_base + 2ull * (uint64_t)step;
  const bool drop = TRAIN && !(st_flags & STEP_FLAG_NO_DROPOUT);
  // the role is wave-uniform by construction; readfirstlane makes it a scalar branch, so each wave
  // passes only its own role's barriers
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int MW = PIPE_MFMA_WAVES, VT = K::THREADS - 64 * MW;   // MFMA waves, VALU threads
  if (wave < MW) {
    // ---- S2-S4, MFMA waves: strip after strip
#ifdef TRUNK_PIPE_PRIO
    __builtin_amdgcn_s_setprio(TRUNK_PIPE_PRIO);
#endif
#pragma unroll 1
    for (int s = 0; s < 3; ++s) {
      pipe_mfma_pool<16 / MW>(s, wave & 3, (wave >> 2) * (16 / MW), tid & 63, a1s, w2s, bias2, pool_s, flag_s);
      PHASE_MARK(3 + 2 * s);
      __syncthreads();
      PHASE_MARK(4 + 2 * s);
    }
  } else {
#ifdef TRUNK_PIPE_VPRIO
    __builtin_amdgcn_s_setprio(TRUNK_PIPE_VPRIO);
#endif
    const int t = tid - 64 * MW;
    // S2: conv1 rows 10-17 (strip 1 needs 8-17); S3: rows 18-25 (strip 2 needs 16-25)
    pipe_conv1_rows<TRAIN, (STRIP + 2) * H1, (2 * STRIP + 2) * H1, VT>(t, xs, wp, bp, a1s, a.a1_out, b, wt);
    PHASE_MARK_BY(64 * MW, 10);
    __syncthreads();
    pipe_conv1_rows<TRAIN, (2 * STRIP + 2) * H1, K::A1_ROWS * H1, VT>(t, xs, wp, bp, a1s, a.a1_out, b, wt);
    PHASE_MARK_BY(64 * MW, 11);
    __syncthreads();
    // S4: strips 0 and 1 are pooled
    if (t < (VT >= 384 ? 384 : 192)) pipe_dropout<TRAIN>(t / 192, t % 192, a, b, pool_s, flag_s, pm_s, seed, off, drop, wt);
    PHASE_MARK_BY(64 * MW, 12);
    __syncthreads();
  }
  // ---- S5: strip 2, then the workgroup's pmask words as whole 16-B lanes
  if (VT >= 384) {
    if (tid < 192) pipe_dropout<TRAIN>(2, tid, a, b, pool_s, flag_s, pm_s, seed, off, drop, wt);
  } else if (tid < 384) {                // strip 0 went in S4; strips 1 and 2 here
    pipe_dropout<TRAIN>(1 + tid / 192, tid % 192, a, b, pool_s, flag_s, pm_s, seed, off, drop, wt);
  }
  if (TRAIN) {
    lds_barrier();
    if (tid < K::PM_BYTES / 16)
      store16(wt, a.pmask_out, (int64_t)b * NFLAT + tid * 16, reinterpret_cast<const uint4*>(smem + K::PM_OFF)[tid]);
  }
  PHASE_MARK(9);
  if (a.wait_a && b == (int)gridDim.y - 1 && tid == 0)
    spin_until_geq(a.wait_a, __hip_atomic_load(a.wait_b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                   a.wait_err);
}


}  // namespace mnist

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <class T> static T* dev_fill(size_t n, T v) {
  std::vector<T> h(n, v);
  T* d; CK(hipMalloc(&d, n * sizeof(T))); CK(hipMemcpy(d, h.data(), n * sizeof(T), hipMemcpyHostToDevice)); return d;
}

int main(int argc, char** argv) {
  using namespace mnist;
  const int B = argc > 1 ? atoi(argv[1]) : 200;
  if (B < 1 || B > TRUNK_IMG_MAX_B) { printf("B must be in [1, %d] (the whole-image form)\n", TRUNK_IMG_MAX_B); return 1; }
  const int N = 1024;
  std::vector<uint8_t> img((size_t)N * 784);
  srand(7);
  for (auto& x : img) x = (uint8_t)(rand() & 0xFF);
  uint8_t* d_img; CK(hipMalloc(&d_img, img.size())); CK(hipMemcpy(d_img, img.data(), img.size(), hipMemcpyHostToDevice));
  std::vector<int32_t> idx(B); for (int i = 0; i < B; ++i) idx[i] = (i * 7) % N;
  int32_t* d_idx; CK(hipMalloc(&d_idx, B * 4)); CK(hipMemcpy(d_idx, idx.data(), B * 4, hipMemcpyHostToDevice));
  StepState st{0, 0, 0x1234, 0};
  StepState* d_st; CK(hipMalloc(&d_st, sizeof(st))); CK(hipMemcpy(d_st, &st, sizeof(st), hipMemcpyHostToDevice));
  // random weights (bf16 conv2 weights from small random floats) so the pool argmax / ReLU paths vary
  std::vector<float> w1(32 * 9), b1(32), b2(64);
  std::vector<uint16_t> w2(64 * 9 * 32);
  for (auto& v : w1) v = (rand() / (float)RAND_MAX - 0.5f) * 0.6f;
  for (auto& v : b1) v = (rand() / (float)RAND_MAX - 0.5f) * 0.2f;
  for (auto& v : b2) v = (rand() / (float)RAND_MAX - 0.5f) * 0.2f;
  for (auto& v : w2) { const float f = (rand() / (float)RAND_MAX - 0.5f) * 0.2f; uint32_t u; memcpy(&u, &f, 4); v = (uint16_t)(u >> 16); }
  float *w1c, *b1c, *b2c; uint16_t* w2f;
  CK(hipMalloc(&w1c, w1.size() * 4)); CK(hipMemcpy(w1c, w1.data(), w1.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&b1c, b1.size() * 4)); CK(hipMemcpy(b1c, b1.data(), b1.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&b2c, b2.size() * 4)); CK(hipMemcpy(b2c, b2.data(), b2.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&w2f, w2.size() * 2)); CK(hipMemcpy(w2f, w2.data(), w2.size() * 2, hipMemcpyHostToDevice));
  const size_t na1 = (size_t)B * 26 * 26 * 32, np = (size_t)B * 9216;
  uint16_t* a1 = dev_fill<uint16_t>(na1, 0);
  uint16_t* p = dev_fill<uint16_t>(np, 0);
  uint8_t* pm = dev_fill<uint8_t>(np, 0);
  TrunkFwdArgs a{d_img, d_idx, 0, d_st, w1c, b1c, w2f, b2c, a1, p, pm, nullptr};
  auto classic = [&]() { launch_trunk_fwd(a, B, true, nullptr); };
  auto piped = [&]() { hipLaunchKernelGGL((trunk_fwd_pipe_kernel<true, TX_IDX>), dim3(1, B), dim3(768), 0, nullptr, a); };

  // bitwise: a1 copy, pooled + dropped activations, pmask
  std::vector<uint16_t> a1c(na1), a1p(na1), pc(np), pp(np);
  std::vector<uint8_t> pmc(np), pmp(np);
  classic(); CK(hipDeviceSynchronize());
  CK(hipMemcpy(a1c.data(), a1, na1 * 2, hipMemcpyDeviceToHost)); CK(hipMemcpy(pc.data(), p, np * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(pmc.data(), pm, np, hipMemcpyDeviceToHost));
  CK(hipMemset(a1, 0, na1 * 2)); CK(hipMemset(p, 0, np * 2)); CK(hipMemset(pm, 0, np));
  piped(); CK(hipDeviceSynchronize());
  CK(hipMemcpy(a1p.data(), a1, na1 * 2, hipMemcpyDeviceToHost)); CK(hipMemcpy(pp.data(), p, np * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(pmp.data(), pm, np, hipMemcpyDeviceToHost));
  const bool same = a1c == a1p && pc == pp && pmc == pmp;
  size_t nz = 0; for (auto v : pc) nz += v != 0;
  printf("B=%d  MFMA waves %d  bitwise equal to the product kernel: %s (a1 %s, p %s, pmask %s; %zu of %zu p nonzero)\n", B,
         PIPE_MFMA_WAVES, same ? "yes" : "NO", a1c == a1p ? "=" : "!=", pc == pp ? "=" : "!=", pmc == pmp ? "=" : "!=", nz, np);

  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](auto f) {
    for (int it = 0; it < 5; ++it) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, nullptr));
    for (int it = 0; it < 50; ++it) f();
    CK(hipEventRecord(e1, nullptr));
    CK(hipDeviceSynchronize());
    float ms = 0; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000 / 50;
  };
  const float tc = timeit(classic), tp = timeit(piped), tc2 = timeit(classic), tp2 = timeit(piped);
  printf("  kernel (events, mean of 50 back-to-back): classic %.2f / %.2f us, pipelined %.2f / %.2f us\n", tc, tc2, tp, tp2);
  const int nwg = B;
  constexpr int S = kPhaseSlots;
  std::vector<uint64_t> t((size_t)nwg * S);
  CK(hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_phase_times), t.size() * 8));   // the last pipelined launch
  auto span = [&](const char* name, int a0, int b0) {
    std::vector<double> d;
    for (int w = 0; w < nwg; ++w) d.push_back((double)(int64_t)(t[w * S + b0] - t[w * S + a0]));
    std::sort(d.begin(), d.end());
    printf("  %-40s median %7.0f  p90 %7.0f ticks\n", name, d[nwg / 2], d[nwg * 9 / 10]);
  };
  span("WG lifetime", 0, 9);
  span("S0 loads + staging", 0, 1);
  span("S1 conv1 rows 0-9 (12 waves)", 1, 2);
  span("S2 MFMA wave: strip 0 conv2 + pool", 2, 3);
  span("S2 VALU wave: conv1 rows 10-17", 2, 10);
  span("S2 end (barrier)", 2, 4);
  span("S3 MFMA wave: strip 1 conv2 + pool", 4, 5);
  span("S3 VALU wave: conv1 rows 18-25", 4, 11);
  span("S3 end (barrier)", 4, 6);
  span("S4 MFMA wave: strip 2 conv2 + pool", 6, 7);
  span("S4 VALU wave: dropout", 6, 12);
  span("S4 end (barrier)", 6, 8);
  span("S5 dropout + pmask", 8, 9);
  return same ? 0 : 2;
}
