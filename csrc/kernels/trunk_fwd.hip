// Fused conv trunk forward: gather+normalise -> conv1+bias+ReLU -> conv2 (MFMA implicit GEMM)
// -> +bias -> ReLU -> maxpool 2x2 -> dropout(0.25) -> flatten.
//
// Replaces reference mnist_ddp.py:49-56 (conv1, relu, conv2, relu, max_pool2d, dropout1, flatten)
// plus the DataLoader's ToTensor/Normalize (mnist_ddp.py:153-156) and the H2D copy (:68).
//
// One workgroup (4 waves) = one image x one strip of 8 conv2-output rows (3 strips per image).
//   * the 12x28 input rows are gathered from the HBM-resident uint8 dataset by index and normalised;
//   * conv1 (K=9, too small for MFMA) runs on the VALU in fp32 straight into an NHWC bf16 LDS tile;
//   * conv2 is an implicit GEMM on v_mfma_f32_16x16x32_bf16: M = 192 pixels, N = 64 channels,
//     K = 9 taps x 32 channels; one 32-deep k-step is exactly one tap, so every A fragment is one
//     16-byte LDS read of 8 contiguous channels at (pixel + tap offset);
//   * the M index is ordered pool-window-major (m = 4*window + q), so each lane's 4 accumulator
//     registers hold one whole 2x2 window: max-pool + argmax happen in registers;
//   * dropout uses Philox-4x32-10 keyed by (seed, per-step offset, element index), so the mask is a
//     pure function of (step, position) and identical across launch geometries and graph replays.
#include "../include/device_utils.h"
#include "../include/kernels.h"

namespace mnist {

namespace {
constexpr int STRIP = 8;                      // conv2 output rows per workgroup
constexpr int A1_ROWS = STRIP + 2;            // 10 conv1 rows
constexpr int X_ROWS = STRIP + 4;             // 12 input rows
constexpr int WIN = (STRIP / 2) * HP;         // 48 pool windows per strip

// LDS carve (bytes, all 16-aligned)
constexpr int XS_OFF = 0, XS_BYTES = X_ROWS * IMG * 4;                     // 1344
constexpr int A1S_OFF = XS_OFF + XS_BYTES, A1S_BYTES = A1_ROWS * H1 * C1 * 2;   // 16640
constexpr int W2S_OFF = A1S_OFF + A1S_BYTES, W2S_BYTES = C2 * 9 * C1 * 2;      // 36864
constexpr int POOL_OFF = W2S_OFF + W2S_BYTES, POOL_BYTES = C2 * WIN * 4;       // 12288
constexpr int FLAG_OFF = POOL_OFF + POOL_BYTES, FLAG_BYTES = C2 * WIN;         // 3072
constexpr int LDS_TOTAL = FLAG_OFF + FLAG_BYTES;

// 16-byte-chunk XOR swizzles (4 chunks of 8 channels per 64-byte row) against ds_read_b128 bank
// conflicts: a1 rows are indexed by pixel, w2 rows by (channel, tap).
__device__ __forceinline__ int swz_a1(int pix) { return 0 * pix; }   // model: no XOR beats (p>>2)&3
__device__ __forceinline__ int swz_w2(int n) { return (4 - ((n >> 2) & 3)) & 3; }
}  // namespace

template <bool TRAIN>
__global__ __launch_bounds__(256) void trunk_fwd_kernel(TrunkFwdArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_TOTAL];
  float* xs = reinterpret_cast<float*>(smem + XS_OFF);
  uint16_t* a1s = reinterpret_cast<uint16_t*>(smem + A1S_OFF);
  uint16_t* w2s = reinterpret_cast<uint16_t*>(smem + W2S_OFF);
  float* pool_s = reinterpret_cast<float*>(smem + POOL_OFF);
  uint8_t* flag_s = smem + FLAG_OFF;

  const int tid = threadIdx.x;
  const int strip = blockIdx.x;   // 0..2
  const int b = blockIdx.y;       // row in batch
  const int step = a.state ? a.state->step : 0;

  // ---- phase 0: issue every global load first (conv2 weights, conv1 weights, the gathered image
  // rows), then fill LDS: conv2 weights swizzled, input rows normalised to fp32.
  const int c = tid & 3;                         // conv1: fixed 8-channel chunk per thread
  float w[8][9], bias[8];
  {
    const uint4* src = reinterpret_cast<const uint4*>(a.w2f);
    uint4 wv[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) wv[i] = src[tid + 256 * i];
    const float4* w1v = reinterpret_cast<const float4*>(a.w1c + c * 72);
#pragma unroll
    for (int k = 0; k < 18; ++k) {
      const float4 f = w1v[k];
      const float fv[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) w[(4 * k + e) / 9][(4 * k + e) % 9] = fv[e];
    }
    const float4* b1v = reinterpret_cast<const float4*>(a.b1c + c * 8);
    const float4 b0 = b1v[0], b1 = b1v[1];
    bias[0] = b0.x; bias[1] = b0.y; bias[2] = b0.z; bias[3] = b0.w;
    bias[4] = b1.x; bias[5] = b1.y; bias[6] = b1.z; bias[7] = b1.w;
    uint4 xv = {0u, 0u, 0u, 0u};
    float4 xf = {0.f, 0.f, 0.f, 0.f};
    constexpr int XCH = X_ROWS * IMG / 16;       // 21 16-byte chunks (image rows are 16-B aligned)
    if (a.xin) {                                  // module API: fp32 input rows (84 float4)
      if (tid < X_ROWS * IMG / 4)
        xf = *reinterpret_cast<const float4*>(a.xin + (int64_t)b * (IMG * IMG) + strip * STRIP * IMG + tid * 4);
    } else {
      const int img = a.idx[(int64_t)step * a.idx_step_stride + b];
      if (tid < XCH)
        xv = *reinterpret_cast<const uint4*>(a.data_u8 + (int64_t)img * (IMG * IMG) + strip * STRIP * IMG + tid * 16);
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int ch = tid + 256 * i;                // 2304 chunks of 16 B
      const int row = ch >> 2, kc = ch & 3;        // row = n*9 + tap
      const int n = row / 9;
      *reinterpret_cast<uint4*>(w2s + row * 32 + ((kc ^ swz_w2(n)) * 8)) = wv[i];
    }
    if (a.xin) {
      if (tid < X_ROWS * IMG / 4) *reinterpret_cast<float4*>(xs + tid * 4) = xf;
    } else if (tid < XCH) {
      const uint32_t words[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float4 f;
        f.x = normalize_u8((uint8_t)(words[k] & 0xFF));
        f.y = normalize_u8((uint8_t)((words[k] >> 8) & 0xFF));
        f.z = normalize_u8((uint8_t)((words[k] >> 16) & 0xFF));
        f.w = normalize_u8((uint8_t)(words[k] >> 24));
        *reinterpret_cast<float4*>(xs + tid * 16 + 4 * k) = f;
      }
    }
  }
  __syncthreads();

  // ---- phase 1: conv1 + bias + ReLU (fp32 VALU) -> a1 tile (bf16 NHWC, swizzled) [+ HBM copy]
  {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int pidx = (tid >> 2) + 64 * i;
      if (pidx < A1_ROWS * H1) {
        const int r = pidx / H1, col = pidx - r * H1;
        const float* xp = xs + r * IMG + col;
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = fmaxf(conv1_preact(xp, IMG, w[j], bias[j]), 0.0f);
        uint4 v;
        v.x = pack2bf(o[0], o[1]); v.y = pack2bf(o[2], o[3]);
        v.z = pack2bf(o[4], o[5]); v.w = pack2bf(o[6], o[7]);
        *reinterpret_cast<uint4*>(a1s + pidx * 32 + ((c ^ swz_a1(pidx)) * 8)) = v;
        if (TRAIN && (r < STRIP || strip == 2)) {
          const int grow = strip * STRIP + r;
          *reinterpret_cast<uint4*>(a.a1_out + (((int64_t)b * H1 + grow) * H1 + col) * C1 + c * 8) = v;
        }
      }
    }
  }
  __syncthreads();

  // ---- phase 2: conv2 implicit GEMM on MFMA. wave w owns M-tiles 3w..3w+2 (16 pixels = 4 windows
  // each) x all 4 N-tiles (64 channels); K loop = 9 taps of 32 channels.
  const int wave = tid >> 6, lane = tid & 63;
  const int m = lane & 15, kg = lane >> 4;
  int pix_base[3];
#pragma unroll
  for (int mt = 0; mt < 3; ++mt) {
    const int win = 4 * (3 * wave + mt) + (m >> 2), q = m & 3;
    const int pr = win / HP, pc = win - pr * HP;
    pix_base[mt] = (2 * pr + (q >> 1)) * H1 + 2 * pc + (q & 1);
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
      A[mt] = ld16(a1s + pix * 32 + ((kg ^ swz_a1(pix)) * 8));
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

  // ---- phase 3: bias + ReLU + 2x2 max-pool (in registers) -> LDS staging [channel][window]
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int n = nt * 16 + m;
    const float bias = a.b2c[n];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) {
      const int win = 4 * (3 * wave + mt) + kg;
      float best = fmaxf(acc[mt][nt][0] + bias, 0.0f);
      int arg = 0;
#pragma unroll
      for (int r = 1; r < 4; ++r) {
        const float v = fmaxf(acc[mt][nt][r] + bias, 0.0f);
        if (v > best) { best = v; arg = r; }   // first max wins, as torch max_pool2d
      }
      pool_s[n * WIN + win] = best;
      flag_s[n * WIN + win] = (uint8_t)(arg | ((best > 0.0f) ? 8 : 0));
    }
  }
  __syncthreads();

  // ---- phase 4: dropout + coalesced stores (4 contiguous flat elements = one Philox block)
  const uint64_t seed = a.state ? a.state->seed : 0;
  const uint64_t off = a.state ? a.state->rng_base + 2ull * (uint64_t)step : 0;
  const bool drop = TRAIN && !(a.state && (a.state->flags & STEP_FLAG_NO_DROPOUT));
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int qd = tid + 256 * i;           // 768 quads
    const int n = qd / 12, j4 = (qd - n * 12) * 4;
    const int flat = n * NPOOL + strip * WIN + j4;
    const float4 pv = *reinterpret_cast<const float4*>(pool_s + n * WIN + j4);
    const uint32_t fl = *reinterpret_cast<const uint32_t*>(flag_s + n * WIN + j4);
    float o[4] = {pv.x, pv.y, pv.z, pv.w};
    uint32_t mk = fl;
    if (TRAIN) {
      u32x4 rw = {0u, 0u, 0u, 0u};
      if (drop) rw = dropout_words(seed, off, ((uint64_t)b * NFLAT + flat) >> 2);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool keep = rw[k] < KEEP1_THR;
        o[k] = keep ? (drop ? o[k] * (1.0f / KEEP1) : o[k]) : 0.0f;
        if (keep) mk |= 4u << (8 * k);
      }
      *reinterpret_cast<uint32_t*>(a.pmask_out + (int64_t)b * NFLAT + flat) = mk;
    }
    uint2 st;
    st.x = pack2bf(o[0], o[1]);
    st.y = pack2bf(o[2], o[3]);
    *reinterpret_cast<uint2*>(a.p_out + (int64_t)b * NFLAT + flat) = st;
  }
}

void launch_trunk_fwd(const TrunkFwdArgs& a, int B, bool train, hipStream_t s) {
  dim3 grid(3, B), block(256);
  if (train)
    hipLaunchKernelGGL(trunk_fwd_kernel<true>, grid, block, 0, s, a);
  else
    hipLaunchKernelGGL(trunk_fwd_kernel<false>, grid, block, 0, s, a);
}

}  // namespace mnist
