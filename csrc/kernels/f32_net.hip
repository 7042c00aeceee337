// fp32 training / eval step (--dtype fp32): the reference's own precision (mnist_ddp.py trains the
// Net in fp32) on gfx950's f32-input matrix cores instead of stock torch ops.
//
// Replaces, for the fp32 mode: reference mnist_ddp.py:49-61 (forward), :71-72 (nll_loss +
// backward) and :89-105 (test forward).  The bf16 engine (trunk_fwd.hip, fc_head.hip, conv_bwd.hip)
// stays the performance path; this one keeps every operand in fp32.
//
// Design:
//   * every GEMM-shaped op - conv2 forward (implicit im2col), fc1, fc1 weight / input gradients,
//     conv2 weight (implicit im2col, split-K) / input gradients (implicit transposed conv), conv1
//     weight gradient - is ONE LDS-tiled GEMM template on v_mfma_f32_16x16x4_f32 (exact f32: a
//     k-ordered fma chain, no xf32 on CDNA4) whose operand loaders and epilogue are small policy
//     structs: no im2col buffer, the gathers happen in the tile loads;
//   * elementwise / per-row work (conv1 + ReLU, ReLU + max-pool + dropout, the fc head with
//     log_softmax + NLL + their backward, bias sums) are VALU kernels;
//   * dropout draws the same Philox-4x32-10 bytes as the bf16 engine (device_utils.h), so both
//     engines drop the same units of the same step; every reduction runs in a fixed order
//     (split-K partial slabs summed by one kernel), so the step is bitwise repeatable.
// Layouts (fp32): a1 [B][26][26][32] (NHWC, ReLU applied; its storage is reused for the conv1
// pre-activation gradient), y2 / dy2 [B][24][24][64] (conv2 pre-activation / its gradient, shared
// storage), p [B][9216] torch flatten order, pm u8 [B][144][64] position-major (bits 0-1 argmax,
// 2 keep, 3 pooled > 0).
#include "../include/device_utils.h"
#include "../include/kernels.h"

#include <algorithm>
#include <stdexcept>

namespace mnist {

namespace {
constexpr int BK = 16;                 // split-K chunk granularity (the GEMM k-tile is 16 or 32)
constexpr int NPIX1 = H1 * H1;         // 676 conv1 output pixels
constexpr int NPIX2 = H2 * H2;         // 576 conv2 output pixels
constexpr int K2 = 9 * C1;             // 288 conv2 reduction length (tap, ci)
constexpr int WG_N = C2 * K2 + C2;     // conv2 weight + bias gradient slab (18496)

__device__ __forceinline__ const StepState* state_of(const F32Step& a) {
  return a.state ? a.state : &g_zero_state;
}

// row b of the current step: pre-gathered rows (idx == null) or the dataset through the index vector
__device__ __forceinline__ const uint8_t* image_row(const F32Step& a, int step, int b) {
  const int64_t row = (int64_t)step * a.idx_step_stride + b;
  const int64_t img = a.idx ? (int64_t)a.idx[row] : row;
  return a.data_u8 + img * (IMG * IMG);
}

// ---------------------------------------------------------------------------------------------
// GEMM template: C[M][N] = sum_k A(m, k) B(k, n) over k in [z*kc, min(K, (z+1)*kc)) (z = blockIdx.z).
// Workgroup tile BM x BN (4 waves, each 32 x 32 = 2 x 2 tiles of 16 x 16), k-tile 16 staged in LDS
// as [k][m] / [k][n] rows, so every MFMA operand read is 16 consecutive floats per 16-lane group.
// The policy P provides M, N, K, kc, put(m, n, v, z), prepare(), whether A / B are contiguous along
// k (A_KF / B_KF), and the operands as 16-B vectors along their contiguous axis:
//   a4(m, k) = A(m, k..k+3) when A_KF, else A(m..m+3, k);  b4(k, n) = B(k..k+3, n) when B_KF, else
//   B(k, n..n+3)
// so each gather (the implicit im2col / transposed-conv index math, its bounds test) serves 4
// elements: the scalar form spent more VALU issue on addressing than the MFMAs took (the conv GEMMs
// ran at 30-38 % of the f32 matrix peak).  Vector axes are 4-aligned (M, N, K multiples of 4 on
// them, split-K chunks multiples of 16); a policy whose vector crosses its bound zero-fills itself.
template <class P, class = void>
struct has_put4 { static constexpr bool value = false; };
template <class P>
struct has_put4<P, decltype(void(P::PUT4))> { static constexpr bool value = P::PUT4; };

// 4 waves in a WGM x (4 / WGM) grid, each owning a (BM / WGM) x (BN * WGM / 4) tile of TM x TN
// 16 x 16 MFMA blocks: wider per-wave tiles read fewer LDS operands per MFMA
template <int BM, int BN, int BK, int WGM, class P>
__global__ __launch_bounds__(256) void f32_gemm_kernel(P p) {
  RW_ENTRY();
  constexpr int WN = 4 / WGM, TM = BM / WGM / 16, TN = BN / WN / 16;
  static_assert(WGM * WN == 4 && TM >= 1 && TN >= 1 && TM * WGM * 16 == BM && TN * WN * 16 == BN, "wave tiling");
  constexpr int NA = BM * BK / 4, NB = BN * BK / 4;            // float4s per operand tile
  constexpr int EA = (NA + 255) / 256, EB = (NB + 255) / 256;
  __shared__ __attribute__((aligned(16))) float As[BK][BM + 4];
  __shared__ __attribute__((aligned(16))) float Bs[BK][BN + 4];
  p.prepare();
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int k_lo = blockIdx.z * p.kc;
  const int k_hi = min(p.K, k_lo + p.kc);
  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // register prefetch: the next k-tile's gathers are issued before this tile's MFMAs, so their
  // latency hides under the matrix work instead of sitting between the two barriers
  float4 ra[EA], rb[EB];
#define F32_GEMM_LOAD(K0)                                                                                    \
  _Pragma("unroll") for (int e = 0; e < EA; ++e) {                                                          \
    const int x = tid + 256 * e;                                                                            \
    const int m = P::A_KF ? x / (BK / 4) : (x % (BM / 4)) * 4, k = P::A_KF ? (x % (BK / 4)) * 4 : x / (BM / 4); \
    const int gm = m0 + m, gk = (K0) + k;                                                                   \
    ra[e] = (x < NA && gm < p.M && gk < k_hi) ? p.a4(gm, gk) : make_float4(0.f, 0.f, 0.f, 0.f);             \
  }                                                                                                         \
  _Pragma("unroll") for (int e = 0; e < EB; ++e) {                                                          \
    const int x = tid + 256 * e;                                                                            \
    const int n = P::B_KF ? x / (BK / 4) : (x % (BN / 4)) * 4, k = P::B_KF ? (x % (BK / 4)) * 4 : x / (BN / 4); \
    const int gn = n0 + n, gk = (K0) + k;                                                                   \
    rb[e] = (x < NB && gn < p.N && gk < k_hi) ? p.b4(gk, gn) : make_float4(0.f, 0.f, 0.f, 0.f);            \
  }
  if (k_lo < k_hi) { F32_GEMM_LOAD(k_lo) }
  for (int k0 = k_lo; k0 < k_hi; k0 += BK) {
    lds_barrier();                                // the previous k-tile's reads are done
#pragma unroll
    for (int e = 0; e < EA; ++e) {
      const int x = tid + 256 * e;
      if (x >= NA) continue;
      if (P::A_KF) {
        const int m = x / (BK / 4), k = (x % (BK / 4)) * 4;
        As[k][m] = ra[e].x; As[k + 1][m] = ra[e].y; As[k + 2][m] = ra[e].z; As[k + 3][m] = ra[e].w;
      } else {
        *reinterpret_cast<float4*>(&As[x / (BM / 4)][(x % (BM / 4)) * 4]) = ra[e];
      }
    }
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int x = tid + 256 * e;
      if (x >= NB) continue;
      if (P::B_KF) {
        const int n = x / (BK / 4), k = (x % (BK / 4)) * 4;
        Bs[k][n] = rb[e].x; Bs[k + 1][n] = rb[e].y; Bs[k + 2][n] = rb[e].z; Bs[k + 3][n] = rb[e].w;
      } else {
        *reinterpret_cast<float4*>(&Bs[x / (BN / 4)][(x % (BN / 4)) * 4]) = rb[e];
      }
    }
    lds_barrier();
    if (k0 + BK < k_hi) { F32_GEMM_LOAD(k0 + BK) }   // in flight under the MFMAs below
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      float av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = As[kk + (lane >> 4)][wm * (16 * TM) + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < TN; ++j) bv[j] = Bs[kk + (lane >> 4)][wn * (16 * TN) + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  }
  // C/D map of the 16 x 16 MFMA: column = lane & 15, row = 4 * (lane >> 4) + register
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int mb = m0 + wm * (16 * TM) + i * 16 + 4 * (lane >> 4);
      const int n = n0 + wn * (16 * TN) + j * 16 + (lane & 15);
      if constexpr (has_put4<P>::value) {       // the lane's 4 consecutive rows at once (M % 4 == 0)
        if (mb < p.M && n < p.N) p.put4(mb, n, acc[i][j], blockIdx.z);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (mb + r < p.M && n < p.N) p.put(mb + r, n, acc[i][j][r], blockIdx.z);
      }
    }
}

// k-tile: P::KT when the policy sets one (the thin fc GEMMs: fewer, fuller k-iterations), else 16
// (4 MFMA k-steps per barrier pair; 32 for every GEMM measured the same step time: 0.3367-0.3388 vs
// 0.3360-0.3367 ms)
template <class P, class = void>
struct kt_of { static constexpr int value = 16; };
template <class P>
struct kt_of<P, decltype(void(P::KT))> { static constexpr int value = P::KT; };

template <int BM, int BN, class P, int WGM = BM / 32>
void gemm(const P& p, int splits, hipStream_t s) {
  const dim3 grid((p.M + BM - 1) / BM, (p.N + BN - 1) / BN, splits);
  hipLaunchKernelGGL((f32_gemm_kernel<BM, BN, kt_of<P>::value, WGM, P>), grid, dim3(256), 0, s, p);
}

// ---- policies
// conv2 forward: y2[(b, oy, ox)][co] = b2[co] + sum_(tap, ci) a1[b][oy+ky][ox+kx][ci] w2[co][ci][tap]
struct PConv2Fwd {
  static constexpr bool A_KF = true, B_KF = false;
  int M, N, K, kc;
  const float* a1;
  const float* w2fwd;   // [tap][ci][co]
  const float* b2;
  float* y2;
  __device__ void prepare() {}
  __device__ float4 a4(int m, int k) const {
    const int b = m / NPIX2, pix = m - b * NPIX2, oy = pix / H2, ox = pix - oy * H2;
    const int tap = k >> 5, ci = k & 31, ky = tap / 3, kx = tap - 3 * ky;
    return *reinterpret_cast<const float4*>(a1 + (((int64_t)b * H1 + oy + ky) * H1 + ox + kx) * C1 + ci);
  }
  __device__ float4 b4(int k, int n) const { return *reinterpret_cast<const float4*>(w2fwd + k * C2 + n); }
  __device__ void put(int m, int n, float v, int) const { y2[(int64_t)m * C2 + n] = v + b2[n]; }
};

// fc1 forward, split-K partial sums: z1part[z][b][o] = sum_(i in split z) p[b][i] w1[o][i]
struct PFc1 {
  static constexpr bool A_KF = true, B_KF = true;
  static constexpr int KT = 32;
  int M, N, K, kc;
  const float* p;
  const float* w1;
  float* z1part;
  __device__ void prepare() {}
  __device__ float4 a4(int m, int k) const { return *reinterpret_cast<const float4*>(p + (int64_t)m * NFLAT + k); }
  __device__ float4 b4(int k, int n) const { return *reinterpret_cast<const float4*>(w1 + (int64_t)n * NFLAT + k); }
  __device__ void put(int m, int n, float v, int z) const { z1part[((int64_t)z * M + m) * NH + n] = v; }
};

// fc1 weight gradient: g[o][i] = sum_b dz1[b][o] p[b][i]
struct PFc1W {
  static constexpr bool A_KF = false, B_KF = false;
  static constexpr int KT = 32;
  int M, N, K, kc;
  const float* dz1;
  const float* p;
  float* g;
  __device__ void prepare() {}
  __device__ float4 a4(int m, int k) const { return *reinterpret_cast<const float4*>(dz1 + (int64_t)k * NH + m); }
  __device__ float4 b4(int k, int n) const { return *reinterpret_cast<const float4*>(p + (int64_t)k * NFLAT + n); }
  __device__ void put(int m, int n, float v, int) const { g[(int64_t)m * NFLAT + n] = v; }
};

// fc1 input gradient dp[b][j] = sum_o dz1[b][o] w1[o][j], through dropout-1 and the max-pool +
// ReLU backward in the epilogue: the 2 x 2 window's four conv2-output gradients (one non-zero).
// Computed TRANSPOSED - rows = fc1 inputs j in position-major order (j' = pos * 64 + c, A operand =
// the w1p copy), columns = images - so each lane's four MFMA accumulators are 4 consecutive channels
// of one pooled position of one image: the four dense NHWC dy2 stores are 16-B vectors (put4).
// (In torch order the lanes were 2 pixels = 512 B apart: 29.5 MB of scattered 4-byte stores took
// 79.5 us of a 555 us step at B = 200; position-major 4-byte stores 22-24 us.  A compact dy2 decoded
// inside the conv2 GEMM loads instead cost those GEMMs more VALU than the stores it saved: 27 us.)
struct PFc1X {
  static constexpr bool A_KF = false, B_KF = true, PUT4 = true;
  static constexpr int KT = 32;
  int M, N, K, kc;      // M = 9216 (j'), N = B, K = 128
  const float* dz1;
  const float* w1p;
  const uint8_t* pm;
  float* dy2;
  const StepState* st;
  float dscale;
  __device__ void prepare() {
    const StepState* s = st ? st : &g_zero_state;
    dscale = (s->flags & STEP_FLAG_NO_DROPOUT) ? 1.0f : (1.0f / KEEP1);
  }
  __device__ float4 a4(int m, int k) const { return *reinterpret_cast<const float4*>(w1p + (int64_t)k * NFLAT + m); }
  __device__ float4 b4(int k, int n) const { return *reinterpret_cast<const float4*>(dz1 + (int64_t)n * NH + k); }
  __device__ void put4(int m, int n, const floatx4& v, int) const {
    const int c = m & (C2 - 1), pos = m >> 6, py = pos / HP, px = pos - py * HP;
    const uint32_t f4 = *reinterpret_cast<const uint32_t*>(pm + (int64_t)n * NFLAT + m);   // pm[n][pos][c..c+3]
    uint32_t fl[4];
    float g[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      fl[j] = (f4 >> (8 * j)) & 0xffu;
      g[j] = ((fl[j] & 12u) == 12u) ? v[j] * dscale : 0.0f;       // kept by dropout, ReLU alive
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int y = 2 * py + (q >> 1), x = 2 * px + (q & 1);
      *reinterpret_cast<float4*>(dy2 + (((int64_t)n * H2 + y) * H2 + x) * C2 + c) =
          make_float4((int)(fl[0] & 3u) == q ? g[0] : 0.0f, (int)(fl[1] & 3u) == q ? g[1] : 0.0f,
                      (int)(fl[2] & 3u) == q ? g[2] : 0.0f, (int)(fl[3] & 3u) == q ? g[3] : 0.0f);
    }
  }
};

// conv2 weight + bias gradient, split-K over the B*576 output pixels:
// part[z][co][n] = sum_m dy2[m][co] im2col(a1)[m][n] (n < 288), sum_m dy2[m][co] (n = 288)
struct PConv2W {
  static constexpr int KT = 32;   // 600 steps 281.3 -> 274.4-274.9 us (the input-gradient / forward GEMMs: no gain / slower)
  static constexpr bool A_KF = false, B_KF = false;
  int M, N, K, kc;
  const float* dy2;
  const float* a1;
  float* part;
  __device__ void prepare() {}
  __device__ float4 a4(int m, int k) const { return *reinterpret_cast<const float4*>(dy2 + (int64_t)k * C2 + m); }
  __device__ float4 b4(int k, int n) const {
    if (n >= K2) return make_float4(1.0f, 0.0f, 0.0f, 0.0f);      // the bias column (n = 288) + padding
    const int b = k / NPIX2, pix = k - b * NPIX2, oy = pix / H2, ox = pix - oy * H2;
    const int tap = n >> 5, ci = n & 31, ky = tap / 3, kx = tap - 3 * ky;
    return *reinterpret_cast<const float4*>(a1 + (((int64_t)b * H1 + oy + ky) * H1 + ox + kx) * C1 + ci);
  }
  __device__ void put(int m, int n, float v, int z) const { part[((int64_t)z * C2 + m) * (K2 + 1) + n] = v; }
};

// conv2 input gradient (transposed conv) times the conv1 ReLU mask, in place over a1:
// da1[(b, iy, ix)][ci] = [a1 > 0] sum_(tap, co) dy2[b][iy-ky][ix-kx][co] w2[co][ci][tap]
struct PConv2X {
  static constexpr bool A_KF = true, B_KF = false;
  int M, N, K, kc;
  const float* dy2;
  const float* w2bwd;   // [tap][co][ci]
  const float* a1;      // the ReLU mask operand
  float* dx1;
  __device__ void prepare() {}
  __device__ float4 a4(int m, int k) const {
    const int b = m / NPIX1, pix = m - b * NPIX1, iy = pix / H1, ix = pix - iy * H1;
    const int tap = k >> 6, co = k & 63, ky = tap / 3, kx = tap - 3 * ky;
    const int oy = iy - ky, ox = ix - kx;
    return (oy >= 0 && oy < H2 && ox >= 0 && ox < H2)
               ? *reinterpret_cast<const float4*>(dy2 + (((int64_t)b * H2 + oy) * H2 + ox) * C2 + co)
               : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __device__ float4 b4(int k, int n) const { return *reinterpret_cast<const float4*>(w2bwd + k * C1 + n); }
  __device__ void put(int m, int n, float v, int) const {
    const int64_t e = (int64_t)m * C1 + n;
    dx1[e] = (a1[e] > 0.0f) ? v : 0.0f;
  }
};

// ---------------------------------------------------------------------------------------------
// conv2 weight in the two GEMM B layouts: w2fwd[tap][ci][co], w2bwd[tap][co][ci] ...
// ... and fc1.weight position-major for the fc1 input gradient: w1p[o][pos][c] = w1[o][c * 144 + pos]
// (threads walk the destination: coalesced 16-B stores, gathered 4-B loads from L2)
__global__ __launch_bounds__(256) void f32_prep_kernel(F32Step a, int train) {
  RW_ENTRY();
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t < C2 * K2) {
    const int co = t / K2, r = t - co * K2, ci = r / 9, tap = r - 9 * ci;   // torch [co][ci][ky][kx]
    const float w = a.param[OFF_CONV2_W + t];
    a.w2fwd[(tap * C1 + ci) * C2 + co] = w;
    a.w2bwd[(tap * C2 + co) * C1 + ci] = w;
  }
  const int u = t - ((C2 * K2 + 255) / 256) * 256;              // the w1p blocks follow
  if (!train || u < 0 || u >= NH * NFLAT / 4) return;
  const int o = u / (NFLAT / 4), j = 4 * (u - o * (NFLAT / 4)), pos = j >> 6, c = j & 63;
  const float* src = a.param + OFF_FC1_W + (int64_t)o * NFLAT + pos;
  *reinterpret_cast<float4*>(a.w1p + (int64_t)o * NFLAT + j) =
      make_float4(src[c * NPOOL], src[(c + 1) * NPOOL], src[(c + 2) * NPOOL], src[(c + 3) * NPOOL]);
}

// conv1 + bias + ReLU: workgroup = 32 output pixels of one image, thread = 4 channels of one pixel
// (the bf16 engine's fma order).  The image is normalised once into LDS (784 LUT loads per workgroup
// instead of 9 per thread), and 8 consecutive lanes cover a pixel's 32 channels, so each float4 store
// instruction writes 8 whole pixels (1 KB contiguous)
constexpr int C1_PIX_PER_WG = 32, C1_WG_PER_IMG = (NPIX1 + C1_PIX_PER_WG - 1) / C1_PIX_PER_WG;   // 22
__global__ __launch_bounds__(256) void f32_conv1_kernel(F32Step a, int B) {
  RW_ENTRY();
  __shared__ float img[IMG * IMG];
  const int b = blockIdx.x / C1_WG_PER_IMG, part = blockIdx.x - b * C1_WG_PER_IMG;
  const uint8_t* src = image_row(a, state_of(a)->step, b);
  for (int i = threadIdx.x; i < IMG * IMG; i += 256) img[i] = normalize_u8(src[i]);   // (LUT: the same bits)
  __syncthreads();
  const int pix = part * C1_PIX_PER_WG + (threadIdx.x >> 3), c4 = threadIdx.x & 7;
  if (pix >= NPIX1) return;
  const int y = pix / H1, x = pix - y * H1;
  float xv[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) xv[k] = img[(y + k / 3) * IMG + x + k % 3];
  const float* w = a.param + OFF_CONV1_W;
  const float* bias = a.param + OFF_CONV1_B;
  float o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = fmaxf(conv1_preact(xv, 3, w + (4 * c4 + j) * 9, bias[4 * c4 + j]), 0.0f);
  reinterpret_cast<float4*>(a.a1 + ((int64_t)b * NPIX1 + pix) * C1)[c4] = make_float4(o[0], o[1], o[2], o[3]);
}

// ReLU + 2x2 max-pool (first max wins, as torch) + dropout(0.25): one thread = 16 consecutive
// flat elements of one channel = one Philox block (the trunk's rule: counter rng_base + 2 step)
template <bool TRAIN>
__global__ __launch_bounds__(256) void f32_pool_kernel(F32Step a, int B) {
  RW_ENTRY();
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)B * C2 * (NPOOL / 16)) return;
  // lanes = channels: each y2 load instruction reads one pixel's 64 channels (256 contiguous bytes;
  // with lanes walking positions of one channel every load touched 64 lines for 4 bytes each)
  const int b = (int)(t / (C2 * (NPOOL / 16))), u = (int)(t - (int64_t)b * (C2 * (NPOOL / 16)));
  const int c = u & (C2 - 1), j = u >> 6;
  const int flat0 = c * NPOOL + 16 * j;
  const StepState* st = state_of(a);
  const bool drop = TRAIN && !(st->flags & STEP_FLAG_NO_DROPOUT);
  u32x4 rw = {0u, 0u, 0u, 0u};
  if (drop) rw = dropout_block(st->seed, st->rng_base + 2ull * (uint64_t)st->step, ((uint64_t)b * NFLAT + flat0) >> 4);
  const float* y2 = a.y2 + (int64_t)b * NPIX2 * C2 + c;
  float out[16];
  uint32_t fl[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int pos = 16 * j + q, py = pos / HP, px = pos - py * HP;
    float best = 0.0f;
    int arg = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = fmaxf(y2[((2 * py + (r >> 1)) * H2 + 2 * px + (r & 1)) * C2], 0.0f);
      if (r == 0 || v > best) { best = v; arg = r; }
    }
    bool keep = true;
    if (TRAIN) keep = dropout_byte(rw, q) < KEEP1_THR8;
    out[q] = keep ? (drop ? best * (1.0f / KEEP1) : best) : 0.0f;
    fl[q >> 2] |= (uint32_t)(arg | (keep ? 4 : 0) | (best > 0.0f ? 8 : 0)) << (8 * (q & 3));
  }
  float4* dst = reinterpret_cast<float4*>(a.p + (int64_t)b * NFLAT + flat0);
#pragma unroll
  for (int q = 0; q < 4; ++q) dst[q] = make_float4(out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]);
  // flags position-major (pm[b][pos][c]: each byte store instruction writes 64 consecutive channels),
  // the layout the fc1 input-gradient epilogue reads 4 channels at a time
  if (TRAIN) {
    uint8_t* pmb = a.pm + (int64_t)b * NFLAT + (16 * j) * C2 + c;
#pragma unroll
    for (int q = 0; q < 16; ++q) pmb[q * C2] = (uint8_t)(fl[q >> 2] >> (8 * (q & 3)));
  }
}

__device__ __forceinline__ void log_softmax10_f32(const float* x, float* lp) {
  float mx = x[0];
#pragma unroll
  for (int c = 1; c < NCLS; ++c) mx = fmaxf(mx, x[c]);
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < NCLS; ++c) se += expf(x[c] - mx);
  const float lse = logf(se);
#pragma unroll
  for (int c = 0; c < NCLS; ++c) lp[c] = (x[c] - mx) - lse;
}

// fc1 bias + ReLU + dropout(0.5) + fc2 + log_softmax + NLL (+ backward to dz1): one wave = one row.
// TRAIN writes h, dz1, dl = d loss / d logits (scaled by inv_batch = 1/(B*world)) and the row's
// loss; eval writes the row's summed-NLL term and whether argmax (first max) == label.
template <bool TRAIN>
__global__ __launch_bounds__(256) void f32_head_kernel(F32Step a, int B, int S) {
  RW_ENTRY();
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= B) return;
  const StepState* st = state_of(a);
  const int step = st->step;
  const bool no_drop = !TRAIN || (st->flags & STEP_FLAG_NO_DROPOUT);
  const uint64_t off = st->rng_base + 2ull * (uint64_t)step + 1ull;
  const int64_t row = (int64_t)step * a.idx_step_stride + b;
  const int y = a.labels[a.idx ? (int64_t)a.idx[row] : row];
  const float* P = a.param;
  float z[2], h[2];
  bool keep[2];
  float zs[2] = {0.f, 0.f};                           // split-K partials in fixed order, 24 loads in flight
  for (int c0 = 0; c0 < S; c0 += 12) {
    float v[12][2];
#pragma unroll
    for (int k = 0; k < 12; ++k)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        v[k][j] = c0 + k < S ? a.z1part[((int64_t)(c0 + k) * B + b) * NH + lane + 64 * j] : 0.0f;
#pragma unroll
    for (int k = 0; k < 12; ++k)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (c0 + k < S) zs[j] += v[k][j];
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int o = lane + 64 * j;
    z[j] = P[OFF_FC1_B + o] + zs[j];
    float hv = fmaxf(z[j], 0.0f);
    keep[j] = true;
    if (!no_drop) {
      const u32x4 w = dropout_block(st->seed, off, ((uint64_t)b * NH + o) >> 4);
      keep[j] = dropout_byte(w, o & 15) < KEEP2_THR8;
      hv = keep[j] ? hv * (1.0f / KEEP2) : 0.0f;
    }
    h[j] = hv;
  }
  float logit[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c)
    logit[c] = wave_sum(h[0] * P[OFF_FC2_W + c * NH + lane] + h[1] * P[OFF_FC2_W + c * NH + lane + 64]) +
               P[OFF_FC2_B + c];
  float lp[NCLS];
  log_softmax10_f32(logit, lp);
  if (!TRAIN) {
    if (lane == 0) {
      int arg = 0;
#pragma unroll
      for (int c = 1; c < NCLS; ++c) arg = lp[c] > lp[arg] ? c : arg;
      a.loss_rows[b] = -lp[y];
      a.correct[b] = arg == y ? 1 : 0;
    }
    return;
  }
  float dl[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) {                    // nll(mean) + log_softmax backward
    const float go = (c == y) ? -a.inv_batch : 0.0f;
    dl[c] = go - expf(lp[c]) * (-a.inv_batch);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int o = lane + 64 * j;
    float dh = 0.f;
#pragma unroll
    for (int c = 0; c < NCLS; ++c) dh = __builtin_fmaf(dl[c], P[OFF_FC2_W + c * NH + o], dh);
    a.dz1[(int64_t)b * NH + o] = (keep[j] && z[j] > 0.0f) ? (no_drop ? dh : dh * (1.0f / KEEP2)) : 0.0f;
    a.h[(int64_t)b * NH + o] = h[j];
  }
  if (lane < 16) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < NCLS; ++c) v = (lane == c) ? dl[c] : v;
    a.dl[(int64_t)b * 16 + lane] = v;
  }
  if (lane == 0) a.loss_rows[b] = -lp[y];
}

// fixed-order workgroup sum of 256 per-thread values (wave sums, then waves 0..3)
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return ((red[0] + red[1]) + red[2]) + red[3];
}

// fc2 weight / bias, fc1 bias gradients and the step's mean loss: workgroup o = hidden unit o
__global__ __launch_bounds__(256) void f32_fc_small_kernel(F32Step a, int B) {
  RW_ENTRY();
  __shared__ float red[4];
  const int o = blockIdx.x;
  float acc[NCLS + 1];
#pragma unroll
  for (int c = 0; c <= NCLS; ++c) acc[c] = 0.f;
  for (int b = threadIdx.x; b < B; b += 256) {
    const float hv = a.h[(int64_t)b * NH + o];
#pragma unroll
    for (int c = 0; c < NCLS; ++c) acc[c] = __builtin_fmaf(a.dl[(int64_t)b * 16 + c], hv, acc[c]);
    acc[NCLS] += a.dz1[(int64_t)b * NH + o];
  }
#pragma unroll
  for (int c = 0; c <= NCLS; ++c) {
    const float s = block_sum(acc[c], red);
    if (threadIdx.x == 0) a.grad[c < NCLS ? OFF_FC2_W + c * NH + o : OFF_FC1_B + o] = s;
  }
  if (o != 0) return;
  float d2[NCLS + 1];
#pragma unroll
  for (int c = 0; c <= NCLS; ++c) d2[c] = 0.f;
  for (int b = threadIdx.x; b < B; b += 256) {
#pragma unroll
    for (int c = 0; c < NCLS; ++c) d2[c] += a.dl[(int64_t)b * 16 + c];
    d2[NCLS] += a.loss_rows[b];
  }
#pragma unroll
  for (int c = 0; c <= NCLS; ++c) {
    const float s = block_sum(d2[c], red);
    if (threadIdx.x == 0) {
      if (c < NCLS) a.grad[OFF_FC2_B + c] = s;
      else if (a.loss_log) a.loss_log[state_of(a)->step] = s / (float)B;
    }
  }
}

// conv1 weight + bias gradient (M = 32 channels, N = 9 taps + bias, K = B*676 pixels: far too thin
// for the GEMM tile, whose 64 x 64 MFMA tiles were 92 % padding): F32_C1W_BLOCKS workgroups, g sums
// pixels [g*P/G, (g+1)*P/G) on the VALU.  Each image the range touches is normalised once into LDS
// (the 784 inputs through the constant LUT: bitwise the fp32 divisions), then thread = (pixel lane
// 0..7, channel) takes a coalesced 128-B da1 row per pixel and its 3x3 patch as LDS broadcast reads,
// 4 pixels' loads in flight; the 8 pixel lanes are added in fixed order through LDS:
// part[g][c][0..9].  (One thread per channel doing its own 64-bit index math and 9 IEEE-division
// normalisations per pixel: 40 us at B = 200.)
__global__ __launch_bounds__(256) void f32_conv1w_kernel(F32Step a, int B, int G) {
  RW_ENTRY();
  __shared__ float red[8][C1 * 10];
  __shared__ float img[IMG * IMG];
  const int g = blockIdx.x, tid = threadIdx.x, c = tid & 31, pl = tid >> 5;
  const int P = B * NPIX1;                                       // < 2^31 for any batch the engine takes
  const int lo = (int)((int64_t)P * g / G), hi = (int)((int64_t)P * (g + 1) / G);
  const int step = state_of(a)->step;
  float acc[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) acc[j] = 0.f;
  for (int b = lo / NPIX1; b * NPIX1 < hi; ++b) {               // workgroup-uniform
    const uint8_t* src = image_row(a, step, b);
    __syncthreads();                                             // the previous image's reads are done
    for (int i = tid; i < IMG * IMG; i += 256) img[i] = normalize_u8(src[i]);
    __syncthreads();
    const int p0 = max(lo, b * NPIX1), p1 = min(hi, (b + 1) * NPIX1);
    constexpr int U = 4;
    for (int m0 = p0 + pl; m0 < p1; m0 += 8 * U) {
      float d[U];
      int off[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int m = m0 + 8 * u;
        const bool ok = m < p1;
        const int pix = (ok ? m : p0) - b * NPIX1, iy = pix / H1, ix = pix - iy * H1;
        off[u] = iy * IMG + ix;
        d[u] = ok ? a.dx1[(int64_t)(ok ? m : p0) * C1 + c] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int k = 0; k < 9; ++k) acc[k] = __builtin_fmaf(d[u], img[off[u] + (k / 3) * IMG + k % 3], acc[k]);
        acc[9] += d[u];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 10; ++j) red[pl][c * 10 + j] = acc[j];
  __syncthreads();
  for (int e = tid; e < C1 * 10; e += 256) {
    float s = red[0][e];
#pragma unroll
    for (int q = 1; q < 8; ++q) s += red[q][e];
    a.c1part[(int64_t)g * C1 * 10 + e] = s;
  }
}

// split-K slabs -> the flat gradient in torch layouts (fixed order).
//   blocks [0, RED2_BLOCKS): conv2 weight + bias, 64 output columns x 4 slab phases per workgroup:
//     thread (column, q) sums slabs z = q, q+4, .. (8 loads in flight), the 4 phases added in order
//     through LDS (was one thread per output walking all ~128 slabs: 31 us);
//   the rest: conv1 weight + bias (F32_C1W_BLOCKS slabs), 4 outputs x 64 slab phases per workgroup,
//     a fixed-order LDS tree over the 64 phases.
constexpr int RED2_BLOCKS = (WG_N + 63) / 64;
constexpr int RED1_BLOCKS = C1 * 10 / 4;
__global__ __launch_bounds__(256) void f32_conv_reduce_kernel(F32Step a, int s2, int s1) {
  RW_ENTRY();
  __shared__ float red[256];
  const int tid = threadIdx.x;
  if (blockIdx.x < RED2_BLOCKS) {
    const int col = tid & 63, q = tid >> 6;
    const int t = blockIdx.x * 64 + col;
    const bool live = t < WG_N;
    const int co = live ? t / (K2 + 1) : 0, n = live ? t - co * (K2 + 1) : 0;
    const float* src = a.c2part + (int64_t)co * (K2 + 1) + n;
    float s = 0.f;
    for (int z0 = q; z0 < s2; z0 += 32) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int z = z0 + 4 * k;
        v[k] = z < s2 ? src[(int64_t)z * (C2 * (K2 + 1))] : 0.0f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[k];
    }
    red[tid] = s;
    __syncthreads();
    if (q != 0 || !live) return;
    s = ((red[col] + red[64 + col]) + red[128 + col]) + red[192 + col];
    if (n < K2) a.grad[OFF_CONV2_W + co * K2 + (n & 31) * 9 + (n >> 5)] = s;
    else a.grad[OFF_CONV2_B + co] = s;
    return;
  }
  const int o = (blockIdx.x - RED2_BLOCKS) * 4 + (tid & 3), q = tid >> 2;   // output, phase 0..63
  const float* src = a.c1part + o;
  float s = 0.f;
  for (int z0 = q; z0 < s1; z0 += 64 * 8) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int z = z0 + 64 * k;
      v[k] = z < s1 ? src[(int64_t)z * (C1 * 10)] : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
  }
  red[tid] = s;
  __syncthreads();
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {                 // fixed-order tree over the 64 phases
    if (q < w) red[tid] = red[tid] + red[tid + 4 * w];
    __syncthreads();
  }
  if (q == 0) {
    const int c = o / 10, j = o - c * 10;
    if (j < 9) a.grad[OFF_CONV1_W + c * 9 + j] = red[tid];
    else a.grad[OFF_CONV1_B + c] = red[tid];
  }
}

inline int kchunk(int64_t K, int max_splits) {
  const int64_t per = (K + max_splits - 1) / max_splits;
  return (int)((per + BK - 1) / BK * BK);
}
inline int nsplit(int64_t K, int kc) { return (int)((K + kc - 1) / kc); }
inline unsigned blocks(int64_t n) { return (unsigned)((n + 255) / 256); }
}  // namespace

int f32_fc1_splits(int B) { return B <= 1024 ? 36 : 9; }
int f32_conv2w_splits(int B) { return nsplit((int64_t)B * NPIX2, kchunk((int64_t)B * NPIX2, F32_MAX_SPLITS)); }
int f32_conv1w_splits(int B) { return F32_C1W_BLOCKS; }

void launch_f32_forward(const F32Step& a, int B, bool train, hipStream_t s) {
  if (B < 1) throw std::runtime_error("f32 forward: empty batch");
  // (training: + the position-major fc1 weight copy for the backward)
  hipLaunchKernelGGL(f32_prep_kernel, dim3(blocks(C2 * K2) + (train ? blocks(NH * NFLAT / 4) : 0)), dim3(256), 0, s,
                     a, train ? 1 : 0);
  hipLaunchKernelGGL(f32_conv1_kernel, dim3(B * C1_WG_PER_IMG), dim3(256), 0, s, a, B);
  gemm<64, 64>(PConv2Fwd{B * NPIX2, C2, K2, K2, a.a1, a.w2fwd, a.param + OFF_CONV2_B, a.y2}, 1, s);
  if (train)
    hipLaunchKernelGGL(f32_pool_kernel<true>, dim3(blocks((int64_t)B * C2 * 9)), dim3(256), 0, s, a, B);
  else
    hipLaunchKernelGGL(f32_pool_kernel<false>, dim3(blocks((int64_t)B * C2 * 9)), dim3(256), 0, s, a, B);
  const int s1 = f32_fc1_splits(B);
  gemm<64, 64>(PFc1{B, NH, NFLAT, NFLAT / s1, a.p, a.param + OFF_FC1_W, a.z1part}, s1, s);
  if (train)
    hipLaunchKernelGGL(f32_head_kernel<true>, dim3((B + 3) / 4), dim3(256), 0, s, a, B, s1);
  else
    hipLaunchKernelGGL(f32_head_kernel<false>, dim3((B + 3) / 4), dim3(256), 0, s, a, B, s1);
}

// fc gradients (fc2 weight / bias, fc1 bias, fc1 weight): after these the fc update may start
void launch_f32_fc_small(const F32Step& a, int B, hipStream_t s) {
  hipLaunchKernelGGL(f32_fc_small_kernel, dim3(NH), dim3(256), 0, s, a, B);
}
void launch_f32_fc1w(const F32Step& a, int B, hipStream_t s) {
  gemm<64, 64>(PFc1W{NH, NFLAT, B, (B + BK - 1) / BK * BK, a.dz1, a.p, a.grad + OFF_FC1_W}, 1, s);
}
void launch_f32_backward_fc(const F32Step& a, int B, hipStream_t s) {
  launch_f32_fc_small(a, B, s);
  launch_f32_fc1w(a, B, s);
}

// the rest: fc1 input gradient (reads the w1p copy, not the fc1 parameters the update rewrites),
// conv2 weight / input gradients, conv1 weight gradient, slab reduce
void launch_f32_fc1x(const F32Step& a, int B, hipStream_t s) {
  gemm<64, 64>(PFc1X{NFLAT, B, NH, NH, a.dz1, a.w1p, a.pm, a.y2, a.state, 1.0f}, 1, s);
}
namespace {
int conv2w_kc(int B) { return kchunk((int64_t)B * NPIX2, F32_MAX_SPLITS); }
}  // namespace
void launch_f32_conv2w(const F32Step& a, int B, hipStream_t s) {
  gemm<64, 64>(PConv2W{C2, K2 + 1, B * NPIX2, conv2w_kc(B), a.y2, a.a1, a.c2part}, f32_conv2w_splits(B), s);
}
void launch_f32_conv2x_conv1w(const F32Step& a, int B, hipStream_t s) {
  gemm<128, 32>(PConv2X{B * NPIX1, C1, 9 * C2, 9 * C2, a.y2, a.w2bwd, a.a1, a.dx1}, 1, s);
  const int s1 = f32_conv1w_splits(B);
  hipLaunchKernelGGL(f32_conv1w_kernel, dim3(s1), dim3(256), 0, s, a, B, s1);
}
void launch_f32_conv_reduce(const F32Step& a, int B, hipStream_t s) {
  hipLaunchKernelGGL(f32_conv_reduce_kernel, dim3(RED2_BLOCKS + RED1_BLOCKS), dim3(256), 0, s, a, f32_conv2w_splits(B),
                     f32_conv1w_splits(B));
}
void launch_f32_backward_conv(const F32Step& a, int B, hipStream_t s) {
  launch_f32_fc1x(a, B, s);
  launch_f32_conv2w(a, B, s);
  launch_f32_conv2x_conv1w(a, B, s);
  launch_f32_conv_reduce(a, B, s);
}

void launch_f32_backward(const F32Step& a, int B, hipStream_t s) {
  launch_f32_backward_fc(a, B, s);
  launch_f32_backward_conv(a, B, s);
}

// load this translation unit's gfx950 code object now (startup prewarm thread) instead of at its
// first launch inside the timed run
void preload_f32() {
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&f32_prep_kernel));
}

}  // namespace mnist
