// Conv trunk backward.
//
// Replaces the autograd backward of reference mnist_ddp.py:50-55 (dropout1, max_pool2d, relu, conv2,
// relu, conv1): max_pool2d_with_indices_backward, threshold_backward x2, convolution_backward x2.
//
//  * conv2_dgrad_kernel  (WG = image x strip of 7 conv1 rows): builds the un-pooled gradient dy
//    (zero except at each window's argmax) in a zero-padded NHWC LDS tile, runs the transposed
//    convolution as an MFMA implicit GEMM (M = pixels, N = 32 ci, K = 9 taps x 64 co), applies the
//    conv1 ReLU mask (conv1 recomputed bit-identically from the input, never stored), and folds
//    the conv1 weight/bias gradient (K = 9 tiny) into the epilogue as per-workgroup partials.
//  * conv2_wgrad_kernel  (G persistent WGs, each looping over half-images): dW2 = dy^T (x) im2col(a1),
//    contraction over pixels.  Both operands are pixel-major NHWC tiles in LDS; fragments come
//    from ds_read_b64_tr_b16 with per-lane row addresses, so the im2col gather is free.
//  * conv_grad_reduce_kernel: fixed-order (deterministic) sum of the partial slabs into the flat
//    fp32 gradient buffer, scaled by 1/world_size (DDP averaging).
#include "../include/device_utils.h"
#include "../include/kernels.h"

namespace mnist {

namespace {
constexpr int DG_ROWS = 7;                              // conv1-output rows per dgrad WG (4 strips)
constexpr int DG_TROWS = DG_ROWS + 2;                   // dy rows incl. halo (top 2)
constexpr int DG_TCOLS = H2 + 4;                        // 28 (2 zero columns each side)
constexpr int DYS_BYTES = DG_TROWS * DG_TCOLS * C2 * 2; // 32256
constexpr int W2DS_BYTES = 9 * C1 * C2 * 2;             // 36864
constexpr int XS2_BYTES = DG_TROWS * IMG * 4;           // 1008 -> pad 1024
constexpr int RED_BYTES = 4 * 32 * 10 * 4;              // 5120
constexpr int DG_LDS = DYS_BYTES + W2DS_BYTES + 1024 + RED_BYTES;

constexpr int WG_HALF_ROWS = 12;                        // dy rows per wgrad unit
constexpr int WDYS_BYTES = WG_HALF_ROWS * H2 * C2 * 2;  // 36864
constexpr int WA1S_BYTES = (WG_HALF_ROWS + 2) * H1 * C1 * 2;  // 23296
constexpr int WG_LDS = WDYS_BYTES + WA1S_BYTES;
constexpr int W2PART_STRIDE = 18432 + 64;
}  // namespace

int conv_wgrad_groups(int B) {
  const int units = 2 * B;
  int g = units < 128 ? units : 128;
  if (B >= 2048) g = 256;
  return g;
}

// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv2_dgrad_kernel(ConvBwdArgs a, int B) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[DG_LDS];
  uint16_t* dys = reinterpret_cast<uint16_t*>(smem);
  uint16_t* w2ds = reinterpret_cast<uint16_t*>(smem + DYS_BYTES);
  float* xs = reinterpret_cast<float*>(smem + DYS_BYTES + W2DS_BYTES);
  float* red = reinterpret_cast<float*>(smem + DYS_BYTES + W2DS_BYTES + 1024);

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int strip = blockIdx.x, b = blockIdx.y;
  const int r0 = strip * DG_ROWS;
  const int nrows = (strip == 3) ? (H1 - 3 * DG_ROWS) : DG_ROWS;   // 7,7,7,5
  const int npix = nrows * H1;
  const int step = a.state ? a.state->step : 0;

  // ---- phase 0: zero dy tile, stage w2d, gather input rows
  {
    uint4 z = {0u, 0u, 0u, 0u};
    for (int c = tid; c < DYS_BYTES / 16; c += 256) reinterpret_cast<uint4*>(dys)[c] = z;
    const uint4* src = reinterpret_cast<const uint4*>(a.w2d);
#pragma unroll
    for (int i = 0; i < 9; ++i) reinterpret_cast<uint4*>(w2ds)[tid + 256 * i] = src[tid + 256 * i];
    const int img = a.idx[(int64_t)step * a.idx_step_stride + b];
    const uint8_t* src8 = a.data_u8 + (int64_t)img * (IMG * IMG);
    for (int e = tid; e < DG_TROWS * IMG; e += 256) {
      const int row = r0 + e / IMG;
      xs[e] = (row < IMG) ? normalize_u8(src8[r0 * IMG + e]) : 0.0f;
    }
  }
  __syncthreads();
  // ---- phase 1: un-pool the gradient into the padded NHWC tile (rows r0-2 .. r0+6)
  {
    const int py0 = (r0 >= 2) ? (r0 - 2) >> 1 : 0;
    const int py1 = min(HP - 1, (r0 + DG_ROWS - 1) >> 1);
    const int per_c = (py1 - py0 + 1) * HP;
    const int total = per_c * C2;
    const uint16_t* gb = a.g + (int64_t)b * NFLAT;
    const uint8_t* mb = a.pmask + (int64_t)b * NFLAT;
    for (int e = tid; e < total; e += 256) {
      const int c = e / per_c, s = e - c * per_c;
      const int flat = c * NPOOL + py0 * HP + s;
      const uint16_t gv = gb[flat];
      if (gv == 0) continue;
      const int mk = mb[flat];
      const int py = py0 + s / HP, px = s % HP;
      const int y = 2 * py + ((mk >> 1) & 1), x = 2 * px + (mk & 1);
      const int ly = y - r0 + 2;
      if (ly >= 0 && ly < DG_TROWS) dys[(ly * DG_TCOLS + x + 2) * C2 + c] = gv;
    }
  }
  __syncthreads();

  // ---- phase 2: transposed conv on MFMA: M-tiles 3w..3w+2 (16 pixels), N = 2 tiles of 16 ci
  const int m = lane & 15, kg = lane >> 4;
  int qy[3], qx[3];
#pragma unroll
  for (int mt = 0; mt < 3; ++mt) {
    int q = 16 * (3 * wave + mt) + m;
    if (q >= npix) q = 0;
    qy[mt] = q / H1;
    qx[mt] = q - qy[mt] * H1;
  }
  floatx4 acc[3][2];
#pragma unroll
  for (int mt = 0; mt < 3; ++mt) acc[mt][0] = acc[mt][1] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 18; ++ks) {
    const int t = ks >> 1, co0 = 32 * (ks & 1);
    const int ky = t / 3, kx = t % 3;
    bf16x8 A[3], Bf[2];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
      A[mt] = ld16(dys + ((qy[mt] + 2 - ky) * DG_TCOLS + (qx[mt] + 2 - kx)) * C2 + co0 + 8 * kg);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) Bf[nt] = ld16(w2ds + (t * C1 + nt * 16 + m) * C2 + co0 + 8 * kg);
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma16x16x32(A[mt], Bf[nt], acc[mt][nt]);
  }

  // ---- phase 3: conv1 ReLU mask (recomputed) + conv1 weight/bias gradient partials
  float w[2][9], bias[2], sdw[2][9], sdb[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int ci = nt * 16 + m;
    bias[nt] = a.b1c[ci];
    sdb[nt] = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) { w[nt][t] = a.w1c[ci * 9 + t]; sdw[nt][t] = 0.f; }
  }
#pragma unroll
  for (int mt = 0; mt < 3; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = 16 * (3 * wave + mt) + 4 * kg + r;
      if (q < npix) {
        const int py = q / H1, px = q - py * H1;
        const float* xp = xs + py * IMG + px;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const float z = conv1_preact(xp, IMG, w[nt], bias[nt]);
          const float d = (z > 0.0f) ? acc[mt][nt][r] : 0.0f;
          sdb[nt] += d;
#pragma unroll
          for (int t = 0; t < 9; ++t) sdw[nt][t] = __builtin_fmaf(d, xp[(t / 3) * IMG + (t % 3)], sdw[nt][t]);
        }
      }
    }
  // lanes l, l^16, l^32, l^48 share a channel
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    sdb[nt] += __shfl_xor(sdb[nt], 16, 64);
    sdb[nt] += __shfl_xor(sdb[nt], 32, 64);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      sdw[nt][t] += __shfl_xor(sdw[nt][t], 16, 64);
      sdw[nt][t] += __shfl_xor(sdw[nt][t], 32, 64);
    }
  }
  if (kg == 0) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      float* dst = red + (wave * 32 + nt * 16 + m) * 10;
#pragma unroll
      for (int t = 0; t < 9; ++t) dst[t] = sdw[nt][t];
      dst[9] = sdb[nt];
    }
  }
  __syncthreads();
  for (int e = tid; e < 320; e += 256) {
    const float s = red[e] + red[e + 320] + red[e + 640] + red[e + 960];
    a.c1part[((int64_t)b * 4 + strip) * 320 + e] = s;
  }
}

// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv2_wgrad_kernel(ConvBwdArgs a, int B) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[WG_LDS];
  uint16_t* dys = reinterpret_cast<uint16_t*>(smem);                // [12][24][64]
  uint16_t* a1s = reinterpret_cast<uint16_t*>(smem + WDYS_BYTES);   // [14][26][32]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int gq = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int mt0 = 2 * (wave & 1), nt0 = 9 * (wave >> 1);
  const int G = gridDim.x;
  floatx4 acc[2][9];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;   // conv2 bias grad partial for channel tid>>2 (4 lanes per channel)
  const int bc = tid >> 2, bsub = tid & 3;

  for (int u = blockIdx.x; u < 2 * B; u += G) {
    const int b = u >> 1, h = u & 1;
    {
      uint4 z = {0u, 0u, 0u, 0u};
      for (int c = tid; c < WDYS_BYTES / 16; c += 256) reinterpret_cast<uint4*>(dys)[c] = z;
      const uint4* src = reinterpret_cast<const uint4*>(a.a1 + ((int64_t)b * H1 + WG_HALF_ROWS * h) * H1 * C1);
      for (int c = tid; c < WA1S_BYTES / 16; c += 256) reinterpret_cast<uint4*>(a1s)[c] = src[c];
    }
    __syncthreads();
    {
      const uint16_t* gb = a.g + (int64_t)b * NFLAT + bc * NPOOL + 6 * h * HP;
      const uint8_t* mb = a.pmask + (int64_t)b * NFLAT + bc * NPOOL + 6 * h * HP;
#pragma unroll 2
      for (int k = 0; k < 18; ++k) {
        const int s = bsub + 4 * k;           // 0..71 within the 6 pooled rows
        const uint16_t gv = gb[s];
        if (gv != 0) {
          bsum += bf2f(gv);
          const int mk = mb[s];
          const int py = s / HP, px = s - py * HP;
          const int y = 2 * py + ((mk >> 1) & 1), x = 2 * px + (mk & 1);
          dys[(y * H2 + x) * C2 + bc] = gv;
        }
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int ks = 0; ks < 9; ++ks) {
      const int plo = 32 * ks + 8 * gq + q, phi = plo + 4;
      const int ylo = plo / H2, xlo = plo - ylo * H2;
      const int yhi = phi / H2, xhi = phi - yhi * H2;
      bf16x8 A[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int cb = 16 * (mt0 + i) + 4 * pp;
        A[i] = tr_frag(dys + plo * C2 + cb, dys + phi * C2 + cb);
      }
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int nt = nt0 + j, t = nt >> 1, ci0 = 16 * (nt & 1) + 4 * pp;
        const int ky = t / 3, kx = t % 3;
        const bf16x8 Bf = tr_frag(a1s + ((ylo + ky) * H1 + xlo + kx) * C1 + ci0,
                                  a1s + ((yhi + ky) * H1 + xhi + kx) * C1 + ci0);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][j] = mfma16x16x32(A[i], Bf, acc[i][j]);
      }
    }
    __syncthreads();
  }
  float* out = a.w2part + (int64_t)blockIdx.x * W2PART_STRIDE;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int nt = nt0 + j, t = nt >> 1, ci = 16 * (nt & 1) + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = 16 * (mt0 + i) + 4 * gq + r;
        out[co * 288 + ci * 9 + t] = acc[i][j][r];
      }
    }
  bsum += __shfl_xor(bsum, 1, 64);
  bsum += __shfl_xor(bsum, 2, 64);
  if (bsub == 0) out[18432 + bc] = bsum;
}

// --------------------------------------------------------------------------------------------
// roles: [0, 72) conv2.weight columns, 72: conv2.bias, [73, 93): conv1 weight+bias (16 outputs each)
__global__ __launch_bounds__(256) void conv_grad_reduce_kernel(ConvBwdArgs a, int B) {
  __shared__ float red[256];
  const int tid = threadIdx.x, bid = blockIdx.x;
  const int G = a.wgrad_groups;
  const float sc = a.grad_scale;
  if (bid < 72) {
    const int e = bid * 256 + tid;
    float s = 0.f;
    for (int g0 = 0; g0 < G; ++g0) s += a.w2part[(int64_t)g0 * W2PART_STRIDE + e];
    a.grad[OFF_CONV2_W + e] = s * sc;
  } else if (bid == 72) {
    if (tid < 64) {
      float s = 0.f;
      for (int g0 = 0; g0 < G; ++g0) s += a.w2part[(int64_t)g0 * W2PART_STRIDE + 18432 + tid];
      a.grad[OFF_CONV2_B + tid] = s * sc;
    }
  } else {
    const int j = (bid - 73) * 16 + (tid & 15), sl = tid >> 4;
    const int nslab = 4 * B;
    float s = 0.f;
    for (int k = sl; k < nslab; k += 16) s += a.c1part[(int64_t)k * 320 + j];
    red[tid] = s;
    __syncthreads();
    if (tid < 16) {
      float t = 0.f;
      for (int k = 0; k < 16; ++k) t += red[k * 16 + tid];
      const int ci = j / 10, kk = j - ci * 10;
      if (kk < 9) a.grad[OFF_CONV1_W + ci * 9 + kk] = t * sc;
      else a.grad[OFF_CONV1_B + ci] = t * sc;
    }
  }
}

void launch_conv_bwd(const ConvBwdArgs& a, int B, hipStream_t s) {
  hipLaunchKernelGGL(conv2_dgrad_kernel, dim3(4, B), dim3(256), 0, s, a, B);
  hipLaunchKernelGGL(conv2_wgrad_kernel, dim3(a.wgrad_groups), dim3(256), 0, s, a, B);
}

void launch_conv_grad_reduce(const ConvBwdArgs& a, int B, hipStream_t s) {
  hipLaunchKernelGGL(conv_grad_reduce_kernel, dim3(93), dim3(256), 0, s, a, B);
}

}  // namespace mnist
