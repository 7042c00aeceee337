// Conv trunk backward.
//
// Replaces the autograd backward of reference mnist_ddp.py:50-55 (dropout1, max_pool2d, relu, conv2,
// relu, conv1): max_pool2d_with_indices_backward, threshold_backward x2, convolution_backward x2.
//
//  * conv2_dgrad_kernel  (WG = image x strip of 7 conv1 rows): stages the dense un-pooled gradient dy
//    (written by fc_bwd) into a zero-padded NHWC LDS tile with 16-B copies, runs the transposed
//    convolution as an MFMA implicit GEMM (M = pixels, N = 32 ci, K = 9 taps x 64 co), applies the
//    conv1 ReLU mask (stored bf16 a1 > 0, prefetched under the MFMA loop), and folds
//    the conv1 weight/bias gradient into the epilogue as a second 16x16x16 MFMA fed straight
//    from the masked accumulators (per-workgroup partials).
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

// 16-byte-chunk XOR swizzles against ds_read_b128 / ds_read_b64_tr_b16 bank conflicts (rows of
// 128 B = 8 chunks, or 64 B = 4 chunks).  Chosen with tools/lds_banks.py (gfx950 lane-group model).
__device__ __forceinline__ int swz8(int row) { return row & 7; }
__device__ __forceinline__ int swz_dy(int pix) { return (pix ^ (pix >> 1)) & 7; }
}  // namespace

// As few groups (= partial slabs for the reduce) as keep the per-group unit count minimal:
// B=200 -> 400 units -> 200 groups x 2 units (not 256 groups doing 1 or 2).
int conv_wgrad_groups(int B) {
  const int units = 2 * B;
  const int per = (units + 255) / 256;
  return (units + per - 1) / per;
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

  // ---- phase 0: stage the padded dy tile (rows r0-2..r0+6, cols -2..25), w2d and the input rows.
  // All global loads are independent 16-B loads issued before any LDS store.
  {
    constexpr int NCH = DG_TROWS * DG_TCOLS * 8;   // 2016 16-B chunks
    uint4 v[8];
    const uint4 z = {0u, 0u, 0u, 0u};
    const uint16_t* dyb = a.dy + (int64_t)b * H2 * H2 * C2;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = tid + 256 * k;
      const int ly = c / (DG_TCOLS * 8), rem = c - ly * (DG_TCOLS * 8), col = rem >> 3, c8 = rem & 7;
      const int y = r0 - 2 + ly, x = col - 2;
      v[k] = z;
      if (c < NCH && y >= 0 && y < H2 && x >= 0 && x < H2)
        v[k] = *reinterpret_cast<const uint4*>(dyb + (y * H2 + x) * C2 + c8 * 8);
    }
    uint4 w[9];
    const uint4* src = reinterpret_cast<const uint4*>(a.w2d);
#pragma unroll
    for (int i = 0; i < 9; ++i) w[i] = src[tid + 256 * i];
    if (a.xin) {
      const float* srcf = a.xin + (int64_t)b * (IMG * IMG);
      for (int e = tid; e < DG_TROWS * IMG; e += 256) {
        const int row = r0 + e / IMG;
        xs[e] = (row < IMG) ? srcf[r0 * IMG + e] : 0.0f;
      }
    } else {
      const int img = a.idx[(int64_t)step * a.idx_step_stride + b];
      const uint8_t* src8 = a.data_u8 + (int64_t)img * (IMG * IMG);
      for (int e = tid; e < DG_TROWS * IMG; e += 256) {
        const int row = r0 + e / IMG;
        xs[e] = (row < IMG) ? normalize_u8(src8[r0 * IMG + e]) : 0.0f;
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = tid + 256 * k;
      if (c < NCH) {
        const int row = c >> 3, c8 = c & 7;
        reinterpret_cast<uint4*>(dys)[row * 8 + (c8 ^ swz8(row))] = v[k];
      }
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int c = tid + 256 * i, row = c >> 3, c8 = c & 7;
      reinterpret_cast<uint4*>(w2ds)[row * 8 + (c8 ^ swz8(row))] = w[i];
    }
  }
  __syncthreads();

  // ---- phase 2: transposed conv on MFMA: M-tiles 3w..3w+2 (16 pixels of the 26-wide strip),
  // N = 2 tiles of 16 ci, K = 9 taps x 64 co.  (Enumerating M over the 28-wide padded grid is
  // bank-conflict free but needs 13 tiles per strip - an unbalanced, branchy split that measured
  // slower; this balanced split keeps the row&7 swizzle at ~1.6x the ideal read cost.)
  const int m = lane & 15, kg = lane >> 4;
  constexpr int MT = 3;
  int qbase[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    int q = 16 * (3 * wave + i) + m;
    if (q >= npix) q = 0;
    const int qy = q / H1, qx = q - qy * H1;
    qbase[i] = (qy + 2) * DG_TCOLS + qx + 2;     // LDS row of the un-shifted pixel
  }
  floatx4 acc[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i][0] = acc[i][1] = floatx4{0.f, 0.f, 0.f, 0.f};
  // conv1 ReLU mask for the epilogue = (a1 > 0): prefetch the stored bf16 a1 values now so the
  // loads overlap the MFMA loop (no conv1 recompute)
  uint16_t a1v[MT][4][2];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int q = 16 * (3 * wave + i) + 4 * kg + r;
      q = q < npix ? q : npix - 1;
      const uint16_t* src = a.a1 + ((int64_t)b * H1 * H1 + r0 * H1 + q) * C1 + m;
      a1v[i][r][0] = src[0];
      a1v[i][r][1] = src[16];
    }
#pragma unroll
  for (int ks = 0; ks < 18; ++ks) {
    const int t = ks >> 1, co0 = 32 * (ks & 1);
    const int toff = (t / 3) * DG_TCOLS + (t % 3);
    const int ch = (co0 >> 3) + kg;
    bf16x8 A[MT], Bf[2];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int row = qbase[i] - toff;
      A[i] = ld16(dys + row * C2 + ((ch ^ swz8(row)) << 3));
    }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int row = t * C1 + nt * 16 + m;
      Bf[nt] = ld16(w2ds + row * C2 + ((ch ^ swz8(row)) << 3));
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) acc[i][nt] = mfma16x16x32(A[i], Bf[nt], acc[i][nt]);
  }

  // ---- phase 3: conv1 ReLU mask (a1 > 0), then the conv1 weight/bias gradient of this strip as a
  // second, tiny MFMA: D[tap][ci] = sum_px X[px][tap] * d[px][ci] on v_mfma_f32_16x16x16_bf16
  // (row 9 of X = ones -> the bias gradient).  That instruction's B-operand layout (lane l holds
  // k = 4(l>>4)+j, n = l&15) is exactly the C layout of the dgrad accumulators, so the masked
  // accumulators feed it straight from registers (bf16-rounded operands, fp32 accumulation).
  floatx4 dw[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
  {
    const int tap = lane & 15, ty = tap / 3, tx = tap - 3 * ty;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      short4_t ax, bd[2];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = 16 * (3 * wave + i) + 4 * kg + j;
        const int qc = q < npix ? q : npix - 1;
        const int py = qc / H1, px = qc - py * H1;
        const float xv = (tap < 9) ? xs[(py + ty) * IMG + px + tx] : ((tap == 9) ? 1.0f : 0.0f);
        ax[j] = (short)f2bf(xv);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const uint16_t av = a1v[i][j][nt];
          const float d = (q < npix && av != 0 && !(av & 0x8000)) ? acc[i][nt][j] : 0.0f;
          bd[nt][j] = (short)f2bf(d);
        }
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) dw[nt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ax, bd[nt], dw[nt], 0, 0, 0);
    }
  }
  // dw[nt]: lane l holds D[tap = 4(l>>4) + r][ci = 16nt + (l&15)]
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = 4 * kg + r;
      if (t < 10) red[(wave * 32 + nt * 16 + m) * 10 + t] = dw[nt][r];
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
  // conv2 bias partial: each thread always stages channels 8*(tid&7)..+7 of the dy tile
  float bsum[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum[j] = 0.f;
  constexpr int DY_CH = WDYS_BYTES / 16;   // 2304 = 9 per thread
  // per-lane fragment offsets (elements), hoisted out of the unit and k-step loops
  const int clo = 8 * gq + q, chi = clo + 4;
  int aoff_lo[2], aoff_hi[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int cb = 16 * (mt0 + i) + 4 * pp;
    aoff_lo[i] = clo * C2 + ((((cb >> 3) ^ swz_dy(clo)) << 3) | (cb & 7));
    aoff_hi[i] = chi * C2 + ((((cb >> 3) ^ swz_dy(chi)) << 3) | (cb & 7));
  }
  constexpr int A1_CH = WA1S_BYTES / 16;   // 1456

  for (int u = blockIdx.x; u < 2 * B; u += G) {
    const int b = u >> 1, h = u & 1;
    {
      const uint4* dsrc = reinterpret_cast<const uint4*>(a.dy + ((int64_t)b * H2 + WG_HALF_ROWS * h) * H2 * C2);
      const uint4* asrc = reinterpret_cast<const uint4*>(a.a1 + ((int64_t)b * H1 + WG_HALF_ROWS * h) * H1 * C1);
      uint4 vd[9], va[6];
#pragma unroll
      for (int k = 0; k < 9; ++k) vd[k] = dsrc[tid + 256 * k];
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int c = tid + 256 * k;
        va[k] = asrc[c < A1_CH ? c : A1_CH - 1];   // clamped: no conditional load (keeps va in VGPRs)
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int c = tid + 256 * k, pix = c >> 3;
        reinterpret_cast<uint4*>(dys)[pix * 8 + ((c & 7) ^ swz_dy(pix))] = vd[k];
        const uint32_t w4[4] = {vd[k].x, vd[k].y, vd[k].z, vd[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bsum[2 * j] += bf2f((uint16_t)(w4[j] & 0xFFFF));
          bsum[2 * j + 1] += bf2f((uint16_t)(w4[j] >> 16));
        }
      }
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int c = tid + 256 * k;
        if (c < A1_CH) reinterpret_cast<uint4*>(a1s)[c] = va[k];
      }
      (void)DY_CH;
    }
    __syncthreads();
#pragma unroll 1
    for (int ks = 0; ks < 9; ++ks) {
      // A: dy rows (pixels) 32ks + c; the chunk swizzle (c ^ c>>1) & 7 does not depend on ks
      bf16x8 A[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) A[i] = tr_frag(dys + ks * 32 * C2 + aoff_lo[i], dys + ks * 32 * C2 + aoff_hi[i]);
      // B: a1 pixel of dy pixel p = 32ks + c shifted by the tap = p + 2*(p/24) + (ky*26 + kx)
      const int plo = 32 * ks + clo, phi = plo + 4;
      const uint16_t* blo = a1s + (plo + 2 * (plo / H2)) * C1 + 4 * pp;
      const uint16_t* bhi = a1s + (phi + 2 * (phi / H2)) * C1 + 4 * pp;
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int nt = nt0 + j, t = nt >> 1, ci0 = 16 * (nt & 1);
        const int toff = ((t / 3) * H1 + (t % 3)) * C1 + ci0;
        const bf16x8 Bf = tr_frag(blo + toff, bhi + toff);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][j] = mfma16x16x32(A[i], Bf, acc[i][j]);
      }
    }
    __syncthreads();
  }
  // slab layout = MFMA-native [co-tile 4][n-tile 18][lane 64][4]: one coalesced float4 per tile
  float* out = a.w2part + (int64_t)blockIdx.x * W2PART_STRIDE;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int tile = (mt0 + i) * 18 + nt0 + j;
      *reinterpret_cast<floatx4*>(out + (tile * 64 + lane) * 4) = acc[i][j];
    }
  // bias: threads with equal tid&7 hold the same 8 channels -> reduce 32 such threads via LDS
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int j = 0; j < 8; ++j) red[j * 256 + tid] = bsum[j];
  __syncthreads();
  if (tid < 64) {
    const int c8 = tid >> 3, j = tid & 7;     // channel = 8*c8 + j
    float s = 0.f;
    for (int k = 0; k < 32; ++k) s += red[j * 256 + k * 8 + c8];
    out[18432 + 8 * c8 + j] = s;
  }
}

// --------------------------------------------------------------------------------------------
// Deterministic fixed-order reduction of the partial slabs into the flat fp32 gradient buffer.
// Latency-bound by construction (19 MB of partials at B=200, mostly MALL-resident), so every
// thread issues all of its float4 loads before the first add:
//   [0, 289): conv2 weight+bias slab columns, 16 float4 columns x 16 slab slices per WG
//             (<= 16 loads in flight per thread for G <= 256), fixed-order LDS tree over slices
//   [289, 309): conv1 weight+bias, 4 float4 columns x 64 slices of the 4*B dgrad partials
namespace {
constexpr int RED_W2_WGS = (W2PART_STRIDE / 4 + 15) / 16;   // 289
constexpr int RED_C1_WGS = 320 / 16;                         // 20
}  // namespace

__global__ __launch_bounds__(256) void conv_grad_reduce_kernel(ConvBwdArgs a, int B) {
  __shared__ float4 red[256];
  const int tid = threadIdx.x, bid = blockIdx.x;
  const float sc = a.grad_scale;
  if (bid < RED_W2_WGS) {
    const int G = a.wgrad_groups;
    const int col = bid * 16 + (tid & 15), sl = tid >> 4;          // float4 column, slab slice
    const float4* src = reinterpret_cast<const float4*>(a.w2part) + col;
    constexpr int S4 = W2PART_STRIDE / 4;
    float4 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int g = sl + 16 * k;
      v[k] = (g < G) ? src[(int64_t)g * S4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float4 t = v[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) { t.x += v[k].x; t.y += v[k].y; t.z += v[k].z; t.w += v[k].w; }
    for (int g = sl + 256; g < G; g += 16) {          // G > 256 never happens today; kept general
      const float4 u = src[(int64_t)g * S4];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    red[tid] = t;
    __syncthreads();
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1) {                 // fixed-order tree over the 16 slices
      if (sl < w) {
        const float4 u = red[tid + 16 * w];
        t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
        red[tid] = t;
      }
      __syncthreads();
    }
    if (sl == 0) {
      const int e = 4 * col;
      const float o[4] = {t.x * sc, t.y * sc, t.z * sc, t.w * sc};
      if (e < 18432) {
        // slab element e = ((mtile*18 + ntile)*64 + lane)*4 + r  ->  co, ci, tap
        const int ln = (e >> 2) & 63, tile = e >> 8;
        const int mtile = tile / 18, ntile = tile - mtile * 18;
        const int co0 = 16 * mtile + 4 * (ln >> 4);
        const int ci = 16 * (ntile & 1) + (ln & 15), tap = ntile >> 1;
#pragma unroll
        for (int r = 0; r < 4; ++r) a.grad[OFF_CONV2_W + (co0 + r) * 288 + ci * 9 + tap] = o[r];
      } else if (e < 18432 + C2) {
#pragma unroll
        for (int r = 0; r < 4; ++r) a.grad[OFF_CONV2_B + (e - 18432) + r] = o[r];
      }
    }
  } else {
    const int col = (bid - RED_W2_WGS) * 4 + (tid & 3), sl = tid >> 2;   // 80 float4 columns, 64 slices
    const int nslab = 4 * B;
    const float4* src = reinterpret_cast<const float4*>(a.c1part) + col;
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k0 = sl; k0 < nslab; k0 += 64 * 16) {
      float4 v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int r = k0 + 64 * k;
        v[k] = (r < nslab) ? src[(int64_t)r * 80] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) { t.x += v[k].x; t.y += v[k].y; t.z += v[k].z; t.w += v[k].w; }
    }
    red[tid] = t;
    __syncthreads();
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
      if (sl < w) {
        const float4 u = red[tid + 4 * w];
        t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
        red[tid] = t;
      }
      __syncthreads();
    }
    if (sl == 0) {
      const float o[4] = {t.x * sc, t.y * sc, t.z * sc, t.w * sc};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = 4 * col + r, ci = j / 10, kk = j - ci * 10;
        if (kk < 9) a.grad[OFF_CONV1_W + ci * 9 + kk] = o[r];
        else a.grad[OFF_CONV1_B + ci] = o[r];
      }
    }
  }
}

void launch_conv_dgrad(const ConvBwdArgs& a, int B, hipStream_t s) {
  hipLaunchKernelGGL(conv2_dgrad_kernel, dim3(4, B), dim3(256), 0, s, a, B);
}
void launch_conv_wgrad(const ConvBwdArgs& a, int B, hipStream_t s) {
  hipLaunchKernelGGL(conv2_wgrad_kernel, dim3(a.wgrad_groups), dim3(256), 0, s, a, B);
}
void launch_conv_bwd(const ConvBwdArgs& a, int B, hipStream_t s) {
  launch_conv_dgrad(a, B, s);
  launch_conv_wgrad(a, B, s);
}

void launch_conv_grad_reduce(const ConvBwdArgs& a, int B, hipStream_t s) {
  hipLaunchKernelGGL(conv_grad_reduce_kernel, dim3(RED_W2_WGS + RED_C1_WGS), dim3(256), 0, s, a, B);
}

}  // namespace mnist
