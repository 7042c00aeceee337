// Conv trunk backward.
//
// Replaces the autograd backward of reference mnist_ddp.py:50-55 (dropout1, max_pool2d, relu, conv2,
// relu, conv1): max_pool2d_with_indices_backward, threshold_backward x2, convolution_backward x2.
//
//  * conv2_dgrad_persist_kernel (items = image x strip of 7 conv1 rows): expands the compact un-pooled gradient
//    (pooled grads + argmax codes written by fc_bwd) into a zero-padded NHWC LDS tile, runs the transposed
//    convolution as an MFMA implicit GEMM (M = pixels, N = 32 ci, K = 9 taps x 64 co), applies the
//    conv1 ReLU mask (stored bf16 a1 > 0, prefetched under the MFMA loop), and folds
//    the conv1 weight/bias gradient into the epilogue as a second 16x16x16 MFMA fed straight
//    from the masked accumulators (per-workgroup partials).
//  * conv2_wgrad_lean_kernel / _lstag_kernel (G <= 256 WGs, each a contiguous range of dy rows of
//    the whole batch, in 8-row chunks through a double-buffered LDS pipeline): dW2 = dy^T (x) im2col(a1), contraction
//    over pixels.  Both operands are pixel-major NHWC tiles in LDS; fragments come
//    from ds_read_b64_tr_b16 with per-lane row addresses, so the im2col gather is free.
//  * conv_grad_reduce_kernel: fixed-order (deterministic) sum of the partial slabs into the flat
//    fp32 gradient buffer, scaled by grad_scale (1.0 from the engine, whose head already carries
//    the 1/(B*world) DDP averaging).
#include "../include/device_utils.h"
#include "../include/kernels.h"
#include "../include/timeline.h"
#include "conv_grad_reduce.h"

#include <stdexcept>
#include <stdlib.h>

namespace mnist {

// Phase timing of the dgrad item (tools/dgrad_phase.hip compiles a copy of this file with
// MNIST_DGRAD_PHASE_TIMING): thread 0 of every workgroup records s_memtime at each phase boundary.
#ifdef MNIST_DGRAD_PHASE_TIMING
constexpr int kDgPhaseMaxWG = 32768;
__device__ uint64_t g_dg_phase[kDgPhaseMaxWG * 8];
#define DG_MARK(i)                                                                             \
  if (threadIdx.x == 0 && blockIdx.y * gridDim.x + blockIdx.x < kDgPhaseMaxWG)                 \
    g_dg_phase[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] = __builtin_amdgcn_s_memtime();
#else
#define DG_MARK(i)
#endif
// Phase timing of the wgrad kernels (tools/wgrad_phase.hip: MNIST_WGRAD_PHASE_TIMING).
#ifdef MNIST_WGRAD_PHASE_TIMING
constexpr int kWgPhaseMaxWG = 1024;
__device__ uint64_t g_wg_phase[kWgPhaseMaxWG * 8];
#define WG_MARK(i)                                                                             \
  if (threadIdx.x == 0 && blockIdx.x < kWgPhaseMaxWG)                                         \
    g_wg_phase[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memtime();
#else
#define WG_MARK(i)
#endif

namespace {
constexpr int DG_ROWS = 7;                              // conv1-output rows per dgrad WG (4 strips)
constexpr int DG_TROWS = DG_ROWS + 2;                   // dy rows incl. halo (top 2)
constexpr int DG_TCOLS = H2 + 4;                        // 28 (2 zero columns each side)
// LDS row pitch of the dy tile (pixels).  A pitch of 34 makes a 16-pixel M-tile that wraps from
// column 25 of one strip row to column 0 of the next advance the LDS row by 9 = 1 mod 8, so the
// row&7 swizzle continues as on a contiguous run (A-fragment reads 6.2 -> 4.3 modelled LDS cycles,
// ideal 4) - and measured slower (B = 8192 dgrad 407 -> 420 us): the kernel is not bound by these
// reads' bank conflicts.  28 = the tile's width.
constexpr int DG_PITCH = 28;
constexpr int DYS_BYTES = DG_TROWS * DG_PITCH * C2 * 2; // 32256
constexpr int W2DS_BYTES = 9 * C1 * C2 * 2;             // 36864
constexpr int XS2_BYTES = 256 * 4;                     // DG_TROWS * IMG = 252 input pixels + 4 zeros
constexpr int RED_BYTES = 4 * 32 * 10 * 4;              // 5120
constexpr int DG_LDS = DYS_BYTES + W2DS_BYTES + 1024;   // 70144: two per CU; the conv1-gradient
                                                        // reduction scratch aliases the dy tile
static_assert(RED_BYTES <= DYS_BYTES && 2 * DG_LDS <= 160 * 1024, "dgrad LDS carve");

// wgrad: every workgroup owns a contiguous range of dy rows of the whole batch (rows of
// consecutive images are contiguous in both dy [B*24 rows] and a1 [B*26 rows]), processed in
// chunks of up to 8 rows (192 px = 6 k-steps) through a double-buffered LDS pipeline.
constexpr int WG_CH = 8;                                     // dy rows per chunk
constexpr int WG_CHPX = WG_CH * H2;                          // 192 px
constexpr int WG_A1ROWS = WG_CH + 4;                         // + 2 halo rows + 2 image-boundary rows
constexpr int WDY_BYTES = WG_CHPX * C2 * 2;                  // 24576
constexpr int WA1_BYTES = WG_A1ROWS * H1 * C1 * 2;           // 19968
constexpr int WBUF_BYTES = WDY_BYTES + WA1_BYTES;            // 44544
constexpr int WG_LDS = 2 * WBUF_BYTES;                       // 89088 (one workgroup per CU)
constexpr int WG_THREADS = 512;                              // 8 waves: 2 per SIMD hide LDS latency
constexpr int WDY_V = WDY_BYTES / 16 / WG_THREADS;           // 3 x 16 B per thread
constexpr int WA1_V = (WA1_BYTES / 16 + WG_THREADS - 1) / WG_THREADS;   // 3 x 16 B (1248 used)
static_assert(WDY_BYTES % (16 * WG_THREADS) == 0, "dy chunk staging");

// 16-byte-chunk XOR swizzles against ds_read_b128 / ds_read_b64_tr_b16 bank conflicts (rows of
// 128 B = 8 chunks, or 64 B = 4 chunks).  Chosen with tools/lds_banks.py (gfx950 lane-group model).
__device__ __forceinline__ int swz8(int row) { return row & 7; }
__device__ __forceinline__ int swz_dy(int pix) { return (pix ^ (pix >> 1)) & 7; }
}  // namespace

// Expand one 16-B chunk of the compact un-pooled gradient (8 channels of one pooled position) to
// the dense chunk of window pixel q (0..3): channel j keeps its value iff its argmax code == q.
// The chunk's codes arrive as two bit planes r16 (bit j = code bit 0 of channel j, bit 8 + j = code
// bit 1; kernels.h DYC_ROUTE).  v_perm_b32's sign selectors (8 / 9 = 0xFF iff bit 15 / 31 of src1
// is set) expand a match flag straight into a 16-bit lane mask, so for output word k (channels 2k,
// 2k + 1) the flags only need to sit at bits 15 / 31: rr = r16 | (r16 >> 1) << 16 puts channel
// 2k + 1's bit 0 at 16 + 2k next to channel 2k's at 2k, and its bit 1 at 24 + 2k next to channel
// 2k's at 8 + 2k; rr << (15 - 2k) and rr << (7 - 2k) bring them to 15 / 31 (tests/test_dyc_expand_cpu.py).
__device__ __forceinline__ uint32_t dyc_rr(uint32_t r16) { return r16 | ((r16 >> 1) << 16); }
__device__ __forceinline__ uint4 dyc_expand_flags(uint4 g, uint32_t bx, uint32_t by) {
  // bx / by: rr or ~rr (code bit 0 / 1 == the pixel's); a match needs both at bits 15 / 31
  uint4 o;
  o.x = g.x & __builtin_amdgcn_perm(0u, (bx << 15) & (by << 7), 0x09090808u);
  o.y = g.y & __builtin_amdgcn_perm(0u, (bx << 13) & (by << 5), 0x09090808u);
  o.z = g.z & __builtin_amdgcn_perm(0u, (bx << 11) & (by << 3), 0x09090808u);
  o.w = g.w & __builtin_amdgcn_perm(0u, (bx << 9) & (by << 1), 0x09090808u);
  return o;
}
// one pixel q (0..3), or nothing (q = 4: the lean wgrad zeroes rows past a chunk this way)
__device__ __forceinline__ uint4 dyc_expand(uint4 g, uint32_t r16, int q) {
  const uint32_t rr = dyc_rr(r16);
  const uint32_t none = q < 4 ? ~0u : 0u;
  return dyc_expand_flags(g, ((q & 1) ? rr : ~rr) & none, (q & 2) ? rr : ~rr);
}
// all four window pixels of one chunk share rr (conv2_dgrad's staging by pooled record)
template <int Q>
__device__ __forceinline__ uint4 dyc_expand_q(uint4 g, uint32_t rr) {
  return dyc_expand_flags(g, (Q & 1) ? rr : ~rr, (Q & 2) ? rr : ~rr);
}
__device__ __forceinline__ const uint8_t* dyc_record(const uint8_t* dyc, int b, int y, int x) {
  return dyc + (int64_t)b * DYC_BYTES_PER_IMAGE + ((y >> 1) * HP + (x >> 1)) * DYC_REC;
}

// One workgroup per CU, each owning >= 8 dy rows (B=200: 4800 rows -> 256 groups x 18-19 rows).
// Monotonic in B, so a workspace sized for the largest batch fits every smaller one.
int conv_wgrad_groups(int B) {
  const int rows = H2 * B;
  const int g = (rows + WG_CH - 1) / WG_CH;
  return g < 256 ? g : 256;
}

// --------------------------------------------------------------------------------------------
// input-row source of the conv1 gradient: pre-gathered epoch rows, rows by index, or fp32 module input
enum DgX { DGX_PRE = 0, DGX_IDX = 1, DGX_XIN = 2 };

// Global loads of one (image, strip) item of the 4-strip dgrad: the padded dy tile's 16-B chunks
// (rows r0-2..r0+6, cols -2..25, compact records + argmax routes) and this thread's input pixel.
// Every load is unconditional (clamped address, validity applied at the LDS store) so all of them
// are in flight at once; the input row (state -> [index] -> pixel, a dependent chain) is issued last.
// Staging by pooled record: the tile's dy rows r0-2..r0+6 lie under 5 pooled rows (py0..py0+4,
// py0 = floor((r0-2)/2)) x 12 pooled columns; job = (pooled row, pooled column, 16-B channel chunk):
// 480 jobs, 2 per thread.  Each job loads its record chunk + argmax routes ONCE and expands them into
// the (up to) 4 pixels of its 2x2 window (the per-pixel form loaded every record 4 times and paid the
// pixel addressing 8 times per thread); pooled rows outside [0, 12) stage zeros (the padding rows),
// and the 4 padding columns are zero-filled separately (288 chunks).  Same LDS bytes as before.
constexpr int DG_JOBS = 5 * HP * 8;                // 480
struct DgLoad {
  uint4 v[2];
  uint32_t rt[2];                                 // the chunk's code planes (r16)
  uint32_t okm;                                   // bit j: job j's pooled row is inside the image
  float xv;                                       // fp32 module input, or the raw pixel byte
};

template <int XM>
__device__ __forceinline__ void dgrad_fetch(const ConvBwdArgs& a, int strip, int b, int step, int tid, DgLoad& L) {
  const int r0 = strip * DG_ROWS;
  const int py0 = (r0 - 2) >> 1;                  // arithmetic shift: floor
  L.okm = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int jb = tid + 256 * k;
    const int j = jb < DG_JOBS ? jb : 0;
    const int c8 = j & 7, pc = (j >> 3) % HP, pr = (j >> 3) / HP;
    const int py = py0 + pr;
    const bool ok = jb < DG_JOBS && py >= 0 && py < HP;
    L.okm |= (ok ? 1u : 0u) << k;
    const uint8_t* rec = a.dyc + (int64_t)b * DYC_BYTES_PER_IMAGE + ((ok ? py : 0) * HP + pc) * DYC_REC;
    L.v[k] = *reinterpret_cast<const uint4*>(rec + c8 * 16);
    L.rt[k] = *reinterpret_cast<const uint16_t*>(rec + DYC_ROUTE + c8 * 2);
  }
  const int e = tid < DG_TROWS * IMG ? tid : 0;   // DG_TROWS * IMG = 252 <= 256
  const bool okx = tid < DG_TROWS * IMG && r0 + e / IMG < IMG;
  const int off = r0 * IMG + (okx ? e : 0);
  if constexpr (XM == DGX_XIN) {
    L.xv = a.xin[(int64_t)b * (IMG * IMG) + off];
  } else {
    const int64_t row = (int64_t)step * a.idx_step_stride + b;
    const int64_t img = (XM == DGX_IDX) ? (int64_t)a.idx[row] : row;
    L.xv = __builtin_bit_cast(float, (uint32_t)a.data_u8[img * (IMG * IMG) + off]);
  }
  if (!okx) L.xv = (XM == DGX_XIN) ? 0.0f : __builtin_bit_cast(float, 0x100u);   // 0x100: "outside"
}

__device__ __forceinline__ void dgrad_w2d_load(const ConvBwdArgs& a, int tid, uint4 (&w)[9]) {
  const uint4* src = reinterpret_cast<const uint4*>(a.w2d);
#pragma unroll
  for (int i = 0; i < 9; ++i) w[i] = src[tid + 256 * i];
}
__device__ __forceinline__ void dgrad_w2d_store(unsigned char* smem, int tid, const uint4 (&w)[9]) {
  uint16_t* w2ds = reinterpret_cast<uint16_t*>(smem + DYS_BYTES);
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int c = tid + 256 * i, row = c >> 3, c8 = c & 7;
    reinterpret_cast<uint4*>(w2ds)[row * 8 + (c8 ^ swz8(row))] = w[i];
  }
}
__device__ __forceinline__ void dgrad_dy_store(unsigned char* smem, int strip, int tid, const DgLoad& L) {
  uint4* dys = reinterpret_cast<uint4*>(smem);    // the dy tile is at the start of smem
  const int r0 = strip * DG_ROWS;
  const int py0 = (r0 - 2) >> 1;
  const uint4 z = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int jb = tid + 256 * k;
    if (jb < DG_JOBS) {
      const int c8 = jb & 7, pc = (jb >> 3) % HP, pr = (jb >> 3) / HP;
      const int ly0 = 2 * (py0 + pr) - (r0 - 2);  // tile row of the window's top pixel row (-1..9)
      const bool ok = (L.okm >> k) & 1u;
      const uint32_t rr = dyc_rr(L.rt[k]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ly = ly0 + (q >> 1);
        if (ly >= 0 && ly < DG_TROWS) {
          const int row = ly * DG_PITCH + 2 * pc + (q & 1) + 2;
          uint4 e = q == 0 ? dyc_expand_q<0>(L.v[k], rr) : q == 1 ? dyc_expand_q<1>(L.v[k], rr)
                  : q == 2 ? dyc_expand_q<2>(L.v[k], rr) : dyc_expand_q<3>(L.v[k], rr);
          const uint32_t okm = ok ? ~0u : 0u;           // per component (a select of the uint4 went
          e.x &= okm; e.y &= okm; e.z &= okm; e.w &= okm;   // through scratch memory)
          dys[row * 8 + (c8 ^ swz8(row))] = e;
        }
      }
    }
  }
  // padding columns 0, 1, 26, 27 of every tile row: 9 x 4 x 8 = 288 zero chunks
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int jz = tid + 256 * k;
    if (jz < DG_TROWS * 4 * 8) {
      const int c8 = jz & 7, pcol = (jz >> 3) & 3, ly = jz >> 5;
      const int row = ly * DG_PITCH + (pcol < 2 ? pcol : pcol + 24);
      dys[row * 8 + (c8 ^ swz8(row))] = z;
    }
  }
}

// MFMA loop + conv1 gradient epilogue of one item whose dy tile and the conv2 weights are in LDS
// (after a barrier).  Ends with the item's c1part row written; the LDS reads of the dy tile are all
// done once every wave has passed this function's first barrier.  ``prefetch()`` runs right after
// the a1 mask loads are issued (the persistent kernel issues the next item's loads there, so the
// epilogue's wait for the mask does not also wait for them).
// Input-row value staged for the conv1-gradient epilogue (raw pixel byte -> normalised fp32).
template <int XM>
__device__ __forceinline__ float dgrad_xs_value(float xv) {
  if (XM == DGX_XIN) return xv;
  const uint32_t u = __builtin_bit_cast(uint32_t, xv);
  return u > 0xFFu ? 0.0f : normalize_u8_alu(u);
}

// Fixed-order sum of the 4 waves' conv1-gradient partials -> the item's c1part row (256 threads).
// 80 lanes x 4 consecutive values, the same per-element sum order; 16-B write-through stores (read
// by the conv reduce kernels only: 42 MB a step at B = 8192 no longer left dirty in L2)
__device__ __forceinline__ void dgrad_red_reduce(const ConvBwdArgs& a, int strip, int b, const float* red, int ltid,
                                                 bool wt) {
  if (ltid < 80) {
    const float4* r4 = reinterpret_cast<const float4*>(red);
    const float4 x0 = r4[ltid], x1 = r4[80 + ltid], x2 = r4[160 + ltid], x3 = r4[240 + ltid];
    const floatx4 s = {x0.x + x1.x + x2.x + x3.x, x0.y + x1.y + x2.y + x3.y, x0.z + x1.z + x2.z + x3.z,
                       x0.w + x1.w + x2.w + x3.w};
    store16(wt, a.c1part, (((int64_t)b * 4 + strip) * 320 + 4 * ltid) * 4, s);
  }
}

// STAG = false: the whole item on one 4-wave workgroup (xs store, barriers, reduce inside).
// STAG = true: xs is already staged and no barriers are taken; the item ends with the waves'
// partials in red (the caller reduces them later).  The staggered-halves dgrad that used this
// (one 8-wave workgroup per CU, halves alternating MFMA and staging phases) measured slower than
// two independent per-item workgroups per CU (B = 8192: 1.56 vs 1.24 ms/step) and was removed.
// conv1 ReLU mask operand of the epilogue = the stored bf16 a1 values of this wave's 3 M-tiles
// (lane: channel m and m + 16 of pixels 4kg..4kg+3 of each tile)
constexpr int DG_MT = 3;
struct DgMask {
  uint16_t v[DG_MT][4][2];
};
__device__ __forceinline__ void dgrad_mask_load(const ConvBwdArgs& a, int strip, int b, int wave, DgMask& M) {
  const int lane = threadIdx.x & 63, m = lane & 15, kg = lane >> 4;
  const int r0 = strip * DG_ROWS;
  const int npix = ((strip == 3) ? (H1 - 3 * DG_ROWS) : DG_ROWS) * H1;
#pragma unroll
  for (int i = 0; i < DG_MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int q = 16 * (3 * wave + i) + 4 * kg + r;
      q = q < npix ? q : npix - 1;
      const uint16_t* src = a.a1 + ((int64_t)b * H1 * H1 + r0 * H1 + q) * C1 + m;
      M.v[i][r][0] = src[0];
      M.v[i][r][1] = src[16];
    }
}

// PRE: the caller issued the mask loads (dgrad_mask_load) before staging, so their HBM latency
// hides under the staging phase too; else they are issued here, ahead of the MFMA loop.
template <int XM, bool STAG, bool PRE, class Prefetch>
__device__ __forceinline__ void dgrad_compute_p(const ConvBwdArgs& a, int strip, int b, uint16_t* dys,
                                                const uint16_t* w2ds, float* xs, float* red, int wave,
                                                int ltid, float xv, const DgMask& pre, Prefetch prefetch) {
  const int lane = threadIdx.x & 63, tid = ltid;
  const int nrows = (strip == 3) ? (H1 - 3 * DG_ROWS) : DG_ROWS;   // 7,7,7,5
  const int npix = nrows * H1;

  // ---- transposed conv on MFMA: M-tiles 3w..3w+2 (16 pixels of the 26-wide strip),
  // N = 2 tiles of 16 ci, K = 9 taps x 64 co.  (Enumerating M over the 28-wide padded grid is
  // bank-conflict free but needs 13 tiles per strip - an unbalanced, branchy split that measured
  // slower; this balanced split keeps the row&7 swizzle at ~1.6x the ideal read cost.)
  const int m = lane & 15, kg = lane >> 4;
  constexpr int MT = DG_MT;
  // A-fragment addresses without per-read VALU: for tap t = 3d + c the LDS row is R_c - 28d with
  // R_c = qbase - c, and (R_c - 28d) & 7 = (R_c & 7) ^ 4(d & 1), so the swizzled chunk of co-half h is
  // ((kg ^ (R_c & 7)) ^ 4(h ^ (d & 1))): per (M-tile, c) two base addresses (chunk bit 2 clear / set)
  // at row R_c - 56, and every read of the loop is base + an immediate (1792 elements per d step).
  static_assert(DG_PITCH % 8 == 4, "row step of one tap row = 4 mod 8");
  const uint16_t* abase[MT][3][2];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int q = 16 * (3 * wave + i) + m;
    const int qy = q / H1, qx = q - qy * H1;
    // LDS row of the un-shifted pixel.  A pixel past the strip reads a window of padding zeros
    // (rows 1-3, columns 27 / 0 / 1: every tap lands on one), so its accumulator row is exactly 0
    // and the epilogue needs no pixel-range mask.
    const int qbase = q < npix ? (qy + 2) * DG_PITCH + qx + 2 : 3 * DG_PITCH + 1;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int rc = qbase - c;
      const int e = (rc - 2 * DG_PITCH) * C2 + ((kg ^ (rc & 7)) << 3);
      abase[i][c][0] = dys + e;
      abase[i][c][1] = dys + (e ^ 32);
    }
  }
  // B fragments: row t*32 + 16nt + m has swizzle key m & 7 for every t, nt
  const int be = m * C2 + ((kg ^ (m & 7)) << 3);
  const uint16_t* bbase[2] = {w2ds + be, w2ds + (be ^ 32)};
  floatx4 acc[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i][0] = acc[i][1] = floatx4{0.f, 0.f, 0.f, 0.f};
  // conv1 ReLU mask for the epilogue = (a1 > 0): the stored bf16 a1 values, loaded ahead so the
  // loads overlap the MFMA loop (no conv1 recompute)
  DgMask own;
  if constexpr (!PRE) dgrad_mask_load(a, strip, b, wave, own);
  const DgMask& mk = PRE ? pre : own;
  prefetch();
#ifdef DG_UB_AREUSE   // A/B upper bound only (wrong results): one A read per tap row, reused for c = 1, 2
  bf16x8 Arow[2][MT];
#endif
#pragma unroll
  for (int ks = 0; ks < 18; ++ks) {
    const int t = ks >> 1, h = ks & 1, d = t / 3, c = t % 3;
    bf16x8 A[MT], Bf[2];
#ifdef DG_UB_AREUSE
    if (c == 0 && (DG_UB_AREUSE == 1 || t == 0)) {   // (=2: one A read for the whole loop)
#pragma unroll
      for (int i = 0; i < MT; ++i) Arow[h][i] = ld16(abase[i][c][h ^ (d & 1)] + (2 - d) * DG_PITCH * C2);
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) A[i] = Arow[h][i];
#else
#pragma unroll
    for (int i = 0; i < MT; ++i) A[i] = ld16(abase[i][c][h ^ (d & 1)] + (2 - d) * DG_PITCH * C2);
#endif
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) Bf[nt] = ld16(bbase[h] + (t * C1 + nt * 16) * C2);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) acc[i][nt] = mfma16x16x32(A[i], Bf[nt], acc[i][nt]);
  }
  DG_MARK(3);

  if constexpr (!STAG) {
    xs[tid] = dgrad_xs_value<XM>(xv);             // input rows (entries 252-255: zeros), first read below
    lds_barrier();
  }
  DG_MARK(5);

  // ---- conv1 ReLU mask (a1 > 0), then the conv1 weight/bias gradient of this strip as a
  // second, tiny MFMA: D[tap][ci] = sum_px X[px][tap] * d[px][ci] on v_mfma_f32_16x16x16_bf16
  // (row 9 of X = ones -> the bias gradient).  That instruction's B-operand layout (lane l holds
  // k = 4(l>>4)+j, n = l&15) is exactly the C layout of the dgrad accumulators, so the masked
  // accumulators feed it straight from registers (bf16-rounded operands, fp32 accumulation).
  floatx4 dw[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
  {
    const int tap = lane & 15, ty = tap / 3, tx = tap - 3 * ty;
    const int toff = tap < 9 ? ty * IMG + tx : 0;          // xs offset of the tap (any valid one past 8)
    const float xconst = tap == 9 ? 1.0f : 0.0f;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      // xs index of input pixel (py + ty, px + tx) of output pixel q = 26 py + px is q + 2 py + toff;
      // the lane's 4 pixels q0..q0+3 step along a row and wrap at most once (+2 past the row end).
      // Pixels past the strip read any in-range entry (their gradient rows are 0, see qbase).
      const int q0 = 16 * (3 * wave + i) + 4 * kg;
      const int qy0 = q0 / H1, qx0 = q0 - qy0 * H1;
      const int a0 = q0 + 2 * qy0 + toff;
      float xf[4], df[2][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int aj = min(a0 + j + (qx0 + j >= H1 ? 2 : 0), 255);
        const float xr = xs[aj];
        xf[j] = tap < 9 ? xr : xconst;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)       // conv1 ReLU mask: bf16 a1 > 0 <=> as int16 > 0
          df[nt][j] = (int16_t)mk.v[i][j][nt] > 0 ? acc[i][nt][j] : 0.0f;
      }
      // bf16 operands two at a time (one v_cvt_pk_bf16_f32 per pair)
      const short4_t ax = __builtin_bit_cast(short4_t, uint2{pack2bf(xf[0], xf[1]), pack2bf(xf[2], xf[3])});
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const short4_t bd = __builtin_bit_cast(short4_t, uint2{pack2bf(df[nt][0], df[nt][1]), pack2bf(df[nt][2], df[nt][3])});
        dw[nt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ax, bd, dw[nt], 0, 0, 0);
      }
    }
  }
  DG_MARK(6);
  // dw[nt]: lane l holds D[tap = 4(l>>4) + r][ci = 16nt + (l&15)]
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = 4 * kg + r;
      if (t < 10) red[(wave * 32 + nt * 16 + m) * 10 + t] = dw[nt][r];
    }
  if constexpr (!STAG) {
    lds_barrier();
    dgrad_red_reduce(a, strip, b, red, tid, a.c1_rows <= 4 * WT_MAX_B);   // (c1_rows = 4B)
  }
}

template <int XM, bool PRE = false, class Prefetch>
__device__ __forceinline__ void dgrad_compute(const ConvBwdArgs& a, int strip, int b, unsigned char* smem, float xv,
                                              const DgMask& pre, Prefetch prefetch) {
  uint16_t* dys = reinterpret_cast<uint16_t*>(smem);
  const uint16_t* w2ds = reinterpret_cast<const uint16_t*>(smem + DYS_BYTES);
  float* xs = reinterpret_cast<float*>(smem + DYS_BYTES + W2DS_BYTES);
  float* red = reinterpret_cast<float*>(smem);   // aliases the dy tile: written after the barrier
                                                  // that ends every wave's MFMA loop
  dgrad_compute_p<XM, false, PRE>(a, strip, b, dys, w2ds, xs, red, threadIdx.x >> 6, threadIdx.x, xv, pre, prefetch);
}

// Persistent dgrad: G <= 2 x CUs workgroups (two fit a CU by LDS), each staging the
// conv2 weights (36.9 KB) into LDS ONCE and then walking items it = blockIdx.x, +G, ... of the 4B
// (image, strip) items (strip = it & 3, image = it >> 2).  The next item's dy / input loads are
// issued right after the current tile's barrier, so they are in flight under the MFMA loop; the
// co-resident workgroup of the CU overlaps the LDS stores.  Per item the math (K order, masks,
// conv1-gradient MFMA, c1part row) does not depend on the grid: any G gives the same bits.
template <int XM>
__global__ __launch_bounds__(256, 2) void conv2_dgrad_persist_kernel(ConvBwdArgs a, int B) {
  TL_SCOPE(TL_DGRAD);
  __shared__ __attribute__((aligned(16))) unsigned char smem[DG_LDS];
  const int tid = threadIdx.x, n = 4 * B, G = gridDim.x;
  int it = blockIdx.x;
  if (a.signal_ctr && it == 0 && tid == 0)
    (RW_SIGNAL(), __hip_atomic_fetch_add(a.signal_ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT));
  RW_ENTRY();
  const StepState* st = a.state ? a.state : &g_zero_state;
  const int step = st->step;
  uint4 w[9];
  dgrad_w2d_load(a, tid, w);
  DgLoad L;
  dgrad_fetch<XM>(a, it & 3, it >> 2, step, tid, L);
  dgrad_w2d_store(smem, tid, w);
  for (; it < n; it += G) {
    dgrad_dy_store(smem, it & 3, tid, L);
    const float xv = L.xv;
    lds_barrier();
    const int nx = (it + G < n) ? it + G : it;   // clamped: the last item's prefetch is a re-read
    dgrad_compute<XM>(a, it & 3, it >> 2, smem, xv, DgMask{}, [&] { dgrad_fetch<XM>(a, nx & 3, nx >> 2, step, tid, L); });
    lds_barrier();                              // the next dy store must not overtake the red reads
  }
}

int conv_dgrad_c1_rows(int B) { return 4 * B; }

// Grid of the persistent dgrad: 2 x CUs workgroups, or fewer when 4B items are fewer (measured
// B = 200: 80.4 vs 82.6 us/step against the per-item grid; B = 8192, with the branch-free conv1-gradient
// epilogue, 0.980 vs 1.062 ms/step).  set_dgrad_grid(n > 0) overrides it (tests: ragged item rounds).
static int g_dgrad_grid_override = 0;
void set_dgrad_grid(int n) { g_dgrad_grid_override = n > 0 ? n : 0; }
static int dgrad_persist_grid(int B, bool full) {
  int g = g_dgrad_grid_override;
  if (g <= 0) {
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess) dev = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    }
    // equal item counts: as many rounds as 2 x CUs workgroups need, spread over the fewest workgroups
    // that keep that round count (B = 200: 800 items on 400 workgroups instead of 512 with 288 doing
    // two; the CUs left free run the comm stream's conv2 reduce + update, whose waves do not fit beside
    // two dgrad workgroups: 600 steps 63.3 -> 62.6 us/step; 448 / 360 / 320 / 272: 62.9 / 64.2 /
    // 65.1 / 65.4, profiles/r5/ab/dgrad_grid.txt).  B = 8192: 64 rounds of 512 either way.
    // The DDP schedules keep 2 x CUs (ConvBwdArgs::dgrad_full_grid: world-1 XGMI 68.6-68.8 us/step
    // with it, 69.5-71.5 with the equal-count grid - its conv2 part is the 124-VGPR xGMI kernel).
    const int n = 4 * B, g2 = 2 * cus, rounds = (n + g2 - 1) / g2;
    g = full ? g2 : (n + rounds - 1) / rounds;
  }
  return g < 4 * B ? g : 4 * B;
}

// --------------------------------------------------------------------------------------------
namespace {
// first a1 row (global, [B*26]) under dy row R (global, [B*24])
__device__ __forceinline__ int a1_row_of(int R) { return R + 2 * (R / H2); }

}  // namespace

// --------------------------------------------------------------------------------------------
// conv2_wgrad, VALU-lean form (below the staggered threshold).  G <= 256 workgroups, each a
// contiguous range of dy rows of the whole batch in 8-row chunks through a double-buffered LDS
// pipeline; 8 waves = 2 co-tile pairs x 4 groups of the 18 (tap, ci-half) n-tiles.  The round-2
// lockstep kernel of the same geometry had the VALU work that made it issue-bound (removed; numbers
// in docs/PERF_NOTES.md) (PMC at B = 200: ~1570 VALU instructions per wave against 133 MFMAs; a
// wave64 VALU instruction holds its SIMD for 2-4 cycles, so VALU issue - not the MFMA pipe or the
// LDS - set the kernel's time; tools/wgrad_phase.hip):
//  * staging: every chunk-invariant part of a thread's three dense dy chunks (row / column inside
//    the chunk, LDS slot, 2x2-window code) is computed once; per chunk a record offset costs a
//    compare against the (scalar) image boundary.  Rows past the chunk are zeroed by expanding with
//    window code 4, which matches no argmax route; a1 loads are clamped into the chunk's own rows
//    (finite values under zero dy) instead of masked;
//  * conv2 bias gradient on the MFMA pipe: one extra n-tile of ones, computed by the two waves
//    whose n-group has 4 tiles (so every SIMD issues 10 + 10 or 10 + 8 MFMAs per k-step), instead
//    of 16 VALU per staged chunk plus an LDS reduction;
//  * MFMA loop: k-steps unrolled, the n-group a template parameter, so every fragment read is a
//    base register + an immediate; the B-row base of each (k-step, lo/hi) lane row is precomputed
//    once per kernel and only the image-boundary shift (52 a1 pixels) is selected per chunk.
namespace {
constexpr int WL_KS = WG_CHPX / 32;                         // 6 k-steps per full chunk
// a1 tile planar by channel half ([ci / 16][pixel][16 ci], 32 B per pixel): with the k -> pixel map
// below, lanes 0-31 of a B-fragment read take 8 consecutive pixels = all 64 banks once (the NHWC
// tile's 64-B pixel pitch put lanes 0-3 and 8-11 on the same banks: 2-way conflicts on 10 of the
// 14 fragment reads per k-step)
constexpr int WL_PLANE = WG_A1ROWS * H1 * 16 * 2;            // 9984 B
template <int NTH>
struct WlPlanT {
  static constexpr int VD = WDY_BYTES / 16 / NTH;
  // record byte offset in the image row pair (x / 2, channel chunk; < 4096) | 2x2-window code << 12 |
  // chunk row << 16
  int rec[VD];
  int dst0;           // LDS uint4 index of chunk 0 (chunk i: + NTH i; the dy swizzle repeats every 8 pixels)
};
template <int NTH>
struct WlChunkT {
  static constexpr int VD = WDY_BYTES / 16 / NTH, VA = (WA1_BYTES / 16 + NTH - 1) / NTH;
  uint4 vd[VD], va[VA];
  uint32_t rt[VD];                                 // code planes (r16) of each dy chunk
};
// chunk-invariant staging plan of thread tid (dense dy chunk c = tid + NTH i: pixel c >> 3, channels
// 8(c & 7)..; every chunk of the workgroup starts on a row of the parity of r0 (chunks are 8 rows),
// so the 2x2-window code of each pixel is fixed)
template <int NTH>
__device__ __forceinline__ void wl_plan(WlPlanT<NTH>& P, int tid, int r0) {
  const int c8 = tid & 7;
  static_assert((NTH / 8) % 8 == 0, "pixel step of the chunks keeps the dy swizzle");
  P.dst0 = (tid >> 3) * 8 + (c8 ^ swz_dy(tid >> 3));
#pragma unroll
  for (int i = 0; i < WlPlanT<NTH>::VD; ++i) {
    const int pix = (tid >> 3) + (NTH / 8) * i;
    const int pr = pix / H2, x = pix - pr * H2;
    static_assert((HP - 1) * DYC_REC + 7 * 16 < 4096, "record offset below the code bits");
    P.rec[i] = (x >> 1) * DYC_REC + c8 * 16 + (((((r0 + pr) & 1) << 1) | (x & 1)) << 12) + (pr << 16);
  }
}
// global loads of chunk [c0, c1): records of rows past the chunk are clamped into it (zeroed at the
// store), a1 chunks past the chunk's rows clamped to its last one (finite, only met by zero dy)
template <int NTH>
__device__ __forceinline__ void wl_fetch(const ConvBwdArgs& a, const WlPlanT<NTH>& P, int tid, int c0, int c1,
                                         WlChunkT<NTH>& k) {
  const int b0 = c0 / H2, y0 = c0 - b0 * H2;               // scalar
  const uint8_t* recb = a.dyc + (int64_t)b0 * DYC_BYTES_PER_IMAGE;
  const int c8 = tid & 7;
#pragma unroll
  for (int i = 0; i < WlChunkT<NTH>::VD; ++i) {
    const int t = y0 + min(P.rec[i] >> 16, c1 - c0 - 1);
    const bool nx = t >= H2;
    const int y = nx ? t - H2 : t;
    const int off = (nx ? (int)DYC_BYTES_PER_IMAGE : 0) + (y >> 1) * (HP * DYC_REC) + (P.rec[i] & 0xFFF);
    k.vd[i] = *reinterpret_cast<const uint4*>(recb + off);
    k.rt[i] = *reinterpret_cast<const uint16_t*>(recb + off + DYC_ROUTE - c8 * 14);   // + 128 + 2 c8 - 16 c8
  }
  const int A0 = a1_row_of(c0), A1 = a1_row_of(c1 - 1) + 3;
  const int na1 = (A1 - A0) * H1 * 4;
  const uint4* asrc = reinterpret_cast<const uint4*>(a.a1 + (int64_t)A0 * H1 * C1);
#pragma unroll
  for (int i = 0; i < WlChunkT<NTH>::VA; ++i) k.va[i] = asrc[min(tid + NTH * i, na1 - 1)];
}
template <int NTH>
__device__ __forceinline__ void wl_store(const WlPlanT<NTH>& P, unsigned char* buf, int tid, int c0, int c1,
                                         const WlChunkT<NTH>& k) {
  uint4* dys = reinterpret_cast<uint4*>(buf);
  uint4* a1s = reinterpret_cast<uint4*>(buf + WDY_BYTES);
#pragma unroll
  for (int i = 0; i < WlChunkT<NTH>::VD; ++i) {
    const int code = (P.rec[i] >> 16) < c1 - c0 ? (P.rec[i] >> 12) & 3 : 4;   // 4: no route matches -> 0
    dys[P.dst0 + NTH * i] = dyc_expand(k.vd[i], k.rt[i], code);
  }
#pragma unroll
  for (int i = 0; i < WlChunkT<NTH>::VA; ++i) {
    const int c = tid + NTH * i;                     // NHWC chunk: pixel c >> 2, channels 8(c & 3)..
    if (c < WA1_BYTES / 16) a1s[(c >> 1) & 1 ? WL_PLANE / 16 + (c >> 2) * 2 + (c & 1) : (c >> 2) * 2 + (c & 1)] = k.va[i];
  }
}
// per-lane fragment bases.  k -> pixel: k = 8 gq + j holds pixel 4 gq + j (j < 4, the "lo" read) or
// 16 + 4 gq + j - 4 (the "hi" read), so each read's lanes 0-31 / 32-63 take 8 consecutive pixels
// (A and B agree).  A: dy rows lo / hi of co-tiles mt0, mt0 + 1 (bytes); B: plane-0 byte offset of the
// a1 pixel under each (k-step, lo / hi) lane row, before the image-boundary shift, and its dy row
struct WlFrag {
  int aoffb[2];       // co-tiles mt0, mt0 + 1, lo row (the hi row, pixel + 16, is + 2048 B: same swizzle)
  uint32_t tb[WL_KS / 2][2];   // B pixel byte offsets (< 2^13) of k-steps 2m (low half) and 2m + 1
  int c[2];           // the lane's lo / hi pixel inside a k-step: row of pixel 32 ks + c = (32 ks + c) / 24
  __device__ __forceinline__ int tbo(int ks, int h) const { return (int)((tb[ks >> 1][h] >> (16 * (ks & 1))) & 0xFFFFu); }
};
__device__ __forceinline__ void wl_frag(WlFrag& F, int lane, int mt0) {
  const int gq = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int clo = 4 * gq + q, chi = clo + 16;
  F.c[0] = clo;
  F.c[1] = chi;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int cb = 16 * (mt0 + i) + 4 * pp;
    F.aoffb[i] = (clo * C2 + ((((cb >> 3) ^ swz_dy(clo)) << 3) | (cb & 7))) * 2;
  }
#pragma unroll
  for (int m = 0; m < WL_KS / 2; ++m)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t v = 0;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int p = 32 * (2 * m + e) + (h ? chi : clo), r = p / H2;
        v |= (uint32_t)((p + 2 * r) * 32 + 8 * pp) << (16 * e);   // a1 pixel p + 2r of the 26-wide tile
      }
      F.tb[m][h] = v;
    }
}

// MFMA loop of one staged chunk: n-tiles NT0..NT0+NN-1 of co-tiles mt0, mt0+1 (acc[i][j]); BIAS bit i:
// also accumulate co-tile mt0+i against a tile of ones (the conv2 bias gradient, every column equal)
// (NB = 1: the one bias tile goes to accb[0]).  A lane row is past the image boundary when its dy row
// (32 ks + c) / 24 >= bnd, i.e. c >= 24 bnd - 32 ks (a scalar per k-step)
template <int NT0, int NN, int BIAS, int NJ, int NB>
__device__ __forceinline__ void wl_mfma(const unsigned char* buf, int nks, int bnd, const WlFrag& F,
                                        floatx4 (&acc)[2][NJ], floatx4 (&accb)[NB]) {
  const unsigned char* pa[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) pa[i][h] = buf + F.aoffb[i] + h * 16 * C2 * 2;
  const u32x4 ones_u = {0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u};
  const bf16x8 ones = __builtin_bit_cast(bf16x8, ones_u);
#pragma unroll
  for (int ks = 0; ks < WL_KS; ++ks) {
    if (ks < nks) {                                       // wave-uniform
      bf16x8 A[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        A[i] = tr_frag(reinterpret_cast<const uint16_t*>(pa[i][0] + ks * 32 * C2 * 2),
                       reinterpret_cast<const uint16_t*>(pa[i][1] + ks * 32 * C2 * 2));
      const unsigned char* pb[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) pb[h] = buf + WDY_BYTES + F.tbo(ks, h) + (F.c[h] >= H2 * bnd - 32 * ks ? 52 * 32 : 0);
#pragma unroll
      for (int j = 0; j < NN; ++j) {
        const int nt = NT0 + j, t = nt >> 1;
        const int toffb = ((t / 3) * H1 + (t % 3)) * 32 + (nt & 1) * WL_PLANE;
        const bf16x8 Bf = tr_frag(reinterpret_cast<const uint16_t*>(pb[0] + toffb),
                                  reinterpret_cast<const uint16_t*>(pb[1] + toffb));
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][j] = mfma16x16x32(A[i], Bf, acc[i][j]);
        // NN = 9 (staggered form): at most 3 B fragments in flight, which keeps the kernel at
        // <= 224 VGPRs (two waves per SIMD then leave 64 registers a lane for the comm stream's fc
        // Adadelta waves, 61 VGPRs; at 250 they could not co-reside and the overlapped update was held
        // back until wgrad ended: B = 8192 0.986 -> 1.051 ms/step)
        if (NN == 9 && j % 3 == 2) __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
        if (BIAS & (1 << i)) accb[NB == 1 ? 0 : i] = mfma16x16x32(A[i], ones, accb[NB == 1 ? 0 : i]);
    }
  }
}

}  // namespace

__global__ __launch_bounds__(WG_THREADS) void conv2_wgrad_lean_kernel(ConvBwdArgs a, int B) {
  TL_SCOPE(TL_WGRAD);
  __shared__ __attribute__((aligned(16))) unsigned char smem[WG_LDS];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // 8 waves = 2 co-tile pairs x 4 groups of the 18 (tap, ci-half) n-tiles (5, 5, 4, 4); the two
  // waves of group 2 also carry the bias tile (10 MFMAs per k-step like groups 0 and 1)
  const int mt0 = 2 * (wave & 1), ng = wave >> 1;
  const int nt0 = (ng < 2) ? 5 * ng : 10 + 4 * (ng - 2), nn = (ng < 2) ? 5 : 4;
  const int G = gridDim.x, g = blockIdx.x;
  if (a.signal_ctr && g == 0 && tid == 0)
    (RW_SIGNAL(), __hip_atomic_fetch_add(a.signal_ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT));
  RW_ENTRY();
  const int rows = H2 * B;
  const int r0 = (int)((int64_t)g * rows / G), r1 = (int)((int64_t)(g + 1) * rows / G);
  const int nchunks = (r1 - r0 + WG_CH - 1) / WG_CH;

  WlPlanT<WG_THREADS> P;
  wl_plan(P, tid, r0);
  WlChunkT<WG_THREADS> k;
  WlFrag F;
  wl_frag(F, lane, mt0);
  floatx4 acc[2][5], accb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    accb[i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  WG_MARK(0);
  if (nchunks > 0) {
    wl_fetch(a, P, tid, r0, min(r0 + WG_CH, r1), k);
    wl_store(P, smem, tid, r0, min(r0 + WG_CH, r1), k);
  }
  __syncthreads();
  WG_MARK(1);
  for (int ch = 0; ch < nchunks; ++ch) {
    const int c0 = r0 + ch * WG_CH, c1 = min(c0 + WG_CH, r1);
    const bool more = ch + 1 < nchunks;
    if (more) wl_fetch(a, P, tid, c1, min(c1 + WG_CH, r1), k);   // in flight under the MFMAs
    const unsigned char* buf = smem + (ch & 1) * WBUF_BYTES;
    const int nks = ((c1 - c0) * H2 + 31) / 32;
    const int bnd = H2 - (c0 - (c0 / H2) * H2);             // first chunk row of the next image
    switch (ng) {                                           // wave-uniform
      case 0: wl_mfma<0, 5, 0>(buf, nks, bnd, F, acc, accb); break;
      case 1: wl_mfma<5, 5, 0>(buf, nks, bnd, F, acc, accb); break;
      case 2: wl_mfma<10, 4, 3>(buf, nks, bnd, F, acc, accb); break;
      default: wl_mfma<14, 4, 0>(buf, nks, bnd, F, acc, accb); break;
    }
#ifdef MNIST_WGRAD_PHASE_TIMING
    if (ch == 0) { WG_MARK(2); }
#endif
    if (more) wl_store(P, smem + ((ch + 1) & 1) * WBUF_BYTES, tid, c1, min(c1 + WG_CH, r1), k);
    __syncthreads();
#ifdef MNIST_WGRAD_PHASE_TIMING
    if (ch == 0) { WG_MARK(3); }
#endif
  }
  WG_MARK(4);
  float* out = a.w2part + (int64_t)g * W2PART_STRIDE;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j)
      if (j < nn) {
        const int tile = (mt0 + i) * 18 + nt0 + j;
        store16(B <= WT_MAX_B, out, (int64_t)((tile * 64 + lane) * 4) * 4, acc[i][j]);   // slabs
      }
  // bias: column 0 of the ones-tile accumulators (every column holds the same row sums)
  if (ng == 2 && (lane & 15) == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      store16(B <= WT_MAX_B, out, (int64_t)(18432 + 16 * (mt0 + i) + 4 * (lane >> 4)) * 4, accb[i]);
  }
  WG_MARK(5);
}

// conv2_wgrad, staggered halves (B >= 342), VALU-lean: conv2_wgrad_stag_kernel's schedule (two
// 4-wave halves alternating MFMA and staging phases on alternate chunks, half 1 handing its sums to
// half 0 at the end) on the lean staging plan, fragment bases and planar a1 tile of
// conv2_wgrad_lean_kernel.  Each wave carries one bias tile (co-tile mt0 + hw/2: 19 MFMAs per
// k-step on every wave).
// <= 224 VGPRs: two waves per SIMD then leave 64 registers a lane, so the comm stream's fc Adadelta
// waves (61 VGPRs) stay co-resident under it (at 250 they could not, and the overlapped update was
// held back until wgrad ended: B = 8192 0.986 -> 1.051 ms/step)
__global__ __launch_bounds__(WG_THREADS) void conv2_wgrad_lstag_kernel(ConvBwdArgs a, int B) {
  TL_SCOPE(TL_WGRAD);
  __shared__ __attribute__((aligned(16))) unsigned char smem[WG_LDS];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int half = wave >> 2, hw = wave & 3, htid = tid & 255;
  const int mt0 = 2 * (hw & 1), nt0 = 9 * (hw >> 1);
  const int G = gridDim.x, g = blockIdx.x;
  if (a.signal_ctr && g == 0 && tid == 0)
    (RW_SIGNAL(), __hip_atomic_fetch_add(a.signal_ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT));
  RW_ENTRY();
  const int rows = H2 * B;
  const int r0 = (int)((int64_t)g * rows / G), r1 = (int)((int64_t)(g + 1) * rows / G);
  const int nchunks = (r1 - r0 + WG_CH - 1) / WG_CH;

  floatx4 acc[2][9], accb[1] = {floatx4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  WlPlanT<256> P;
  wl_plan(P, htid, r0);
  WlChunkT<256> k;
  WlFrag F;
  wl_frag(F, lane, mt0);
  auto chunk_lo = [&](int ch) { return r0 + ch * WG_CH; };
  auto chunk_hi = [&](int ch) { return min(r0 + (ch + 1) * WG_CH, r1); };
  unsigned char* mybuf = smem + half * WBUF_BYTES;

  // prologue: half 0 stages chunk 0 and prefetches chunk 2; half 1 prefetches chunk 1
  if (half == 0) {
    if (nchunks > 0) {
      wl_fetch(a, P, htid, chunk_lo(0), chunk_hi(0), k);
      wl_store(P, mybuf, htid, chunk_lo(0), chunk_hi(0), k);
    }
    if (nchunks > 2) wl_fetch(a, P, htid, chunk_lo(2), chunk_hi(2), k);
  } else if (nchunks > 1) {
    wl_fetch(a, P, htid, chunk_lo(1), chunk_hi(1), k);
  }
  __syncthreads();
  for (int ph = 0; ph < nchunks; ++ph) {
    if ((ph & 1) == half) {                             // MFMAs of chunk ph (half-uniform)
      const int c0 = chunk_lo(ph), c1 = chunk_hi(ph);
      const int nks = ((c1 - c0) * H2 + 31) / 32;
      const int bnd = H2 - (c0 - (c0 / H2) * H2);
      switch (hw) {                                     // wave-uniform
        case 0: wl_mfma<0, 9, 1>(mybuf, nks, bnd, F, acc, accb); break;
        case 1: wl_mfma<0, 9, 1>(mybuf, nks, bnd, F, acc, accb); break;
        case 2: wl_mfma<9, 9, 2>(mybuf, nks, bnd, F, acc, accb); break;
        default: wl_mfma<9, 9, 2>(mybuf, nks, bnd, F, acc, accb); break;
      }
    } else if (ph + 1 < nchunks) {                      // stage chunk ph+1, prefetch chunk ph+3
      wl_store(P, mybuf, htid, chunk_lo(ph + 1), chunk_hi(ph + 1), k);
      if (ph + 3 < nchunks) wl_fetch(a, P, htid, chunk_lo(ph + 3), chunk_hi(ph + 3), k);
    }
    __syncthreads();
  }
  // half 1 -> half 0 through LDS ([hw][i][j][lane] float4 + [hw][lane] bias), half 0 adds in fixed order
  floatx4* xch = reinterpret_cast<floatx4*>(smem);
  floatx4* xb = xch + 4 * 18 * 64;
  static_assert((4 * 18 * 64 + 4 * 64) * 16 <= WG_LDS, "accumulator exchange fits the chunk buffers");
  const int bi = hw >> 1;                               // this wave's bias tile: co-tile mt0 + bi
  const floatx4 mb = accb[0];
  if (half == 1) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 9; ++j) xch[((hw * 2 + i) * 9 + j) * 64 + lane] = acc[i][j];
    xb[hw * 64 + lane] = mb;
  }
  __syncthreads();
  float* out = a.w2part + (int64_t)g * W2PART_STRIDE;
  if (half == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const floatx4 o = xch[((hw * 2 + i) * 9 + j) * 64 + lane];
        const floatx4 v = {acc[i][j][0] + o[0], acc[i][j][1] + o[1], acc[i][j][2] + o[2], acc[i][j][3] + o[3]};
        const int tile = (mt0 + i) * 18 + nt0 + j;
        store16(B <= WT_MAX_B, out, (int64_t)((tile * 64 + lane) * 4) * 4, v);   // slabs
      }
    if ((lane & 15) == 0) {
      const floatx4 o = xb[hw * 64 + lane];
      const floatx4 v = {mb[0] + o[0], mb[1] + o[1], mb[2] + o[2], mb[3] + o[3]};
      store16(B <= WT_MAX_B, out, (int64_t)(18432 + 16 * (mt0 + bi) + 4 * (lane >> 4)) * 4, v);
    }
  }
}

// --------------------------------------------------------------------------------------------
// Stand-alone reduce (the DDP schedule all-reduces the conv bucket between it and the update).
__global__ __launch_bounds__(256) void conv_grad_reduce_kernel(ConvBwdArgs a, int B, int bid0) {
  TL_SCOPE(TL_CONV_REDUCE);
  RW_ENTRY();
  __shared__ float4 red[256];
  float* grad = a.grad;
  reduce_conv_grads(a, B, blockIdx.x + bid0, red, [grad](int64_t e, float v) { grad[e] = v; });
}

static void launch_c1_prereduce(const ConvBwdArgs& a, int B, hipStream_t s);

// c1red[j] = sum of the conv1 partial rows [j*R, (j+1)*R) (R = ceil(4B / C1_PRE_SLABS)) in fixed
// order: thread (column, slice) sums rows slice, slice+3, ... in batches of 16 independent loads,
// then the 3 slices are added in order.
__global__ __launch_bounds__(256) void c1_prereduce_kernel(const float* __restrict__ c1part, int nslab,
                                                           float* __restrict__ c1red) {
  TL_SCOPE(TL_C1_PRE);
  RW_ENTRY();
  __shared__ float4 sh[240];
  const int j = blockIdx.x, tid = threadIdx.x;
  const int R = (nslab + C1_PRE_SLABS - 1) / C1_PRE_SLABS;
  const int r0 = j * R, r1 = min(r0 + R, nslab);
  const int col = tid % 80, sl = tid / 80;       // 80 float4 columns x 3 slices (240 threads)
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if (sl < 3) {
    const float4* src = reinterpret_cast<const float4*>(c1part) + col;
    for (int k0 = r0 + sl; k0 < r1; k0 += 3 * 16) {
      float4 v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int r = k0 + 3 * k;
        v[k] = (r < r1) ? src[(int64_t)r * 80] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) { t.x += v[k].x; t.y += v[k].y; t.z += v[k].z; t.w += v[k].w; }
    }
    sh[tid] = t;
  }
  __syncthreads();
  if (tid < 80) {
    const float4 a = sh[tid], b = sh[tid + 80], c = sh[tid + 160];
    reinterpret_cast<float4*>(c1red)[(int64_t)j * 80 + tid] =
        make_float4((a.x + b.x) + c.x, (a.y + b.y) + c.y, (a.z + b.z) + c.z, (a.w + b.w) + c.w);
  }
}

static void launch_c1_prereduce(const ConvBwdArgs& a, int B, hipStream_t s) {
  if (a.c1red) hipLaunchKernelGGL(c1_prereduce_kernel, dim3(C1_PRE_SLABS), dim3(256), 0, s, a.c1part, a.c1_rows, a.c1red);
}

void launch_conv_dgrad(const ConvBwdArgs& a, int B, hipStream_t s) {
  if (a.c1_rows != 4 * B) throw std::runtime_error("conv_dgrad: c1_rows must be conv_dgrad_c1_rows(B)");
  const dim3 g(dgrad_persist_grid(B, a.dgrad_full_grid != 0));
  if (a.xin)
    hipLaunchKernelGGL((conv2_dgrad_persist_kernel<DGX_XIN>), g, dim3(256), 0, s, a, B);
  else if (a.idx)
    hipLaunchKernelGGL((conv2_dgrad_persist_kernel<DGX_IDX>), g, dim3(256), 0, s, a, B);
  else
    hipLaunchKernelGGL((conv2_dgrad_persist_kernel<DGX_PRE>), g, dim3(256), 0, s, a, B);
  launch_c1_prereduce(a, B, s);
}
// Staggered halves pay once every half has >= 2 chunks of its own (rows per workgroup >= 32, i.e.
// B >= 342 at 256 groups): measured B = 8192 1263-1266 -> 1214-1216 us/step, B = 2048 367-370 ->
// 355-363; at B = 200 (2-3 chunks per workgroup) the single-buffer-pair form stays (78.5-78.9 vs
// 80.3-80.8).  set_wgrad_form(0 / 1) forces either form (tests: the two forms agree), -1 = by batch.
static int g_wgrad_form = -1;
void set_wgrad_form(int f) { g_wgrad_form = (f == 0 || f == 1) ? f : -1; }
static bool wgrad_staggered(const ConvBwdArgs& a, int B) {
  if (g_wgrad_form >= 0) return g_wgrad_form == 1;
  return (int64_t)H2 * B >= (int64_t)4 * WG_CH * a.wgrad_groups;
}
void launch_conv_wgrad(const ConvBwdArgs& a, int B, hipStream_t s) {
  if (wgrad_staggered(a, B))
    hipLaunchKernelGGL(conv2_wgrad_lstag_kernel, dim3(a.wgrad_groups), dim3(WG_THREADS), 0, s, a, B);
  else
    hipLaunchKernelGGL(conv2_wgrad_lean_kernel, dim3(a.wgrad_groups), dim3(WG_THREADS), 0, s, a, B);
}
void launch_conv_bwd(const ConvBwdArgs& a, int B, hipStream_t s) {
  launch_conv_dgrad(a, B, s);
  launch_conv_wgrad(a, B, s);
}

void launch_conv_grad_reduce(const ConvBwdArgs& a, int B, hipStream_t s) {
  hipLaunchKernelGGL(conv_grad_reduce_kernel, dim3(RED_WGS), dim3(256), 0, s, a, B, 0);
}
void launch_conv_grad_reduce_parts(const ConvBwdArgs& a, int B, int lo, int hi, hipStream_t s) {
  if (lo < 0 || hi > RED_WGS || lo >= hi) throw std::runtime_error("conv_grad_reduce: bad part range");
  hipLaunchKernelGGL(conv_grad_reduce_kernel, dim3(hi - lo), dim3(256), 0, s, a, B, lo);
}

TL_DEFINE_HOST(conv_bwd)

// load this translation unit's gfx950 code object now (startup prewarm thread) instead of at its
// first launch inside the timed run
void preload_conv_bwd() {
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&conv_grad_reduce_kernel));
}

}  // namespace mnist
