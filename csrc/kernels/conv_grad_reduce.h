// Deterministic fixed-order reduction of the conv gradient partial slabs (shared by the stand-alone
// reduce kernel in conv_bwd.hip and the fused reduce+Adadelta launch in adadelta.hip).
// Latency-bound by construction (19 MB of partials at B=200, mostly MALL-resident), so every
// thread issues all of its float4 loads before the first add:
//   [0, 289): conv2 weight+bias slab columns, 16 float4 columns x 16 slab slices per WG
//             (<= 16 loads in flight per thread for G <= 256), fixed-order LDS tree over slices
//   [289, 309): conv1 weight+bias, 4 float4 columns x 64 slices of the c1_rows dgrad partials (or of
//               their C1_PRE_SLABS group sums, ConvBwdArgs::c1red)
// Each final (scaled) value is handed to sink(flat_element_index, value).
#pragma once
#include "../include/device_utils.h"
#include "../include/kernels.h"

namespace mnist {

constexpr int W2PART_STRIDE = 18432 + 64;
constexpr int RED_W2_WGS = (W2PART_STRIDE / 4 + 15) / 16;   // 289
constexpr int RED_C1_WGS = 320 / 16;                         // 20
constexpr int RED_WGS = RED_W2_WGS + RED_C1_WGS;             // 309
static_assert(RED_W2_WGS == RED_W2_PARTS && RED_WGS == RED_ALL_PARTS, "kernels.h mirrors the partition");

// Flat parameter index of the r-th (0..3) value lane `tid` of reduce block `bid` hands to the sink,
// or -1 (lanes that sink nothing, the padding column).  Shared with callers that prefetch the
// update's optimizer state before the slab loads complete.
__device__ __forceinline__ int64_t conv_sink_index(int bid, int tid, int r) {
  if (bid < RED_W2_WGS) {
    if ((tid >> 4) != 0) return -1;
    const int col = bid * 16 + (tid & 15), e = 4 * col;
    if (e < 18432) {
      // slab element e = ((mtile*18 + ntile)*64 + lane)*4 + r  ->  co, ci, tap
      const int ln = (e >> 2) & 63, tile = e >> 8;
      const int mtile = tile / 18, ntile = tile - mtile * 18;
      const int co0 = 16 * mtile + 4 * (ln >> 4);
      const int ci = 16 * (ntile & 1) + (ln & 15), tap = ntile >> 1;
      return (int64_t)OFF_CONV2_W + (co0 + r) * 288 + ci * 9 + tap;
    }
    if (e < 18432 + C2) return (int64_t)OFF_CONV2_B + (e - 18432) + r;
    return -1;
  }
  if ((tid >> 2) != 0) return -1;
  const int col = (bid - RED_W2_WGS) * 4 + (tid & 3);
  const int j = 4 * col + r, ci = j / 10, kk = j - ci * 10;
  return kk < 9 ? (int64_t)OFF_CONV1_W + ci * 9 + kk : (int64_t)OFF_CONV1_B + ci;
}

// All slab loads are unconditional (clamped row; the out-of-range values are replaced by 0 in the
// sum, as before) and issued before `pre()` - the caller's own loads (e.g. the optimizer state the
// sink updates) - so the sums wait for the slabs alone: a branch-guarded load would end in vmcnt(0)
// and split the kernel into dependent round trips.
template <class Pre, class Sink>
__device__ __forceinline__ void reduce_conv_grads(const ConvBwdArgs& a, int B, int bid, float4* red, Pre&& pre,
                                                  Sink&& sink) {
  const int tid = threadIdx.x;
  const float sc = a.grad_scale;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (bid < RED_W2_WGS) {
    const int G = a.wgrad_groups;
    const int col = bid * 16 + (tid & 15), sl = tid >> 4;          // float4 column, slab slice
    const float4* src = reinterpret_cast<const float4*>(a.w2part) + col;
    constexpr int S4 = W2PART_STRIDE / 4;
    float4 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int g = sl + 16 * k;
      v[k] = src[(int64_t)(g < G ? g : 0) * S4];
    }
    pre();
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (sl + 16 * k >= G) v[k] = z4;
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
    if (sl == 0 && 4 * col < 18432 + C2) {
      const float o[4] = {t.x * sc, t.y * sc, t.z * sc, t.w * sc};
#pragma unroll
      for (int r = 0; r < 4; ++r) sink(conv_sink_index(bid, tid, r), o[r]);
    }
  } else {
    const int col = (bid - RED_W2_WGS) * 4 + (tid & 3), sl = tid >> 2;   // 80 float4 columns, 64 slices
    const int nslab = a.c1red ? C1_PRE_SLABS : a.c1_rows;
    const float4* src = reinterpret_cast<const float4*>(a.c1red ? a.c1red : a.c1part) + col;
    float4 t = z4;
    bool first = true;
    for (int k0 = sl; k0 < nslab; k0 += 64 * 16) {
      float4 v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int r = k0 + 64 * k;
        v[k] = src[(int64_t)(r < nslab ? r : 0) * 80];
      }
      if (first) pre();
      first = false;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k0 + 64 * k >= nslab) v[k] = z4;
#pragma unroll
      for (int k = 0; k < 16; ++k) { t.x += v[k].x; t.y += v[k].y; t.z += v[k].z; t.w += v[k].w; }
    }
    if (first) pre();
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
      for (int r = 0; r < 4; ++r) sink(conv_sink_index(bid, tid, r), o[r]);
    }
  }
}

template <class Sink>
__device__ __forceinline__ void reduce_conv_grads(const ConvBwdArgs& a, int B, int bid, float4* red, Sink&& sink) {
  reduce_conv_grads(a, B, bid, red, [] {}, sink);
}

// bf16 shadows of one updated conv2.weight element: forward layout w2f [co][tap][ci] and dgrad
// layout w2d [tap][ci][co]
__device__ __forceinline__ void conv2_shadow(const AdadeltaArgs& a, int64_t e, float v) {
  const int rel = (int)(e - OFF_CONV2_W);
  if (rel < 0 || rel >= C2 * C1 * 9) return;
  const int co = rel / 288, rem = rel - co * 288, ci = rem / 9, t = rem - ci * 9;
  const uint16_t h = f2bf(v);
  a.w2f[(co * 9 + t) * C1 + ci] = h;
  a.w2d[(t * C1 + ci) * C2 + co] = h;
}

// Reduce part `bid` of the conv gradients and apply the Adadelta step to each finished element
// (grad buffer, param, optimizer state, bf16 shadows).  The optimizer state of the <= 4 elements a
// lane sinks is loaded before (and in flight with) the slab loads.
__device__ __forceinline__ void conv_reduce_update(const AdadeltaArgs& a, const ConvBwdArgs& c, int B, int bid,
                                                   float4* red) {
  float* gbuf = c.grad;
  float pp[4], ps[4], pa[4], lr = 0.f;
  auto pre = [&] {                      // issued right after the slab loads, unconditionally
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int64_t e = conv_sink_index(bid, threadIdx.x, r);
      e = e >= 0 ? e : OFF_CONV1_W;
      pp[r] = a.param[e];
      ps[r] = a.square_avg[e];
      pa[r] = a.acc_delta[e];
    }
    lr = *a.lr;
  };
  int k = 0;
  reduce_conv_grads(c, B, bid, red, pre, [&](int64_t e, float g) {
    const Ada ad{a.rho, a.eps, a.weight_decay, lr};
    gbuf[e] = g;                        // the flat gradient buffer stays complete (p.grad views)
    float p = pp[k], sq = ps[k], acc = pa[k];
    ++k;
    ad.step(p, g, sq, acc);
    a.param[e] = p;
    a.square_avg[e] = sq;
    a.acc_delta[e] = acc;
    conv2_shadow(a, e, p);
  });
}

}  // namespace mnist
