// Fused multi-tensor Adadelta over the flat fp32 parameter buffer + bf16 shadow-weight refresh.
//
// Replaces optim.Adadelta(model.parameters(), lr) .step() (reference mnist_ddp.py:176, :73), which on
// the GPU is a chain of ~11 torch._foreach_* kernels (torch/optim/adadelta.py _multi_tensor_adadelta),
// and the weight casts the forward would otherwise need.  Per element, in torch's foreach order:
//     sq  = sq*rho + (1-rho)*g*g
//     d   = sqrt(acc+eps) / sqrt(sq+eps) * g
//     acc = acc*rho + (1-rho)*d*d
//     p  += -lr * d
// One read of g, read-modify-write of sq/acc/p, and in the same pass the bf16 copies the next
// forward/backward consume are written in the layouts their MFMA fragments want:
//   fc1.weight -> w1 [128][9216] and w1t [9216][128] (64x32 tiles transposed through LDS),
//   conv2.weight -> w2f [64][9][32] and w2d [9][32][64].
// lr is read from device memory so a captured graph picks up StepLR changes.
#include "../include/device_utils.h"
#include "../include/kernels.h"
#include "../include/timeline.h"
#include "conv_grad_reduce.h"

#include <stdexcept>

namespace mnist {

namespace {
constexpr int FC1_TILES = 2 * (NFLAT / 32);                       // 576 64(o) x 32(i) tiles of fc1.weight
constexpr int64_t FC_TAIL_N = OFF_CONV1_W - OFF_FC1_B;            // 1472 (fc1.b, fc2.w, fc2.b + pad)
constexpr int64_t CONV_N = PARAM_TOTAL - OFF_CONV1_W;             // 18880
constexpr int CONV_WGS = (int)((CONV_N / 4 + 255) / 256);         // 19

// Per-element math: Ada (device_utils.h), contraction off so every launch path is bitwise equal.

template <bool UPDATE>
__device__ __forceinline__ void elementwise(const AdadeltaArgs& a, const Ada& ad, int64_t begin, int64_t n,
                                            int wg, int nwg) {
  for (int64_t v = (int64_t)wg * 256 + threadIdx.x; v < n / 4; v += (int64_t)nwg * 256) {
    const int64_t e = begin + 4 * v;
    float4 p = *reinterpret_cast<float4*>(a.param + e);
    if (UPDATE) {
      const float4 g = *reinterpret_cast<const float4*>(a.grad + e);
      float4 sq = *reinterpret_cast<float4*>(a.square_avg + e);
      float4 ac = *reinterpret_cast<float4*>(a.acc_delta + e);
      ad.step(p.x, g.x, sq.x, ac.x);
      ad.step(p.y, g.y, sq.y, ac.y);
      ad.step(p.z, g.z, sq.z, ac.z);
      ad.step(p.w, g.w, sq.w, ac.w);
      store16(a.wt, a.param, e * 4, make_floatx4(p));        // write-through: read by later kernels
      store16(a.wt, a.square_avg, e * 4, make_floatx4(sq));
      store16(a.wt, a.acc_delta, e * 4, make_floatx4(ac));
    }
    if (e + 3 >= OFF_CONV2_W && e < OFF_CONV2_W + C2 * C1 * 9) {
      conv2_shadow(a, e, p.x);
      conv2_shadow(a, e + 1, p.y);
      conv2_shadow(a, e + 2, p.z);
      conv2_shadow(a, e + 3, p.w);
    }
  }
}

template <bool UPDATE>
__device__ __forceinline__ void fc1_tile(const AdadeltaArgs& a, const Ada& ad, int tile, uint16_t* ts) {
  constexpr int TS = 72;  // padded LDS row (bf16 elements): ts[32 i][64 o]
  const int ot = tile / (NFLAT / 32), it = tile - ot * (NFLAT / 32);
  const int t = threadIdx.x;
  const int ol = t >> 2, ic = (t & 3) * 8;
  const int o = 64 * ot + ol, i0 = 32 * it;
  const int64_t e0 = OFF_FC1_W + (int64_t)o * NFLAT + i0 + ic;
  float4 p[2], g[2], sq[2], ac[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    p[j] = *reinterpret_cast<float4*>(a.param + e0 + 4 * j);
    if (UPDATE) {
      g[j] = *reinterpret_cast<const float4*>(a.grad + e0 + 4 * j);
      sq[j] = *reinterpret_cast<float4*>(a.square_avg + e0 + 4 * j);
      ac[j] = *reinterpret_cast<float4*>(a.acc_delta + e0 + 4 * j);
    }
  }
  float v[8];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (UPDATE) {
      ad.step(p[j].x, g[j].x, sq[j].x, ac[j].x);
      ad.step(p[j].y, g[j].y, sq[j].y, ac[j].y);
      ad.step(p[j].z, g[j].z, sq[j].z, ac[j].z);
      ad.step(p[j].w, g[j].w, sq[j].w, ac[j].w);
      store16(a.wt, a.param, (e0 + 4 * j) * 4, make_floatx4(p[j]));   // write-through (later kernels)
      store16(a.wt, a.square_avg, (e0 + 4 * j) * 4, make_floatx4(sq[j]));
      store16(a.wt, a.acc_delta, (e0 + 4 * j) * 4, make_floatx4(ac[j]));
    }
    v[4 * j] = p[j].x; v[4 * j + 1] = p[j].y; v[4 * j + 2] = p[j].z; v[4 * j + 3] = p[j].w;
  }
  uint4 lo;
  lo.x = pack2bf(v[0], v[1]); lo.y = pack2bf(v[2], v[3]); lo.z = pack2bf(v[4], v[5]); lo.w = pack2bf(v[6], v[7]);
  store16(a.wt, a.w1, ((int64_t)o * NFLAT + i0 + ic) * 2, lo);
#pragma unroll
  for (int j = 0; j < 8; ++j) ts[(ic + j) * TS + ol] = f2bf(v[j]);
  __syncthreads();
  const int il = t >> 3, oc = (t & 7) * 8;
  store16(a.wt, a.w1t, ((int64_t)(i0 + il) * NH + 64 * ot + oc) * 2, *reinterpret_cast<const uint4*>(ts + il * TS + oc));
}
}  // namespace

template <bool UPDATE>
__global__ __launch_bounds__(256) void adadelta_kernel(AdadeltaArgs a, int region) {
  TL_SCOPE(region == ADA_FC ? TL_ADA_FC : region == ADA_CONV ? TL_ADA_CONV : TL_ADA_ALL);
  __shared__ __attribute__((aligned(16))) uint16_t ts[32 * 72];
  Ada ad{a.rho, a.eps, a.weight_decay, UPDATE ? *a.lr : 0.0f};
  int bid = blockIdx.x;
  if (a.state_inc && !a.hold_a && bid == 0 && threadIdx.x == 0) a.state_inc->step += 1;
  if (a.signal_start && bid == 0 && threadIdx.x == 0)      // the previous launch on the stream is done
    (RW_SIGNAL(), __hip_atomic_fetch_add(a.signal_start, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT));
  RW_ENTRY();
  bool done = false;
  if (region == ADA_FC && gridDim.x < FC1_TILES + 1) {
    // fc bucket on fewer workgroups than tiles (grid-stride): the overlapped single-GPU / RCCL update
    // runs beside wgrad / dgrad and only has to finish before the next step's trunk_fwd ends
    for (int t = bid; t < FC1_TILES + 1; t += gridDim.x) {
      if (t < FC1_TILES) fc1_tile<UPDATE>(a, ad, t, ts);
      else elementwise<UPDATE>(a, ad, OFF_FC1_B, FC_TAIL_N, 0, 1);
      __syncthreads();                            // ts is rewritten by the next tile
    }
    done = true;
  } else if (region != ADA_CONV) {
    if (bid < FC1_TILES) {
      fc1_tile<UPDATE>(a, ad, bid, ts);
      done = true;
    } else {
      bid -= FC1_TILES;
      if (bid == 0) {
        elementwise<UPDATE>(a, ad, OFF_FC1_B, FC_TAIL_N, 0, 1);
        done = true;
      }
      bid -= 1;
    }
  }
  if (!done) elementwise<UPDATE>(a, ad, OFF_CONV1_W, CONV_N, bid, CONV_WGS);
  // optional completion hold (single-GPU OVERLAP chain: the fc update completes only once the
  // compute stream's dgrad has started, so conv2's reduce + update follows with no wait launch)
  if (a.hold_a && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0)
    spin_until_geq(a.hold_a, __hip_atomic_load(a.hold_b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + a.hold_delta,
                   a.hold_err);
}

// Single-GPU step tail in ONE launch: the fc-tile / fc-tail updates of adadelta_kernel next to the
// conv-gradient slab reduction, whose workgroups apply the update to each conv parameter as soon as
// its gradient is final (no grad round trip, no extra kernel boundary; both halves are memory-
// bound and overlap).  Same per-element math as the two-kernel path, so results are bitwise equal.
// conv_only: reduce + update parts [bid0, bid0 + grid) of the conv bucket only (the overlapped
// single-GPU schedule updates the fc parameters on the comm stream and splits conv2 / conv1)
__global__ __launch_bounds__(256) void adadelta_reduce_kernel(AdadeltaArgs a, ConvBwdArgs c, int B, int conv_only,
                                                              int bid0) {
  TL_SCOPE(!conv_only ? TL_RED_ALL : bid0 < RED_W2_WGS ? TL_RED_CONV2 : TL_RED_CONV1);
  __shared__ __attribute__((aligned(16))) uint16_t ts[32 * 72];
  __shared__ float4 red[256];
  int bid = blockIdx.x;
  if (a.state_inc && !a.hold_a && bid == 0 && threadIdx.x == 0) a.state_inc->step += 1;
  if (a.signal_start && bid == 0 && threadIdx.x == 0)
    (RW_SIGNAL(), __hip_atomic_fetch_add(a.signal_start, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT));
  RW_ENTRY();
  if (!conv_only) {
    const Ada ad{a.rho, a.eps, a.weight_decay, *a.lr};
    if (bid < FC1_TILES) { fc1_tile<true>(a, ad, bid, ts); return; }
    bid -= FC1_TILES;
    if (bid == 0) { elementwise<true>(a, ad, OFF_FC1_B, FC_TAIL_N, 0, 1); return; }
    bid -= 1;
  }
  conv_reduce_update(a, c, B, bid + bid0, red);
  // single-GPU side-conv2 schedule: the step's last kernel completes only once the comm stream has
  // published this step's conv2 update, so the next trunk_fwd (stream order) reads the new weights
  // With a hold the step index advances after it: the comm stream's readers of this step's index
  // (fc_bwd's role C writing loss_log[step] in the side-weight-gradient schedule) are ordered before
  // the conv2 update that releases it.
  if (a.hold_a && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    spin_until_geq(a.hold_a, __hip_atomic_load(a.hold_b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), a.hold_err);
    if (a.state_inc) a.state_inc->step += 1;
  }
}

void launch_adadelta_reduce(const AdadeltaArgs& a, const ConvBwdArgs& c, int B, hipStream_t s) {
  hipLaunchKernelGGL(adadelta_reduce_kernel, dim3(FC1_TILES + 1 + RED_WGS), dim3(256), 0, s, a, c, B, 0, 0);
}

void launch_adadelta_reduce_parts(const AdadeltaArgs& a, const ConvBwdArgs& c, int B, int lo, int hi, hipStream_t s) {
  if (lo < 0 || hi > RED_WGS || lo >= hi) throw std::runtime_error("adadelta_reduce: bad part range");
  // (a 60-VGPR conv2-part kernel that fits beside the persistent dgrad's resident workgroups and so
  // runs under dgrad from its start measured slower than this one, which waits for dgrad's
  // one-item workgroups to retire: 600 steps 68.2-68.7 vs 67.1-67.8 us/step, same box)
  hipLaunchKernelGGL(adadelta_reduce_kernel, dim3(hi - lo), dim3(256), 0, s, a, c, B, 1, lo);
}

// conv1's reduce + update (the conv1 parts of adadelta_reduce_kernel, bitwise equal) on 80 one-wave
// workgroups: workgroup = one float4 column of the 320 conv1 gradient values, lane = slab slice.  Each
// lane sums rows slice, slice + 64, ... as the 256-thread parts do, and the fixed tree over the 64
// slices (slice s += slice s + w, w = 32 .. 1) runs on cross-lane moves instead of LDS round trips
// and barriers; the step's last compute launch at small batches, so its 20 x 4 KB-per-CU load bursts
// became 80 x 1 KB and its six barriers none.
__global__ __launch_bounds__(64) void adadelta_c1_kernel(AdadeltaArgs a, ConvBwdArgs c) {
  TL_SCOPE(TL_RED_CONV1);
  const int col = blockIdx.x, sl = threadIdx.x;
  if (a.state_inc && !a.hold_a && col == 0 && sl == 0) a.state_inc->step += 1;
  RW_ENTRY();
  const int nslab = c.c1red ? C1_PRE_SLABS : c.c1_rows;
  const float4* src = reinterpret_cast<const float4*>(c.c1red ? c.c1red : c.c1part) + col;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 t = z4;
  int64_t e[4];
  float pp[4], ps[4], pa[4], lr = 0.f;
  bool first = true;
  auto pre = [&] {                        // the update's operands, in flight with the slab loads
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 4 * col + r, ci = j / 10, kk = j - ci * 10;
      e[r] = kk < 9 ? (int64_t)OFF_CONV1_W + ci * 9 + kk : (int64_t)OFF_CONV1_B + ci;
      pp[r] = a.param[e[r]];
      ps[r] = a.square_avg[e[r]];
      pa[r] = a.acc_delta[e[r]];
    }
    lr = *a.lr;
  };
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
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {     // lanes >= w compute values nobody reads
    t.x += __shfl_down(t.x, w, 64);
    t.y += __shfl_down(t.y, w, 64);
    t.z += __shfl_down(t.z, w, 64);
    t.w += __shfl_down(t.w, w, 64);
  }
  if (sl == 0) {
    const float sc = c.grad_scale;
    const float o[4] = {t.x * sc, t.y * sc, t.z * sc, t.w * sc};
    const Ada ad{a.rho, a.eps, a.weight_decay, lr};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float p = pp[r], sq = ps[r], acc = pa[r];
      c.grad[e[r]] = o[r];                // the flat gradient buffer stays complete (p.grad views)
      ad.step(p, o[r], sq, acc);
      a.param[e[r]] = p;
      a.square_avg[e[r]] = sq;
      a.acc_delta[e[r]] = acc;
    }
  }
  // as adadelta_reduce_kernel: the launch completes only once the comm stream has published this
  // step's conv2 update, then the step index advances
  if (a.hold_a && col == gridDim.x - 1 && sl == 0) {
    spin_until_geq(a.hold_a, __hip_atomic_load(a.hold_b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), a.hold_err);
    if (a.state_inc) a.state_inc->step += 1;
  }
}

void launch_adadelta_c1(const AdadeltaArgs& a, const ConvBwdArgs& c, int B, hipStream_t s) {
  (void)B;
  hipLaunchKernelGGL(adadelta_c1_kernel, dim3(80), dim3(64), 0, s, a, c);
}

static int adadelta_grid(int region) {
  if (region == ADA_FC) return FC1_TILES + 1;
  if (region == ADA_CONV) return CONV_WGS;
  return FC1_TILES + 1 + CONV_WGS;
}

void launch_adadelta(const AdadeltaArgs& a, int region, hipStream_t s, int grid) {
  if (grid > 0 && (region != ADA_FC || grid > FC1_TILES + 1))
    throw std::runtime_error("adadelta: a reduced grid is for the fc region only");
  hipLaunchKernelGGL(adadelta_kernel<true>, dim3(grid > 0 ? grid : adadelta_grid(region)), dim3(256), 0, s, a, region);
}

void launch_refresh_shadows(const AdadeltaArgs& a, hipStream_t s) {
  AdadeltaArgs b = a;
  b.state_inc = nullptr;
  hipLaunchKernelGGL(adadelta_kernel<false>, dim3(adadelta_grid(ADA_ALL)), dim3(256), 0, s, b, (int)ADA_ALL);
}

__global__ void set_step_kernel(StepState* st, int step) { st->step = step; }
void launch_set_step(StepState* st, int step, hipStream_t s) {
  hipLaunchKernelGGL(set_step_kernel, dim3(1), dim3(1), 0, s, st, step);
}
// the whole StepState from kernel arguments: stream ordered, no host buffer to keep alive, no sync
__global__ void set_state_kernel(StepState* st, StepState v) { *st = v; }
void launch_set_state(StepState* st, const StepState& v, hipStream_t s) {
  hipLaunchKernelGGL(set_state_kernel, dim3(1), dim3(1), 0, s, st, v);
}

TL_DEFINE_HOST(adadelta)

// load this translation unit's gfx950 code object now (startup prewarm thread) instead of at its
// first launch inside the timed run
void preload_adadelta() {
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&set_step_kernel));
}

}  // namespace mnist
