// Direct xGMI all-reduce for the DDP gradient buckets (runtime/xgmi_comm.cpp).
//
// MI355X GPUs in a node are fully connected by point-to-point xGMI links (7 per GPU), so a ring
// (what RCCL picks for a 4.7 MB bucket) drives only 2 of them per GPU and pays 2(W-1) latency-bound
// hops.  Here every rank maps every peer's bucket (IPC) and the sum is two direct phases:
//   phase 1 (reduce-scatter): rank r reads shard r of all W input buckets over the W-1 links at
//            once, sums them in rank order 0..W-1 (same bits on every rank, run to run) and writes
//            shard r of its OUTPUT bucket;
//   phase 2 (all-gather):     rank r reads shard p of rank p's output bucket for every p != r.
// Inputs and outputs are separate buffers, so the only hand-offs are "every rank's inputs are
// final" (stage 0) and "every rank's shard is reduced" (stage 1): a rank's next-step producer
// kernels overwrite only its input bucket, which peers read before stage 1 completes, and its
// next call writes its output shard only after stage 0 of that call (= after every peer left
// phase 2 of this one).
//
// Hand-offs are per workgroup: WG b of every rank covers the same index set in both phases, so WG b
// waits only for WG b of the peers (no grid-wide barrier, no co-residency requirement).  Payload
// loads/stores are buffer ops with sc0 sc1 (system-coherent: bypass this GPU's caches and write
// through), drained with s_waitcnt vmcnt(0) before the workgroup barrier that precedes the flag
// stores; flags are system-scope atomics carrying a per-WG call counter (monotonic, no reset, so
// graph replays need no host work).  A wait that exceeds the timeout sets *err and returns; every
// later call then returns at once and the host raises (XgmiComm::check).
#include "../include/device_utils.h"
#include "../include/kernels.h"
#include "conv_grad_reduce.h"

namespace mnist {

namespace {
typedef __attribute__((ext_vector_type(4))) float f4;
constexpr int SYS = 17;   // cache policy bits: sc0 | sc1 (system scope)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f4 ld_sys(__amdgpu_buffer_rsrc_t r, int64_t i) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 16), 0, SYS));
}
__device__ __forceinline__ void st_sys(__amdgpu_buffer_rsrc_t r, int64_t i, f4 v) {
  typedef __attribute__((ext_vector_type(4))) unsigned u4;
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), r, (int)(i * 16), 0, SYS);
}

// Stage hand-off of workgroup b: lane p (< world) publishes this WG's call counter into rank p's
// flag slot [stage][my rank][b], then polls its own slot [stage][p][b].  Returns false (and sets
// *err) on timeout.
__device__ bool xgmi_stage(const XgmiArgs& a, int stage, int b, int e) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's write-through stores are done
  __syncthreads();
  bool ok = true;
  const int p = threadIdx.x;
  if (p < a.world) {
    __hip_atomic_store(a.flags[p] + (stage * XGMI_MAX_RANKS + a.rank) * XGMI_MAX_WG + b, e, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    const int* slot = a.flags[a.rank] + (stage * XGMI_MAX_RANKS + p) * XGMI_MAX_WG + b;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();            // 100 MHz
    while (__hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
        __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
        break;
      }
    }
  }
  return __syncthreads_and(ok);
}
}  // namespace

// Fused Adadelta on one float4 of reduced gradients at flat parameter index e (+ conv2 bf16 shadows);
// pr / sq / ac are the element's current param / square_avg / acc_delta (loaded by the caller, so the
// one-shot kernel can issue those local loads before it waits for its peers)
__device__ __forceinline__ void ada_update4(const XgmiArgs& a, const Ada& ad, int64_t e, f4 g, float4 pr,
                                            float4 sq, float4 ac) {
  ad.step(pr.x, g.x, sq.x, ac.x);
  ad.step(pr.y, g.y, sq.y, ac.y);
  ad.step(pr.z, g.z, sq.z, ac.z);
  ad.step(pr.w, g.w, sq.w, ac.w);
  *reinterpret_cast<float4*>(a.ada.param + e) = pr;
  *reinterpret_cast<float4*>(a.ada.square_avg + e) = sq;
  *reinterpret_cast<float4*>(a.ada.acc_delta + e) = ac;
  const float pv[4] = {pr.x, pr.y, pr.z, pr.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {             // conv2.weight -> w2f [64][9][32], w2d [9][32][64]
    const int rel = (int)(e + q - OFF_CONV2_W);
    if (rel < 0 || rel >= C2 * C1 * 9) continue;
    const int co = rel / 288, rem = rel - co * 288, ci = rem / 9, t = rem - ci * 9;
    const uint16_t h = f2bf(pv[q]);
    a.ada.w2f[(co * 9 + t) * C1 + ci] = h;
    a.ada.w2d[(t * C1 + ci) * C2 + co] = h;
  }
}

// W is a template parameter so the per-peer loads unroll into one straight batch (a runtime
// `p < world` guard makes hipcc wait vmcnt(0) after every load).  Buffer ops are bounds-checked by
// the descriptor: loads past the bucket return 0 and stores past it are dropped, so the shard
// edges need no guards, and a zero-length descriptor turns a load into a no-op.
template <int W>
__global__ __launch_bounds__(256) void xgmi_allreduce_kernel(XgmiArgs a) {
  __shared__ int s_epoch, s_err;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) {
    const int e = a.ctr[b] + 1;          // only this lane of this WG touches ctr[b]; calls are stream ordered
    a.ctr[b] = e;
    s_epoch = e;
    s_err = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (s_err) return;
  const int e = s_epoch;
  const int r = a.rank;
  const int64_t S4 = (a.nvec + W - 1) / W;                 // float4s per shard
  const int64_t step = (int64_t)gridDim.x * 256;
  const int64_t bytes = a.nvec * 16;
  const __amdgpu_buffer_rsrc_t out = rsrc(a.out[r], bytes);

  if (!xgmi_stage(a, 0, b, e)) return;
  // ---- phase 1: shard r of the sum -> my output
  {
    __amdgpu_buffer_rsrc_t in[W];
#pragma unroll
    for (int p = 0; p < W; ++p) in[p] = rsrc(a.in[p], bytes);
    const int64_t hi = (r + 1) * S4;
    for (int64_t i = r * S4 + (int64_t)b * 256 + tid; i < hi; i += 2 * step) {
      const int64_t i2 = i + step;
      f4 v[W], w[W];
#pragma unroll
      for (int p = 0; p < W; ++p) {
        v[p] = ld_sys(in[p], i);
        w[p] = ld_sys(in[p], i2);
      }
      f4 s = v[0], t = w[0];
#pragma unroll
      for (int p = 1; p < W; ++p) {
        s += v[p];
        t += w[p];
      }
      st_sys(out, i, s);
      if (i2 < hi) st_sys(out, i2, t);
    }
  }
  if (!xgmi_stage(a, 1, b, e)) return;
  // ---- phase 2: every other rank's reduced shard -> my output (the same index set per WG)
  if (!a.fuse_ada) {
    __amdgpu_buffer_rsrc_t src[W];
#pragma unroll
    for (int p = 0; p < W; ++p) src[p] = rsrc(a.out[p], p == r ? 0 : bytes);   // own shard: no-op load
    for (int64_t k = (int64_t)b * 256 + tid; k < S4; k += step) {
      f4 v[W];
#pragma unroll
      for (int p = 0; p < W; ++p) v[p] = ld_sys(src[p], p * S4 + k);
#pragma unroll
      for (int p = 0; p < W; ++p)
        if (p != r) st_sys(out, p * S4 + k, v[p]);
    }
    return;
  }
  // fused Adadelta: the gathered sums (own shard re-read from the local output) are the gradients
  if (b == 0 && tid == 0 && a.ada.state_inc) a.ada.state_inc->step += 1;   // end-of-step marker
  const Ada ad{a.ada.rho, a.ada.eps, a.ada.weight_decay, *a.ada.lr};
  __amdgpu_buffer_rsrc_t src[W];
#pragma unroll
  for (int p = 0; p < W; ++p) src[p] = rsrc(a.out[p], bytes);
  for (int64_t k = (int64_t)b * 256 + tid; k < S4; k += step) {
    f4 v[W];
#pragma unroll
    for (int p = 0; p < W; ++p) v[p] = ld_sys(src[p], p * S4 + k);
#pragma unroll
    for (int p = 0; p < W; ++p) {
      const int64_t j = p * S4 + k;
      if (j >= a.nvec) continue;
      if (p != r) st_sys(out, j, v[p]);
      const int64_t e = a.ada_base + 4 * j;
      ada_update4(a, ad, e, v[p], *reinterpret_cast<float4*>(a.ada.param + e),
                  *reinterpret_cast<float4*>(a.ada.square_avg + e), *reinterpret_cast<float4*>(a.ada.acc_delta + e));
    }
  }
}

// One-shot: WG b owns the float4 index set {b*256 + tid + m*grid*256}.  It copies its part of this
// rank's input into staging slot (call parity) with write-through stores, publishes stage 0, then
// reads that part of every rank's slot and sums in rank order.  A slot is rewritten two calls later,
// after stage 0 of the call in between, i.e. after every peer's WG b finished reading it - so one
// hand-off per call suffices (the two-shot kernel needs two).
template <int W>
__global__ __launch_bounds__(256) void xgmi_oneshot_kernel(XgmiArgs a) {
  __shared__ int s_epoch, s_err;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) {
    const int e = a.ctr[b] + 1;
    a.ctr[b] = e;
    s_epoch = e;
    s_err = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (s_err) return;
  const int e = s_epoch, r = a.rank;
  const int64_t step = (int64_t)gridDim.x * 256, bytes = a.nvec * 16;
  const int64_t slot = (e & 1) * a.slot_floats;
  const int64_t k0 = (int64_t)b * 256 + tid;
  constexpr int KMAX = 4;                      // float4s per lane kept in registers (host-checked)
  f4 mine[KMAX];
  float4 pr[KMAX], sq[KMAX], ac[KMAX];           // fused update: local state loaded before the wait
#pragma unroll
  for (int m = 0; m < KMAX; ++m) {
    const int64_t k = k0 + m * step;
    if (k < a.nvec) {
      mine[m] = *reinterpret_cast<const f4*>(a.in[r] + 4 * k);
      st_sys(rsrc(a.stage[r] + slot, bytes), k, mine[m]);
      if (a.fuse_ada) {
        const int64_t el = a.ada_base + 4 * k;
        pr[m] = *reinterpret_cast<const float4*>(a.ada.param + el);
        sq[m] = *reinterpret_cast<const float4*>(a.ada.square_avg + el);
        ac[m] = *reinterpret_cast<const float4*>(a.ada.acc_delta + el);
      }
    }
  }
  if (!xgmi_stage(a, 0, b, e)) return;
  __amdgpu_buffer_rsrc_t src[W];
#pragma unroll
  for (int p = 0; p < W; ++p) src[p] = rsrc(a.stage[p] + slot, p == r ? 0 : bytes);   // own: registers
  if (a.fuse_ada && b == 0 && tid == 0 && a.ada.state_inc) a.ada.state_inc->step += 1;
  const Ada ad{a.ada.rho, a.ada.eps, a.ada.weight_decay, a.fuse_ada ? *a.ada.lr : 0.0f};
  const __amdgpu_buffer_rsrc_t out = rsrc(a.out[r], bytes);
#pragma unroll
  for (int m = 0; m < KMAX; ++m) {
    const int64_t k = k0 + m * step;
    if (k >= a.nvec) break;
    f4 v[W];
#pragma unroll
    for (int p = 0; p < W; ++p) v[p] = ld_sys(src[p], k);
    f4 s = (r == 0) ? mine[m] : v[0];
#pragma unroll
    for (int p = 1; p < W; ++p) s += (p == r) ? mine[m] : v[p];
    if (a.fuse_ada) ada_update4(a, ad, a.ada_base + 4 * k, s, pr[m], sq[m], ac[m]);
    else st_sys(out, k, s);
  }
}

void launch_xgmi_allreduce_oneshot(const XgmiArgs& a, hipStream_t s) {
  const dim3 g((unsigned)((a.nvec + 255) / 256 < XGMI_MAX_WG ? (a.nvec + 255) / 256 : XGMI_MAX_WG)), blk(256);
  switch (a.world) {
    case 1: hipLaunchKernelGGL(xgmi_oneshot_kernel<1>, g, blk, 0, s, a); break;
    case 2: hipLaunchKernelGGL(xgmi_oneshot_kernel<2>, g, blk, 0, s, a); break;
    case 3: hipLaunchKernelGGL(xgmi_oneshot_kernel<3>, g, blk, 0, s, a); break;
    case 4: hipLaunchKernelGGL(xgmi_oneshot_kernel<4>, g, blk, 0, s, a); break;
    case 5: hipLaunchKernelGGL(xgmi_oneshot_kernel<5>, g, blk, 0, s, a); break;
    case 6: hipLaunchKernelGGL(xgmi_oneshot_kernel<6>, g, blk, 0, s, a); break;
    case 7: hipLaunchKernelGGL(xgmi_oneshot_kernel<7>, g, blk, 0, s, a); break;
    case 8: hipLaunchKernelGGL(xgmi_oneshot_kernel<8>, g, blk, 0, s, a); break;
    default: break;
  }
}

// ---------------------------------------------------------------------------------------------
// fc bucket with the fc Adadelta step fused (two-shot).  The unit of work is a 64(o) x 32(i) tile
// of fc1.weight (576 tiles) plus one pseudo-tile for the tail (fc1.b, fc2.w, fc2.b; 368 float4):
// shard p = units [p*577/W, (p+1)*577/W).  Phase 1: WG b reduces units b, b+G, .. of shard r (rank
// order) into its output bucket; stage 1; phase 2: WG b gathers units b, b+G, .. of EVERY shard
// (all loads in flight at once), applies Ada::step with the gathered sums as gradients and writes
// param / square_avg / acc_delta plus the bf16 shadows w1 [128][9216] and w1t [9216][128] (tile
// transposed through LDS) - exactly the adadelta kernel's fc1 tile math, so bitwise equal to the
// all-reduce + separate update it replaces.  The fc branch of the DDP step loses a launch and a
// 4.7 MB gradient re-read.
namespace {
constexpr int FCU_TILES = 2 * (NFLAT / 32);                      // 576
constexpr int FCU_UNITS = FCU_TILES + 1;                         // + tail
constexpr int FCU_TAIL_F4 = (int)((OFF_CONV1_W - OFF_FC1_B) / 4);  // 368
constexpr int FCU_TS = 72;                                       // padded LDS row (bf16) of a tile

__device__ __forceinline__ int fcu_lo(int p, int W) { return p * FCU_UNITS / W; }
// float4 index (in the bucket) of this thread's h-th float4 of unit u (h = 0, 1)
__device__ __forceinline__ int fcu_f4(int u, int h, int tid) {
  if (u < FCU_TILES) {
    const int ot = u / (NFLAT / 32), it = u - ot * (NFLAT / 32);
    const int o = 64 * ot + (tid >> 2), i = 32 * it + (tid & 3) * 8;
    return (o * NFLAT + i) / 4 + h;
  }
  const int q = tid + 256 * h;                                   // tail: 368 float4
  return q < FCU_TAIL_F4 ? (int)(OFF_FC1_B / 4) + q : -1;
}
}  // namespace

template <int W>
__global__ __launch_bounds__(256) void xgmi_fc_fused_kernel(XgmiArgs a) {
  constexpr int UMAX = W == 1 ? 3 : W == 2 ? 2 : 1;              // units per shard per WG (host grid)
  __shared__ int s_epoch, s_err;
  __shared__ __attribute__((aligned(16))) uint16_t ts[W * UMAX][32 * FCU_TS];
  const int b = blockIdx.x, tid = threadIdx.x, G = gridDim.x;
  if (tid == 0) {
    const int e = a.ctr[b] + 1;
    a.ctr[b] = e;
    s_epoch = e;
    s_err = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (s_err) return;
  const int e = s_epoch, r = a.rank;
  const int64_t bytes = a.nvec * 16;
  const __amdgpu_buffer_rsrc_t out = rsrc(a.out[r], bytes);
  if (!xgmi_stage(a, 0, b, e)) return;
  // ---- phase 1: my shard's units, rank-order sums -> my output
  {
    __amdgpu_buffer_rsrc_t in[W];
#pragma unroll
    for (int p = 0; p < W; ++p) in[p] = rsrc(a.in[p], bytes);
    const int lo = fcu_lo(r, W), hi = fcu_lo(r + 1, W);
#pragma unroll
    for (int m = 0; m < UMAX; ++m) {
      const int u = lo + b + m * G;
      if (u >= hi) break;
      f4 v[2][W];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int q = fcu_f4(u, h, tid);
#pragma unroll
        for (int p = 0; p < W; ++p) v[h][p] = ld_sys(in[p], q < 0 ? a.nvec : q);   // q < 0: past the end -> 0
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int q = fcu_f4(u, h, tid);
        f4 t = v[h][0];
#pragma unroll
        for (int p = 1; p < W; ++p) t += v[h][p];
        if (q >= 0) st_sys(out, q, t);
      }
    }
  }
  if (!xgmi_stage(a, 1, b, e)) return;
  // ---- phase 2: every shard's units of this WG, PG shards at a time: gathered sums + local
  // optimizer state all in flight per group.  PG bounds the registers (~100 VGPRs) so this kernel,
  // which runs on the comm stream beside the conv backward, co-resides with wgrad / dgrad
  // workgroups instead of taking whole CUs from them.
  const Ada ad{a.ada.rho, a.ada.eps, a.ada.weight_decay, *a.ada.lr};
  constexpr int PG = W < 2 ? W : 2;
#pragma unroll
  for (int p0 = 0; p0 < W; p0 += PG) {
    f4 g[PG][UMAX][2];
    float4 pr[PG][UMAX][2], sq[PG][UMAX][2], ac[PG][UMAX][2];
#pragma unroll
    for (int pp = 0; pp < PG; ++pp) {
      const int p = p0 + pp;
      if (p >= W) break;
      const __amdgpu_buffer_rsrc_t src = rsrc(a.out[p], bytes);
#pragma unroll
      for (int m = 0; m < UMAX; ++m) {
        const int u = fcu_lo(p, W) + b + m * G;
        if (u >= fcu_lo(p + 1, W)) continue;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int q = fcu_f4(u, h, tid);
          if (q < 0) continue;
          g[pp][m][h] = ld_sys(src, q);
          pr[pp][m][h] = reinterpret_cast<const float4*>(a.ada.param)[q];
          sq[pp][m][h] = reinterpret_cast<const float4*>(a.ada.square_avg)[q];
          ac[pp][m][h] = reinterpret_cast<const float4*>(a.ada.acc_delta)[q];
        }
      }
    }
#pragma unroll
    for (int pp = 0; pp < PG; ++pp) {
      const int p = p0 + pp;
      if (p >= W) break;
#pragma unroll
      for (int m = 0; m < UMAX; ++m) {
        const int u = fcu_lo(p, W) + b + m * G;
        if (u >= fcu_lo(p + 1, W)) continue;
        float v8[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int q = fcu_f4(u, h, tid);
          if (q < 0) continue;
          float4 P = pr[pp][m][h], S = sq[pp][m][h], A = ac[pp][m][h];
          const f4 G4 = g[pp][m][h];
          ad.step(P.x, G4.x, S.x, A.x);
          ad.step(P.y, G4.y, S.y, A.y);
          ad.step(P.z, G4.z, S.z, A.z);
          ad.step(P.w, G4.w, S.w, A.w);
          reinterpret_cast<float4*>(a.ada.param)[q] = P;
          reinterpret_cast<float4*>(a.ada.square_avg)[q] = S;
          reinterpret_cast<float4*>(a.ada.acc_delta)[q] = A;
          v8[4 * h] = P.x; v8[4 * h + 1] = P.y; v8[4 * h + 2] = P.z; v8[4 * h + 3] = P.w;
        }
        if (u < FCU_TILES) {                                        // bf16 shadows of the fc1 tile
          const int ot = u / (NFLAT / 32), it = u - ot * (NFLAT / 32);
          const int ol = tid >> 2, ic = (tid & 3) * 8, o = 64 * ot + ol, i0 = 32 * it;
          uint4 lo4;
          lo4.x = pack2bf(v8[0], v8[1]); lo4.y = pack2bf(v8[2], v8[3]);
          lo4.z = pack2bf(v8[4], v8[5]); lo4.w = pack2bf(v8[6], v8[7]);
          *reinterpret_cast<uint4*>(a.ada.w1 + (int64_t)o * NFLAT + i0 + ic) = lo4;
          uint16_t* t = ts[p * UMAX + m];
#pragma unroll
          for (int j = 0; j < 8; ++j) t[(ic + j) * FCU_TS + ol] = f2bf(v8[j]);
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < W; ++p) {
#pragma unroll
    for (int m = 0; m < UMAX; ++m) {
      const int u = fcu_lo(p, W) + b + m * G;
      if (u >= fcu_lo(p + 1, W) || u >= FCU_TILES) continue;
      const int ot = u / (NFLAT / 32), it = u - ot * (NFLAT / 32);
      const int il = tid >> 3, oc = (tid & 7) * 8;
      *reinterpret_cast<uint4*>(a.ada.w1t + (int64_t)(32 * it + il) * NH + 64 * ot + oc) =
          *reinterpret_cast<const uint4*>(ts[p * UMAX + m] + il * FCU_TS + oc);
    }
  }
}

int xgmi_fc_fused_workgroups(int world) {
  const int per = (FCU_UNITS + world - 1) / world;
  return per < XGMI_MAX_WG ? per : XGMI_MAX_WG;
}

void launch_xgmi_fc_fused(const XgmiArgs& a, hipStream_t s) {
  const dim3 g(xgmi_fc_fused_workgroups(a.world)), blk(256);
  switch (a.world) {
    case 1: hipLaunchKernelGGL(xgmi_fc_fused_kernel<1>, g, blk, 0, s, a); break;
    case 2: hipLaunchKernelGGL(xgmi_fc_fused_kernel<2>, g, blk, 0, s, a); break;
    case 3: hipLaunchKernelGGL(xgmi_fc_fused_kernel<3>, g, blk, 0, s, a); break;
    case 4: hipLaunchKernelGGL(xgmi_fc_fused_kernel<4>, g, blk, 0, s, a); break;
    case 5: hipLaunchKernelGGL(xgmi_fc_fused_kernel<5>, g, blk, 0, s, a); break;
    case 6: hipLaunchKernelGGL(xgmi_fc_fused_kernel<6>, g, blk, 0, s, a); break;
    case 7: hipLaunchKernelGGL(xgmi_fc_fused_kernel<7>, g, blk, 0, s, a); break;
    case 8: hipLaunchKernelGGL(xgmi_fc_fused_kernel<8>, g, blk, 0, s, a); break;
    default: break;
  }
}

// ---------------------------------------------------------------------------------------------
// conv bucket, fully fused: WG b runs conv_grad_reduce's WG b (same slab partition and summation
// order -> the same bits), keeps its <= 4 finished gradients per lane in registers, publishes them
// into this rank's staging slot (call parity; 4-byte write-through stores at their bucket index),
// hands off once (stage 0: WG b of every rank is done with the same indices), then sums every
// rank's values at those indices in rank order and applies Ada::step + the conv2 bf16 shadows.
// Replaces conv_grad_reduce + the one-shot all-reduce: one launch less on the DDP critical path.
namespace {
__device__ __forceinline__ void st_sys1(__amdgpu_buffer_rsrc_t r, int64_t i, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), r, (int)(i * 4), 0, SYS);
}
__device__ __forceinline__ float ld_sys1(__amdgpu_buffer_rsrc_t r, int64_t i) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)(i * 4), 0, SYS));
}
}  // namespace

template <int W>
__global__ __launch_bounds__(256) void xgmi_conv_reduce_fused_kernel(XgmiArgs a, ConvBwdArgs c, int B) {
  __shared__ float4 red[256];
  __shared__ int s_epoch, s_err;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) {
    const int e = a.ctr[b] + 1;
    a.ctr[b] = e;
    s_epoch = e;
    s_err = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // (s_err is read after the reduce's barriers; a poisoned communicator skips the exchange)
  float vals[4];
  int64_t idx[4];
  int nv = 0;
  reduce_conv_grads(c, B, b, red, [&](int64_t el, float v) {
    vals[nv] = v;
    idx[nv] = el - a.ada_base;
    ++nv;
  });
  __syncthreads();
  if (s_err) return;
  const int e = s_epoch, r = a.rank;
  const int64_t slot = (e & 1) * a.slot_floats;
  const int64_t bytes = a.nvec * 16;
  {
    const __amdgpu_buffer_rsrc_t mine = rsrc(a.stage[r] + slot, bytes);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < nv) st_sys1(mine, idx[k], vals[k]);
  }
  // the update's local state, loaded before the hand-off wait
  float pr[4], sq[4], ac[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (k < nv) {
      const int64_t el = a.ada_base + idx[k];
      pr[k] = a.ada.param[el];
      sq[k] = a.ada.square_avg[el];
      ac[k] = a.ada.acc_delta[el];
    }
  if (!xgmi_stage(a, 0, b, e)) return;
  if (b == 0 && tid == 0 && a.ada.state_inc) a.ada.state_inc->step += 1;   // end-of-step marker
  if (nv == 0) return;
  __amdgpu_buffer_rsrc_t src[W];
#pragma unroll
  for (int p = 0; p < W; ++p) src[p] = rsrc(a.stage[p] + slot, p == r ? 0 : bytes);   // own: registers
  float v[4][W];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int p = 0; p < W; ++p) v[k][p] = ld_sys1(src[p], k < nv ? idx[k] : 0);
  const Ada ad{a.ada.rho, a.ada.eps, a.ada.weight_decay, *a.ada.lr};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k >= nv) break;
    float g = (r == 0) ? vals[k] : v[k][0];
#pragma unroll
    for (int p = 1; p < W; ++p) g += (p == r) ? vals[k] : v[k][p];
    const int64_t el = a.ada_base + idx[k];
    float P = pr[k], S = sq[k], A = ac[k];
    ad.step(P, g, S, A);
    a.ada.param[el] = P;
    a.ada.square_avg[el] = S;
    a.ada.acc_delta[el] = A;
    const int rel = (int)(el - OFF_CONV2_W);
    if (rel >= 0 && rel < C2 * C1 * 9) {
      const int co = rel / 288, rem = rel - co * 288, ci = rem / 9, t = rem - ci * 9;
      const uint16_t h = f2bf(P);
      a.ada.w2f[(co * 9 + t) * C1 + ci] = h;
      a.ada.w2d[(t * C1 + ci) * C2 + co] = h;
    }
  }
}

void launch_xgmi_conv_reduce_fused(const XgmiArgs& a, const ConvBwdArgs& c, int B, hipStream_t s) {
  static_assert(RED_WGS <= XGMI_MAX_WG, "one flag slot per reduce workgroup");
  const dim3 g(RED_WGS), blk(256);
  switch (a.world) {
    case 1: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<1>, g, blk, 0, s, a, c, B); break;
    case 2: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<2>, g, blk, 0, s, a, c, B); break;
    case 3: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<3>, g, blk, 0, s, a, c, B); break;
    case 4: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<4>, g, blk, 0, s, a, c, B); break;
    case 5: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<5>, g, blk, 0, s, a, c, B); break;
    case 6: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<6>, g, blk, 0, s, a, c, B); break;
    case 7: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<7>, g, blk, 0, s, a, c, B); break;
    case 8: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<8>, g, blk, 0, s, a, c, B); break;
    default: break;
  }
}

int xgmi_workgroups(int64_t nvec, int world, bool fuse_ada) {
  const int64_t s4 = (nvec + world - 1) / world;
  // >= 2 float4 per lane per phase-1 pass; with the fused update (W elementwise Adadelta steps per
  // index) spread wider so its dependent load -> update -> store chains run on more CUs
  int64_t g = fuse_ada ? (s4 + 127) / 128 : (s4 + 511) / 512;
  if (g < 1) g = 1;
  if (g > XGMI_MAX_WG) g = XGMI_MAX_WG;
  return (int)g;
}

void launch_xgmi_allreduce(const XgmiArgs& a, hipStream_t s) {
  const dim3 g(xgmi_workgroups(a.nvec, a.world, a.fuse_ada != 0)), blk(256);
  switch (a.world) {
    case 1: hipLaunchKernelGGL(xgmi_allreduce_kernel<1>, g, blk, 0, s, a); break;
    case 2: hipLaunchKernelGGL(xgmi_allreduce_kernel<2>, g, blk, 0, s, a); break;
    case 3: hipLaunchKernelGGL(xgmi_allreduce_kernel<3>, g, blk, 0, s, a); break;
    case 4: hipLaunchKernelGGL(xgmi_allreduce_kernel<4>, g, blk, 0, s, a); break;
    case 5: hipLaunchKernelGGL(xgmi_allreduce_kernel<5>, g, blk, 0, s, a); break;
    case 6: hipLaunchKernelGGL(xgmi_allreduce_kernel<6>, g, blk, 0, s, a); break;
    case 7: hipLaunchKernelGGL(xgmi_allreduce_kernel<7>, g, blk, 0, s, a); break;
    case 8: hipLaunchKernelGGL(xgmi_allreduce_kernel<8>, g, blk, 0, s, a); break;
    default: break;   // the host rejects world sizes outside 1..XGMI_MAX_RANKS
  }
}

}  // namespace mnist
