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
//
// Cross-device ordering: why no release / acquire fence is needed by default.  Each rule below is
// the gfx942/gfx950 mapping of the LLVM AMDGPU memory model (AMDGPUUsage, "memory model gfx942")
// or a measured gfx950 fact from docs (MI355X_MICROARCH.md, visibility tables):
//  R1  every buffer a peer reads or writes (input / output buckets, staging slots, flag blocks) is
//      allocated hipDeviceMallocUncached (XgmiComm ctor): MTYPE UC, so no L2 of either GPU ever
//      holds a line of it - the only stale-data path the system-scope fences exist for (buffer_wbl2
//      writes back dirty L2 lines, buffer_inv sc0 sc1 drops clean non-coherent ones) has nothing to
//      act on.  RCCL relies on the same property for its LL/LL128 FIFOs on MI300-class GPUs
//      (uncached, peer-mapped, polled without reader-side invalidates).
//  R2  every payload store a peer reads is `sc0 sc1` (st_sys / st_sys1) - the gfx942 mapping of a
//      system-scope monotonic atomic store - or a plain store into an R1 buffer by a kernel that
//      COMPLETED before this launch on the same stream (the gradient producers writing the input
//      bucket: kernel boundary);
//  R3  every storing wave runs `s_waitcnt vmcnt(0)` (gfx9 counts stores in vmcnt: the wait returns
//      once each store is acknowledged by the memory side) and the workgroup barrier follows, before
//      the ONE lane per peer that stores the flag - a system-scope atomic store;
//  R4  the reader polls the flag with system-scope atomic loads and issues its payload loads only
//      after the poll matched (and the workgroup barrier after it); every payload load is `sc0 sc1`
//      (ld_sys / ld_sys1) - the gfx942 mapping of a system-scope monotonic atomic load, which must
//      observe the latest value in coherence order and is never served from L1.
// R1 + R2 + R3: when the flag becomes visible at a peer, every payload byte is in the owner's HBM;
// R1 + R4: the peer's loads read HBM, not a cached copy.  The fences stay available as knobs
// (XgmiComm::set_fences: buffer_wbl2 sc0 sc1 before every flag, +13 us per world-1 step, and
// buffer_inv sc0 sc1 after every matched poll - the trainer's fallback when the unfenced schedule
// fails its cross-rank validation) and XgmiComm::ordering() names the mode in use (bench JSON
// "xgmi_ordering").
#include <stdexcept>
#include <string>

#include "../include/device_utils.h"
#include "../include/kernels.h"
#include "../include/timeline.h"
#include "../runtime/host_logic.h"
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
// flag slot [stage][my rank][b], then polls its own slot [stage][p][b].  Returns false on timeout
// and records the first failure as *err = kid << 24 | stage << 16 | peer << 12 | b (XgmiComm::error).
__device__ bool xgmi_stage(const XgmiArgs& a, int stage, int b, int e, int kid) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's write-through stores are done
  __syncthreads();
  bool ok = true;
  const int p = threadIdx.x;
  if (p < a.world) {
    // optional system-scope release before the flag (XgmiArgs::release, XgmiComm::set_fences):
    // off by default - the payload stores are write-through (sc0 sc1) into uncached buckets and
    // drained above; the fence's L2 write-back costs ~13 us per world-1 step
    if (a.release) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(a.flags[p] + (stage * XGMI_MAX_RANKS + a.rank) * XGMI_MAX_WG + b, e, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    const int* slot = a.flags[a.rank] + (stage * XGMI_MAX_RANKS + p) * XGMI_MAX_WG + b;
    const uint64_t tmo = __hip_atomic_load(a.timeout_ticks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();            // 100 MHz
    while (__hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > tmo) {
        int zero = 0;
        __hip_atomic_compare_exchange_strong(a.err, &zero, (kid << 24) | (stage << 16) | (p << 12) | b,
                                             __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
        break;
      }
    }
  }
  const bool all = __syncthreads_and(ok);
  if (a.acquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // opt-in system-scope acquire (R1/R4 above)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: keeps the payload loads below
  return all;
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
  TL_SCOPE(TL_XGMI_TWOSHOT);
  RW_ENTRY();
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

  if (!xgmi_stage(a, 0, b, e, XGMI_K_TWOSHOT)) return;
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
  if (!xgmi_stage(a, 1, b, e, XGMI_K_TWOSHOT)) return;
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
  TL_SCOPE(TL_XGMI_ONESHOT);
  RW_ENTRY();
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
  if (!xgmi_stage(a, 0, b, e, XGMI_K_ONESHOT)) return;
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

namespace {
inline int clamp_grid(int64_t natural, int lo, int cap) {
  int64_t g = natural < cap ? natural : cap;
  if (g < lo) g = lo;
  if (g > XGMI_MAX_WG) g = XGMI_MAX_WG;
  return (int)(g < 1 ? 1 : g);
}
}  // namespace

void launch_xgmi_allreduce_oneshot(const XgmiArgs& a, hipStream_t s) {
  // <= 4 float4 per lane (KMAX): the grid may shrink to nvec / 1024 workgroups, never below
  const dim3 g(clamp_grid((a.nvec + 255) / 256, (int)((a.nvec + 1023) / 1024), a.max_wg)), blk(256);
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
// shard p = units [p*577/W, (p+1)*577/W).  Workgroup b owns units lo_p + b + m*G of every shard p
// (G = grid, any size: the residency planner may shrink it).
//   phase 1: WG b reduces its units of shard r (rank order) into its output bucket (the peers'
//            phase-2 source) and applies the update to them at once - their gradients are final;
//   stage 1;
//   phase 2: WG b gathers its units of every OTHER shard (gathered sums + local optimizer state in
//            flight together) and applies the update.
// The update is exactly the adadelta kernel's fc1 tile math (Ada::step, param / square_avg /
// acc_delta, bf16 shadows w1 [128][9216] and w1t [9216][128], the tile transposed through LDS), so the
// result is bitwise that of the all-reduce + separate update it replaces.  Registers and LDS are kept
// at the single-GPU update's scale (one unit per pass at W <= 2, 4.6 KB of LDS) so the kernel fits
// beside the persistent conv2_dgrad's workgroups (2 x 216 VGPRs per SIMD, 150 KB of LDS per CU) -
// at 103 VGPRs it did not, and dgrad ran 2 us longer beside it (world-1 in-kernel timeline).  Every
// world size is held to <= 80 VGPRs (6 waves per SIMD: beside dgrad's 2 x 216 and wgrad's 2 x 208):
// one phase-2 unit in flight per lane and phase-1 peer loads in groups of 4 (W = 4..8 reached
// 106-113 VGPRs with two phase-2 units in flight, so at N >= 4 the fc branch could not co-run with
// the conv backward at all).
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

__device__ __forceinline__ void fcu_load_state(const XgmiArgs& a, const int q[2], float4 pr[2], float4 sq[2],
                                               float4 ac[2]) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (q[h] < 0) continue;
    pr[h] = reinterpret_cast<const float4*>(a.ada.param)[q[h]];
    sq[h] = reinterpret_cast<const float4*>(a.ada.square_avg)[q[h]];
    ac[h] = reinterpret_cast<const float4*>(a.ada.acc_delta)[q[h]];
  }
}

// Unit u's update from its reduced gradients g (this lane's 2 float4; q = their bucket indices,
// -1 past the tail).  Workgroup-uniform call: two LDS barriers around the w1t transpose in ts.
__device__ __forceinline__ void fcu_update(const XgmiArgs& a, const Ada& ad, int u, int tid, const int q[2],
                                           const f4 g[2], float4 pr[2], float4 sq[2], float4 ac[2], uint16_t* ts) {
  float v8[8];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (q[h] < 0) continue;
    ad.step(pr[h].x, g[h].x, sq[h].x, ac[h].x);
    ad.step(pr[h].y, g[h].y, sq[h].y, ac[h].y);
    ad.step(pr[h].z, g[h].z, sq[h].z, ac[h].z);
    ad.step(pr[h].w, g[h].w, sq[h].w, ac[h].w);
    // write-through 16-B stores at small batches (AdadeltaArgs::wt, as the single-GPU update): the
    // next step's kernels read these, and the kernel-end write-back of dirty lines is a step gap
    store16(a.ada.wt, a.ada.param, (int64_t)q[h] * 16, make_floatx4(pr[h]));
    store16(a.ada.wt, a.ada.square_avg, (int64_t)q[h] * 16, make_floatx4(sq[h]));
    store16(a.ada.wt, a.ada.acc_delta, (int64_t)q[h] * 16, make_floatx4(ac[h]));
    v8[4 * h] = pr[h].x; v8[4 * h + 1] = pr[h].y; v8[4 * h + 2] = pr[h].z; v8[4 * h + 3] = pr[h].w;
  }
  const bool tile = u < FCU_TILES;                               // workgroup-uniform
  const int ot = u / (NFLAT / 32), it = u - ot * (NFLAT / 32);
  if (tile) {                                                    // bf16 shadows of the fc1 tile
    const int ol = tid >> 2, ic = (tid & 3) * 8, o = 64 * ot + ol, i0 = 32 * it;
    uint4 lo4;
    lo4.x = pack2bf(v8[0], v8[1]); lo4.y = pack2bf(v8[2], v8[3]);
    lo4.z = pack2bf(v8[4], v8[5]); lo4.w = pack2bf(v8[6], v8[7]);
    store16(a.ada.wt, a.ada.w1, ((int64_t)o * NFLAT + i0 + ic) * 2, lo4);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) ts[(ic + jj) * FCU_TS + ol] = f2bf(v8[jj]);
  }
  lds_barrier();
  if (tile) {
    const int il = tid >> 3, oc = (tid & 7) * 8;
    store16(a.ada.wt, a.ada.w1t, ((int64_t)(32 * it + il) * NH + 64 * ot + oc) * 2,
            *reinterpret_cast<const uint4*>(ts + il * FCU_TS + oc));
  }
  lds_barrier();                                                 // ts is rewritten by the next unit
}
}  // namespace

template <int W>
#ifndef XGMI_FC_W1_MINBLOCKS   // A/B builds only (-DXGMI_FC_W1_MINBLOCKS=6: the VGPR-capped form at W < 4)
#define XGMI_FC_W1_MINBLOCKS 1
#endif
__global__ __launch_bounds__(256, W >= 4 ? 6 : XGMI_FC_W1_MINBLOCKS) void xgmi_fc_fused_kernel(XgmiArgs a) {
  TL_SCOPE(TL_XGMI_FC);
  RW_ENTRY();
  constexpr int PG = 1;                                          // phase-2 units in flight per lane
  __shared__ int s_epoch, s_err;
  __shared__ __attribute__((aligned(16))) uint16_t ts[32 * FCU_TS];
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
  if (!xgmi_stage(a, 0, b, e, XGMI_K_FC_FUSED)) return;
  const Ada ad{a.ada.rho, a.ada.eps, a.ada.weight_decay, *a.ada.lr};
  // ---- phase 1: my shard's units - rank-order sums -> my output (for the peers), then the update
  {
    __amdgpu_buffer_rsrc_t in[W];
#pragma unroll
    for (int p = 0; p < W; ++p) in[p] = rsrc(a.in[p], bytes);
    const int lo = fcu_lo(r, W), hi = fcu_lo(r + 1, W);
    for (int u = lo + b; u < hi; u += G) {                       // workgroup-uniform
      int q[2];
      f4 g[2];
      float4 pr[2], sq[2], ac[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) q[h] = fcu_f4(u, h, tid);
      fcu_load_state(a, q, pr, sq, ac);                          // local, in flight with the peer loads
      if (W <= 2) {                                              // both halves' peer loads at once
        f4 v[2][W];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int p = 0; p < W; ++p) v[h][p] = ld_sys(in[p], q[h] < 0 ? a.nvec : q[h]);   // -1: 0
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          g[h] = v[h][0];
#pragma unroll
          for (int p = 1; p < W; ++p) g[h] += v[h][p];
        }
      } else {                                                   // one half's loads at a time, in
#pragma unroll                                                   // groups of <= 4 peers (the rank-order
        for (int h = 0; h < 2; ++h) {                            // sum is unchanged; <= 80 VGPRs at W = 8)
#pragma unroll
          for (int p0 = 0; p0 < W; p0 += 4) {
            f4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (p0 + k < W) v[k] = ld_sys(in[p0 + k], q[h] < 0 ? a.nvec : q[h]);
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (p0 + k < W) g[h] = (p0 + k == 0) ? v[0] : g[h] + v[k];
          }
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (q[h] >= 0) st_sys(out, q[h], g[h]);
      fcu_update(a, ad, u, tid, q, g, pr, sq, ac, ts);
    }
  }
  if constexpr (W > 1) {
    if (!xgmi_stage(a, 1, b, e, XGMI_K_FC_FUSED)) return;
    // ---- phase 2: items j over the other shards (p' = j mod (W-1) -> p, m = j / (W-1)): unit
    // lo_p + b + m*G, which peer p's workgroup b reduced; consecutive items come from different
    // peers' links.  Workgroup-uniform loop bounds (the LDS transpose needs the barriers).
    const int M = ((FCU_UNITS + W - 1) / W + G - 1) / G;       // units per shard per WG (upper bound)
    for (int j0 = 0; j0 < (W - 1) * M; j0 += PG) {
      int uu[PG], q[PG][2];
      f4 g[PG][2];
      float4 pr[PG][2], sq[PG][2], ac[PG][2];
#pragma unroll
      for (int k = 0; k < PG; ++k) {
        const int j = j0 + k, pp = j % (W - 1), m = j / (W - 1);
        const int p = pp + (pp >= r ? 1 : 0);
        const int u = fcu_lo(p, W) + b + m * G;
        uu[k] = (j < (W - 1) * M && u < fcu_lo(p + 1, W)) ? u : -1;
        if (uu[k] < 0) continue;
        const __amdgpu_buffer_rsrc_t src = rsrc(a.out[p], bytes);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          q[k][h] = fcu_f4(u, h, tid);
          g[k][h] = ld_sys(src, q[k][h] < 0 ? a.nvec : q[k][h]);
        }
        fcu_load_state(a, q[k], pr[k], sq[k], ac[k]);
      }
#pragma unroll
      for (int k = 0; k < PG; ++k)
        if (uu[k] >= 0) fcu_update(a, ad, uu[k], tid, q[k], g[k], pr[k], sq[k], ac[k], ts);
    }
  }
  // optional completion hold (the XGMI comm chain, as the single-GPU fc update): the launch
  // completes only once *hold_a >= *hold_b + hold_delta (this step's dgrad has started), so the
  // conv2 part that follows on the comm stream needs no wait launch of its own
  if (a.ada.hold_a && b == G - 1 && tid == 0)
    spin_until_geq(a.ada.hold_a,
                   __hip_atomic_load(a.ada.hold_b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + a.ada.hold_delta,
                   a.ada.hold_err);
}

int xgmi_fc_fused_workgroups(int world) {
  // one workgroup per unit of this rank's shard (the residency planner may shrink it).  Not the
  // single-GPU update's lean 144: this kernel's units wait on uncached / peer loads, so fewer
  // workgroups lengthen the fc branch more than they relieve the conv backward (world 1, 600 steps:
  // natural grid 68.5-68.9 us/step, 256 workgroups 69.7-70.8; before the slim kernel 144 was worse too)
  const int per = (FCU_UNITS + world - 1) / world;
  return per < XGMI_MAX_WG ? per : XGMI_MAX_WG;
}

void launch_xgmi_fc_fused(const XgmiArgs& a, hipStream_t s) {
  const dim3 g(clamp_grid(xgmi_fc_fused_workgroups(a.world), 1, a.max_wg)), blk(256);
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
// conv bucket, fully fused: the 309 blocks of conv_grad_reduce's partition become virtual blocks
// vb = b, b + G, .. of workgroup b (same slab partition and summation order per block -> the same
// bits).  Each virtual block's <= 64 finished gradients go to LDS slots (k*64 + lane*4 + r), are
// published into this rank's staging slot (call parity; 4-byte write-through stores at their bucket
// index), ONE hand-off (stage 0: WG b of every rank is done with the same indices), then every rank's
// values at those indices are summed in rank order and Ada::step + the conv2 bf16 shadows applied -
// one slot per lane (<= 512 slots: XGMI_CONV_VB_MAX virtual blocks).  Replaces conv_grad_reduce +
// the one-shot all-reduce + the conv update: one launch on the DDP critical path.
namespace {
__device__ __forceinline__ void st_sys1(__amdgpu_buffer_rsrc_t r, int64_t i, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), r, (int)(i * 4), 0, SYS);
}
__device__ __forceinline__ float ld_sys1(__amdgpu_buffer_rsrc_t r, int64_t i) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)(i * 4), 0, SYS));
}
constexpr int CONV_SLOTS = XGMI_CONV_VB_MAX * 64;
constexpr int CONV_SLOTS_PER_LANE = CONV_SLOTS / 256;
}  // namespace

template <int W>
__global__ __launch_bounds__(256) void xgmi_conv_reduce_fused_kernel(XgmiArgs a, ConvBwdArgs c, int B, XgmiConvPart part) {
  TL_SCOPE(part.lo == 0 ? TL_XGMI_CONV2 : TL_XGMI_CONV);
  __shared__ float4 red[256];
  __shared__ float s_val[CONV_SLOTS];
  __shared__ int s_idx[CONV_SLOTS];
  __shared__ int s_epoch, s_err;
  const int b = blockIdx.x, tid = threadIdx.x, G = gridDim.x;
  // reduce blocks [part.lo, part.hi) of conv_grad_reduce's partition, virtual block lo + b + k*G
  const int nvb = (part.hi - part.lo - b + G - 1) / G;        // <= XGMI_CONV_VB_MAX (host-checked grid)
#pragma unroll
  for (int k = 0; k < CONV_SLOTS_PER_LANE; ++k) s_idx[tid + 256 * k] = -1;
  if (tid == 0) {
    const int e = a.ctr[b] + 1;
    a.ctr[b] = e;
    s_epoch = e;
    s_err = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // XGMI comm chain: "the previous launch on this stream (the fc all-reduce + update) is done",
    // signalled by the first workgroup at its start instead of by a signal launch
    if (b == 0 && a.ada.signal_start)
      (RW_SIGNAL(), __hip_atomic_fetch_add(a.ada.signal_start, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT));
  }
  RW_ENTRY();
  // (the reduce's first barrier orders the slot initialisation before any sink write)
  for (int k = 0; k < nvb; ++k) {
    int nv = 0;
    reduce_conv_grads(c, B, part.lo + b + k * G, red, [&](int64_t el, float v) {   // lanes 0..15, <= 4 each
      const int q = k * 64 + tid * 4 + nv;
      s_idx[q] = (int)(el - a.ada_base);
      s_val[q] = v;
      ++nv;
    });
  }
  __syncthreads();
  if (s_err) return;
  const int e = s_epoch, r = a.rank;
  const int64_t slot = (e & 1) * a.slot_floats;
  const int64_t bytes = a.nvec * 16;
  int idx[CONV_SLOTS_PER_LANE];
  float val[CONV_SLOTS_PER_LANE], pr[CONV_SLOTS_PER_LANE], sq[CONV_SLOTS_PER_LANE], ac[CONV_SLOTS_PER_LANE];
  {
    const __amdgpu_buffer_rsrc_t mine = rsrc(a.stage[r] + slot, bytes);
#pragma unroll
    for (int k = 0; k < CONV_SLOTS_PER_LANE; ++k) {
      const int q = tid + 256 * k;
      idx[k] = q < nvb * 64 ? s_idx[q] : -1;
      if (idx[k] < 0) continue;
      val[k] = s_val[q];
      st_sys1(mine, idx[k], val[k]);
      const int64_t el = a.ada_base + idx[k];                   // the update's local state, loaded
      pr[k] = a.ada.param[el];                                  // before the hand-off wait
      sq[k] = a.ada.square_avg[el];
      ac[k] = a.ada.acc_delta[el];
    }
  }
  if (!xgmi_stage(a, 0, b, e, XGMI_K_CONV_FUSED)) return;
  // end-of-step marker (with a wait: after it, so the comm stream's readers of the step index are done)
  if (b == 0 && tid == 0 && a.ada.state_inc && !part.wait_a) a.ada.state_inc->step += 1;
  __amdgpu_buffer_rsrc_t src[W];
#pragma unroll
  for (int p = 0; p < W; ++p) src[p] = rsrc(a.stage[p] + slot, p == r ? 0 : bytes);   // own: registers
  float v[CONV_SLOTS_PER_LANE][W];
#pragma unroll
  for (int k = 0; k < CONV_SLOTS_PER_LANE; ++k)
#pragma unroll
    for (int p = 0; p < W; ++p) v[k][p] = ld_sys1(src[p], idx[k] < 0 ? 0 : idx[k]);
  const Ada ad{a.ada.rho, a.ada.eps, a.ada.weight_decay, *a.ada.lr};
#pragma unroll
  for (int k = 0; k < CONV_SLOTS_PER_LANE; ++k) {
    if (idx[k] < 0) continue;
    float g = (r == 0) ? val[k] : v[k][0];
#pragma unroll
    for (int p = 1; p < W; ++p) g += (p == r) ? val[k] : v[k][p];
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
  // split schedule: the conv1 launch (compute stream) completes only once the conv2 launch (comm
  // stream) has published its update (device counters, as trunk_fwd's hold), so the next trunk_fwd,
  // which follows it on the compute stream, reads the new conv2 weights
  if (part.wait_a && b == 0 && tid == 0) {
    const int target = __hip_atomic_load(part.wait_b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t tmo = __hip_atomic_load(a.timeout_ticks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(part.wait_a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > tmo) {
        __hip_atomic_store(part.wait_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    if (a.ada.state_inc) a.ada.state_inc->step += 1;
  }
}

namespace {
constexpr int CONV_FUSED_MIN_WG = (RED_WGS + XGMI_CONV_VB_MAX - 1) / XGMI_CONV_VB_MAX;   // 39
}

void launch_xgmi_conv_reduce_fused(const XgmiArgs& a, const ConvBwdArgs& c, int B, hipStream_t s,
                                   const XgmiConvPart& part) {
  static_assert(RED_WGS <= XGMI_MAX_WG, "one flag slot per reduce workgroup");
  const int n = part.hi - part.lo;
  if (part.lo < 0 || part.hi > RED_WGS || n < 1) return;
  const int lo_wg = (n + XGMI_CONV_VB_MAX - 1) / XGMI_CONV_VB_MAX;
  const dim3 g(clamp_grid(n, lo_wg, a.max_wg)), blk(256);
  switch (a.world) {
    case 1: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<1>, g, blk, 0, s, a, c, B, part); break;
    case 2: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<2>, g, blk, 0, s, a, c, B, part); break;
    case 3: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<3>, g, blk, 0, s, a, c, B, part); break;
    case 4: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<4>, g, blk, 0, s, a, c, B, part); break;
    case 5: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<5>, g, blk, 0, s, a, c, B, part); break;
    case 6: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<6>, g, blk, 0, s, a, c, B, part); break;
    case 7: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<7>, g, blk, 0, s, a, c, B, part); break;
    case 8: hipLaunchKernelGGL(xgmi_conv_reduce_fused_kernel<8>, g, blk, 0, s, a, c, B, part); break;
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
  const dim3 g(clamp_grid(xgmi_workgroups(a.nvec, a.world, a.fuse_ada != 0), 1, a.max_wg)), blk(256);
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

// ---------------------------------------------------------------------------------------------
// Residency planner (see XgmiGrids in kernels.h).
namespace {
template <int W>
void occupancies(int* fc, int* conv, int* two, int* one) {
  auto occ = [](const void* f) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, 256, 0) != hipSuccess || n < 1) n = 1;
    return n;
  };
  *fc = occ(reinterpret_cast<const void*>(&xgmi_fc_fused_kernel<W>));
  *conv = occ(reinterpret_cast<const void*>(&xgmi_conv_reduce_fused_kernel<W>));
  *two = occ(reinterpret_cast<const void*>(&xgmi_allreduce_kernel<W>));
  *one = occ(reinterpret_cast<const void*>(&xgmi_oneshot_kernel<W>));
}

}  // namespace

XgmiGrids xgmi_plan_grids(int world, int co_ranks, int64_t oneshot_max_floats, double budget) {
  if (world < 1 || world > XGMI_MAX_RANKS) throw std::runtime_error("xgmi_plan_grids: bad world size");
  if (co_ranks < 1) co_ranks = 1;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    throw std::runtime_error("xgmi_plan_grids: cannot query the device");
  int ofc = 1, oconv = 1, otwo = 1, oone = 1;
  switch (world) {
    case 1: occupancies<1>(&ofc, &oconv, &otwo, &oone); break;
    case 2: occupancies<2>(&ofc, &oconv, &otwo, &oone); break;
    case 3: occupancies<3>(&ofc, &oconv, &otwo, &oone); break;
    case 4: occupancies<4>(&ofc, &oconv, &otwo, &oone); break;
    case 5: occupancies<5>(&ofc, &oconv, &otwo, &oone); break;
    case 6: occupancies<6>(&ofc, &oconv, &otwo, &oone); break;
    case 7: occupancies<7>(&ofc, &oconv, &otwo, &oone); break;
    default: occupancies<8>(&ofc, &oconv, &otwo, &oone); break;
  }
  XgmiGrids g{};
  g.cap_fc_fused = ofc * cus;
  g.cap_conv_fused = oconv * cus;
  g.cap_twoshot = otwo * cus;
  g.cap_oneshot = oone * cus;
  const int one_nat = (int)((oneshot_max_floats / 4 + 255) / 256);
  const int one_min = (int)((oneshot_max_floats / 4 + 1023) / 1024);
  g.fc_fused = xgmi_fc_fused_workgroups(world);
  g.conv_fused = RED_WGS;
  g.twoshot = XGMI_MAX_WG;                                       // cap: launches use min(natural, cap)
  g.oneshot = one_nat < XGMI_MAX_WG ? (one_nat > one_min ? one_nat : one_min) : XGMI_MAX_WG;
  g.load_fused = fit_grid_pair(&g.fc_fused, 8, g.cap_fc_fused, &g.conv_fused, CONV_FUSED_MIN_WG, g.cap_conv_fused,
                          co_ranks, budget);
  g.load_separate = fit_grid_pair(&g.twoshot, 8, g.cap_twoshot, &g.oneshot, one_min > 1 ? one_min : 1, g.cap_oneshot,
                             co_ranks, budget);
  if (g.load_fused > 1.0 || g.load_separate > 1.0)
    throw std::runtime_error("xgmi: the spinning all-reduce grids of " + std::to_string(co_ranks) +
                             " ranks per GPU cannot all be resident");
  return g;
}

TL_DEFINE_HOST(xgmi)

// load this translation unit's gfx950 code object now (startup prewarm thread) instead of at its
// first launch inside the timed run
void preload_xgmi() {
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&xgmi_allreduce_kernel<1>));
}

}  // namespace mnist
