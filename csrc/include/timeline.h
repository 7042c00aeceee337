// In-kernel timeline (debug build only: `python -m pytorch_mnist_ddp_amd._build --timeline` compiles
// every source with -DMNIST_TIMELINE into a separate _C_tl extension; the product build compiles
// the macros below to nothing).
//
// rocprofv3 intercepts every dispatch and perturbs the overlapped schedule (a 412 us profiled
// period against 68 us unprofiled at B = 200), so the overlap of the comm-stream kernels with the
// conv backward has to be observed from inside the kernels: every wave of an instrumented kernel
// reads s_memrealtime (the device-wide 100 MHz constant clock) when it starts and, through the scope
// object's destructor (so early returns are covered), stores {kernel id, start, end} into its own
// slot in device memory with plain vector stores from lane 0.  The host clusters the wave
// records into launches (launches of one kernel id are stream-ordered, so a new launch starts after
// the previous cluster's last end) and rebuilds the per-queue timeline (tools/timeline_tl.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace mnist {

enum TlKernel : int {
  TL_TRUNK = 0, TL_FC1 = 1, TL_HEAD = 2, TL_FC_BWD = 3, TL_WGRAD = 4, TL_DGRAD = 5,
  TL_ADA_FC = 6, TL_ADA_CONV = 7, TL_ADA_ALL = 8, TL_RED_ALL = 9, TL_RED_CONV2 = 10, TL_RED_CONV1 = 11,
  TL_WAIT = 12, TL_SIGNAL = 13, TL_GATHER = 14, TL_XGMI_FC = 15, TL_XGMI_CONV = 16, TL_XGMI_CONV2 = 17,
  TL_CONV_REDUCE = 18, TL_XGMI_TWOSHOT = 19, TL_XGMI_ONESHOT = 20, TL_C1_PRE = 21, TL_NKINDS = 22
};

#ifdef MNIST_TIMELINE
// No atomics: a wave owns the slot (kernel id, flat wave id) and every launch of one kernel id is
// stream-ordered after the previous one, so the slot's launch counter is a plain load at wave start
// and a plain store at the end (a single device-wide atomic counter serialised ~2400 waves per
// launch at the memory-side atomic unit: 180 us/step against 72.5 in the first version).
constexpr int TL_MAXW = 2560;                    // waves per launch recorded (more are dropped)
constexpr int TL_GENS = 48;                      // launches kept per kernel id (ring)

// per translation unit (no relocatable device code): static device symbols
static __device__ unsigned g_tl_cnt[TL_NKINDS][TL_MAXW];
static __device__ ulonglong2 g_tl_rec[TL_NKINDS][TL_MAXW][TL_GENS];

struct TlScope {
  uint64_t t0;
  int kid, wid;
  unsigned gen;
  __device__ explicit TlScope(int k) : t0(__builtin_amdgcn_s_memrealtime()), kid(k) {
    const int wpb = (blockDim.x * blockDim.y * blockDim.z + 63) >> 6;
    wid = (int)((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * wpb +
          (int)((threadIdx.z * blockDim.y + threadIdx.y) * blockDim.x + threadIdx.x) / 64;
    gen = wid < TL_MAXW ? g_tl_cnt[kid][wid] : 0u;      // in flight until the destructor
  }
  __device__ ~TlScope() {
    if ((threadIdx.x & 63) == 0 && wid < TL_MAXW) {
      const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
      g_tl_rec[kid][wid][gen % TL_GENS] = make_ulonglong2(t0 | ((uint64_t)kid << 56), t1);
      g_tl_cnt[kid][wid] = gen + 1;
    }
  }
};
#define TL_SCOPE(kid) ::mnist::TlScope tl_scope_(kid)

// host side of one translation unit: copy its records out (appended to `out` as [kid, t0, t1]
// triples, the last TL_GENS launches per kernel id) and zero its counters
#define TL_DEFINE_HOST(tag)                                                                   \
  void tl_dump_##tag(std::vector<uint64_t>& out) {                                          \
    std::vector<unsigned> cnt((size_t)TL_NKINDS * TL_MAXW);                                   \
    if (hipMemcpyFromSymbol(cnt.data(), HIP_SYMBOL(g_tl_cnt), cnt.size() * sizeof(unsigned)) != hipSuccess) return; \
    std::vector<ulonglong2> r((size_t)TL_NKINDS * TL_MAXW * TL_GENS);                         \
    if (hipMemcpyFromSymbol(r.data(), HIP_SYMBOL(g_tl_rec), r.size() * sizeof(ulonglong2)) != hipSuccess) return; \
    for (size_t s = 0; s < cnt.size(); ++s) {                                                 \
      const unsigned n = cnt[s], g0 = n > (unsigned)TL_GENS ? n - TL_GENS : 0u;               \
      for (unsigned g = g0; g < n; ++g) {                                                     \
        const ulonglong2& x = r[s * TL_GENS + g % TL_GENS];                                   \
        out.push_back(x.x >> 56);                                                             \
        out.push_back(x.x & ((1ull << 56) - 1));                                              \
        out.push_back(x.y);                                                                   \
      }                                                                                       \
    }                                                                                         \
    std::fill(cnt.begin(), cnt.end(), 0u);                                                    \
    hipMemcpyToSymbol(HIP_SYMBOL(g_tl_cnt), cnt.data(), cnt.size() * sizeof(unsigned));       \
  }
#else
#define TL_SCOPE(kid) ((void)0)
#define TL_DEFINE_HOST(tag)
#endif

}  // namespace mnist
