// In-kernel timeline (debug build only: `python -m pytorch_mnist_ddp_amd._build --timeline` compiles
// every source with -DMNIST_TIMELINE into a separate _C_tl extension; the product build compiles
// the macros below to nothing).
//
// rocprofv3 intercepts every dispatch and perturbs the overlapped schedule (a 412 us profiled
// period against 68 us unprofiled at B = 200), so the overlap of the comm-stream kernels with the
// conv backward has to be observed from inside the kernels: every wave of an instrumented kernel
// reads s_memrealtime (the device-wide 100 MHz constant clock) when it starts and, through the scope
// object's destructor (so early returns are covered), appends {kernel id, start, end} to a ring in
// device memory with one vector atomic + one vector store from lane 0.  The host clusters the wave
// records into launches (launches of one kernel id are stream-ordered, so a new launch starts after
// the previous cluster's last end) and rebuilds the per-queue timeline (tools/timeline_tl.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace mnist {

enum TlKernel : int {
  TL_TRUNK = 0, TL_FC1 = 1, TL_HEAD = 2, TL_FC_BWD = 3, TL_WGRAD = 4, TL_DGRAD = 5,
  TL_ADA_FC = 6, TL_ADA_CONV = 7, TL_ADA_ALL = 8, TL_RED_ALL = 9, TL_RED_CONV2 = 10, TL_RED_CONV1 = 11,
  TL_WAIT = 12, TL_SIGNAL = 13, TL_GATHER = 14, TL_XGMI_FC = 15, TL_XGMI_CONV = 16, TL_XGMI_CONV2 = 17,
  TL_CONV_REDUCE = 18, TL_XGMI_TWOSHOT = 19, TL_XGMI_ONESHOT = 20, TL_C1_PRE = 21, TL_NKINDS = 22
};

#ifdef MNIST_TIMELINE
constexpr unsigned TL_CAP = 1u << 17;            // wave records per translation unit (2 MB)

// one ring per translation unit (no relocatable device code): static device symbols
static __device__ unsigned g_tl_n;
static __device__ ulonglong2 g_tl_rec[TL_CAP];

struct TlScope {
  uint64_t t0;
  int kid;
  __device__ explicit TlScope(int k) : t0(__builtin_amdgcn_s_memrealtime()), kid(k) {}
  __device__ ~TlScope() {
    if ((threadIdx.x & 63) == 0) {
      const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
      const unsigned i = atomicAdd(&g_tl_n, 1u);
      if (i < TL_CAP) g_tl_rec[i] = make_ulonglong2(t0 | ((uint64_t)kid << 56), t1);
    }
  }
};
#define TL_SCOPE(kid) ::mnist::TlScope tl_scope_(kid)

// host side of one translation unit: copy its records out (appended to `out` as [kid, t0, t1]
// triples) and rewind its ring
#define TL_DEFINE_HOST(tag)                                                                   \
  void tl_dump_##tag(std::vector<uint64_t>& out) {                                          \
    unsigned n = 0;                                                                           \
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_tl_n), sizeof(n)) != hipSuccess) return;         \
    if (n > TL_CAP) n = TL_CAP;                                                               \
    std::vector<ulonglong2> r(n);                                                             \
    if (n && hipMemcpyFromSymbol(r.data(), HIP_SYMBOL(g_tl_rec), n * sizeof(ulonglong2)) != hipSuccess) return; \
    for (const auto& x : r) {                                                                 \
      out.push_back(x.x >> 56);                                                               \
      out.push_back(x.x & ((1ull << 56) - 1));                                                \
      out.push_back(x.y);                                                                     \
    }                                                                                         \
    const unsigned z = 0;                                                                     \
    hipMemcpyToSymbol(HIP_SYMBOL(g_tl_n), &z, sizeof(z));                                     \
  }
#else
#define TL_SCOPE(kid) ((void)0)
#define TL_DEFINE_HOST(tag)
#endif

}  // namespace mnist
