// Per-phase timing of conv2_wgrad_kernel (the B < 342 form): compiles conv_bwd.hip with
// MNIST_WGRAD_PHASE_TIMING (thread 0 of every workgroup stamps s_memtime at each phase boundary) and
// prints per-phase medians over workgroups plus the kernel's event time (synthetic records + a1).
// build: hipcc -x hip --offload-arch=gfx950 -O3 -fno-slp-vectorize -Icsrc/kernels tools/wgrad_phase.hip -o tools/wgrad_phase.bin
// usage: tools/wgrad_phase.bin [B [G [FORM]]]   (G = workgroups, 0 = conv_wgrad_groups(B); FORM 0: the
//        8-wave lockstep kernel, 1: conv2_wgrad_stag_kernel (event time only), 2: the VALU-lean kernel,
//        3: the VALU-lean staggered kernel (event time only))
#define MNIST_WGRAD_PHASE_TIMING 1
#ifndef WGRAD_SRC
#define WGRAD_SRC "../csrc/kernels/conv_bwd.hip"
#endif
#include WGRAD_SRC

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <class T> T* dev_rand(size_t n, unsigned mask) {
  std::vector<T> h(n);
  for (auto& x : h) x = (T)(rand() & mask);
  T* d; CK(hipMalloc(&d, n * sizeof(T))); CK(hipMemcpy(d, h.data(), n * sizeof(T), hipMemcpyHostToDevice)); return d;
}

int main(int argc, char** argv) {
  using namespace mnist;
  const int B = argc > 1 ? atoi(argv[1]) : 200;
  const int G = argc > 2 && atoi(argv[2]) > 0 ? atoi(argv[2]) : conv_wgrad_groups(B);
  const int form = argc > 3 ? atoi(argv[3]) : 0;   // 0 plain, 1 staggered, 2 lean, 3 lean staggered
  const bool stag = form == 1 || form == 3;
  if (G > kWgPhaseMaxWG || G < 1) { printf("G out of range (max %d)\n", kWgPhaseMaxWG); return 1; }
  std::vector<uint8_t> rec((size_t)B * DYC_BYTES_PER_IMAGE);
  for (size_t i = 0; i < rec.size(); ++i) {
    const size_t o = i % DYC_REC;
    rec[i] = o < DYC_ROUTE ? (uint8_t)((o & 1) ? 0x3B : (rand() & 0xFF)) : (uint8_t)(rand() & 0xFF);   // code bit planes: any byte
  }
  uint8_t* dyc; CK(hipMalloc(&dyc, rec.size())); CK(hipMemcpy(dyc, rec.data(), rec.size(), hipMemcpyHostToDevice));
  uint16_t* a1 = dev_rand<uint16_t>((size_t)B * H1 * H1 * C1, 0x3BFF);
  float* w2part; CK(hipMalloc(&w2part, (size_t)G * W2PART_STRIDE * 4));
  ConvBwdArgs a{};
  a.dyc = dyc; a.a1 = a1; a.w2part = w2part; a.grad_scale = 1.0f; a.wgrad_groups = G;
  auto launch = [&] {
    if (form == 3) hipLaunchKernelGGL(conv2_wgrad_lstag_kernel, dim3(G), dim3(WG_THREADS), 0, nullptr, a, B);
    else if (stag) hipLaunchKernelGGL(conv2_wgrad_stag_kernel, dim3(G), dim3(WG_THREADS), 0, nullptr, a, B);
    else if (form == 2) hipLaunchKernelGGL(conv2_wgrad_lean_kernel, dim3(G), dim3(WG_THREADS), 0, nullptr, a, B);
    else hipLaunchKernelGGL(conv2_wgrad_kernel, dim3(G), dim3(WG_THREADS), 0, nullptr, a, B);
  };
  for (int it = 0; it < 5; ++it) launch();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  constexpr int kReps = 50;
  CK(hipEventRecord(e0, nullptr));
  for (int it = 0; it < kReps; ++it) launch();
  CK(hipEventRecord(e1, nullptr));
  CK(hipDeviceSynchronize());
  float ms = 0; CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= kReps;
  if (stag) {
    printf("B=%d  %s G=%d: %.2f us (events, mean of %d back-to-back)\n", B, form == 3 ? "conv2_wgrad_lstag_kernel" : "conv2_wgrad_stag_kernel", G, ms * 1000, kReps);
    return 0;
  }
  std::vector<uint64_t> t((size_t)G * 8);
  CK(hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_wg_phase), t.size() * 8));
  printf("B=%d  %s G=%d: %.2f us (events, mean of %d back-to-back); s_memtime ticks\n", B, form == 2 ? "conv2_wgrad_lean_kernel" : "conv2_wgrad_kernel", G, ms * 1000, kReps);
  uint64_t lo = ~0ull, hi = 0;
  for (int w = 0; w < G; ++w) { lo = std::min(lo, t[w * 8]); hi = std::max(hi, t[w * 8 + 5]); }
  std::vector<double> st;
  for (int w = 0; w < G; ++w) st.push_back((double)(t[w * 8] - lo));
  std::sort(st.begin(), st.end());
  printf("  span first start -> last end: %.0f ticks; start offsets median %.0f p90 %.0f max %.0f\n", (double)(hi - lo),
         st[G / 2], st[G * 9 / 10], st[G - 1]);
  const char* names[5] = {"prologue fetch+expand+store (chunk 0)", "chunk-0 MFMAs (wave 0)",
                          "chunk-1 store + barrier", "remaining chunks", "slab write + bias reduce"};
  for (int ph = 0; ph < 5; ++ph) {
    std::vector<double> d;
    for (int w = 0; w < G; ++w) d.push_back((double)(t[w * 8 + ph + 1] - t[w * 8 + ph]));
    std::sort(d.begin(), d.end());
    printf("  phase %-40s median %7.0f  p10 %7.0f  p90 %7.0f ticks\n", names[ph], d[G / 2], d[G / 10], d[G * 9 / 10]);
  }
  return 0;
}
