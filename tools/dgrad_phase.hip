// Per-phase timing of the per-item conv2 dgrad (conv2_dgrad_kernel, the B > 256 form): compiles
// conv_bwd.hip with MNIST_DGRAD_PHASE_TIMING (thread 0 of every workgroup stamps s_memtime at each
// phase boundary) and prints per-phase medians over workgroups plus the kernel's event time.
// build: hipcc -x hip --offload-arch=gfx950 -O3 -fno-slp-vectorize -Icsrc/kernels tools/dgrad_phase.hip -o tools/dgrad_phase.bin
// usage: tools/dgrad_phase.bin [B [G [STAGGER]]]   (B <= 8192; synthetic records, masks, weights)
//   G > 0: time the persistent form with G workgroups instead (event time only), the workgroups
//   blockIdx >= G/2 first waiting STAGGER s_memtime ticks
#define MNIST_DGRAD_PHASE_TIMING 1
#ifndef DGRAD_SRC
#define DGRAD_SRC "../csrc/kernels/conv_bwd.hip"
#endif
#include DGRAD_SRC

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
  const int B = argc > 1 ? atoi(argv[1]) : 8192;
  if (4 * B > kDgPhaseMaxWG) { printf("B too large for the timing buffer (max %d)\n", kDgPhaseMaxWG / 4); return 1; }
  const int N = std::max(1024, B);
  uint8_t* img = dev_rand<uint8_t>((size_t)N * IMG * IMG, 0xFF);
  std::vector<int32_t> hidx(B); for (int i = 0; i < B; ++i) hidx[i] = (i * 7) % N;
  int32_t* idx; CK(hipMalloc(&idx, B * 4)); CK(hipMemcpy(idx, hidx.data(), B * 4, hipMemcpyHostToDevice));
  StepState st{0, 0, 0x1234, 0};
  StepState* d_st; CK(hipMalloc(&d_st, sizeof(st))); CK(hipMemcpy(d_st, &st, sizeof(st), hipMemcpyHostToDevice));
  // records: bf16 grads in [0, 0x3C00) (small positive), routes 0..3 per byte
  std::vector<uint8_t> rec((size_t)B * DYC_BYTES_PER_IMAGE);
  for (size_t i = 0; i < rec.size(); ++i) {
    const size_t o = i % DYC_REC;
    rec[i] = o < DYC_ROUTE ? (uint8_t)((o & 1) ? 0x3B : (rand() & 0xFF)) : (uint8_t)(rand() & 0xFF);   // code bit planes: any byte
  }
  uint8_t* dyc; CK(hipMalloc(&dyc, rec.size())); CK(hipMemcpy(dyc, rec.data(), rec.size(), hipMemcpyHostToDevice));
  uint16_t* a1 = dev_rand<uint16_t>((size_t)B * H1 * H1 * C1, 0xBFFF);
  uint16_t* w2d = dev_rand<uint16_t>(9 * C1 * C2, 0x3BFF);
  float* c1part; CK(hipMalloc(&c1part, (size_t)4 * B * 320 * 4));
  ConvBwdArgs a{};
  a.dyc = dyc; a.a1 = a1; a.w2d = w2d; a.data_u8 = img; a.idx = idx; a.idx_step_stride = 0; a.state = d_st;
  a.c1part = c1part; a.grad_scale = 1.0f; a.c1_rows = 4 * B;
  const int G = argc > 2 ? atoi(argv[2]) : 0;
  const int stagger = argc > 3 ? atoi(argv[3]) : 0;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_dg_stagger), &stagger, sizeof(int)));
  auto launch = [&] {
    if (G > 0)
      hipLaunchKernelGGL((conv2_dgrad_persist_kernel<DGX_IDX, true>), dim3(G), dim3(256), 0, nullptr, a, B);
    else
      hipLaunchKernelGGL(conv2_dgrad_kernel<DGX_IDX>, dim3(4, B), dim3(256), 0, nullptr, a, B);
  };
  for (int it = 0; it < 5; ++it) launch();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  constexpr int kReps = 30;
  CK(hipEventRecord(e0, nullptr));
  for (int it = 0; it < kReps; ++it) launch();
  CK(hipEventRecord(e1, nullptr));
  CK(hipDeviceSynchronize());
  float ms = 0; CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= kReps;
  if (G > 0) {
    printf("B=%d  conv2_dgrad_persist_kernel G=%d stagger=%d: %.2f us (events, mean of %d)\n", B, G, stagger, ms * 1000, kReps);
    return 0;
  }
  const int nwg = 4 * B;
  std::vector<uint64_t> t((size_t)nwg * 8);
  CK(hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_dg_phase), t.size() * 8));
  // mark order in a workgroup's life: 0 start, 1 w2d stored, 2 dy tile stored (barrier), 3 wave 0's
  // MFMA loop done, 5 xs barrier (every wave's loop done), 6 mask + conv1-grad MFMA done, 4 end
  const int order[7] = {0, 1, 2, 3, 5, 6, 4};
  const char* names[6] = {"w2d+record loads, w2d store", "dy expand+store, barrier", "MFMA loop (wave 0)",
                          "xs store + barrier (all waves)", "mask (a1 wait) + conv1-grad MFMA", "red + reduce + c1part"};
  printf("B=%d  conv2_dgrad_kernel %.2f us (events, mean of %d), %d WGs; s_memtime ticks (shader clock)\n", B, ms * 1000, kReps, nwg);
  std::vector<double> tot;
  for (int w = 0; w < nwg; ++w) tot.push_back((double)(t[w * 8 + 4] - t[w * 8]));
  std::sort(tot.begin(), tot.end());
  printf("  WG lifetime ticks: median %.0f  p10 %.0f  p90 %.0f\n", tot[nwg / 2], tot[nwg / 10], tot[nwg * 9 / 10]);
  {  // per XCD (WG id % 8): span from first start to last end, and WGs per CU-slot implied
    std::vector<double> sp;
    for (int x = 0; x < 8; ++x) {
      uint64_t lo = ~0ull, hi = 0;
      for (int w = x; w < nwg; w += 8) { lo = std::min(lo, t[w * 8]); hi = std::max(hi, t[w * 8 + 4]); }
      sp.push_back((double)(hi - lo));
    }
    std::sort(sp.begin(), sp.end());
    printf("  per-XCD span %.0f..%.0f ticks; sum of lifetimes / (span x 64 slots) = %.2f\n", sp[0], sp[7],
           [&] { double s = 0; for (double v : tot) s += v; return s / 8 / (sp[7] * 64); }());
  }
  for (int ph = 0; ph < 6; ++ph) {
    std::vector<double> d;
    for (int w = 0; w < nwg; ++w) d.push_back((double)(t[w * 8 + order[ph + 1]] - t[w * 8 + order[ph]]));
    std::sort(d.begin(), d.end());
    printf("  phase %-34s median %7.0f  p10 %7.0f  p90 %7.0f ticks\n", names[ph], d[nwg / 2], d[nwg / 10], d[nwg * 9 / 10]);
  }
  return 0;
}
