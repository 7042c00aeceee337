// Per-phase timing of trunk_fwd: compiles the kernel with MNIST_PHASE_TIMING (thread 0 of every
// workgroup stamps s_memtime at each phase boundary) and prints per-phase medians over workgroups.
// build: hipcc -x hip --offload-arch=gfx950 -O3 -fno-slp-vectorize -Icsrc/kernels tools/phase_timing.hip -o /tmp/phase_timing
// (-DTRUNK_SRC='"path"' times another revision of the kernel, e.g. a `git show` copy; see trunk_ab.sh)
#define MNIST_PHASE_TIMING 1
#ifndef TRUNK_SRC
#define TRUNK_SRC "../csrc/kernels/trunk_fwd.hip"
#endif
#include TRUNK_SRC

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <class T> T* dev_fill(size_t n, T v) {
  std::vector<T> h(n, v);
  T* d; CK(hipMalloc(&d, n * sizeof(T))); CK(hipMemcpy(d, h.data(), n * sizeof(T), hipMemcpyHostToDevice)); return d;
}

int main(int argc, char** argv) {
  using namespace mnist;
  const int B = argc > 1 ? atoi(argv[1]) : 200;
  if (3 * B > mnist::kPhaseMaxWG) { printf("B too large for the timing buffer (max %d)\n", mnist::kPhaseMaxWG / 3); return 1; }
  const int N = std::max(1024, B);
  std::vector<uint8_t> img((size_t)N * 784);
  for (auto& x : img) x = (uint8_t)(rand() & 0xFF);
  uint8_t* d_img; CK(hipMalloc(&d_img, img.size())); CK(hipMemcpy(d_img, img.data(), img.size(), hipMemcpyHostToDevice));
  std::vector<int32_t> idx(B); for (int i = 0; i < B; ++i) idx[i] = (i * 7) % N;
  int32_t* d_idx; CK(hipMalloc(&d_idx, B * 4)); CK(hipMemcpy(d_idx, idx.data(), B * 4, hipMemcpyHostToDevice));
  StepState st{0, 0, 0x1234, 0};
  StepState* d_st; CK(hipMalloc(&d_st, sizeof(st))); CK(hipMemcpy(d_st, &st, sizeof(st), hipMemcpyHostToDevice));
  float* w1c = dev_fill<float>(32 * 9, 0.05f);
  float* b1c = dev_fill<float>(32, 0.01f);
  uint16_t* w2f = dev_fill<uint16_t>(64 * 9 * 32, 0x3C00);   // bf16 0.0078
  float* b2c = dev_fill<float>(64, 0.0f);
  uint16_t* a1 = dev_fill<uint16_t>((size_t)B * 26 * 26 * 32, 0);
  uint16_t* p = dev_fill<uint16_t>((size_t)B * 9216, 0);
  uint8_t* pm = dev_fill<uint8_t>((size_t)B * 9216, 0);
  const bool pre = argc > 2 && atoi(argv[2]) == 1;   // 1: pre-gathered rows (no index load)
  TrunkFwdArgs a{d_img, pre ? nullptr : d_idx, 0, d_st, w1c, b1c, w2f, b2c, a1, p, pm, nullptr};
  for (int it = 0; it < 5; ++it) launch_trunk_fwd(a, B, true, nullptr);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  constexpr int kReps = 50;
  CK(hipEventRecord(e0, nullptr));
  for (int it = 0; it < kReps; ++it) launch_trunk_fwd(a, B, true, nullptr);
  CK(hipEventRecord(e1, nullptr));
  CK(hipDeviceSynchronize());
  float ms = 0; CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= kReps;
  const int nwg = 3 * B / trunk_strips_per_wg(B);
  constexpr int S = kPhaseSlots;
  std::vector<uint64_t> t((size_t)nwg * S);
  CK(hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_phase_times), t.size() * 8));
  const char* names[6] = {"0 loads+W2/x staging", "1 conv1 (VALU)", "1b W2 tail", "2 conv2 MFMA",
                          "3 pool epilogue", "4 dropout+stores"};
  printf("B=%d  kernel %.2f us (events, mean of 50 back-to-back), %d WGs; s_memtime ticks are per-XCD shader clocks\n", B, ms * 1000, nwg);
  std::vector<double> tot;
  for (int w = 0; w < nwg; ++w) tot.push_back((double)(t[w * S + 6] - t[w * S]));
  std::sort(tot.begin(), tot.end());
  printf("  WG lifetime ticks: median %.0f  p10 %.0f  p90 %.0f\n", tot[nwg / 2], tot[nwg / 10], tot[nwg * 9 / 10]);
  {  // per-XCD (WG id % 8 shares a clock) dispatch spread and span
    std::vector<double> st, sp;
    for (int x = 0; x < 8; ++x) {
      uint64_t lo = ~0ull, hi = 0, last_start = 0;
      for (int w = x; w < nwg; w += 8) {
        lo = std::min(lo, t[w * S]); hi = std::max(hi, t[w * S + 6]); last_start = std::max(last_start, t[w * S]);
      }
      st.push_back((double)(last_start - lo)); sp.push_back((double)(hi - lo));
    }
    std::sort(st.begin(), st.end()); std::sort(sp.begin(), sp.end());
    printf("  per-XCD: last WG start after first %.0f..%.0f ticks, first start -> last end %.0f..%.0f ticks\n",
           st[0], st[7], sp[0], sp[7]);
  }
  for (int ph = 0; ph < 6; ++ph) {
    std::vector<double> d;
    for (int w = 0; w < nwg; ++w) d.push_back((double)(t[w * S + ph + 1] - t[w * S + ph]));
    std::sort(d.begin(), d.end());
    printf("  phase %-22s median %7.0f  p90 %7.0f ticks\n", names[ph], d[nwg / 2], d[nwg * 9 / 10]);
  }
  return 0;
}
