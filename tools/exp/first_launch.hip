// Where a process's first kernel launch spends its time (startup inside the reference timer):
// context, code-object load, first launch + sync on the null stream or on a created stream, a second
// launch, the runtime's memset / copy paths.  usage: first_launch [stream|null]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_fill(unsigned* p, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0u;
}
__global__ void k_other(unsigned* p, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1u;
}

int main(int argc, char** argv) {
  const bool on_stream = argc > 1 && !strcmp(argv[1], "stream");
  using clk = std::chrono::steady_clock;
  auto t = clk::now();
  auto lap = [&](const char* what) {
    auto n = clk::now();
    printf("%-34s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  };
  hipSetDevice(0);
  hipFree(nullptr);
  lap("context (hipFree 0)");
  hipFuncAttributes fa;
  hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_fill));
  lap("hipFuncGetAttributes");
  unsigned* d = nullptr;
  hipMalloc(&d, 1 << 20);
  lap("hipMalloc 1 MB");
  hipStream_t s = nullptr;
  if (on_stream) {
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    lap("hipStreamCreate");
  }
  hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, s, d, 1 << 18);
  lap("first launch (enqueue)");
  hipStreamSynchronize(s);
  lap("first launch sync");
  hipLaunchKernelGGL(k_other, dim3(1024), dim3(256), 0, s, d, 1 << 18);
  hipStreamSynchronize(s);
  lap("second kernel + sync");
  hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, s, d, 1 << 18);
  hipStreamSynchronize(s);
  lap("third launch + sync");
  std::vector<char> h(1 << 20, 1);
  hipMemcpy(d, h.data(), 1 << 20, hipMemcpyHostToDevice);
  lap("first pageable H2D 1 MB");
  hipMemsetAsync(d, 0, 1 << 20, s);
  hipStreamSynchronize(s);
  lap("first hipMemsetAsync + sync");
  hipMemcpy(h.data(), d, 4096, hipMemcpyDeviceToHost);
  lap("first D2H 4 KB");
  hipMemcpyAsync(d + 1024, d, 4096, hipMemcpyDeviceToDevice, s);
  hipStreamSynchronize(s);
  lap("first D2D 4 KB + sync");
  return 0;
}
