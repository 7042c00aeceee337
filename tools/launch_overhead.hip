// Fixed cost of a dependent kernel boundary inside a replayed hipGraph on gfx950: N back-to-back
// launches of a near-empty kernel (each workgroup writes one word, vector store) captured into one
// graph, replayed R times; prints us per launch for several grid sizes and block sizes.
// build: hipcc -x hip --offload-arch=gfx950 -O3 tools/launch_overhead.hip -o tools/launch_overhead.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void touch_kernel(int* out, int v) {
  if (threadIdx.x == 0) out[blockIdx.x] = v;
}

// same, with LDS use forcing fewer workgroups per CU (models the real kernels' residency)
__global__ void touch_lds_kernel(int* out, int v) {
  __shared__ int s[16384];   // 64 KB -> 2 workgroups per CU
  s[threadIdx.x] = v;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s[(threadIdx.x + 1) % blockDim.x];
}

int main() {
  int* d;
  CK(hipMalloc(&d, 1 << 20));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grids[] = {1, 64, 256, 512, 800, 2048};
  const int blocks[] = {64, 256, 768};
  const int N = 20, R = 200;
  for (int lds = 0; lds < 2; ++lds)
    for (int bi = 0; bi < 3; ++bi)
      for (int gi = 0; gi < 6; ++gi) {
        const int G = grids[gi], T = blocks[bi];
        if (lds && T == 768) continue;
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < N; ++i) {
          if (lds)
            hipLaunchKernelGGL(touch_lds_kernel, dim3(G), dim3(T), 0, s, d, i);
          else
            hipLaunchKernelGGL(touch_kernel, dim3(G), dim3(T), 0, s, d, i);
        }
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int w = 0; w < 5; ++w) CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < R; ++r) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipStreamSynchronize(s));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%s grid %5d block %4d: %.2f us per launch\n", lds ? "lds64K" : "plain ", G, T, ms * 1000.0 / (N * R));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
      }
  return 0;
}
