// Small kernels of the DDP gradient reducer (runtime/bucket_reducer.cpp): the copy of one
// parameter's gradient into its bucket view, pre-scaled by 1/world_size (torch DDP's
// "divide before all-reduce", reducer.hpp copy_grad_to_bucket), 16 B per lane where aligned.
#include "../include/kernels.h"

namespace mnist {

__global__ __launch_bounds__(256) void scale_copy_kernel(float* __restrict__ dst, const float* __restrict__ src,
                                                          int64_t n, float s) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool vec = ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0;
  if (vec) {
    const int64_t n4 = n >> 2;
    for (int64_t i = i0; i < n4; i += stride) {
      float4 v = reinterpret_cast<const float4*>(src)[i];
      v.x *= s; v.y *= s; v.z *= s; v.w *= s;
      reinterpret_cast<float4*>(dst)[i] = v;
    }
    for (int64_t i = (n4 << 2) + i0; i < n; i += stride) dst[i] = src[i] * s;
  } else {
    for (int64_t i = i0; i < n; i += stride) dst[i] = src[i] * s;
  }
}

void launch_scale_copy(float* dst, const float* src, int64_t n, float s, hipStream_t stream) {
  if (n <= 0) return;
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(scale_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, dst, src, n, s);
}

}  // namespace mnist
