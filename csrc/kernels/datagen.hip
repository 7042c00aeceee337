// Device render of the synthetic MNIST split (generator v3): one workgroup per image, each of 196
// lanes renders 4 consecutive pixels of it and stores them as one 4-byte word.  The per-pixel math
// is csrc/data/synth_render.h - the same expression the host generator evaluates, contraction off,
// so the bytes equal the host render's (tests/test_gpu_datagen.py).  The plan (96 B per sample) and
// the templates (1 MB) come from the host generator; the images (47 MB for the train split) are
// written straight into HBM, where the fused engine keeps them - no 47 MB host-to-device copy inside
// the reference's timer.
#include <hip/hip_runtime.h>

#include "../data/synth_render.h"
#include "../include/device_utils.h"
#include "../include/kernels.h"

namespace mnist {

namespace {
__global__ __launch_bounds__(256) void synth_render_kernel(const synth::Sample* __restrict__ plan,
                                                           const float* __restrict__ tmpl, uint32_t* __restrict__ out) {
  RW_ENTRY();
  const int64_t img = blockIdx.x;
  const int q = threadIdx.x;                     // pixels 4q .. 4q+3
  if (q >= synth::IMG * synth::IMG / 4) return;
  const synth::Sample s = plan[img];
  uint32_t v = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) v |= (uint32_t)synth::render_pixel(s, tmpl, 4 * q + j) << (8 * j);
  out[img * (synth::IMG * synth::IMG / 4) + q] = v;
}
}  // namespace

void launch_synth_render(const void* plan, const float* templates, int64_t n, uint8_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(synth_render_kernel, dim3((unsigned)n), dim3(256), 0, s,
                     static_cast<const synth::Sample*>(plan), templates, reinterpret_cast<uint32_t*>(out));
}

}  // namespace mnist
