// Shared constants and device helpers for the MI355X (gfx950 / CDNA4) MNIST kernels.
//
// Model = the reference `Net` (reference mnist_ddp.py:39-62):
//   conv1 1->32 3x3 -> relu -> conv2 32->64 3x3 -> relu -> maxpool 2x2 -> dropout(0.25)
//   -> flatten(9216) -> fc1 9216->128 -> relu -> dropout(0.5) -> fc2 128->10 -> log_softmax
//
// Layout conventions (all chosen for 64-wide wavefronts and MFMA fragment shapes):
//   a1      bf16 [B][26][26][32]   NHWC conv1 output (8 contiguous channels = one 16-B MFMA fragment)
//   p       bf16 [B][9216]         pooled+dropout output in torch flatten order (c*144 + y*12 + x)
//   pmask   u8   [B][36][64][4]    (pooled position / 4, channel, position % 4) bits 0-1 argmax in the
//                                   2x2 window, bit 2 dropout keep, bit 3 pooled>0 (functional.pmask_flat
//                                   gives the channel-major [B][9216] view)
//   w2f     bf16 [64][9][32]       conv2 weight, forward B operand  (co, tap, ci)
//   w2d     bf16 [9][32][64]       conv2 weight, dgrad B operand    (tap, ci, co)
//   w1      bf16 [128][9216]       fc1 weight (torch layout) - forward B operand
//   w1t     bf16 [9216][128]       fc1 weight transposed - dgrad B operand
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mnist {

constexpr int IMG = 28, H1 = 26, C1 = 32, H2 = 24, C2 = 64, HP = 12;
constexpr int NPOOL = HP * HP;          // 144
constexpr int NFLAT = C2 * NPOOL;       // 9216
constexpr int NH = 128, NCLS = 10;
constexpr float MNIST_MEAN = 0.1307f, MNIST_STD = 0.3081f;
constexpr float KEEP1 = 0.75f, KEEP2 = 0.5f;          // dropout(0.25), dropout(0.5)
// Dropout draws one random byte per element (16 elements per Philox-4x32-10 call); keep <=> byte < thr.
// 192/256 = 0.75 and 128/256 = 0.5 exactly, so the keep probabilities are exact.
constexpr uint32_t KEEP1_THR8 = 192u;
constexpr uint32_t KEEP2_THR8 = 128u;

// Flat fp32 parameter buffer: every tensor starts on a 64-element (256 B) boundary.
// Bucket 0 (fc params, ready first in backward) = [0, OFF_CONV1_W); bucket 1 = conv params.
constexpr int64_t OFF_FC1_W = 0, OFF_FC1_B = 1179648, OFF_FC2_W = 1179776, OFF_FC2_B = 1181056;
constexpr int64_t OFF_CONV1_W = 1181120, OFF_CONV1_B = 1181440, OFF_CONV2_W = 1181504,
                  OFF_CONV2_B = 1199936, PARAM_TOTAL = 1200000;

// Per-step device state read by every step kernel (so one captured graph can be replayed).
constexpr int32_t STEP_FLAG_NO_DROPOUT = 1;

struct StepState {
  int32_t step;        // step index within the epoch (advanced on device by the optimizer)
  int32_t flags;       // bit 0: dropout disabled (parity tests); other bits reserved
  uint64_t seed;       // dropout Philox key
  uint64_t rng_base;   // Philox counter base for this epoch; step s uses base + 2s (+1 for dropout2)
};

}  // namespace mnist
