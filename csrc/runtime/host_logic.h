// Pure host-side logic of the runtime, kept free of HIP calls so it can be unit-tested on the CPU
// under AddressSanitizer / UndefinedBehaviorSanitizer (csrc/tests/host_logic_test.cpp,
// tools/sanitize_host.sh):
//   * the engine's workspace carve (offsets of every activation buffer for a batch capacity);
//   * the xGMI IPC export record: encode / decode / validation against this communicator;
//   * the residency planner's grid fitting;
//   * the DDP gradient scaling constants the engine hands its kernels.
#pragma once
#include <stdint.h>
#include <string.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "../include/kernels.h"

namespace mnist {

// ---------------------------------------------------------------------------- DDP gradient scaling
// The engine folds DDP's 1/world averaging into the head's loss-gradient scale: every rank's head
// scales by 1/(B * world) and the all-reduce SUMS, so each row's bf16 gradient operands are bitwise
// those of the world-1 run on the world*B batch.  The GEMM / slab-reduce epilogues then get 1.0
// (FcBwdArgs::grad_scale, ConvBwdArgs::grad_scale) - a caller that also divided there would
// average twice.
inline float ddp_head_inv_batch(int batch, int world) {
  if (batch < 1 || world < 1) throw std::runtime_error("ddp scale: bad batch / world");
  return 1.0f / (float)(batch * world);
}
constexpr float kDdpEpilogueScale = 1.0f;

// ---------------------------------------------------------------------------- engine workspace
struct WorkspaceLayout {
  int64_t a1, p, pmask, z1part, loss_rows, dz1, h_bf, dl_bf, dyc, c1part, w2part, fcpart, sync, w2d_alt, c1red,
      w1t_alt;
  int64_t total;   // bytes
};

inline int64_t ws_align256(int64_t x) { return (x + 255) & ~int64_t(255); }

// wgrad_groups = conv_wgrad_groups(max_batch), fc_splits = fc_bwd_splits(max_batch) (both monotonic in B)
inline WorkspaceLayout compute_workspace_layout(int max_batch, int max_test_batch, int wgrad_groups, int fc_splits) {
  if (max_batch < 1 || max_test_batch < 0 || wgrad_groups < 1 || fc_splits < 1)
    throw std::runtime_error("workspace layout: bad sizes");
  auto round_up = [](int64_t x, int64_t m) { return (x + m - 1) / m * m; };
  // forward activations (p, fc1 partials) serve the training and the eval batch; backward-only
  // buffers only the training batch
  const int64_t Ma = max_batch > max_test_batch ? max_batch : max_test_batch;
  const int64_t M = max_batch;
  const int64_t Mp = round_up(M, 64), Map = round_up(Ma, 64);
  WorkspaceLayout L{};
  int64_t off = 0;
  auto carve = [&](int64_t bytes) { int64_t o = off; off += ws_align256(bytes); return o; };
  L.a1 = carve(M * H1 * H1 * C1 * 2);
  L.p = carve(Map * NFLAT * 2);
  L.pmask = carve(M * NFLAT);
  L.z1part = carve((int64_t)FC1_KSPLIT * Ma * NH * 4);
  L.loss_rows = carve(M * 4);
  L.dz1 = carve(Mp * NH * 2);
  L.h_bf = carve(Mp * NH * 2);
  L.dl_bf = carve(Mp * 16 * 2);
  L.dyc = carve(M * DYC_BYTES_PER_IMAGE);   // compact dy records
  L.c1part = carve(4 * M * 320 * 4);
  L.w2part = carve((int64_t)wgrad_groups * (18432 + 64) * 4);
  L.fcpart = carve(fc_splits > 1 ? (int64_t)fc_splits * FCB_PART_STRIDE * 4 : 256);   // large-batch partials
  L.sync = carve(256);                                                                // hand-off counters
  L.w2d_alt = carve((int64_t)9 * C1 * C2 * 2);                                         // alternate w2d
  L.c1red = carve((int64_t)C1_PRE_SLABS * 320 * 4);                                    // conv1 group sums
  L.w1t_alt = carve((int64_t)NFLAT * NH * 2);                                          // alternate w1t
  L.total = off;
  return L;
}

// ---------------------------------------------------------------------------- xGMI export block
// Everything a peer reads or writes lives in ONE exported allocation per rank, so a peer maps it
// with one hipIpcOpenMemHandle (W-1 per rank instead of 4(W-1): the IPC import is the dominant
// per-peer setup cost inside the reference's timer).  Regions 4 KiB aligned:
//   in [numel f32] | out [numel f32] | flags [channels][XGMI_FLAG_INTS] | stage [channels][2][oneshot_max] (+4) | sig [4][4 int32]
struct XgmiBlockLayout {
  int64_t in_off, out_off, flags_off, stage_off, sig_off, bytes;
};
constexpr int64_t kXgmiSigBytes = 16;
inline XgmiBlockLayout xgmi_block_layout(int64_t numel, int channels, int64_t oneshot_max) {
  if (numel < 4 || channels < 1 || oneshot_max < 0) throw std::runtime_error("xgmi block layout: bad sizes");
  auto al = [](int64_t x) { return (x + 4095) & ~int64_t(4095); };
  XgmiBlockLayout L{};
  L.in_off = 0;
  L.out_off = al(L.in_off + 4 * numel);
  L.flags_off = al(L.out_off + 4 * numel);
  L.stage_off = al(L.flags_off + 4LL * XGMI_FLAG_INTS * channels);
  L.sig_off = al(L.stage_off + 4LL * (2 * oneshot_max + 4) * channels);
  L.bytes = al(L.sig_off + 4 * kXgmiSigBytes);
  return L;
}

// ---------------------------------------------------------------------------- xGMI export record
// What one rank publishes (through the c10d store) about its block; peers map it with IPC.
struct XgmiRecord {
  hipIpcMemHandle_t blk_h;
  int64_t blk_off;                                  // the block's offset inside the IPC allocation
  XgmiBlockLayout layout;
  int64_t numel, oneshot_max;
  int32_t world, rank, channels, pid, device;
  int32_t grid_fc, grid_conv, grid_two, grid_one;   // residency-planned grids (must agree across ranks)
  char host[64];                                    // IPC mappings only exist between the GPUs of one node
};

inline std::vector<uint8_t> encode_record(const XgmiRecord& r) {
  const uint8_t* b = reinterpret_cast<const uint8_t*>(&r);
  return std::vector<uint8_t>(b, b + sizeof(r));
}

// Decode peer q's record and check it against this communicator; throws with the reason.
inline XgmiRecord decode_record(const std::vector<uint8_t>& bytes, int q, int world, int64_t numel, int channels,
                                int64_t oneshot_max, const XgmiGrids& grids, const char* my_host) {
  if (bytes.size() != sizeof(XgmiRecord)) throw std::runtime_error("xgmi: bad record size");
  XgmiRecord r;
  memcpy(&r, bytes.data(), sizeof(r));
  if (r.rank != q || r.world != world || r.numel != numel || r.channels != channels || r.oneshot_max != oneshot_max)
    throw std::runtime_error("xgmi: peer record does not match this communicator");
  const XgmiBlockLayout L = xgmi_block_layout(numel, channels, oneshot_max);
  if (r.blk_off < 0 || r.blk_off % 256 || memcmp(&r.layout, &L, sizeof(L)) != 0)
    throw std::runtime_error("xgmi: peer record has a different buffer layout");
  if (r.grid_fc != grids.fc_fused || r.grid_conv != grids.conv_fused || r.grid_two != grids.twoshot ||
      r.grid_one != grids.oneshot)
    throw std::runtime_error("xgmi: ranks planned different kernel grids (mixed GPUs or co_ranks?)");
  if (memchr(r.host, 0, sizeof(r.host)) == nullptr) throw std::runtime_error("xgmi: peer host name not terminated");
  if (strncmp(my_host, r.host, sizeof(r.host)) != 0)
    throw std::runtime_error("xgmi: ranks span more than one node (peer on " + std::string(r.host) + ")");
  return r;
}

// ---------------------------------------------------------------------------- residency planner
// Shrink grids a (minimum amin, capacity ca) and b so that co * (a/ca + b/cb) <= budget; returns
// the resulting load (may stay above budget when the minimums do not fit).
inline double fit_grid_pair(int* a, int amin, int ca, int* b, int bmin, int cb, int co, double budget) {
  if (ca < 1 || cb < 1 || co < 1 || budget <= 0.0) throw std::runtime_error("fit_grid_pair: bad arguments");
  auto load = [&] { return co * ((double)*a / ca + (double)*b / cb); };
  if (load() > budget) {
    const double s = budget / load();
    const int na = (int)(*a * s), nb = (int)(*b * s);
    *a = na > amin ? na : amin;
    *b = nb > bmin ? nb : bmin;
  }
  return load();
}

}  // namespace mnist
