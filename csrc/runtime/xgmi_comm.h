// Direct xGMI gradient all-reduce between the GPUs of one node (kernels/xgmi_allreduce.hip).
//
// The reference averages DDP gradients with ProcessGroupNCCL's ring all-reduce (mnist_ddp.py:173,
// reducer at :72).  On MI355X every GPU pair has its own xGMI link, so this communicator maps every
// peer's gradient buckets into its address space once (hipIpc handles exchanged through the c10d
// store) and reduces with one kernel per bucket: a reduce-scatter that pulls shard r of all peers
// over all links at once, then an all-gather of the reduced shards - two direct hops instead of the
// ring's 2(W-1).  Input (the producers' gradient buffer) and output (what the optimizer reads) are
// separate buffers, which removes the end-of-call barrier an in-place version needs.
//
// Channels: independent flag / counter sets, one per bucket that may be in flight concurrently with
// another (the engine's fc bucket on the comm stream, conv bucket on the compute stream).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>

#include "../include/kernels.h"

namespace mnist {

class XgmiComm {
 public:
  // The communicator owns this rank's flat input and output buffers (`numel` floats each, in() /
  // out(): the engine's gradient producers write in(), the optimizer reads out()).
  // Buckets of at most `oneshot_max` floats use the one-shot kernel (one hand-off per call; staging
  // slots allocated here, 2 per channel); larger ones the two-shot reduce-scatter + all-gather.
  // co_ranks: how many ranks drive this rank's GPU (1 in production; > 1 in the one-GPU multi-process
  // rehearsal) - the kernel grids are sized so every rank's spinning workgroups fit at once
  // (xgmi_plan_grids, `budget` = fraction of the GPU's workgroup slots they may take).
  XgmiComm(int world, int rank, int device, int64_t numel, int channels, int64_t oneshot_max = 32768,
           int co_ranks = 1, double budget = 0.5);
  ~XgmiComm();
  XgmiComm(const XgmiComm&) = delete;
  XgmiComm& operator=(const XgmiComm&) = delete;

  std::vector<uint8_t> record() const;                               // this rank's export record
  void connect(const std::vector<std::vector<uint8_t>>& records);   // every rank's, in rank order
  bool connected() const { return connected_; }

  // out[offset, offset+count) = sum over ranks of in[offset, offset+count); offset and count in
  // floats, multiples of 4.  Graph-capturable (no host work beyond the launch).
  // With `ada` (conv bucket of the engine): the kernel also applies the Adadelta step to the reduced
  // elements (flat parameter index = offset + bucket index) - see XgmiArgs::fuse_ada.
  void allreduce(int channel, int64_t offset, int64_t count, hipStream_t stream,
                 const AdadeltaArgs* ada = nullptr);
  // The engine's fc bucket (flat [0, OFF_CONV1_W)) with the fc Adadelta step and the w1 / w1t bf16
  // shadow refresh fused into the gather phase (launch_xgmi_fc_fused).
  void allreduce_fc_fused(int channel, hipStream_t stream, const AdadeltaArgs& ada);
  // The engine's conv bucket straight from the conv gradient slabs: slab reduce + one-shot
  // all-reduce + Adadelta + conv2 shadows in one launch (launch_xgmi_conv_reduce_fused).
  void conv_reduce_fused(int channel, const ConvBwdArgs& conv, int B, hipStream_t stream, const AdadeltaArgs& ada,
                         const XgmiConvPart& part = XgmiConvPart{});
  int channels() const { return channels_; }
  // device error code (0 = ok; else the first stage wait that timed out on this rank:
  // kernel id << 24 | stage << 16 | peer << 12 | workgroup); synchronous read
  int error() const;
  // how peer-visible payload is ordered (bench JSON "xgmi_ordering"; rules in xgmi_allreduce.hip)
  std::string ordering() const;
  // system-scope release fence before every stage flag + acquire after every matched poll (off by
  // default: rules R1-R4 in xgmi_allreduce.hip).  Read at launch / capture time: graphs captured
  // before a change keep the old mode.  The trainer turns it on when the unfenced schedule fails its
  // cross-rank validation with wrong sums (not a timeout) and validates again.
  void set_fences(bool on) { fences_ = on; }
  bool fences() const { return fences_; }
  const XgmiGrids& grids() const { return grids_; }
  // stage-wait timeout; kept in device memory and read by every stage wait, so it also applies to
  // graphs captured earlier (synchronous 8-byte copy: call while no xGMI kernel is running)
  void set_timeout_seconds(double s);
  // Buffer recycling.  The exported buffers are never returned to the allocator (a peer's import
  // cache could not tell a new allocation at the same address from the old one); a later
  // communicator of the same shape may reuse them - but only once EVERY peer has unmapped them, or a
  // late write of a peer's old kernel could satisfy a new wait.  close_peers() waits for this
  // device's work and unmaps the peers' buffers; after a barrier that every rank enters only after
  // its own close_peers(), mark_recyclable() lets the destructor hand the buffers to the free list
  // (without it they are leaked, as before).
  void close_peers();
  void mark_recyclable() { recyclable_ = true; }
  // broadcast helpers (host-ordered copies; the caller barriers between them): out()[0, count) =
  // buf on the root; buf = peer's out()[0, count) on the others
  void stage_out(const float* buf, int64_t count, hipStream_t stream);
  void read_peer_out(int peer, float* buf, int64_t count, hipStream_t stream);
  int world_size() const { return world_; }
  int rank() const { return rank_; }
  float* in() const { return in_; }
  float* out() const { return out_; }
  int64_t numel() const { return numel_; }
  int device() const { return device_; }

 private:
  int world_, rank_, device_, channels_;
  char* block_ = nullptr;    // the one IPC-exported allocation (host_logic.h xgmi_block_layout)
  int64_t block_bytes_ = 0;
  float *in_ = nullptr, *out_ = nullptr;
  int64_t numel_;
  int* flags_ = nullptr;     // [channels][XGMI_FLAG_INTS]
  float* stage_ = nullptr;   // [channels][2][oneshot_max_]
  bool recyclable_ = false;
  bool fences_ = false;
  int64_t oneshot_max_;
  int* ctr_ = nullptr;       // [channels][XGMI_MAX_WG], local
  int* err_ = nullptr;
  uint64_t* timeout_ = nullptr;   // device: stage-wait timeout in s_memrealtime ticks (100 MHz)
  XgmiGrids grids_;
  bool connected_ = false;
  std::vector<const float*> peer_in_;
  std::vector<float*> peer_out_;
  std::vector<int*> peer_flags_;
  std::vector<float*> peer_stage_;
  std::vector<void*> opened_;   // IPC mappings to close
  XgmiArgs args(int channel, int64_t offset, int64_t count) const;
  static constexpr int32_t kSigMagic = 0x58474d49;   // "XGMI"
};

}  // namespace mnist
