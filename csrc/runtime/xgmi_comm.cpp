#include "xgmi_comm.h"

#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "../include/kernels.h"
#include "host_logic.h"

namespace mnist {

namespace {
void ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("xgmi: ") + what + ": " + hipGetErrorString(e));
}

// Process-wide free list of exported buffers, keyed by (device, bytes).  Exported buffers are never
// returned to the allocator (see the constructor); a communicator whose ranks all unmapped each
// other (close_peers + barrier + mark_recyclable) hands them to a later communicator of the same
// shape, so the test communicators of a long-lived process do not grow device memory by ~9.6 MB
// each.  Reuse hands out the SAME memory under the SAME IPC handle, so a peer's import cache maps
// the right pages; the 16-byte signatures are rewritten by every new communicator, so a peer that
// kept a stale mapping of an older communicator's buffer is still refused by connect().
std::mutex g_pool_mu;
std::map<std::pair<int, size_t>, std::vector<void*>> g_pool;

void* pool_take(int device, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  auto it = g_pool.find({device, bytes});
  if (it == g_pool.end() || it->second.empty()) return nullptr;
  void* p = it->second.back();
  it->second.pop_back();
  return p;
}

void pool_give(int device, size_t bytes, void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  g_pool[{device, bytes}].push_back(p);
}

void export_ptr(const void* p, hipIpcMemHandle_t* h, int64_t* off) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  ok(hipMemGetAddressRange(&base, &size, const_cast<void*>(p)), "hipMemGetAddressRange");
  ok(hipIpcGetMemHandle(h, base), "hipIpcGetMemHandle");
  *off = (int64_t)((const char*)p - (const char*)base);
}
}  // namespace

XgmiComm::XgmiComm(int world, int rank, int device, int64_t numel, int channels, int64_t oneshot_max,
                   int co_ranks, double budget)
    : world_(world), rank_(rank), device_(device), channels_(channels), numel_(numel), oneshot_max_(oneshot_max) {
  // the one-shot kernel keeps <= 4 float4 per lane of <= XGMI_MAX_WG workgroups
  if (oneshot_max < 0 || oneshot_max > 4LL * 4 * 256 * XGMI_MAX_WG || (oneshot_max & 3))
    throw std::runtime_error("xgmi: bad one-shot size");
  if (world < 1 || world > XGMI_MAX_RANKS) throw std::runtime_error("xgmi: world size must be 1..8");
  if (rank < 0 || rank >= world) throw std::runtime_error("xgmi: bad rank");
  if (channels < 1) throw std::runtime_error("xgmi: need at least one channel");
  if (numel < 4 || (numel & 3)) throw std::runtime_error("xgmi: numel must be a positive multiple of 4");
  ok(hipSetDevice(device), "hipSetDevice");
  grids_ = xgmi_plan_grids(world, co_ranks, oneshot_max, budget);   // throws when not co-resident
  // Every buffer a peer reads or writes lives in this communicator's own UNCACHED allocation
  // (hipDeviceMallocUncached: no L2 allocation on any XCD of any GPU).  The per-XCD L2s are not
  // coherent: with cached memory a clean line left in one XCD's L2 by an earlier plain access (a
  // fill, the optimizer's read of the reduced bucket, a previous call's gather) is served to a later
  // system-scope load from that XCD even after the owner rewrote the bytes write-through - observed
  // on one GPU as whole shards of stale sums.  Uncached, every load reaches memory.  The block is
  // never returned to the allocator either (never a block of torch's caching allocator): a later
  // allocation at the same address would carry an IPC handle a peer's import cache cannot tell
  // from the old one.  ONE block per rank (in | out | flags | staging | signatures): a peer maps it
  // with a single IPC import.
  const XgmiBlockLayout L = xgmi_block_layout(numel, channels, oneshot_max);
  block_bytes_ = L.bytes;
  block_ = static_cast<char*>(pool_take(device, (size_t)L.bytes));
  if (!block_) ok(hipExtMallocWithFlags(reinterpret_cast<void**>(&block_), (size_t)L.bytes, hipDeviceMallocUncached),
                  "hipExtMallocWithFlags(block)");
  in_ = reinterpret_cast<float*>(block_ + L.in_off);
  out_ = reinterpret_cast<float*>(block_ + L.out_off);
  flags_ = reinterpret_cast<int*>(block_ + L.flags_off);
  stage_ = reinterpret_cast<float*>(block_ + L.stage_off);
  ok(hipMalloc(&ctr_, sizeof(int) * XGMI_MAX_WG * channels), "hipMalloc(ctr)");
  ok(hipMalloc(&err_, sizeof(int)), "hipMalloc(err)");
  ok(hipMalloc(&timeout_, sizeof(uint64_t)), "hipMalloc(timeout)");
  launch_fill(block_, L.sig_off, 0, nullptr);
  launch_fill(ctr_, (int64_t)sizeof(int) * XGMI_MAX_WG * channels, 0, nullptr);
  launch_fill(err_, (int64_t)sizeof(int), 0, nullptr);
  ok(hipGetLastError(), "fill");
  // signatures {magic, rank, pid, region id} that peers read back through their mapping after
  // connect() (a mapping that does not show them is refused)
  int32_t sig[4][4];
  for (int id = 0; id < 4; ++id) {
    sig[id][0] = kSigMagic;
    sig[id][1] = rank;
    sig[id][2] = (int32_t)getpid();
    sig[id][3] = id;
  }
  ok(hipMemcpy(block_ + L.sig_off, sig, sizeof(sig), hipMemcpyHostToDevice), "hipMemcpy(signature)");
  ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
  set_timeout_seconds(60.0);
  if (world == 1) {                       // nothing to map: the kernel runs against itself
    peer_in_.assign(1, in_);
    peer_out_.assign(1, out_);
    peer_flags_.assign(1, flags_);
    peer_stage_.assign(1, stage_);
    connected_ = true;
  }
}

XgmiComm::~XgmiComm() {
  close_peers();
  // the block was exported: never freed (see the constructor); returned to the process-wide free
  // list only when every peer is known to have unmapped it (mark_recyclable)
  if (recyclable_) pool_give(device_, (size_t)block_bytes_, block_);
  if (ctr_) hipFree(ctr_);
  if (err_) hipFree(err_);
  if (timeout_) hipFree(timeout_);
}

void XgmiComm::close_peers() {
  hipSetDevice(device_);
  hipDeviceSynchronize();
  for (void* p : opened_) hipIpcCloseMemHandle(p);
  opened_.clear();
  if (world_ > 1) connected_ = false;
}

void XgmiComm::set_timeout_seconds(double s) {
  const uint64_t t = (uint64_t)(s * 1e8);
  ok(hipSetDevice(device_), "hipSetDevice");
  ok(hipMemcpy(timeout_, &t, sizeof(t), hipMemcpyHostToDevice), "hipMemcpy(timeout)");
}

std::vector<uint8_t> XgmiComm::record() const {
  XgmiRecord r;
  memset(&r, 0, sizeof(r));
  export_ptr(block_, &r.blk_h, &r.blk_off);
  r.layout = xgmi_block_layout(numel_, channels_, oneshot_max_);
  r.numel = numel_;
  r.oneshot_max = oneshot_max_;
  r.world = world_;
  r.rank = rank_;
  r.channels = channels_;
  r.pid = (int32_t)getpid();
  r.device = device_;
  r.grid_fc = grids_.fc_fused;
  r.grid_conv = grids_.conv_fused;
  r.grid_two = grids_.twoshot;
  r.grid_one = grids_.oneshot;
  gethostname(r.host, sizeof(r.host) - 1);
  return encode_record(r);
}

void XgmiComm::connect(const std::vector<std::vector<uint8_t>>& records) {
  if ((int)records.size() != world_) throw std::runtime_error("xgmi: need one record per rank");
  ok(hipSetDevice(device_), "hipSetDevice");
  peer_in_.assign(world_, nullptr);
  peer_out_.assign(world_, nullptr);
  peer_flags_.assign(world_, nullptr);
  peer_stage_.assign(world_, nullptr);
  char host[64] = {0};
  gethostname(host, sizeof(host) - 1);
  for (int q = 0; q < world_; ++q) {
    const XgmiRecord r = decode_record(records[q], q, world_, numel_, channels_, oneshot_max_, grids_, host);
    if (q == rank_) {
      peer_in_[q] = in_;
      peer_out_[q] = out_;
      peer_flags_[q] = flags_;
      peer_stage_[q] = stage_;
      continue;
    }
    if (r.device != device_) {
      int can = 0;
      ok(hipDeviceCanAccessPeer(&can, device_, r.device), "hipDeviceCanAccessPeer");
      if (!can) throw std::runtime_error("xgmi: no peer access to device " + std::to_string(r.device));
    }
    void* p = nullptr;
    ok(hipIpcOpenMemHandle(&p, r.blk_h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    opened_.push_back(p);
    char* b = static_cast<char*>(p) + r.blk_off;
    peer_in_[q] = reinterpret_cast<const float*>(b + r.layout.in_off);
    peer_out_[q] = reinterpret_cast<float*>(b + r.layout.out_off);
    peer_flags_[q] = reinterpret_cast<int*>(b + r.layout.flags_off);
    peer_stage_[q] = reinterpret_cast<float*>(b + r.layout.stage_off);
    // read the block's signatures through the new mapping: they must be peer q's
    int32_t sig[4][4];
    ok(hipMemcpy(sig, b + r.layout.sig_off, sizeof(sig), hipMemcpyDeviceToHost), "hipMemcpy(peer signature)");
    for (int id = 0; id < 4; ++id)
      if (sig[id][0] != kSigMagic || sig[id][1] != q || sig[id][2] != r.pid || sig[id][3] != id)
        throw std::runtime_error("xgmi: the IPC mapping of rank " + std::to_string(q) +
                                 "'s block does not show its signature (got rank " + std::to_string(sig[id][1]) +
                                 ", pid " + std::to_string(sig[id][2]) + ", region " + std::to_string(sig[id][3]) +
                                 ")");
  }
  connected_ = true;
}

XgmiArgs XgmiComm::args(int channel, int64_t offset, int64_t count) const {
  if (channel < 0 || channel >= channels_) throw std::runtime_error("xgmi: bad channel");
  if (offset < 0 || count < 0 || offset + count > numel_ || (offset & 3) || (count & 3))
    throw std::runtime_error("xgmi: range must lie in the buffer, offset and count multiples of 4");
  if (!connected_) throw std::runtime_error("xgmi: connect() first");
  XgmiArgs a;
  memset(&a, 0, sizeof(a));
  for (int q = 0; q < world_; ++q) {
    a.in[q] = peer_in_[q] + offset;
    a.out[q] = peer_out_[q] + offset;
    a.flags[q] = peer_flags_[q] + (int64_t)channel * XGMI_FLAG_INTS;
    a.stage[q] = peer_stage_[q] + (int64_t)channel * 2 * oneshot_max_;
  }
  a.slot_floats = oneshot_max_;
  a.ctr = ctr_ + (int64_t)channel * XGMI_MAX_WG;
  a.err = err_;
  a.world = world_;
  a.rank = rank_;
  a.nvec = count / 4;
  a.timeout_ticks = timeout_;
  a.max_wg = XGMI_MAX_WG;
  // system-scope release fence before every stage flag (buffer_wbl2 of the XCD's dirty L2 lines) +
  // acquire after every matched poll: off by default - rules R1-R4 in xgmi_allreduce.hip order the
  // payload without them; the release fence measured +13 us per world-1 step (100.5 vs 87.5)
  a.release = a.acquire = fences_ ? 1 : 0;
  return a;
}

std::string XgmiComm::ordering() const {
  return fences_ ? "uncached+sc0sc1+release+acquire (fenced: the unfenced schedule failed validation)"
                 : "uncached+sc0sc1 (no fence: xgmi_allreduce.hip R1-R4)";
}

void XgmiComm::allreduce_fc_fused(int channel, hipStream_t stream, const AdadeltaArgs& ada) {
  XgmiArgs a = args(channel, OFF_FC1_W, OFF_CONV1_W - OFF_FC1_W);
  a.fuse_ada = 1;
  a.ada_base = OFF_FC1_W;
  a.ada = ada;
  a.max_wg = grids_.fc_fused;
  launch_xgmi_fc_fused(a, stream);
}

void XgmiComm::conv_reduce_fused(int channel, const ConvBwdArgs& conv, int B, hipStream_t stream,
                                 const AdadeltaArgs& ada, const XgmiConvPart& part) {
  XgmiArgs a = args(channel, OFF_CONV1_W, PARAM_TOTAL - OFF_CONV1_W);
  if (PARAM_TOTAL - OFF_CONV1_W > oneshot_max_) throw std::runtime_error("xgmi: conv bucket exceeds the staging slots");
  a.fuse_ada = 1;
  a.ada_base = OFF_CONV1_W;
  a.ada = ada;
  a.max_wg = grids_.conv_fused;
  launch_xgmi_conv_reduce_fused(a, conv, B, stream, part);
}

void XgmiComm::allreduce(int channel, int64_t offset, int64_t count, hipStream_t stream, const AdadeltaArgs* ada) {
  XgmiArgs a = args(channel, offset, count);
  if (count == 0) return;
  if (ada) {
    a.fuse_ada = 1;
    a.ada_base = offset;
    a.ada = *ada;
  }
  if (count <= oneshot_max_) {
    a.max_wg = grids_.oneshot;
    launch_xgmi_allreduce_oneshot(a, stream);
  } else {
    a.max_wg = grids_.twoshot;
    launch_xgmi_allreduce(a, stream);
  }
}

void XgmiComm::stage_out(const float* buf, int64_t count, hipStream_t stream) {
  if (count < 0 || count > numel_) throw std::runtime_error("xgmi: stage_out count out of range");
  ok(hipMemcpyAsync(out_, buf, sizeof(float) * count, hipMemcpyDeviceToDevice, stream), "hipMemcpyAsync(stage_out)");
}

void XgmiComm::read_peer_out(int peer, float* buf, int64_t count, hipStream_t stream) {
  if (!connected_) throw std::runtime_error("xgmi: connect() first");
  if (peer < 0 || peer >= world_ || count < 0 || count > numel_) throw std::runtime_error("xgmi: read_peer_out range");
  ok(hipMemcpyAsync(buf, peer_out_[peer], sizeof(float) * count, hipMemcpyDeviceToDevice, stream),
     "hipMemcpyAsync(read_peer_out)");
}

int XgmiComm::error() const {
  int v = 0;
  ok(hipMemcpy(&v, err_, sizeof(int), hipMemcpyDeviceToHost), "hipMemcpy(err)");
  return v;
}

}  // namespace mnist
