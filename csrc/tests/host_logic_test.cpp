// Host-logic unit test, built and run under AddressSanitizer + UndefinedBehaviorSanitizer on the CPU
// (tools/sanitize_host.sh; tests/test_host_sanitizers.py).  Covers the parts of the native runtime
// that parse peer data or carve memory by hand (csrc/runtime/host_logic.h):
//   * the engine workspace layout for every batch capacity 1..9000 (+ eval capacities): buffers are
//     256-B aligned, disjoint, inside the allocation, and large enough for their contents;
//   * the xGMI record decoder: round trip, and rejection of truncated / oversized / mismatched /
//     unterminated records, plus random byte soup (must throw, never read out of bounds);
//   * the residency planner's grid fitting.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <utility>

#include "../runtime/host_logic.h"

using namespace mnist;

static int failures = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      fprintf(stderr, "%s:%d CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                     \
    }                                                                 \
  } while (0)

static int wgrad_groups(int B) {   // conv_bwd.hip's conv_wgrad_groups (monotonic, <= 256)
  const int g = (24 * B + 7) / 8;   // rows = H2 * B, WG_CH = 8 rows per chunk
  return g < 256 ? g : 256;
}

static void test_workspace() {
  const int caps[] = {0, 1, 1000, 10000};
  for (int B = 1; B <= 9000; B += (B < 300 ? 1 : 97)) {
    for (int T : caps) {
      const WorkspaceLayout L = compute_workspace_layout(B, T, wgrad_groups(B), fc_bwd_splits(B));
      const int64_t Ma = std::max<int64_t>(B, T);
      std::vector<std::pair<int64_t, int64_t>> bufs = {
          {L.a1, (int64_t)B * H1 * H1 * C1 * 2}, {L.p, ((Ma + 63) / 64 * 64) * NFLAT * 2},
          {L.pmask, (int64_t)B * NFLAT},          {L.z1part, (int64_t)FC1_KSPLIT * Ma * NH * 4},
          {L.loss_rows, (int64_t)B * 4},          {L.dz1, ((B + 63) / 64 * 64) * NH * 2},
          {L.h_bf, ((B + 63) / 64 * 64) * NH * 2}, {L.dl_bf, ((B + 63) / 64 * 64) * 16 * 2},
          {L.dyc, (int64_t)B * DYC_BYTES_PER_IMAGE}, {L.c1part, 4LL * B * 320 * 4},
          {L.w2part, (int64_t)wgrad_groups(B) * (18432 + 64) * 4},
          {L.fcpart, fc_bwd_splits(B) > 1 ? (int64_t)fc_bwd_splits(B) * FCB_PART_STRIDE * 4 : 4},
          {L.sync, 64},                           {L.w2d_alt, 9LL * C1 * C2 * 2},
          {L.c1red, (int64_t)C1_PRE_SLABS * 320 * 4}, {L.w1t_alt, (int64_t)NFLAT * NH * 2}};
      std::sort(bufs.begin(), bufs.end());
      int64_t end = 0;
      for (auto& b : bufs) {
        CHECK(b.first % 256 == 0);
        CHECK(b.first >= end);                    // disjoint
        end = b.first + b.second;
      }
      CHECK(end <= L.total);
    }
  }
  bool threw = false;
  try {
    compute_workspace_layout(0, 0, 1, 1);
  } catch (const std::runtime_error&) {
    threw = true;
  }
  CHECK(threw);
}

static XgmiGrids grids() {
  XgmiGrids g{};
  g.fc_fused = 73; g.conv_fused = 309; g.twoshot = 145; g.oneshot = 19;
  return g;
}

static XgmiRecord make_record(int q) {
  XgmiRecord r;
  memset(&r, 0, sizeof(r));
  r.blk_off = 0; r.layout = xgmi_block_layout(1200000, 2, 32768); r.numel = 1200000; r.oneshot_max = 32768;
  r.world = 8; r.rank = q; r.channels = 2; r.pid = 1234; r.device = q;
  const XgmiGrids g = grids();
  r.grid_fc = g.fc_fused; r.grid_conv = g.conv_fused; r.grid_two = g.twoshot; r.grid_one = g.oneshot;
  snprintf(r.host, sizeof(r.host), "node-a");
  return r;
}

static bool rejects(const std::vector<uint8_t>& bytes, int q) {
  try {
    decode_record(bytes, q, 8, 1200000, 2, 32768, grids(), "node-a");
  } catch (const std::runtime_error&) {
    return true;
  }
  return false;
}

static void test_records() {
  for (int q = 0; q < 8; ++q) {
    const std::vector<uint8_t> enc = encode_record(make_record(q));
    const XgmiRecord back = decode_record(enc, q, 8, 1200000, 2, 32768, grids(), "node-a");
    CHECK(back.rank == q && back.layout.out_off >= back.layout.in_off + 4800000 && back.device == q);
    CHECK(back.layout.bytes % 4096 == 0 && back.layout.sig_off + 64 <= back.layout.bytes);
    CHECK(rejects(enc, (q + 1) % 8));                                   // wrong rank slot
    std::vector<uint8_t> shorter(enc.begin(), enc.end() - 1), longer = enc;
    longer.push_back(0);
    CHECK(rejects(shorter, q));
    CHECK(rejects(longer, q));
    CHECK(rejects({}, q));
    XgmiRecord r = make_record(q);
    r.numel = 4; CHECK(rejects(encode_record(r), q));
    r = make_record(q); r.grid_conv = 87; CHECK(rejects(encode_record(r), q));
    r = make_record(q); r.blk_off = -256; CHECK(rejects(encode_record(r), q));
    r = make_record(q); r.blk_off = 6; CHECK(rejects(encode_record(r), q));
    r = make_record(q); r.layout.out_off += 4096; CHECK(rejects(encode_record(r), q));
    r = make_record(q); r.layout.bytes -= 4096; CHECK(rejects(encode_record(r), q));
    r = make_record(q); snprintf(r.host, sizeof(r.host), "node-b"); CHECK(rejects(encode_record(r), q));
    r = make_record(q); memset(r.host, 'x', sizeof(r.host)); CHECK(rejects(encode_record(r), q));   // no NUL
  }
  std::mt19937_64 rng(7);
  for (int it = 0; it < 20000; ++it) {                                  // byte soup: reject, never crash
    std::vector<uint8_t> junk(rng() % (2 * sizeof(XgmiRecord) + 1));
    for (auto& b : junk) b = (uint8_t)rng();
    if (junk.size() == sizeof(XgmiRecord) && it % 2 == 0) {            // plausible header, garbage rest
      XgmiRecord r = make_record(3);
      memcpy(junk.data(), &r, offsetof(XgmiRecord, blk_off));
    }
    (void)rejects(junk, 3);
  }
}

static void test_ddp_scale() {
  // world W: head 1/(B*W), epilogues 1.0 - the W-rank SUM of per-rank gradients is the mean-NLL
  // gradient of the W*B batch; the same constant as the world-1 run on W*B rows (bitwise)
  CHECK(ddp_head_inv_batch(200, 8) == 1.0f / 1600.0f);
  CHECK(ddp_head_inv_batch(1600, 1) == ddp_head_inv_batch(200, 8));
  CHECK(ddp_head_inv_batch(200, 1) == 1.0f / 200.0f);
  CHECK(kDdpEpilogueScale == 1.0f);
  bool threw = false;
  try {
    ddp_head_inv_batch(0, 8);
  } catch (const std::runtime_error&) {
    threw = true;
  }
  CHECK(threw);
}

static void test_fit() {
  int a = 145, b = 309;
  double l = fit_grid_pair(&a, 8, 1024, &b, 39, 1024, 1, 0.5);
  CHECK(a == 145 && b == 309 && l < 0.5);                               // one rank per GPU: untouched
  a = 145; b = 309;
  l = fit_grid_pair(&a, 8, 1024, &b, 39, 1024, 4, 0.5);
  CHECK(l <= 0.5 + 1e-9 && a >= 8 && b >= 39 && a < 145 && b < 309);  // four ranks: shrunk to fit
  a = 512; b = 512;
  l = fit_grid_pair(&a, 400, 100, &b, 400, 100, 8, 0.5);
  CHECK(a == 400 && b == 400 && l > 1.0);                               // minimums cannot fit: reported
  bool threw = false;
  try {
    fit_grid_pair(&a, 1, 0, &b, 1, 1, 1, 0.5);
  } catch (const std::runtime_error&) {
    threw = true;
  }
  CHECK(threw);
}

int main() {
  test_workspace();
  test_records();
  test_fit();
  test_ddp_scale();
  if (failures) {
    fprintf(stderr, "HOST_LOGIC_TEST FAILED (%d)\n", failures);
    return 1;
  }
  printf("HOST_LOGIC_TEST PASS\n");
  return 0;
}
