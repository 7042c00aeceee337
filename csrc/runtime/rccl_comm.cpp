#include "rccl_comm.h"

#include <dlfcn.h>
#include <stdexcept>
#include <string.h>
#include <time.h>

namespace mnist {

namespace {
// Minimal RCCL ABI (stable since NCCL 2.x): opaque comm, 128-byte unique id.
typedef void* ncclComm_t;
struct ncclUniqueId { char internal[RcclComm::kUniqueIdBytes]; };
typedef int ncclResult_t;
enum { ncclFloat32 = 7, ncclBfloat16 = 9 };   // ncclDataType_t values (rccl.h)
enum { ncclSum = 0 };
constexpr ncclResult_t ncclInProgress = 7;

// ncclConfig_t as of NCCL 2.17 (the config ABI is versioned: the library reads a config of an older
// version field by field and defaults the rest), so the layout does not depend on which RCCL torch
// bundles (2.26 in this image) or on /opt/rocm's header (2.27)
struct ConfigV21700 {
  size_t size;
  unsigned int magic;
  unsigned int version;
  int blocking;
  int cgaClusterSize;
  int minCTAs;
  int maxCTAs;
  const char* netName;
  int splitShare;
};
constexpr int kUndefInt = (int)0x80000000;   // NCCL_CONFIG_UNDEF_INT (INT_MIN)

struct Api {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitRankConfig)(ncclComm_t*, int, ncclUniqueId, int, ConfigV21700*) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GetVersion)(int*) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  bool ok = false;
};

void* find_sym(const char* name) {
  void* p = dlsym(RTLD_DEFAULT, name);
  if (!p) {
    static void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
    if (h) p = dlsym(h, name);
  }
  return p;
}

Api& api() {
  static Api a = [] {
    Api x;
    x.GetUniqueId = (decltype(x.GetUniqueId))find_sym("ncclGetUniqueId");
    x.CommInitRank = (decltype(x.CommInitRank))find_sym("ncclCommInitRank");
    x.CommInitRankConfig = (decltype(x.CommInitRankConfig))find_sym("ncclCommInitRankConfig");
    x.CommGetAsyncError = (decltype(x.CommGetAsyncError))find_sym("ncclCommGetAsyncError");
    x.CommAbort = (decltype(x.CommAbort))find_sym("ncclCommAbort");
    x.CommDestroy = (decltype(x.CommDestroy))find_sym("ncclCommDestroy");
    x.AllReduce = (decltype(x.AllReduce))find_sym("ncclAllReduce");
    x.Broadcast = (decltype(x.Broadcast))find_sym("ncclBroadcast");
    x.GetVersion = (decltype(x.GetVersion))find_sym("ncclGetVersion");
    x.GetErrorString = (decltype(x.GetErrorString))find_sym("ncclGetErrorString");
    x.ok = x.GetUniqueId && x.CommInitRank && x.CommDestroy && x.AllReduce && x.Broadcast;
    return x;
  }();
  return a;
}

void check(ncclResult_t r, const char* what) {
  if (r != 0) {
    const char* s = api().GetErrorString ? api().GetErrorString(r) : "?";
    throw std::runtime_error(std::string("RCCL ") + what + " failed: " + s);
  }
}
int dt(int dtype) { return dtype == 1 ? ncclBfloat16 : ncclFloat32; }

double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

typedef int (*roctx_push_t)(const char*);
typedef int (*roctx_pop_t)();
}  // namespace

bool RcclComm::available() { return api().ok; }

std::string RcclComm::version() {
  int v = 0;
  if (api().GetVersion) api().GetVersion(&v);
  return std::to_string(v);
}

std::vector<uint8_t> RcclComm::unique_id() {
  if (!available()) throw std::runtime_error("RCCL symbols not found (import torch first)");
  ncclUniqueId id;
  check(api().GetUniqueId(&id), "ncclGetUniqueId");
  return std::vector<uint8_t>(id.internal, id.internal + kUniqueIdBytes);
}

RcclComm::RcclComm(const std::vector<uint8_t>& uid, int world_size, int rank, int device, double init_timeout_s,
                   bool wait)
    : world_(world_size), rank_(rank) {
  if (!available()) throw std::runtime_error("RCCL symbols not found (import torch first)");
  if (uid.size() != kUniqueIdBytes) throw std::runtime_error("bad ncclUniqueId size");
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
  ncclUniqueId id;
  memcpy(id.internal, uid.data(), kUniqueIdBytes);
  ncclComm_t c = nullptr;
  const Api& a = api();
  if (a.CommInitRankConfig && a.CommGetAsyncError && a.CommAbort) {
    // non-blocking communicator: the init (socket bootstrap, topology, channels) runs in RCCL's own
    // thread and is polled here, so a peer that never arrives ends in ncclCommAbort after
    // init_timeout_s instead of a thread stuck in ncclCommInitRank; every later call that returns
    // ncclInProgress is completed the same way (finish) before anything else is enqueued
    ConfigV21700 cfg{sizeof(ConfigV21700), 0xcafebeef, 21700, 0, kUndefInt, kUndefInt, kUndefInt, nullptr, kUndefInt};
    ncclResult_t r = a.CommInitRankConfig(&c, world_size, id, rank, &cfg);
    if (r != 0 && r != ncclInProgress) check(r, "ncclCommInitRankConfig");
    comm_ = c;
    nonblocking_ = true;
    if (wait) finish(r, "ncclCommInitRankConfig", init_timeout_s);
  } else {
    check(a.CommInitRank(&c, world_size, id, rank), "ncclCommInitRank");
    comm_ = c;
  }
}

RcclComm::~RcclComm() {
  if (!comm_) return;
  // a communicator whose init failed or is still running is aborted (ncclCommDestroy would wait for it)
  if (nonblocking_ && init_status() != 0) abort();
  else api().CommDestroy((ncclComm_t)comm_);
}

int RcclComm::init_status() const {
  if (!comm_) return -1;
  if (!nonblocking_ || !api().CommGetAsyncError) return 0;
  ncclResult_t st = 0;
  ncclResult_t r = api().CommGetAsyncError((ncclComm_t)comm_, &st);
  return r != 0 ? r : st;
}

std::string RcclComm::error_string(int code) {
  if (code == -1) return "communicator aborted";
  const char* s = api().GetErrorString ? api().GetErrorString(code) : nullptr;
  return s ? s : ("RCCL error " + std::to_string(code));
}

void RcclComm::finish(int r, const char* what, double timeout_s) {
  if (r == ncclInProgress) {
    const double t0 = now_s();
    ncclResult_t st = ncclInProgress;
    for (;;) {
      check(api().CommGetAsyncError((ncclComm_t)comm_, &st), "ncclCommGetAsyncError");
      if (st != ncclInProgress) break;
      if (now_s() - t0 > timeout_s) {
        abort();
        throw std::runtime_error(std::string("RCCL ") + what + " did not complete within " +
                                 std::to_string((int)timeout_s) + " s (communicator aborted)");
      }
      timespec ts{0, 200000};   // 0.2 ms
      nanosleep(&ts, nullptr);
    }
    r = st;
  }
  check(r, what);
}

void RcclComm::live(const char* what) const {
  if (!comm_) throw std::runtime_error(std::string("RCCL ") + what + ": the communicator was aborted");
}

void RcclComm::allreduce_sum(void* buf, int64_t count, int dtype, hipStream_t stream) {
  live("ncclAllReduce");
  finish(api().AllReduce(buf, buf, (size_t)count, dt(dtype), ncclSum, (ncclComm_t)comm_, stream), "ncclAllReduce");
}

void RcclComm::broadcast(void* buf, int64_t count, int dtype, int root, hipStream_t stream) {
  live("ncclBroadcast");
  finish(api().Broadcast(buf, buf, (size_t)count, dt(dtype), root, (ncclComm_t)comm_, stream), "ncclBroadcast");
}

void RcclComm::abort() {
  // ncclCommAbort raises the communicator's abort flag, which RCCL's device-side wait loops poll:
  // a collective stuck on a peer that never arrives returns, so the streams behind it drain
  if (!comm_) return;
  if (api().CommAbort) api().CommAbort((ncclComm_t)comm_);
  else api().CommDestroy((ncclComm_t)comm_);
  comm_ = nullptr;
  aborted_ = true;
}

int RcclComm::async_error() const {
  if (!comm_ || !api().CommGetAsyncError) return 0;
  ncclResult_t st = 0;
  api().CommGetAsyncError((ncclComm_t)comm_, &st);
  return st;
}

namespace {
// roctx entry points: the rocprofiler-sdk library (what rocprofv3 --marker-trace intercepts) first,
// then the legacy libroctx64 (torch ships one), then whatever the process already has loaded
void* roctx_sym(const char* name) {
  static void* lib = [] {
    for (const char* so : {"librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
                           "libroctx64.so.4", "libroctx64.so"}) {
      if (void* h = dlopen(so, RTLD_NOW | RTLD_GLOBAL)) return h;
    }
    return (void*)nullptr;
  }();
  void* f = lib ? dlsym(lib, name) : nullptr;
  return f ? f : dlsym(RTLD_DEFAULT, name);
}
}  // namespace

void roctx_push(const char* name) {
  static roctx_push_t f = (roctx_push_t)roctx_sym("roctxRangePushA");
  if (f) f(name);
}
void roctx_pop() {
  static roctx_pop_t f = (roctx_pop_t)roctx_sym("roctxRangePop");
  if (f) f();
}

}  // namespace mnist
