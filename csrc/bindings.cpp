// Python bindings (pybind11) for the native MI355X runtime.  Tensors cross the boundary as raw
// device pointers (tensor.data_ptr()) and HIP streams as integer handles
// (torch.cuda.Stream.cuda_stream): the runtime never includes libtorch headers, so it is immune
// to torch C++ ABI details and compiles in seconds.
#include <pybind11/pybind11.h>
#include <chrono>
#include <vector>
#include <pybind11/stl.h>

#include <stdexcept>

#include "include/kernels.h"
#include "runtime/bucket_reducer.h"
#include "runtime/engine.h"
#include "runtime/rccl_comm.h"

namespace py = pybind11;

#ifdef MNIST_TIMELINE
namespace mnist {
void tl_dump_trunk(std::vector<uint64_t>&);
void tl_dump_fc_head(std::vector<uint64_t>&);
void tl_dump_conv_bwd(std::vector<uint64_t>&);
void tl_dump_adadelta(std::vector<uint64_t>&);
void tl_dump_comm(std::vector<uint64_t>&);
void tl_dump_xgmi(std::vector<uint64_t>&);
}  // namespace mnist
#endif
using namespace mnist;

namespace {
template <typename T>
T* P(uintptr_t x) { return reinterpret_cast<T*>(x); }
hipStream_t S(uintptr_t x) { return reinterpret_cast<hipStream_t>(x); }

void check_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("kernel launch failed: ") + hipGetErrorString(e));
}

// ---- minimal DLPack (v0.8 ABI) export of a device fp32 vector; the capsule keeps `owner` alive
struct DLDevice { int32_t device_type; int32_t device_id; };
struct DLDataType { uint8_t code; uint8_t bits; uint16_t lanes; };
struct DLTensor {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor*);
};
constexpr int32_t kDLROCM = 10;
constexpr uint8_t kDLFloat = 2;

struct DLCtx {
  std::shared_ptr<void> owner;
  int64_t shape[1];
  DLManagedTensor mt;
};

void dl_deleter(DLManagedTensor* mt) { delete static_cast<DLCtx*>(mt->manager_ctx); }

py::capsule dlpack_f32(float* data, int64_t n, int device, std::shared_ptr<void> owner) {
  auto* ctx = new DLCtx{std::move(owner), {n}, {}};
  ctx->mt.dl_tensor = DLTensor{data, DLDevice{kDLROCM, device}, 1, DLDataType{kDLFloat, 32, 1}, ctx->shape, nullptr, 0};
  ctx->mt.manager_ctx = ctx;
  ctx->mt.deleter = dl_deleter;
  return py::capsule(&ctx->mt, "dltensor", [](PyObject* cap) {
    // an unconsumed capsule still owns the tensor (a consumer renames it to "used_dltensor")
    if (PyCapsule_IsValid(cap, "dltensor")) {
      auto* mt = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
      if (mt && mt->deleter) mt->deleter(mt);
    }
  });
}

EngineBuffers buffers_from_dict(const py::dict& d) {
  EngineBuffers b;
  auto get = [&](const char* k) -> uintptr_t {
    if (!d.contains(k)) return 0;
    return d[k].cast<uintptr_t>();
  };
  b.param = P<float>(get("param"));
  b.grad = P<float>(get("grad"));
  b.square_avg = P<float>(get("square_avg"));
  b.acc_delta = P<float>(get("acc_delta"));
  b.lr = P<float>(get("lr"));
  b.w2f = P<uint16_t>(get("w2f"));
  b.w2d = P<uint16_t>(get("w2d"));
  b.w1 = P<uint16_t>(get("w1"));
  b.w1t = P<uint16_t>(get("w1t"));
  b.state = P<StepState>(get("state"));
  b.loss_log = P<float>(get("loss_log"));
  b.train_u8 = P<const uint8_t>(get("train_u8"));
  b.train_labels = P<const int32_t>(get("train_labels"));
  b.train_idx = P<const int32_t>(get("train_idx"));
  b.epoch_u8 = P<uint8_t>(get("epoch_u8"));
  b.epoch_labels = P<int32_t>(get("epoch_labels"));
  b.test_u8 = P<const uint8_t>(get("test_u8"));
  b.test_labels = P<const int32_t>(get("test_labels"));
  b.test_idx = P<const int32_t>(get("test_idx"));
  b.test_loss_rows = P<float>(get("test_loss_rows"));
  b.test_correct = P<int32_t>(get("test_correct"));
  if (!b.param || !b.grad || !b.square_avg || !b.acc_delta || !b.lr || !b.w2f || !b.w2d || !b.w1 ||
      !b.w1t || !b.state)
    throw std::runtime_error("engine buffers: missing model/optimizer pointer");
  return b;
}
}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X (gfx950) native kernels + runtime for the MNIST DDP framework";

  m.attr("PARAM_TOTAL") = PARAM_TOTAL;
  m.attr("FC1_KSPLIT") = FC1_KSPLIT;
  m.attr("DYC_REC") = DYC_REC;
  py::dict offs;
  offs["fc1.weight"] = OFF_FC1_W; offs["fc1.bias"] = OFF_FC1_B;
  offs["fc2.weight"] = OFF_FC2_W; offs["fc2.bias"] = OFF_FC2_B;
  offs["conv1.weight"] = OFF_CONV1_W; offs["conv1.bias"] = OFF_CONV1_B;
  offs["conv2.weight"] = OFF_CONV2_W; offs["conv2.bias"] = OFF_CONV2_B;
  m.attr("PARAM_OFFSETS") = offs;
  m.attr("BUCKET_SPLIT") = OFF_CONV1_W;
  m.def("conv_wgrad_groups", &conv_wgrad_groups);
  m.def("set_dgrad_grid", &set_dgrad_grid, "persistent dgrad grid override (0 = 2 x CUs; tests)");
  m.def("set_wgrad_form", &set_wgrad_form, "wgrad form override (-1 = by batch, 0 lean, 1 staggered; tests)");
  m.attr("SCHED_SERIAL") = (int)Engine::SERIAL;
  m.attr("SCHED_OVERLAP") = (int)Engine::OVERLAP;
  m.attr("SCHED_RCCL") = (int)Engine::RCCL;
  m.attr("SCHED_XGMI") = (int)Engine::XGMI;

  // ---------------- per-kernel entry points ----------------
  m.def("trunk_fwd", [](uintptr_t data_u8, uintptr_t idx, int64_t idx_stride, uintptr_t state, uintptr_t w1c,
                        uintptr_t b1c, uintptr_t w2f, uintptr_t b2c, uintptr_t a1_out, uintptr_t p_out,
                        uintptr_t pmask_out, int B, bool train, uintptr_t stream, uintptr_t xin) {
    TrunkFwdArgs a{P<const uint8_t>(data_u8), P<const int32_t>(idx), idx_stride, P<const StepState>(state),
                   P<const float>(w1c), P<const float>(b1c), P<const uint16_t>(w2f), P<const float>(b2c),
                   P<uint16_t>(a1_out), P<uint16_t>(p_out), P<uint8_t>(pmask_out), P<const float>(xin)};
    launch_trunk_fwd(a, B, train, S(stream));
    check_launch();
  }, py::arg("data_u8"), py::arg("idx"), py::arg("idx_stride"), py::arg("state"), py::arg("w1c"), py::arg("b1c"),
     py::arg("w2f"), py::arg("b2c"), py::arg("a1_out"), py::arg("p_out"), py::arg("pmask_out"), py::arg("B"),
     py::arg("train"), py::arg("stream"), py::arg("xin") = 0);
  m.def("fc1_fwd", [](uintptr_t p, uintptr_t w1, uintptr_t z1part, int B, uintptr_t stream) {
    launch_fc1_fwd(P<const uint16_t>(p), P<const uint16_t>(w1), P<float>(z1part), B, S(stream));
    check_launch();
  });
  m.def("head_train", [](uintptr_t z1part, uintptr_t b_fc1, uintptr_t w_fc2, uintptr_t b_fc2, uintptr_t labels,
                         uintptr_t idx, int64_t idx_stride, uintptr_t state, float inv_batch, uintptr_t loss_rows,
                         uintptr_t dz1, uintptr_t h_bf, uintptr_t dl_bf, int B, int Bp, uintptr_t stream,
                         uintptr_t dlogp) {
    HeadArgs a{};
    a.z1part = P<const float>(z1part); a.b_fc1 = P<const float>(b_fc1); a.w_fc2 = P<const float>(w_fc2);
    a.b_fc2 = P<const float>(b_fc2); a.labels = P<const int32_t>(labels); a.idx = P<const int32_t>(idx);
    a.idx_step_stride = idx_stride; a.state = P<const StepState>(state); a.inv_batch = inv_batch;
    a.loss_rows = P<float>(loss_rows); a.dz1 = P<uint16_t>(dz1); a.h_bf = P<uint16_t>(h_bf);
    a.dl_bf = P<uint16_t>(dl_bf); a.dlogp = P<const float>(dlogp);
    launch_head_train(a, B, Bp, S(stream));
    check_launch();
  }, py::arg("z1part"), py::arg("b_fc1"), py::arg("w_fc2"), py::arg("b_fc2"), py::arg("labels"), py::arg("idx"),
     py::arg("idx_stride"), py::arg("state"), py::arg("inv_batch"), py::arg("loss_rows"), py::arg("dz1"),
     py::arg("h_bf"), py::arg("dl_bf"), py::arg("B"), py::arg("Bp"), py::arg("stream"), py::arg("dlogp") = 0);
  m.def("head_fwd", [](uintptr_t z1part, uintptr_t b_fc1, uintptr_t w_fc2, uintptr_t b_fc2, uintptr_t state,
                       uintptr_t logp, int B, bool train, uintptr_t stream) {
    HeadArgs a{};
    a.z1part = P<const float>(z1part); a.b_fc1 = P<const float>(b_fc1); a.w_fc2 = P<const float>(w_fc2);
    a.b_fc2 = P<const float>(b_fc2); a.state = P<const StepState>(state); a.logp_out = P<float>(logp);
    launch_head_fwd(a, B, train, S(stream));
    check_launch();
  });
  m.def("head_eval", [](uintptr_t z1part, uintptr_t b_fc1, uintptr_t w_fc2, uintptr_t b_fc2, uintptr_t labels,
                        uintptr_t idx, uintptr_t loss_rows, uintptr_t correct, uintptr_t logp, int B,
                        uintptr_t stream) {
    HeadArgs a{};
    a.z1part = P<const float>(z1part); a.b_fc1 = P<const float>(b_fc1); a.w_fc2 = P<const float>(w_fc2);
    a.b_fc2 = P<const float>(b_fc2); a.labels = P<const int32_t>(labels); a.idx = P<const int32_t>(idx);
    a.loss_rows = P<float>(loss_rows); a.correct_out = P<int32_t>(correct); a.logp_out = P<float>(logp);
    launch_head_eval(a, B, S(stream));
    check_launch();
  });
  m.def("fc_bwd", [](uintptr_t dz1, uintptr_t p, uintptr_t pmask, uintptr_t w1t, uintptr_t h_bf, uintptr_t dl_bf,
                     uintptr_t loss_rows, uintptr_t state, uintptr_t grad, uintptr_t dyc, uintptr_t loss_log,
                     float grad_scale, float inv_batch, int B, int Bp, uintptr_t stream, int role,
                     uintptr_t part) {
    FcBwdArgs a{P<const uint16_t>(dz1), P<const uint16_t>(p), P<const uint8_t>(pmask), P<const uint16_t>(w1t),
                P<const uint16_t>(h_bf), P<const uint16_t>(dl_bf), P<const float>(loss_rows),
                P<const StepState>(state), P<float>(grad), P<uint8_t>(dyc), P<float>(loss_log), grad_scale,
                inv_batch, P<float>(part)};
    if (role < 0) launch_fc_bwd(a, B, Bp, S(stream));
    else if (role == 3) launch_fc_bwd_dw1(a, B, Bp, S(stream));                  // role A alone, lean kernel
    else if (role == 4) launch_fc_bwd(a, B, Bp, S(stream), false, FCB_ROLE_C | FCB_ROLE_B);   // B > 1024
    else if (role == 5) launch_fc_bwd(a, B, Bp, S(stream), false, FCB_ROLE_C | FCB_ROLE_A);   // weight grads
    else if (role == 6) launch_fc_bwd(a, B, Bp, S(stream), false, FCB_ROLE_B);
    else launch_fc_bwd_role(a, B, Bp, role, S(stream));
    check_launch();
  }, py::arg("dz1"), py::arg("p"), py::arg("pmask"), py::arg("w1t"), py::arg("h_bf"), py::arg("dl_bf"),
     py::arg("loss_rows"), py::arg("state"), py::arg("grad"), py::arg("dyc"), py::arg("loss_log"),
     py::arg("grad_scale"), py::arg("inv_batch"), py::arg("B"), py::arg("Bp"), py::arg("stream"),
     py::arg("role") = -1, py::arg("part") = 0);
  m.def("fc_bwd_splits", &fc_bwd_splits);
  m.attr("FCB_PART_STRIDE") = FCB_PART_STRIDE;
  m.def("conv_bwd", [](uintptr_t dyc, uintptr_t a1, uintptr_t w2d, uintptr_t w1c, uintptr_t b1c,
                       uintptr_t data_u8, uintptr_t idx, int64_t idx_stride, uintptr_t state, uintptr_t c1part,
                       uintptr_t w2part, uintptr_t grad, float grad_scale, int B, uintptr_t stream,
                       uintptr_t xin) {
    ConvBwdArgs a{P<const uint8_t>(dyc), P<const uint16_t>(a1), P<const uint16_t>(w2d),
                  P<const float>(w1c), P<const float>(b1c), P<const uint8_t>(data_u8), P<const int32_t>(idx),
                  idx_stride, P<const StepState>(state), P<float>(c1part), P<float>(w2part), P<float>(grad),
                  grad_scale, conv_wgrad_groups(B), P<const float>(xin)};
    a.c1_rows = conv_dgrad_c1_rows(B);
    launch_conv_bwd(a, B, S(stream));
    launch_conv_grad_reduce(a, B, S(stream));
    check_launch();
  }, py::arg("dy"), py::arg("a1"), py::arg("w2d"), py::arg("w1c"), py::arg("b1c"), py::arg("data_u8"), py::arg("idx"),
     py::arg("idx_stride"), py::arg("state"), py::arg("c1part"), py::arg("w2part"), py::arg("grad"),
     py::arg("grad_scale"), py::arg("B"), py::arg("stream"), py::arg("xin") = 0);
  m.def("adadelta", [](uintptr_t param, uintptr_t grad, uintptr_t sq, uintptr_t acc, uintptr_t lr, float rho,
                       float eps, float wd, uintptr_t w2f, uintptr_t w2d, uintptr_t w1, uintptr_t w1t,
                       uintptr_t state_inc, int region, bool update, uintptr_t stream) {
    AdadeltaArgs a{P<float>(param), P<const float>(grad), P<float>(sq), P<float>(acc), P<const float>(lr), rho,
                   eps, wd, P<uint16_t>(w2f), P<uint16_t>(w2d), P<uint16_t>(w1), P<uint16_t>(w1t),
                   P<StepState>(state_inc)};
    if (update) launch_adadelta(a, region, S(stream));
    else launch_refresh_shadows(a, S(stream));
    check_launch();
  });

  // ---------------- communicator ----------------
  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init([](py::bytes uid, int world, int rank, int device, double init_timeout_s, bool wait) {
             std::string s = uid;
             std::shared_ptr<RcclComm> c;
             {
               // the init waits for its bootstrap: let other Python threads run meanwhile
               // (distributed.PendingRcclComm overlaps it with data / model / trainer setup)
               py::gil_scoped_release nogil;
               c = std::make_shared<RcclComm>(std::vector<uint8_t>(s.begin(), s.end()), world, rank, device,
                                              init_timeout_s, wait);
             }
             return c;
           }),
           py::arg("unique_id"), py::arg("world_size"), py::arg("rank"), py::arg("device"),
           py::arg("init_timeout_s") = 600.0, py::arg("wait") = true)
      .def("abort", [](RcclComm& c) {
        py::gil_scoped_release nogil;
        c.abort();
      })
      .def_property_readonly("aborted", &RcclComm::aborted)
      .def_property_readonly("nonblocking", &RcclComm::nonblocking)
      .def("async_error", &RcclComm::async_error)
      .def("init_status", &RcclComm::init_status, py::call_guard<py::gil_scoped_release>())
      .def_static("error_string", &RcclComm::error_string)
      .def_static("available", &RcclComm::available)
      .def_static("version", &RcclComm::version)
      .def_static("unique_id", []() {
        auto v = RcclComm::unique_id();
        return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
      })
      .def("allreduce_sum", [](RcclComm& c, uintptr_t buf, int64_t count, int dtype, uintptr_t stream) {
        c.allreduce_sum(P<void>(buf), count, dtype, S(stream));
      })
      .def("broadcast", [](RcclComm& c, uintptr_t buf, int64_t count, int dtype, int root, uintptr_t stream) {
        c.broadcast(P<void>(buf), count, dtype, root, S(stream));
      })
      .def_property_readonly("world_size", &RcclComm::world_size)
      .def_property_readonly("rank", &RcclComm::rank);

  py::class_<XgmiComm, std::shared_ptr<XgmiComm>>(m, "XgmiComm", py::dynamic_attr())
      .def(py::init([](int world, int rank, int device, int64_t numel, int channels, int64_t oneshot_max,
                       int co_ranks, double budget) {
             // device allocation + memsets + a device sync: other Python threads run meanwhile
             // (distributed.PendingXgmiComm overlaps the setup with the main thread's)
             py::gil_scoped_release nogil;
             return std::make_shared<XgmiComm>(world, rank, device, numel, channels, oneshot_max, co_ranks,
                                               budget);
           }),
           py::arg("world_size"), py::arg("rank"), py::arg("device"), py::arg("numel"), py::arg("channels") = 2,
           py::arg("oneshot_max") = 32768, py::arg("co_ranks") = 1, py::arg("budget") = 0.5)
      // the communicator's own buffers as DLPack capsules (torch.utils.dlpack.from_dlpack): zero-copy
      // fp32 [numel] views that keep the communicator alive
      .def("dlpack", [](std::shared_ptr<XgmiComm> c, const std::string& which) {
        if (which != "in" && which != "out") throw std::runtime_error("dlpack: which must be 'in' or 'out'");
        return dlpack_f32(which == "in" ? c->in() : c->out(), c->numel(), c->device(), c);
      })
      .def_property_readonly("ordering", &XgmiComm::ordering)
      .def_property_readonly("grids", [](const XgmiComm& c) {
        const XgmiGrids& g = c.grids();
        py::dict d;
        d["fc_fused"] = g.fc_fused; d["conv_fused"] = g.conv_fused; d["twoshot"] = g.twoshot; d["oneshot"] = g.oneshot;
        d["cap_fc_fused"] = g.cap_fc_fused; d["cap_conv_fused"] = g.cap_conv_fused;
        d["cap_twoshot"] = g.cap_twoshot; d["cap_oneshot"] = g.cap_oneshot;
        d["load_fused"] = g.load_fused; d["load_separate"] = g.load_separate;
        return d;
      })
      .def("record", [](const XgmiComm& c) {
        auto v = c.record();
        return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
      })
      .def("connect", [](XgmiComm& c, std::vector<py::bytes> recs) {
        std::vector<std::vector<uint8_t>> v;
        for (auto& r : recs) {
          std::string s = r;
          v.emplace_back(s.begin(), s.end());
        }
        py::gil_scoped_release nogil;   // one IPC import per peer
        c.connect(v);
      })
      .def("allreduce", [](XgmiComm& c, int channel, int64_t offset, int64_t count, uintptr_t stream) {
        c.allreduce(channel, offset, count, S(stream));
      }, py::arg("channel"), py::arg("offset"), py::arg("count"), py::arg("stream"))
      .def("error", &XgmiComm::error)
      .def("set_timeout_seconds", &XgmiComm::set_timeout_seconds)
      .def("set_fences", &XgmiComm::set_fences)
      .def_property_readonly("fences", &XgmiComm::fences)
      .def("close_peers", &XgmiComm::close_peers, py::call_guard<py::gil_scoped_release>())
      .def("mark_recyclable", &XgmiComm::mark_recyclable)
      // rank `root`'s parameters to every rank through the IPC-mapped output buffers (DDP construction
      // broadcast without RCCL): root stages `count` floats of `buf` into its output buffer, then -
      // after the caller's barrier - every other rank copies them out of root's; the caller barriers
      // again before the buffers are reused
      .def("stage_out", [](XgmiComm& c, uintptr_t buf, int64_t count, uintptr_t stream) {
        c.stage_out(P<const float>(buf), count, S(stream));
      })
      .def("read_peer_out", [](XgmiComm& c, int peer, uintptr_t buf, int64_t count, uintptr_t stream) {
        c.read_peer_out(peer, P<float>(buf), count, S(stream));
      })
      .def_property_readonly("connected", &XgmiComm::connected)
      .def_property_readonly("world_size", &XgmiComm::world_size)
      .def_property_readonly("rank", &XgmiComm::rank);

  // ---------------- DDP gradient reducer (module-level path) ----------------
  py::class_<BucketReducer>(m, "BucketReducer")
      .def(py::init([](std::vector<std::vector<int64_t>> numels, int world, std::shared_ptr<RcclComm> comm) {
             return new BucketReducer(numels, world, std::move(comm));
           }),
           py::arg("bucket_numels"), py::arg("world_size"), py::arg("comm") = nullptr)
      .def("prepare", &BucketReducer::prepare)
      .def("mark_ready", [](BucketReducer& r, int b, int slot, uintptr_t grad, uintptr_t out, uintptr_t stream) {
        r.mark_ready(b, slot, P<const float>(grad), P<float>(out), S(stream));
      })
      .def("finalize", [](BucketReducer& r, uintptr_t stream) { r.finalize(S(stream)); })
      .def_property_readonly("num_buckets", &BucketReducer::num_buckets)
      .def("bucket_numel", &BucketReducer::bucket_numel)
      .def("bucket_ptr", &BucketReducer::bucket_ptr)
      .def_property_readonly("launches", &BucketReducer::launches);

  // ---------------- engine ----------------
  py::class_<Engine>(m, "Engine")
      .def(py::init([](py::dict bufs, int max_batch, int max_test_batch, uintptr_t compute, uintptr_t comm,
                       int world, float rho, float eps, float wd, bool fp32) {
             return new Engine(buffers_from_dict(bufs), max_batch, max_test_batch, S(compute), S(comm), world, rho,
                               eps, wd, fp32);
           }),
           py::arg("buffers"), py::arg("max_batch"), py::arg("max_test_batch"), py::arg("compute_stream"),
           py::arg("comm_stream"), py::arg("world_size"), py::arg("rho"), py::arg("eps"), py::arg("weight_decay"),
           py::arg("fp32") = false)
      .def_property_readonly("fp32", &Engine::fp32)
      .def("attach_comm", &Engine::attach_comm)
      .def("attach_xgmi", &Engine::attach_xgmi)
      .def("set_xgmi_fuse_update", &Engine::set_xgmi_fuse_update)
      .def("set_bucket_split", &Engine::set_bucket_split)
      .def("set_rccl_handoff", &Engine::set_rccl_handoff)
      .def_property("fc_dw1_side", &Engine::fc_dw1_side, &Engine::set_fc_dw1_side)
      .def_property("w1t_pingpong", &Engine::w1t_pingpong, &Engine::set_w1t_pingpong)
      .def_property("c1_lanes", &Engine::c1_lanes, &Engine::set_c1_lanes)
      .def("fault_hold", &Engine::fault_hold)
      .def("fault_release", [](Engine& e, uintptr_t stream) { e.fault_release(S(stream)); })
      .def("set_schedule", &Engine::set_schedule, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("schedule", &Engine::schedule)
      .def("reset_counters", &Engine::reset_counters, py::call_guard<py::gil_scoped_release>())
      .def("probe_stream_handoff", &Engine::probe_stream_handoff, py::arg("timeout_s") = 2.0,
           py::call_guard<py::gil_scoped_release>())
      .def("begin_epoch", &Engine::begin_epoch, py::arg("seed"), py::arg("rng_base"), py::arg("step0") = 0, py::arg("flags") = 0)
      .def("train_steps", &Engine::train_steps, py::call_guard<py::gil_scoped_release>())
      .def("capture_train", &Engine::capture_train)
      .def("profile_steps", &Engine::profile_steps, py::call_guard<py::gil_scoped_release>())
      .def("gather_rows", &Engine::gather_rows, py::arg("start"), py::arg("n"))
      .def("replay", &Engine::replay, py::call_guard<py::gil_scoped_release>())
      .def("eval", &Engine::eval)
      .def("capture_eval", &Engine::capture_eval)
      .def("refresh_shadows", &Engine::refresh_shadows)
      .def("broadcast_params", &Engine::broadcast_params)
      .def("synchronize", &Engine::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("sync_streams", &Engine::sync_streams, py::call_guard<py::gil_scoped_release>())
      .def("errors", &Engine::errors)
      .def("check_errors", &Engine::check_errors)
      .def_static("describe_xgmi_error", &Engine::describe_xgmi_error)
      .def_property_readonly("workspace_bytes", &Engine::workspace_bytes);

#ifdef MNIST_TIMELINE
  m.attr("TIMELINE") = true;
  // every instrumented wave since the last dump as little-endian uint64 triples (kernel id, start,
  // end; s_memrealtime ticks of 10 ns); the rings are rewound
  m.def("timeline_dump", []() {
    std::vector<uint64_t> v;
    tl_dump_trunk(v);
    tl_dump_fc_head(v);
    tl_dump_conv_bwd(v);
    tl_dump_adadelta(v);
    tl_dump_comm(v);
    tl_dump_xgmi(v);
    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(uint64_t));
  });
#else
  m.attr("TIMELINE") = false;
#endif
  m.def("hip_prewarm", [](int device) {
    // the HIP runtime + this process's context on `device` and every kernel TU's code object, with
    // the GIL released (the driver's prewarm thread: the main thread keeps building data and model)
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("hip_prewarm: hipSetDevice failed");
    (void)hipFree(nullptr);
    const auto t1 = clk::now();
    preload_trunk();
    preload_fc_head();
    preload_conv_bwd();
    preload_adadelta();
    preload_comm();
    preload_xgmi();
    preload_f32();
    const auto t2 = clk::now();
    // the runtime's own first-use costs the setup would otherwise pay on the main thread: the blit
    // kernels behind hipMemset and the staging path of pageable host copies (measured on the box:
    // 80 ms of first hipMemsets, 28 ms of first pageable H2D copies inside the reference timer)
    clk::time_point tm = t2, th = t2, td = t2;
    {
      constexpr size_t kBytes = 1 << 20;
      void* d = nullptr;
      std::vector<char> h(kBytes, 0);
      if (hipMalloc(&d, kBytes) == hipSuccess) {
        launch_fill(d, kBytes, 0, nullptr);         // (our fill kernel: no blit-kernel load)
        (void)hipDeviceSynchronize();
        tm = clk::now();
        (void)hipMemcpy(d, h.data(), kBytes, hipMemcpyHostToDevice);
        th = clk::now();
        (void)hipMemcpy(h.data(), d, 4096, hipMemcpyDeviceToHost);
        td = clk::now();
        (void)hipFree(d);
      }
    }
    const auto t3 = clk::now();
    auto sec = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); };
    return std::make_tuple(sec(t0, t1), sec(t1, t2), sec(t2, t3), sec(t2, tm), sec(tm, th), sec(th, td));
  }, py::call_guard<py::gil_scoped_release>(), py::arg("device"));
  // physical identity of a device (PCI domain:bus:device.function + UUID) straight from the HIP
  // runtime: callable from any thread, no amdsmi (torch.cuda.get_device_properties counts devices
  // through amdsmi, and from a helper thread it refused a valid index on the box)
  m.def("device_identity", [](int device) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus) - 1, device) != hipSuccess)
      throw std::runtime_error("device_identity: hipDeviceGetPCIBusId failed");
    hipUUID uuid;
    std::string u;
    if (hipDeviceGetUuid(&uuid, device) == hipSuccess) {
      static const char* hx = "0123456789abcdef";
      for (int i = 0; i < 16; ++i) {
        u += hx[((unsigned char)uuid.bytes[i]) >> 4];
        u += hx[((unsigned char)uuid.bytes[i]) & 15];
      }
    }
    return std::string(bus) + "|" + u;
  });
  // raw HIP streams for the engine: "dedicated" = hipExtStreamCreateWithCUMask over every CU (the
  // runtime gives a CU-masked stream a hardware queue of its own instead of sharing a pooled one),
  // else hipStreamCreateWithPriority(non-blocking, priority)
  m.def("create_stream", [](int device, bool dedicated, int priority) {
    if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("create_stream: hipSetDevice failed");
    hipStream_t st = nullptr;
    if (dedicated) {
      int cus = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
        throw std::runtime_error("create_stream: CU count");
      std::vector<uint32_t> mask((cus + 31) / 32, 0xffffffffu);
      if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
      if (hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()) != hipSuccess)
        throw std::runtime_error("hipExtStreamCreateWithCUMask failed");
    } else if (hipStreamCreateWithPriority(&st, hipStreamNonBlocking, priority) != hipSuccess) {
      throw std::runtime_error("hipStreamCreateWithPriority failed");
    }
    return reinterpret_cast<uintptr_t>(st);
  }, py::arg("device"), py::arg("dedicated") = true, py::arg("priority") = 0);
  m.def("destroy_stream", [](uintptr_t s) { (void)hipStreamDestroy(S(s)); });
  // do two streams hand off through device counters (x waits for y's signal, then y for x's)?  False
  // when they share a hardware queue: the first wait times out (timeout_s) before the signal queued
  // behind it runs.  Engine-independent form of Engine::probe_stream_handoff (make_streams).
  m.def("probe_streams", [](uintptr_t xs, uintptr_t ys, double timeout_s) {
    hipStream_t x = S(xs), y = S(ys);
    int* c = nullptr;
    if (hipMalloc(&c, 4 * sizeof(int)) != hipSuccess) throw std::runtime_error("probe_streams: hipMalloc failed");
    launch_fill(c, 4 * sizeof(int), 0, x);
    bool ok = hipStreamSynchronize(x) == hipSuccess;
    launch_stream_wait(c + 0, c + 2, 1, c + 3, x, timeout_s);
    launch_stream_signal(c + 0, y);
    launch_stream_wait(c + 1, c + 2, 1, c + 3, y, timeout_s);
    launch_stream_signal(c + 1, x);
    ok = ok && hipStreamSynchronize(x) == hipSuccess && hipStreamSynchronize(y) == hipSuccess;
    int err = 1;
    if (ok) ok = hipMemcpyAsync(&err, c + 3, sizeof(int), hipMemcpyDeviceToHost, x) == hipSuccess &&
                 hipStreamSynchronize(x) == hipSuccess;
    (void)hipFree(c);
    return ok && err == 0;
  }, py::call_guard<py::gil_scoped_release>(), py::arg("x"), py::arg("y"), py::arg("timeout_s") = 0.5);
  m.def("synth_render", [](uintptr_t plan, uintptr_t templates, int64_t n, uintptr_t out, uintptr_t stream) {
    launch_synth_render(P<const void>(plan), P<const float>(templates), n, P<uint8_t>(out), S(stream));
    check_launch();
  }, py::arg("plan"), py::arg("templates"), py::arg("n"), py::arg("out"), py::arg("stream"),
     "render n synthetic images [n, 784] on the device from a host-made plan (generator v3)");
  m.def("memset_sync", [](uintptr_t ptr, int value, int64_t nbytes) {
    // setup-time buffer initialisation without a torch fill kernel (whose code object would load on
    // first launch inside the reference timer); synchronous
    if (nbytes > 0) {
      launch_fill(reinterpret_cast<void*>(ptr), nbytes, value, nullptr);
      if (hipStreamSynchronize(nullptr) != hipSuccess) throw std::runtime_error("memset_sync: fill failed");
    }
  }, py::call_guard<py::gil_scoped_release>());
  m.def("preload_code_objects", []() {
    preload_trunk();
    preload_fc_head();
    preload_conv_bwd();
    preload_adadelta();
    preload_comm();
    preload_xgmi();
    preload_f32();
  }, py::call_guard<py::gil_scoped_release>(), "load every kernel translation unit's code object on the current device");
  m.def("roctx_push", [](const std::string& s) { roctx_push(s.c_str()); });
  m.def("roctx_pop", []() { roctx_pop(); });
}
