// pybind11 module `_comm`: RCCL communicator manager + Horovod-style fusion engine.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>

#include "comm_manager.h"
#include "fusion_engine.h"
#include "p2p_ring.h"
#include "xgmi_allreduce.h"

namespace {

using pde::FusionEngine;
using pde::P2PRing;
using pde::RcclComm;
using pde::XgmiAllreduce;

int code_of(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kHalf: return 2;
    case at::kDouble: return 3;
    case at::kInt: return 4;
    case at::kLong: return 5;
    case at::kByte: return 6;
    default: TORCH_CHECK(false, "rccl: unsupported dtype");
  }
  return -1;
}

hipStream_t cur(const at::Tensor& t) { return at::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check_gpu(const at::Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "rccl ops need contiguous GPU tensors");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X communication runtime: RCCL communicator manager and tensor-fusion engine";
  m.def("rccl_unique_id", []() { return py::bytes(pde::rccl_unique_id()); });
  m.def("rccl_version", &pde::rccl_version);

  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init<>())
      .def("init",
           [](RcclComm& c, py::bytes uid, int rank, int size, int device, bool blocking) {
             std::string u = uid;
             py::gil_scoped_release nogil;
             c.init(u, rank, size, device, blocking);
           },
           py::arg("uid"), py::arg("rank"), py::arg("size"), py::arg("device"), py::arg("blocking") = true)
      .def("abort", [](RcclComm& c) { py::gil_scoped_release nogil; c.abort(); })
      .def("shrink_from",
           [](RcclComm& c, RcclComm& parent, const std::vector<int>& exclude, bool abort_parent) {
             py::gil_scoped_release nogil;
             return c.shrink_from(parent, exclude, abort_parent);
           },
           py::arg("parent"), py::arg("exclude"), py::arg("abort_parent") = false)
      .def_static("shrink_supported", &RcclComm::shrink_supported)
      .def("split_from",
           [](RcclComm& c, RcclComm& parent, int color, int key, double timeout_s) {
             py::gil_scoped_release nogil;
             return c.split_from(parent, color, key, timeout_s);
           },
           py::arg("parent"), py::arg("color"), py::arg("key"), py::arg("timeout_s") = 300.0)
      .def("destroy", [](RcclComm& c) { py::gil_scoped_release nogil; c.destroy(); })
      .def_property_readonly("valid", &RcclComm::valid)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def_property_readonly("device", &RcclComm::device)
      .def("async_error", &RcclComm::async_error)
      .def("nranks", &RcclComm::nranks)
      // tensor-level collectives, enqueued on the caller's CURRENT torch stream (stream-ordered with
      // the producing kernels; no host synchronisation)
      .def("allreduce_",
           [](RcclComm& c, at::Tensor& t, int op) {
             check_gpu(t);
             c.allreduce(t.data_ptr(), t.data_ptr(), t.numel(), code_of(t), op, cur(t));
             return t;
           },
           py::arg("tensor"), py::arg("op") = 0)
      .def("broadcast_",
           [](RcclComm& c, at::Tensor& t, int root) {
             check_gpu(t);
             c.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), code_of(t), root, cur(t));
             return t;
           })
      .def("allgather",
           [](RcclComm& c, const at::Tensor& t) {
             check_gpu(t);
             std::vector<int64_t> shape = t.sizes().vec();
             if (shape.empty()) shape.push_back(1);
             shape[0] *= c.size();
             at::Tensor out = at::empty(shape, t.options());
             c.allgather(t.data_ptr(), out.data_ptr(), t.numel(), code_of(t), cur(t));
             return out;
           })
      .def("reduce_scatter",
           [](RcclComm& c, const at::Tensor& t, int op) {
             check_gpu(t);
             TORCH_CHECK(t.numel() % c.size() == 0, "reduce_scatter: numel must divide by size");
             at::Tensor out = at::empty({t.numel() / c.size()}, t.options());
             c.reduce_scatter(t.data_ptr(), out.data_ptr(), out.numel(), code_of(t), op, cur(t));
             return out;
           })
      .def("alltoall",
           [](RcclComm& c, const at::Tensor& t) {
             check_gpu(t);
             TORCH_CHECK(t.numel() % c.size() == 0, "alltoall: numel must divide by size");
             at::Tensor out = at::empty_like(t);
             c.alltoall(t.data_ptr(), out.data_ptr(), t.numel() / c.size(), code_of(t), cur(t));
             return out;
           })
      .def("send",
           [](RcclComm& c, const at::Tensor& t, int peer) {
             check_gpu(t);
             c.send(t.data_ptr(), t.numel(), code_of(t), peer, cur(t));
           })
      .def("recv",
           [](RcclComm& c, at::Tensor& t, int peer) {
             check_gpu(t);
             c.recv(t.data_ptr(), t.numel(), code_of(t), peer, cur(t));
             return t;
           })
      .def("group_start", &RcclComm::group_start)
      .def("group_end", &RcclComm::group_end);

  py::class_<XgmiAllreduce, std::shared_ptr<XgmiAllreduce>>(m, "XgmiAllreduce")
      .def(py::init<int, int, int, int64_t, int, double>(), py::arg("rank"), py::arg("size"), py::arg("device"),
           py::arg("max_bytes"), py::arg("blocks") = 64, py::arg("timeout_s") = 5.0)
      .def("ipc_handle", [](XgmiAllreduce& x) { return py::bytes(x.ipc_handle()); })
      .def("open",
           [](XgmiAllreduce& x, const std::vector<py::bytes>& hs) {
             std::vector<std::string> v;
             for (const auto& h : hs) v.emplace_back(std::string(h));
             x.open(v);
           })
      // in place (or src -> dst) on the caller's CURRENT stream; hipGraph-capturable
      .def("allreduce_",
           [](XgmiAllreduce& x, at::Tensor& t, double scale, bool wire_bf16) {
             check_gpu(t);
             TORCH_CHECK(t.scalar_type() == at::kFloat, "xgmi allreduce: fp32 tensors");
             x.allreduce(t.data_ptr<float>(), t.data_ptr<float>(), t.numel(), static_cast<float>(scale), cur(t),
                         wire_bf16);
             return t;
           },
           py::arg("tensor"), py::arg("scale") = 1.0, py::arg("wire_bf16") = false)
      .def("allreduce_twoshot_",
           [](XgmiAllreduce& x, at::Tensor& t, double scale, bool wire_bf16) {
             check_gpu(t);
             TORCH_CHECK(t.scalar_type() == at::kFloat, "xgmi allreduce: fp32 tensors");
             TORCH_CHECK(t.is_contiguous(), "xgmi allreduce: contiguous tensors");
             x.allreduce_twoshot(t.data_ptr<float>(), t.data_ptr<float>(), t.numel(), static_cast<float>(scale),
                                 cur(t), wire_bf16);
             return t;
           },
           py::arg("tensor"), py::arg("scale") = 1.0, py::arg("wire_bf16") = false)
      .def("view",
           [](const XgmiAllreduce& x) {  // flat device view for kernels that fold the exchange in (xgmi_view.h)
             const pde::XgmiView v = x.view();
             std::vector<int64_t> w;
             for (int r = 0; r < pde::kXgmiMaxRanks; ++r) w.push_back(reinterpret_cast<int64_t>(v.base[r]));
             w.push_back(reinterpret_cast<int64_t>(v.state));
             w.push_back(static_cast<int64_t>(v.timeout_ticks));
             w.push_back(v.flag_bytes);
             w.push_back(v.slot_bytes);
             w.push_back(v.rank);
             w.push_back(v.size);
             w.push_back(v.blocks);
             w.push_back(static_cast<int64_t>(v.read_delay_ticks));
             w.push_back(reinterpret_cast<int64_t>(v.host));
             return w;
           })
      .def("set_read_delay_us", &XgmiAllreduce::set_read_delay_us)
      .def("error", [](XgmiAllreduce& x, bool sync) { py::gil_scoped_release nogil; return x.error(sync); },
           py::arg("sync") = true)
      .def("clear_error", [](XgmiAllreduce& x) { py::gil_scoped_release nogil; x.clear_error(); })
      .def("abort", &XgmiAllreduce::abort)
      .def("reset_abort", &XgmiAllreduce::reset_abort)
      .def_property_readonly("aborted", &XgmiAllreduce::aborted)
      .def("close", [](XgmiAllreduce& x) { py::gil_scoped_release nogil; x.close(); })
      .def_property_readonly("rank", &XgmiAllreduce::rank)
      .def_property_readonly("size", &XgmiAllreduce::size)
      .def_property_readonly("max_bytes", &XgmiAllreduce::max_bytes)
      .def_property_readonly("calls", &XgmiAllreduce::calls);

  py::class_<P2PRing, std::shared_ptr<P2PRing>>(m, "P2PRing")
      .def(py::init<int, int64_t, double>(), py::arg("device"), py::arg("slot_bytes"), py::arg("timeout_s") = 60.0)
      .def("ipc_handle", [](P2PRing& r) { return py::bytes(r.ipc_handle()); })
      .def("open", [](P2PRing& r, py::bytes h) { r.open(std::string(h)); })
      .def("open_local", &P2PRing::open_local, py::arg("peer"))
      .def_static("max_wg", &P2PRing::max_wg)
      // both stream-ordered on the caller's CURRENT stream, hipGraph-capturable; raw bytes of the tensor
      .def("send",
           [](P2PRing& r, const at::Tensor& t) {
             check_gpu(t);
             r.send(t.data_ptr(), static_cast<int64_t>(t.numel() * t.element_size()), cur(t));
           })
      .def("recv",
           [](P2PRing& r, at::Tensor& t) {
             check_gpu(t);
             r.recv(t.data_ptr(), static_cast<int64_t>(t.numel() * t.element_size()), cur(t));
             return t;
           })
      .def("error", [](P2PRing& r) { py::gil_scoped_release nogil; return r.error(); })
      .def("close", [](P2PRing& r) { py::gil_scoped_release nogil; r.close(); })
      .def_property_readonly("slot_bytes", &P2PRing::slot_bytes)
      .def_property_readonly("sent", &P2PRing::sent)
      .def_property_readonly("received", &P2PRing::received);

  py::class_<FusionEngine, std::shared_ptr<FusionEngine>>(m, "FusionEngine")
      .def(py::init<int, int, int64_t, const std::string&, double>(), py::arg("rank"), py::arg("size"),
           py::arg("fusion_bytes"), py::arg("timeline_path") = "", py::arg("cycle_ms") = 0.5)
      .def("set_rccl", &FusionEngine::set_rccl)
      .def("set_xgmi", &FusionEngine::set_xgmi, py::arg("xgmi"), py::arg("threshold_bytes"))
      .def("allreduce_inline", &FusionEngine::allreduce_inline, py::arg("tensors"), py::arg("op"),
           py::arg("prescale") = 1.0, py::arg("postscale") = 1.0, py::arg("compress") = false)
      .def("cached", &FusionEngine::cached)
      .def("set_graph_mode", &FusionEngine::set_graph_mode, py::arg("on"), py::arg("tensors"))
      .def("check_xgmi", &FusionEngine::check_xgmi)
      .def("set_py_backend", &FusionEngine::set_py_backend)
      .def("set_control", &FusionEngine::set_control, py::arg("process_group"))
      .def("set_timeout", &FusionEngine::set_timeout)
      .def("set_blocking_wait", &FusionEngine::set_blocking_wait)
      .def("allreduce", &FusionEngine::allreduce, py::arg("tensor"), py::arg("output"), py::arg("name"),
           py::arg("op"), py::arg("prescale") = 1.0, py::arg("postscale") = 1.0, py::arg("compress") = false)
      .def("broadcast", &FusionEngine::broadcast)
      .def("allgather", &FusionEngine::allgather)
      .def("flush", &FusionEngine::flush)
      .def("poll", &FusionEngine::poll)
      .def("wait", &FusionEngine::wait)
      .def("shutdown", &FusionEngine::shutdown, py::arg("abort") = false)
      .def("inject_error", &FusionEngine::inject_error)
      .def_property_readonly("error", &FusionEngine::error)
      .def("stats", &FusionEngine::stats)
      .def_property("fusion_bytes", &FusionEngine::fusion_bytes, &FusionEngine::set_fusion_bytes);
}
