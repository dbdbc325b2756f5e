// Horovod-style fusion engine: see fusion_engine.h.
#include "fusion_engine.h"

#include <c10/hip/HIPCachingAllocator.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <sstream>

#include "pack.h"

namespace pde {

namespace {

int dtype_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kHalf: return 2;
    case at::kDouble: return 3;
    case at::kInt: return 4;
    case at::kLong: return 5;
    case at::kByte: return 6;
    default: throw std::invalid_argument("fusion engine: unsupported dtype");
  }
}

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("fusion engine: ") + what + ": " + hipGetErrorString(e));
}

void record_on(const at::Tensor& t, hipStream_t s, int device) {
  if (!t.defined() || !t.is_cuda()) return;
  c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(),
                                              c10::hip::getStreamFromExternal(s, device));
}

}  // namespace

FusionEngine::FusionEngine(int rank, int size, int64_t fusion_bytes, const std::string& timeline_path)
    : rank_(rank), size_(size), fusion_bytes_(fusion_bytes), t0_(std::chrono::steady_clock::now()) {
  if (!timeline_path.empty()) {
    trace_.open(timeline_path);
    trace_ << "[\n";
  }
  worker_ = std::thread([this] { loop(); });
}

FusionEngine::~FusionEngine() {
  try {
    shutdown();
  } catch (...) {
  }
}

double FusionEngine::now() const {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0_).count();
}

void FusionEngine::trace(const std::string& name, const std::string& phase, double t0, double t1, int64_t bytes) {
  if (!trace_.is_open()) return;
  std::lock_guard<std::mutex> g(trace_mu_);
  if (!trace_first_) trace_ << ",\n";
  trace_first_ = false;
  trace_ << "{\"name\":\"" << phase << "\",\"cat\":\"" << name << "\",\"ph\":\"X\",\"ts\":" << t0
         << ",\"dur\":" << (t1 - t0) << ",\"pid\":" << rank_ << ",\"tid\":\"" << name
         << "\",\"args\":{\"bytes\":" << bytes << "}}";
}

void FusionEngine::set_rccl(std::shared_ptr<RcclComm> comm) {
  comm_ = std::move(comm);
  gpu_backend_ = comm_ != nullptr;
}

void FusionEngine::set_py_backend(py::object allreduce_fn, py::object broadcast_fn, py::object allgather_fn) {
  py_allreduce_ = std::move(allreduce_fn);
  py_broadcast_ = std::move(broadcast_fn);
  py_allgather_ = std::move(allgather_fn);
}

void FusionEngine::close_open_locked() {
  if (!open_.reqs.empty()) {
    closed_.push_back(std::move(open_));
    open_ = Batch();
    cv_.notify_one();
  }
}

int64_t FusionEngine::allreduce(at::Tensor t, at::Tensor out, const std::string& name, int op, double prescale,
                                double postscale, bool compress) {
  TORCH_CHECK(t.is_contiguous() && out.is_contiguous(), "fusion engine: tensors must be contiguous");
  TORCH_CHECK(t.numel() == out.numel(), "fusion engine: output size mismatch");
  Request r;
  r.type = ReqType::ALLREDUCE;
  r.name = name;
  r.tensor = t;
  r.output = out;
  r.op = op;
  r.prescale = prescale;
  r.postscale = postscale;
  r.compress = compress && t.scalar_type() == at::kFloat;
  r.t_enqueue = now();
  if (t.is_cuda()) {
    TORCH_CHECK(gpu_backend_, "fusion engine: GPU tensor but no RCCL communicator");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(t.device());
    hip_ok(hipEventCreateWithFlags(&r.ready, hipEventDisableTiming), "event create");
    hip_ok(hipEventRecord(r.ready, at::hip::getCurrentHIPStream(t.device().index()).stream()), "event record");
  }
  const int64_t bytes = t.numel() * static_cast<int64_t>(r.compress ? 2 : t.element_size());
  std::lock_guard<std::mutex> g(mu_);
  r.handle = next_handle_++;
  handles_[r.handle] = HandleState();
  ++n_requests_;
  // batch key: device, dtype, op, scales, compression -- a change closes the open batch
  if (!open_.reqs.empty()) {
    const Request& h = open_.reqs.front();
    const bool same = h.tensor.device() == t.device() && h.tensor.scalar_type() == t.scalar_type() && h.op == op &&
                      h.prescale == prescale && h.postscale == postscale && h.compress == r.compress;
    if (!same || open_.bytes + bytes > fusion_bytes_.load() ||
        static_cast<int>(open_.reqs.size()) >= kMaxPackSegs * 8)
      close_open_locked();
  }
  const int64_t h = r.handle;
  open_.reqs.push_back(std::move(r));
  open_.bytes += bytes;
  if (open_.bytes >= fusion_bytes_.load()) close_open_locked();
  return h;
}

int64_t FusionEngine::broadcast(at::Tensor t, int root, const std::string& name) {
  TORCH_CHECK(t.is_contiguous(), "fusion engine: tensor must be contiguous");
  Request r;
  r.type = ReqType::BROADCAST;
  r.name = name;
  r.tensor = t;
  r.output = t;
  r.root = root;
  r.t_enqueue = now();
  if (t.is_cuda()) {
    TORCH_CHECK(gpu_backend_, "fusion engine: GPU tensor but no RCCL communicator");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(t.device());
    hip_ok(hipEventCreateWithFlags(&r.ready, hipEventDisableTiming), "event create");
    hip_ok(hipEventRecord(r.ready, at::hip::getCurrentHIPStream(t.device().index()).stream()), "event record");
  }
  std::lock_guard<std::mutex> g(mu_);
  r.handle = next_handle_++;
  handles_[r.handle] = HandleState();
  ++n_requests_;
  close_open_locked();
  Batch b;
  b.bytes = t.numel() * t.element_size();
  const int64_t h = r.handle;
  b.reqs.push_back(std::move(r));
  closed_.push_back(std::move(b));
  cv_.notify_one();
  return h;
}

int64_t FusionEngine::allgather(at::Tensor t, const std::string& name) {
  TORCH_CHECK(t.is_contiguous(), "fusion engine: tensor must be contiguous");
  Request r;
  r.type = ReqType::ALLGATHER;
  r.name = name;
  r.tensor = t;
  std::vector<int64_t> shape = t.sizes().vec();
  if (shape.empty()) shape.push_back(1);
  shape[0] *= size_;
  r.output = at::empty(shape, t.options());
  r.t_enqueue = now();
  if (t.is_cuda()) {
    TORCH_CHECK(gpu_backend_, "fusion engine: GPU tensor but no RCCL communicator");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(t.device());
    hip_ok(hipEventCreateWithFlags(&r.ready, hipEventDisableTiming), "event create");
    hip_ok(hipEventRecord(r.ready, at::hip::getCurrentHIPStream(t.device().index()).stream()), "event record");
  }
  std::lock_guard<std::mutex> g(mu_);
  r.handle = next_handle_++;
  handles_[r.handle] = HandleState();
  ++n_requests_;
  close_open_locked();
  Batch b;
  b.bytes = t.numel() * t.element_size();
  const int64_t h = r.handle;
  b.reqs.push_back(std::move(r));
  closed_.push_back(std::move(b));
  cv_.notify_one();
  return h;
}

void FusionEngine::flush() {
  std::lock_guard<std::mutex> g(mu_);
  close_open_locked();
}

bool FusionEngine::poll(int64_t h) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = handles_.find(h);
  if (it == handles_.end()) return true;
  if (!it->second.done) return false;
  if (it->second.finished != nullptr) return hipEventQuery(it->second.finished) == hipSuccess;
  return true;
}

at::Tensor FusionEngine::wait(int64_t h) {
  HandleState st;
  {
    py::gil_scoped_release nogil;
    std::unique_lock<std::mutex> lk(mu_);
    // a handle still sitting in the open batch is flushed: every rank reaches this point in the same
    // request order, so the cut stays deterministic
    for (const auto& r : open_.reqs)
      if (r.handle == h) {
        close_open_locked();
        break;
      }
    auto it = handles_.find(h);
    TORCH_CHECK(it != handles_.end(), "fusion engine: unknown handle ", h);
    done_cv_.wait(lk, [&] { return handles_[h].done || stop_; });
    st = handles_[h];
    handles_.erase(h);
  }
  if (!st.error.empty()) throw std::runtime_error("HorovodInternalError: " + st.error);
  if (st.finished != nullptr) {
    // order the caller's stream after the collective; no host block
    const int dev = st.output.device().index();
    hipError_t e = hipStreamWaitEvent(at::hip::getCurrentHIPStream(dev).stream(), st.finished, 0);
    (void)hipEventDestroy(st.finished);
    hip_ok(e, "stream wait");
  }
  return st.output;
}

void FusionEngine::shutdown() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) return;
    close_open_locked();
    stop_ = true;
    cv_.notify_all();
  }
  if (worker_.joinable()) {
    if (PyGILState_Check()) {
      py::gil_scoped_release nogil;
      worker_.join();
    } else {
      worker_.join();
    }
  }
  if (trace_.is_open()) {
    trace_ << "\n]\n";
    trace_.close();
  }
}

py::dict FusionEngine::stats() {
  std::lock_guard<std::mutex> g(mu_);
  py::dict d;
  d["requests"] = n_requests_;
  d["batches"] = n_batches_;
  d["fused_requests"] = n_fused_requests_;
  d["bytes"] = n_bytes_;
  d["fusion_bytes"] = fusion_bytes_.load();
  d["backend"] = gpu_backend_ ? "rccl" : "python";
  return d;
}

void FusionEngine::loop() {
  for (;;) {
    Batch b;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !closed_.empty(); });
      if (closed_.empty() && stop_) return;
      b = std::move(closed_.front());
      closed_.pop_front();
    }
    execute(b);
  }
}

void FusionEngine::finish(Batch& b, const std::string& err, bool gpu_done) {
  std::lock_guard<std::mutex> g(mu_);
  ++n_batches_;
  n_bytes_ += b.bytes;
  if (b.reqs.size() > 1) n_fused_requests_ += static_cast<int64_t>(b.reqs.size());
  for (size_t i = 0; i < b.reqs.size(); ++i) {
    Request& r = b.reqs[i];
    HandleState& st = handles_[r.handle];
    st.done = true;
    st.error = err;
    st.output = r.output;
    if (gpu_done) {
      // each handle owns an event (the waiter destroys it)
      hipEvent_t e2 = nullptr;
      if (hipEventCreateWithFlags(&e2, hipEventDisableTiming) == hipSuccess) {
        (void)hipEventRecord(e2, comm_->stream());
        st.finished = e2;
      }
    }
    if (r.ready != nullptr) {
      (void)hipEventDestroy(r.ready);
      r.ready = nullptr;
    }
  }
  done_cv_.notify_all();
}

void FusionEngine::execute(Batch& b) {
  std::string err;
  const bool gpu = b.reqs.front().tensor.is_cuda();
  const double t_start = now();
  try {
    if (gpu) {
      hip_ok(hipSetDevice(comm_->device()), "set device");
      if (b.reqs.front().type == ReqType::ALLREDUCE)
        run_allreduce_gpu(b);
      else
        run_single_gpu(b.reqs.front());
    } else {
      if (b.reqs.front().type == ReqType::ALLREDUCE)
        run_allreduce_cpu(b);
      else
        run_single_cpu(b.reqs.front());
    }
  } catch (py::error_already_set& e) {
    py::gil_scoped_acquire g;
    err = e.what();
  } catch (std::exception& e) {
    err = e.what();
  }
  const double t_end = now();
  if (trace_.is_open()) {
    for (auto& r : b.reqs) {
      trace(r.name, "QUEUE", r.t_enqueue, t_start, 0);
      trace(r.name, b.reqs.front().type == ReqType::ALLREDUCE ? "ALLREDUCE" : "COLLECTIVE", t_start, t_end, b.bytes);
    }
  }
  finish(b, err, gpu && err.empty());
}

void FusionEngine::run_allreduce_gpu(Batch& b) {
  hipStream_t s = comm_->stream();
  const int dev = comm_->device();
  for (auto& r : b.reqs)
    if (r.ready) hip_ok(hipStreamWaitEvent(s, r.ready, 0), "wait producer");
  Request& r0 = b.reqs.front();
  const int dt = dtype_code(r0.tensor);
  if (b.reqs.size() == 1 && !r0.compress && r0.prescale == 1.0 && r0.postscale == 1.0) {
    comm_->allreduce(r0.tensor.data_ptr(), r0.output.data_ptr(), r0.tensor.numel(), dt, r0.op, s);
    record_on(r0.tensor, s, dev);
    record_on(r0.output, s, dev);
    return;
  }
  TORCH_CHECK(dt == 0 || dt == 1, "fusion engine: fused batches support fp32/bf16 tensors");
  const int wire = (r0.compress || dt == 1) ? 1 : 0;
  int64_t total = 0;
  for (auto& r : b.reqs) total += r.tensor.numel();
  const int64_t need = total * (wire == 1 ? 2 : 4);
  if (!fused_.defined() || fused_.device() != r0.tensor.device() || fused_.numel() < need) {
    if (fused_.defined()) hip_ok(hipStreamSynchronize(s), "sync before regrow");
    fused_ = at::empty({need + (1 << 20)}, r0.tensor.options().dtype(at::kByte));
  }
  // pack (pre-scale) in chunks of kMaxPackSegs tensors
  PackTable tab;
  auto each_chunk = [&](auto&& fn) {
    int64_t off = 0;
    size_t i = 0;
    while (i < b.reqs.size()) {
      tab.count = 0;
      for (; i < b.reqs.size() && tab.count < kMaxPackSegs; ++i) {
        PackSeg& sg = tab.seg[tab.count++];
        sg.n = b.reqs[i].tensor.numel();
        sg.offset = off;
        sg.dtype = dt;
        sg.ptr = nullptr;
        off += sg.n;
      }
      fn(i - tab.count);
    }
  };
  const float pre = static_cast<float>(r0.prescale), post = static_cast<float>(r0.postscale);
  each_chunk([&](size_t first) {
    for (int k = 0; k < tab.count; ++k) tab.seg[k].ptr = b.reqs[first + k].tensor.data_ptr();
    hip_ok(fusion_pack(tab, fused_.data_ptr(), wire, pre, s), "pack");
  });
  comm_->allreduce(fused_.data_ptr(), fused_.data_ptr(), total, wire, r0.op, s);
  each_chunk([&](size_t first) {
    for (int k = 0; k < tab.count; ++k) tab.seg[k].ptr = b.reqs[first + k].output.data_ptr();
    hip_ok(fusion_unpack(tab, fused_.data_ptr(), wire, post, s), "unpack");
  });
  for (auto& r : b.reqs) {
    record_on(r.tensor, s, dev);
    record_on(r.output, s, dev);
  }
}

void FusionEngine::run_single_gpu(Request& r) {
  hipStream_t s = comm_->stream();
  if (r.ready) hip_ok(hipStreamWaitEvent(s, r.ready, 0), "wait producer");
  const int dt = dtype_code(r.tensor);
  if (r.type == ReqType::BROADCAST) {
    comm_->broadcast(r.tensor.data_ptr(), r.tensor.data_ptr(), r.tensor.numel(), dt, r.root, s);
  } else {
    comm_->allgather(r.tensor.data_ptr(), r.output.data_ptr(), r.tensor.numel(), dt, s);
  }
  record_on(r.tensor, s, comm_->device());
  record_on(r.output, s, comm_->device());
}

void FusionEngine::run_allreduce_cpu(Batch& b) {
  Request& r0 = b.reqs.front();
  const auto wire = (r0.compress) ? at::kBFloat16 : r0.tensor.scalar_type();
  std::vector<at::Tensor> flats;
  flats.reserve(b.reqs.size());
  for (auto& r : b.reqs) {
    at::Tensor f = r.tensor.reshape({-1});
    if (r.prescale != 1.0) f = f * r.prescale;
    flats.push_back(f.to(wire));
  }
  at::Tensor fused = flats.size() == 1 ? flats[0].clone() : at::cat(flats);
  {
    py::gil_scoped_acquire g;
    py_allreduce_(fused, r0.op);
  }
  int64_t off = 0;
  for (auto& r : b.reqs) {
    const int64_t n = r.tensor.numel();
    at::Tensor part = fused.slice(0, off, off + n).view(r.output.sizes());
    if (r.postscale != 1.0) part = part.to(at::kFloat) * r.postscale;
    r.output.copy_(part);
    off += n;
  }
}

void FusionEngine::run_single_cpu(Request& r) {
  py::gil_scoped_acquire g;
  if (r.type == ReqType::BROADCAST)
    py_broadcast_(r.tensor, r.root);
  else
    py_allgather_(r.tensor, r.output);
}

}  // namespace pde
