// Horovod-style fusion engine with negotiation: see fusion_engine.h.
#include "fusion_engine.h"

#include <c10/hip/HIPCachingAllocator.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

constexpr char kFieldSep = '\x1f';
constexpr char kRecSep = '\x1e';
const char* kTypeNames[] = {"allreduce", "broadcast", "allgather"};

}  // namespace

std::string Request::signature() const {
  std::ostringstream s;
  s << kTypeNames[static_cast<int>(type)] << " dtype=" << c10::toString(tensor.scalar_type())
    << " shape=" << tensor.sizes() << " device=" << (tensor.is_cuda() ? "gpu" : "cpu");
  if (type == ReqType::ALLREDUCE)
    s << " op=" << op << " prescale=" << prescale << " postscale=" << postscale << " compress=" << compress;
  if (type == ReqType::BROADCAST) s << " root=" << root;
  return s.str();
}

FusionEngine::FusionEngine(int rank, int size, int64_t fusion_bytes, const std::string& timeline_path,
                           double cycle_ms)
    : rank_(rank), size_(size), fusion_bytes_(fusion_bytes), cycle_ms_(cycle_ms),
      t0_(std::chrono::steady_clock::now()) {
  if (const char* e = std::getenv("PDE_HVD_IDLE_MS")) idle_ms_ = std::max(0.05, std::atof(e));
  if (const char* e = std::getenv("HOROVOD_STALL_CHECK_TIME_SECONDS")) stall_warn_s_ = std::max(1.0, std::atof(e));
  if (const char* e = std::getenv("HOROVOD_CACHE_CAPACITY")) cache_capacity_ = std::max<int64_t>(0, std::atoll(e));
  if (!timeline_path.empty()) {
    trace_.open(timeline_path);
    trace_ << "[\n";
  }
  worker_ = std::thread([this] { loop(); });
}

FusionEngine::~FusionEngine() {
  try {
    shutdown(false);
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
  gpu_backend_ = comm_ != nullptr || xgmi_ != nullptr;
}

void FusionEngine::set_xgmi(std::shared_ptr<XgmiAllreduce> xgmi, int64_t threshold_bytes) {
  xgmi_ = std::move(xgmi);
  xgmi_threshold_ = xgmi_ ? std::min<int64_t>(threshold_bytes, xgmi_->max_bytes()) : 0;
  gpu_backend_ = comm_ != nullptr || xgmi_ != nullptr;
}

void FusionEngine::set_py_backend(py::object allreduce_fn, py::object broadcast_fn, py::object allgather_fn) {
  py_allreduce_ = std::move(allreduce_fn);
  py_broadcast_ = std::move(broadcast_fn);
  py_allgather_ = std::move(allgather_fn);
}

void FusionEngine::set_control(c10::intrusive_ptr<c10d::ProcessGroup> pg) {
  TORCH_CHECK(pg->getSize() == size_ && pg->getRank() == rank_, "fusion engine: control group rank/size mismatch");
  {
    std::lock_guard<std::mutex> g(mu_);  // the worker reads control_ under mu_ to decide lockstep cycling
    control_ = std::move(pg);
  }
  cv_.notify_all();
}

// ---------------------------------------------------------------------------------------------------
// enqueue side (framework thread)
// ---------------------------------------------------------------------------------------------------
int64_t FusionEngine::enqueue(Request&& r) {
  std::lock_guard<std::mutex> g(mu_);
  if (!error_.empty()) {
    if (r.ready) (void)hipEventDestroy(r.ready);
    throw std::runtime_error("HorovodInternalError: " + error_);
  }
  if (stop_requested_ || stopped_) {
    if (r.ready) (void)hipEventDestroy(r.ready);
    throw std::runtime_error("Horovod has been shut down");
  }
  const bool dup = announced_.count(r.name) > 0 ||
                   std::any_of(cached_pending_.begin(), cached_pending_.end(),
                               [&](const std::pair<const int, Request>& q) { return q.second.name == r.name; }) ||
                   std::any_of(unannounced_.begin(), unannounced_.end(),
                               [&](const Request& q) { return q.name == r.name; });
  if (dup) {
    if (r.ready) (void)hipEventDestroy(r.ready);
    TORCH_CHECK(false, "fusion engine: a request named '", r.name, "' is already outstanding on rank ", rank_);
  }
  r.handle = next_handle_++;
  handles_[r.handle] = HandleState();
  ++n_requests_;
  const int64_t h = r.handle;
  unannounced_.push_back(std::move(r));
  cv_.notify_one();
  return h;
}

static void record_ready(Request& r) {
  if (!r.tensor.is_cuda()) return;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(r.tensor.device());
  hip_ok(hipEventCreateWithFlags(&r.ready, hipEventDisableTiming), "event create");
  hip_ok(hipEventRecord(r.ready, at::hip::getCurrentHIPStream(r.tensor.device().index()).stream()), "event record");
}

int64_t FusionEngine::allreduce(at::Tensor t, at::Tensor out, const std::string& name, int op, double prescale,
                                double postscale, bool compress) {
  TORCH_CHECK(t.is_contiguous() && out.is_contiguous(), "fusion engine: tensors must be contiguous");
  TORCH_CHECK(t.numel() == out.numel(), "fusion engine: output size mismatch");
  if (t.is_cuda()) TORCH_CHECK(gpu_backend_, "fusion engine: GPU tensor but no RCCL communicator");
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
  record_ready(r);
  return enqueue(std::move(r));
}

int64_t FusionEngine::broadcast(at::Tensor t, int root, const std::string& name) {
  TORCH_CHECK(t.is_contiguous(), "fusion engine: tensor must be contiguous");
  if (t.is_cuda()) TORCH_CHECK(gpu_backend_, "fusion engine: GPU tensor but no RCCL communicator");
  Request r;
  r.type = ReqType::BROADCAST;
  r.name = name;
  r.tensor = t;
  r.output = t;
  r.root = root;
  r.t_enqueue = now();
  record_ready(r);
  return enqueue(std::move(r));
}

int64_t FusionEngine::allgather(at::Tensor t, const std::string& name) {
  TORCH_CHECK(t.is_contiguous(), "fusion engine: tensor must be contiguous");
  if (t.is_cuda()) TORCH_CHECK(gpu_backend_, "fusion engine: GPU tensor but no RCCL communicator");
  Request r;
  r.type = ReqType::ALLGATHER;
  r.name = name;
  r.tensor = t;
  std::vector<int64_t> shape = t.sizes().vec();
  if (shape.empty()) shape.push_back(1);
  shape[0] *= size_;
  r.output = at::empty(shape, t.options());
  r.t_enqueue = now();
  record_ready(r);
  return enqueue(std::move(r));
}

void FusionEngine::flush() {
  // negotiation cycles run on their own; kept for API compatibility (wakes the engine early)
  std::lock_guard<std::mutex> g(mu_);
  cv_.notify_one();
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
    auto it = handles_.find(h);
    TORCH_CHECK(it != handles_.end(), "fusion engine: unknown handle ", h);
    done_cv_.wait(lk, [&] { return handles_[h].done; });
    st = handles_[h];
    handles_.erase(h);
  }
  if (!st.error.empty()) {
    if (st.finished) (void)hipEventDestroy(st.finished);
    throw std::runtime_error("HorovodInternalError: " + st.error);
  }
  if (st.finished != nullptr) {
    if (blocking_wait_) {
      // host-side completion poll with liveness checks: a failed peer surfaces HERE
      py::gil_scoped_release nogil;
      const auto t0 = std::chrono::steady_clock::now();
      std::string err;
      for (;;) {
        hipError_t q = hipEventQuery(st.finished);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) {
          err = std::string("GPU error while waiting: ") + hipGetErrorString(q);
          break;
        }
        {
          std::lock_guard<std::mutex> g(mu_);
          if (!error_.empty()) err = error_;
        }
        if (err.empty()) err = xgmi_failure();
        if (err.empty() && comm_) {
          const int ae = comm_->async_error();
          if (ae != ncclSuccess && ae != ncclInProgress) err = std::string("RCCL async error: ") +
                                                                ncclGetErrorString(static_cast<ncclResult_t>(ae));
        }
        if (err.empty() && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s_)
          err = "collective did not complete within " + std::to_string(timeout_s_) + " s";
        if (!err.empty()) break;
        std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
      if (!err.empty()) {
        set_error(err);
        (void)hipEventDestroy(st.finished);
        throw std::runtime_error("HorovodInternalError: " + err);
      }
    } else {
      // order the caller's stream after the collective; no host block (the engine's watchdog aborts the
      // communicator if the batch never completes)
      const int dev = st.output.device().index();
      hipError_t e = hipStreamWaitEvent(at::hip::getCurrentHIPStream(dev).stream(), st.finished, 0);
      hip_ok(e, "stream wait");
    }
    (void)hipEventDestroy(st.finished);
  }
  return st.output;
}

void FusionEngine::inject_error(const std::string& why) { set_error(why); }

void FusionEngine::shutdown(bool abort) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stopped_ && !worker_.joinable()) return;
    stop_requested_ = true;
    cv_.notify_all();
  }
  if (abort) set_error("Horovod has been shut down (abort)");
  if (worker_.joinable()) {
    auto join = [&] {
      if (!abort) {
        worker_.join();
        return;
      }
      // an aborted engine may have its thread inside a control collective with a dead peer: bounded wait
      for (int i = 0; i < 400; ++i) {
        {
          std::lock_guard<std::mutex> g(mu_);
          if (stopped_) break;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
      }
      bool done;
      {
        std::lock_guard<std::mutex> g(mu_);
        done = stopped_;
      }
      if (done)
        worker_.join();
      else
        worker_.detach();  // Python keeps this engine object alive (hvd.core._retired)
    };
    if (PyGILState_Check()) {
      py::gil_scoped_release nogil;
      join();
    } else {
      join();
    }
  }
  for (auto& f : inflight_) (void)hipEventDestroy(f.done);
  inflight_.clear();
  // (own_stream_ is deliberately not destroyed: tensors were recordStream()-ed on it; see RcclComm's dtor)
  if (trace_.is_open()) {
    std::lock_guard<std::mutex> g(trace_mu_);
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
  d["cycles"] = n_cycles_;
  d["fusion_bytes"] = fusion_bytes_.load();
  d["backend"] = gpu_backend_ ? "rccl" : "python";
  d["negotiated"] = control_ ? true : false;
  d["xgmi_batches"] = n_xgmi_batches_;
  d["rccl_batches"] = n_rccl_batches_;
  d["inplace_batches"] = n_inplace_batches_;    // adjacent views of one buffer: no pack / unpack
  d["inline_calls"] = n_inline_calls_;          // graph-mode calls (caller's stream, no negotiation)
  d["string_gathers"] = n_string_gathers_;    // cycles that all-gathered name/signature strings (2 gathers each)
  d["bit_allreduces"] = n_bit_allreduces_;    // cycles negotiated by the cached bit vector alone
  d["cache_hits"] = n_cache_hits_;
  d["cache_evictions"] = n_cache_evictions_;
  d["cache_entries"] = static_cast<int64_t>(cache_.size());
  d["error"] = error_;
  return d;
}

// ---------------------------------------------------------------------------------------------------
// failure state
// ---------------------------------------------------------------------------------------------------
void FusionEngine::fail_all_locked(const std::string& err) {
  for (auto& r : unannounced_)
    if (r.ready) (void)hipEventDestroy(r.ready);
  for (auto& kv : announced_)
    if (kv.second.ready) (void)hipEventDestroy(kv.second.ready);
  for (auto& kv : cached_pending_)
    if (kv.second.ready) (void)hipEventDestroy(kv.second.ready);
  unannounced_.clear();
  announced_.clear();
  cached_pending_.clear();
  table_.clear();
  for (auto& kv : handles_) {
    if (!kv.second.done) {
      kv.second.done = true;
      kv.second.error = err;
    }
  }
  done_cv_.notify_all();
}

void FusionEngine::set_error(const std::string& err) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (error_.empty()) error_ = err;
    fail_all_locked(error_);
  }
  // release any collective hung on a dead peer (kernels spinning on a connection exit on abort; xGMI
  // exchanges give up on the host abort word)
  if (comm_) comm_->abort();
  if (xgmi_) xgmi_->abort();
}

std::string FusionEngine::xgmi_failure() {
  if (xgmi_ && xgmi_->error(false) != 0)
    return "xGMI peer exchange: a wait for a peer timed out (peer dead or stalled); its result was dropped";
  return std::string();
}

void FusionEngine::check_xgmi() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!error_.empty()) throw std::runtime_error("HorovodInternalError: " + error_);
  }
  const std::string err = xgmi_failure();
  if (!err.empty()) {
    set_error(err);
    throw std::runtime_error("HorovodInternalError: " + err);
  }
}

void FusionEngine::set_graph_mode(bool on, const std::vector<at::Tensor>& tensors) {
  int64_t need = 0;
  for (const auto& t : tensors) need += t.numel() * 4;  // fp32 staging covers every wire format
  if (on && !tensors.empty() && tensors.front().is_cuda() && need > 0) {
    c10::hip::HIPGuardMasqueradingAsCUDA guard(tensors.front().device());
    if (!inline_fused_.defined() || inline_fused_.numel() < need) {
      if (inline_fused_.defined()) retired_inline_.push_back(inline_fused_);  // an earlier capture may use it
      inline_fused_ = at::empty({need + 4096}, tensors.front().options().dtype(at::kByte));
    }
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    graph_mode_ = on;
  }
  cv_.notify_all();
}

void FusionEngine::ensure_stage(at::Tensor& stage, const at::Tensor& like, int64_t bytes, hipStream_t s,
                                bool inline_mode) {
  if (stage.defined() && stage.device() == like.device() && stage.numel() >= bytes) return;
  if (inline_mode) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    hip_ok(hipStreamIsCapturing(s, &st), "capture status");
    // growing here would synchronise a capturing stream (breaking the capture) or free storage an earlier
    // capture still points at: graph mode sizes its buffer up front (set_graph_mode)
    TORCH_CHECK(st == hipStreamCaptureStatusNone && !stage.defined(),
                "fusion engine: graph-mode staging buffer too small (", bytes,
                " B); call set_graph_mode with the gradient set before capturing");
  } else if (stage.defined()) {
    hip_ok(hipStreamSynchronize(s), "sync before regrow");
  }
  stage = at::empty({bytes + (1 << 20)}, like.options().dtype(at::kByte));
}

void FusionEngine::check_inflight() {
  if (inflight_.empty()) {
    const std::string e = xgmi_failure();
    if (!e.empty()) set_error(e);
    return;
  }
  std::string err;
  size_t k = 0;
  for (auto& f : inflight_) {
    hipError_t q = hipEventQuery(f.done);
    if (q == hipSuccess) {
      (void)hipEventDestroy(f.done);
      continue;
    }
    if (q != hipErrorNotReady && err.empty()) err = std::string("GPU error: ") + hipGetErrorString(q);
    if (err.empty() && now() - f.t_start > timeout_s_ * 1e6)
      err = "RCCL collective did not complete within " + std::to_string(timeout_s_) + " s";
    inflight_[k++] = f;
  }
  inflight_.resize(k);
  if (err.empty()) err = xgmi_failure();
  if (err.empty() && comm_ && !inflight_.empty()) {
    const int ae = comm_->async_error();
    if (ae != ncclSuccess && ae != ncclInProgress)
      err = std::string("RCCL async error: ") + ncclGetErrorString(static_cast<ncclResult_t>(ae));
  }
  if (!err.empty()) set_error(err);
}

// ---------------------------------------------------------------------------------------------------
// background loop: cycle = (coalesce) -> negotiate -> fuse -> execute
// ---------------------------------------------------------------------------------------------------
void FusionEngine::loop() {
  for (;;) {
    bool stop_local;
    std::vector<Request> announce;
    {
      std::unique_lock<std::mutex> lk(mu_);
      auto has_work = [&] {
        return stop_requested_ || !unannounced_.empty() || !announced_.empty() || !cached_pending_.empty();
      };
      // Multi-rank engines cycle in lockstep whether or not this rank has work: a rank that announced a
      // tensor blocks in the control-plane all-gather until every peer joins the cycle, so an idle peer
      // (running eval, writing a checkpoint) must keep taking part -- Horovod's background loop does the
      // same.  Idle cycles back off to idle_ms_ so an idle job costs one small all-gather per few ms.
      const bool lockstep = size_ > 1 && control_ && error_.empty() && !graph_mode_;
      if (!has_work()) {
        if (lockstep)
          cv_.wait_for(lk, std::chrono::microseconds(static_cast<int64_t>(idle_ms_ * 1e3)), has_work);
        else if (inflight_.empty())
          cv_.wait(lk, has_work);
        else
          cv_.wait_for(lk, std::chrono::milliseconds(5), has_work);
      }
      if (!has_work() && !lockstep) {
        lk.unlock();
        check_inflight();
        continue;
      }
      if (!error_.empty()) {  // failed engine: nothing is negotiated any more
        stopped_ = true;
        done_cv_.notify_all();
        return;
      }
    }
    // coalesce a burst of enqueues (backward hooks) into one cycle, as Horovod's cycle time does
    bool local_work;
    {
      std::lock_guard<std::mutex> g(mu_);
      local_work = !unannounced_.empty();
    }
    if (local_work && cycle_ms_ > 0) std::this_thread::sleep_for(std::chrono::microseconds(static_cast<int64_t>(cycle_ms_ * 1e3)));
    {
      std::lock_guard<std::mutex> g(mu_);
      while (!unannounced_.empty()) {
        announce.push_back(std::move(unannounced_.front()));
        unannounced_.pop_front();
      }
      stop_local = stop_requested_;
    }
    std::vector<Request> ready;
    bool stop = stop_local;
    const double tn = now();
    bool have_control;
    {
      std::lock_guard<std::mutex> g(mu_);
      have_control = static_cast<bool>(control_);
    }
    if (size_ == 1 || !have_control) {
      ready = std::move(announce);
    } else {
      try {
        negotiate(announce, ready, stop);
      } catch (std::exception& e) {
        set_error(std::string("control plane: ") + e.what());
        std::lock_guard<std::mutex> g(mu_);
        stopped_ = true;
        done_cv_.notify_all();
        return;
      }
    }
    ++n_cycles_;
    if (trace_.is_open() && !ready.empty()) trace("engine", "NEGOTIATE", tn, now(), 0);
    std::vector<Batch> batches = make_batches(ready);
    for (auto& b : batches) execute(b);
    check_inflight();
    if (stop) {
      std::lock_guard<std::mutex> g(mu_);
      stopped_ = true;
      fail_all_locked("Horovod has been shut down");
      return;
    }
  }
}

void FusionEngine::negotiate(std::vector<Request>& announce, std::vector<Request>& ready, bool& stop) {
  const double tn = now();
  // 0. response cache: requests whose (name, signature) negotiated before ride on their cache id's word
  std::vector<Request> uncached;
  int nbits = 0;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& r : announce) {
      auto c = cache_.find(r.name);
      if (c != cache_.end() && c->second.signature == r.signature()) {
        ++n_cache_hits_;
        cached_pending_.emplace(c->second.id, std::move(r));
      } else {
        uncached.push_back(std::move(r));
      }
    }
    nbits = cache_ids_;
  }
  announce.clear();
  auto i32 = at::TensorOptions().dtype(at::kInt);
  at::Tensor bits = at::zeros({nbits + 2}, i32);
  int32_t* bw = bits.data_ptr<int32_t>();
  {
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& kv : cached_pending_) bw[kv.first] = 1;
  }
  bw[nbits] = stop ? -1 : 0;
  bw[nbits + 1] = uncached.empty() ? 0 : -1;
  {
    std::vector<at::Tensor> v{bits};
    c10d::AllreduceOptions o;
    o.reduceOp = c10d::ReduceOp::MIN;
    control_->allreduce(v, o)->wait();
  }
  bool any_stop = bw[nbits] < 0;
  const bool any_uncached = bw[nbits + 1] < 0;
  {  // cached tensors every rank announced: ready, in cache-id order (identical on every rank)
    std::lock_guard<std::mutex> g(mu_);
    for (int id = 0; id < nbits; ++id) {
      if (bw[id] != 1) continue;
      auto it = cached_pending_.find(id);
      if (it == cached_pending_.end()) continue;  // cannot happen: the AND includes this rank's word
      ready.push_back(std::move(it->second));
      cached_pending_.erase(it);
    }
  }
  if (!any_uncached) {
    ++n_bit_allreduces_;
    stop = any_stop;
    return;
  }
  ++n_string_gathers_;
  // 1. this rank's message: stop flag + (name, signature) records, in local enqueue order
  std::string msg(1, stop ? 'S' : '-');
  for (const auto& r : uncached) {
    msg += r.name;
    msg += kFieldSep;
    msg += r.signature();
    msg += kRecSep;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& r : uncached) {
      std::string name = r.name;
      announced_.emplace(std::move(name), std::move(r));
    }
  }
  uncached.clear();
  // 2. all-gather the lengths, then the padded payloads, over the gloo control group
  auto i64 = at::TensorOptions().dtype(at::kLong);
  std::vector<at::Tensor> len_in{at::full({1}, static_cast<int64_t>(msg.size()), i64)};
  std::vector<std::vector<at::Tensor>> len_out(1);
  for (int i = 0; i < size_; ++i) len_out[0].push_back(at::empty({1}, i64));
  control_->allgather(len_out, len_in)->wait();
  std::vector<int64_t> lens(size_);
  int64_t L = 1;
  for (int i = 0; i < size_; ++i) {
    lens[i] = len_out[0][i].data_ptr<int64_t>()[0];
    L = std::max(L, lens[i]);
  }
  auto u8 = at::TensorOptions().dtype(at::kByte);
  at::Tensor payload = at::zeros({L}, u8);
  std::memcpy(payload.data_ptr(), msg.data(), msg.size());
  std::vector<at::Tensor> pay_in{payload};
  std::vector<std::vector<at::Tensor>> pay_out(1);
  for (int i = 0; i < size_; ++i) pay_out[0].push_back(at::empty({L}, u8));
  control_->allgather(pay_out, pay_in)->wait();
  // 3. the decentralised coordinator: every rank applies the same rule to the same table
  for (int r = 0; r < size_; ++r) {
    const char* p = reinterpret_cast<const char*>(pay_out[0][r].data_ptr());
    std::string m(p, static_cast<size_t>(lens[r]));
    if (m.empty()) continue;
    any_stop |= m[0] == 'S';
    size_t pos = 1;
    while (pos < m.size()) {
      size_t fs = m.find(kFieldSep, pos), rs = m.find(kRecSep, pos);
      if (fs == std::string::npos || rs == std::string::npos || fs > rs) break;
      std::string name = m.substr(pos, fs - pos), sig = m.substr(fs + 1, rs - fs - 1);
      pos = rs + 1;
      {  // a cached name announced through the strings (its signature changed on some rank): evict it on
         // every rank; this rank's pending cached request for it is re-announced through the strings
        std::lock_guard<std::mutex> g(mu_);
        auto c = cache_.find(name);
        if (c != cache_.end()) {
          auto p = cached_pending_.find(c->second.id);
          if (p != cached_pending_.end()) {
            unannounced_.push_front(std::move(p->second));
            cached_pending_.erase(p);
          }
          cache_.erase(c);
          ++n_cache_evictions_;
        }
      }
      auto it = table_.find(name);
      if (it == table_.end()) {
        NegEntry e;
        e.signature = sig;
        e.count = 1;
        e.order = order_seq_++;
        e.t_first = tn;
        table_.emplace(name, std::move(e));
      } else {
        if (it->second.signature != sig && it->second.error.empty())
          it->second.error = "mismatched request for tensor '" + name + "': rank " + std::to_string(r) + " sent [" +
                             sig + "] but another rank sent [" + it->second.signature + "]";
        ++it->second.count;
      }
    }
  }
  std::vector<std::pair<int64_t, std::string>> complete;
  for (auto& kv : table_) {
    if (kv.second.count >= size_) {
      complete.emplace_back(kv.second.order, kv.first);
    } else if (!kv.second.warned && tn - kv.second.t_first > stall_warn_s_ * 1e6) {
      // stall inspector: a tensor some ranks announced long ago and others never did is reported, not fatal
      kv.second.warned = true;
      if (rank_ == 0)
        std::fprintf(stderr, "[hvd] stall: tensor '%s' announced by %d of %d ranks for over %.0f s\n", kv.first.c_str(),
                     kv.second.count, size_, stall_warn_s_);
    }
  }
  std::sort(complete.begin(), complete.end());
  {
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& c : complete) {
      auto te = table_.find(c.second);
      auto it = announced_.find(c.second);
      if (it != announced_.end()) {
        Request r = std::move(it->second);
        r.error = te->second.error;
        announced_.erase(it);
        ready.push_back(std::move(r));
      }
      // cache ids in completion order: the same assignment on every rank
      if (te->second.error.empty() && static_cast<int64_t>(cache_.size()) < cache_capacity_)
        cache_[c.second] = CacheEntry{cache_ids_++, te->second.signature};
      table_.erase(te);
    }
  }
  stop = any_stop;
}

std::vector<Batch> FusionEngine::make_batches(std::vector<Request>& ready) {
  std::vector<Batch> out;
  Batch open;
  auto close = [&] {
    if (!open.reqs.empty()) {
      out.push_back(std::move(open));
      open = Batch();
    }
  };
  for (auto& r : ready) {
    const int64_t bytes = r.tensor.numel() * static_cast<int64_t>(r.compress ? 2 : r.tensor.element_size());
    if (r.type != ReqType::ALLREDUCE || !r.error.empty()) {
      close();
      Batch b;
      b.bytes = r.tensor.numel() * r.tensor.element_size();
      b.reqs.push_back(std::move(r));
      out.push_back(std::move(b));
      continue;
    }
    if (!open.reqs.empty()) {
      const Request& h = open.reqs.front();
      const bool same = h.tensor.device() == r.tensor.device() && h.tensor.scalar_type() == r.tensor.scalar_type() &&
                        h.op == r.op && h.prescale == r.prescale && h.postscale == r.postscale &&
                        h.compress == r.compress;
      if (!same || open.bytes + bytes > fusion_bytes_.load() ||
          static_cast<int>(open.reqs.size()) >= kMaxPackSegs * 8)
        close();
    }
    open.bytes += bytes;
    open.reqs.push_back(std::move(r));
    if (open.bytes >= fusion_bytes_.load()) close();
  }
  close();
  return out;
}

void FusionEngine::finish(Batch& b, const std::string& err, bool gpu_done) {
  hipEvent_t watch = nullptr;
  hipStream_t cs = gpu_done ? engine_stream() : nullptr;
  if (gpu_done && hipEventCreateWithFlags(&watch, hipEventDisableTiming) == hipSuccess)
    (void)hipEventRecord(watch, cs);
  std::lock_guard<std::mutex> g(mu_);
  ++n_batches_;
  n_bytes_ += b.bytes;
  if (b.reqs.size() > 1) n_fused_requests_ += static_cast<int64_t>(b.reqs.size());
  for (size_t i = 0; i < b.reqs.size(); ++i) {
    Request& r = b.reqs[i];
    auto hs = handles_.find(r.handle);
    if (hs != handles_.end() && !hs->second.done) {
      HandleState& st = hs->second;
      st.done = true;
      st.error = err;
      st.output = r.output;
      if (gpu_done) {
        // each handle owns an event (the waiter destroys it)
        hipEvent_t e2 = nullptr;
        if (hipEventCreateWithFlags(&e2, hipEventDisableTiming) == hipSuccess) {
          (void)hipEventRecord(e2, cs);
          st.finished = e2;
        }
      }
    }
    if (r.ready != nullptr) {
      (void)hipEventDestroy(r.ready);
      r.ready = nullptr;
    }
  }
  if (watch) inflight_.push_back({watch, now()});
  done_cv_.notify_all();
}

void FusionEngine::execute(Batch& b) {
  const Request& r0 = b.reqs.front();
  if (!r0.error.empty()) {
    finish(b, r0.error, false);
    return;
  }
  std::string err;
  const bool gpu = r0.tensor.is_cuda();
  const double t_start = now();
  try {
    if (gpu) {
      hip_ok(hipSetDevice(r0.tensor.device().index()), "set device");
      if (r0.type == ReqType::ALLREDUCE) {
        run_allreduce_gpu(b, engine_stream(), fused_, false);
      } else if (comm_) {
        TORCH_CHECK(comm_->valid(), "RCCL communicator is not valid (aborted?)");
        run_single_gpu(b.reqs.front());
      } else {
        single_gpu_via_host(b.reqs.front());
      }
    } else {
      if (r0.type == ReqType::ALLREDUCE)
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
      trace(r.name, r0.type == ReqType::ALLREDUCE ? "ALLREDUCE" : "COLLECTIVE", t_start, t_end, b.bytes);
    }
  }
  finish(b, err, gpu && err.empty());
  if (!err.empty() && gpu) set_error(err);  // a failed RCCL call leaves the communicator unusable
}

hipStream_t FusionEngine::engine_stream() {
  if (comm_) return comm_->stream();
  if (own_stream_ == nullptr) {
    int lo = 0, hi = 0;
    hip_ok(hipDeviceGetStreamPriorityRange(&lo, &hi), "stream priority range");
    hip_ok(hipStreamCreateWithPriority(&own_stream_, hipStreamNonBlocking, hi), "engine stream");
  }
  return own_stream_;
}

// The batch's tensors are consecutive, in-place views of one buffer (a fused model's flat gradients):
// reduce the span in place -- no pack, no unpack.
static bool adjacent_inplace(const Batch& b) {
  const Request& r0 = b.reqs.front();
  const char* p = static_cast<const char*>(r0.tensor.data_ptr());
  for (const auto& r : b.reqs) {
    if (r.tensor.data_ptr() != r.output.data_ptr() || r.tensor.scalar_type() != r0.tensor.scalar_type() ||
        static_cast<const char*>(r.tensor.data_ptr()) != p)
      return false;
    p += r.tensor.numel() * r.tensor.element_size();
  }
  return true;
}

void FusionEngine::run_allreduce_gpu(Batch& b, hipStream_t s, at::Tensor& stage, bool inline_mode) {
  const int dev = b.reqs.front().tensor.device().index();
  for (auto& r : b.reqs)
    if (r.ready) hip_ok(hipStreamWaitEvent(s, r.ready, 0), "wait producer");
  Request& r0 = b.reqs.front();
  const int dt = dtype_code(r0.tensor);
  int64_t total = 0;
  for (auto& r : b.reqs) total += r.tensor.numel();
  const bool span = adjacent_inplace(b);
  // one-shot xGMI exchange for latency-bound fp32 batches (Sum / Average; pre/post scale folded in)
  if (xgmi_ && dt == 0 && (r0.op == 0 || r0.op == 1) && total * 4 <= xgmi_threshold_) {
    const float scale = static_cast<float>(r0.prescale * r0.postscale * (r0.op == 1 ? 1.0 / size_ : 1.0));
    ++n_xgmi_batches_;
    if (span) {
      ++n_inplace_batches_;
      float* p = static_cast<float*>(r0.tensor.data_ptr());
      xgmi_->allreduce(p, p, total, scale, s, r0.compress);
    } else {
      ensure_stage(stage, r0.tensor, total * 4, s, inline_mode);
      PackTable tab;
      int64_t off = 0;
      size_t i = 0;
      while (i < b.reqs.size()) {  // pack in chunks of kMaxPackSegs tensors
        tab.count = 0;
        const int64_t off0 = off;
        const size_t first = i;
        for (; i < b.reqs.size() && tab.count < kMaxPackSegs; ++i) {
          PackSeg& sg = tab.seg[tab.count++];
          sg.n = b.reqs[i].tensor.numel();
          sg.offset = off;
          sg.dtype = 0;
          sg.ptr = b.reqs[i].tensor.data_ptr();
          off += sg.n;
        }
        (void)off0;
        (void)first;
        hip_ok(fusion_pack(tab, stage.data_ptr(), 0, 1.0f, s), "pack");
      }
      float* f = static_cast<float*>(stage.data_ptr());
      xgmi_->allreduce(f, f, total, scale, s, r0.compress);
      off = 0;
      i = 0;
      while (i < b.reqs.size()) {
        tab.count = 0;
        for (; i < b.reqs.size() && tab.count < kMaxPackSegs; ++i) {
          PackSeg& sg = tab.seg[tab.count++];
          sg.n = b.reqs[i].tensor.numel();
          sg.offset = off;
          sg.dtype = 0;
          sg.ptr = b.reqs[i].output.data_ptr();
          off += sg.n;
        }
        hip_ok(fusion_unpack(tab, stage.data_ptr(), 0, 1.0f, s), "unpack");
      }
    }
    for (auto& r : b.reqs) {
      record_on(r.tensor, s, dev);
      record_on(r.output, s, dev);
    }
    return;
  }
  TORCH_CHECK(comm_ && comm_->valid(), "RCCL communicator is not valid (aborted?) and the batch (",
              total * r0.tensor.element_size(), " B) exceeds the xGMI one-shot threshold");
  ++n_rccl_batches_;
  if ((b.reqs.size() == 1 || span) && !r0.compress && r0.prescale == 1.0 && r0.postscale == 1.0) {
    if (span && b.reqs.size() > 1) ++n_inplace_batches_;
    comm_->allreduce(r0.tensor.data_ptr(), r0.output.data_ptr(), total, dt, r0.op, s);
    for (auto& r : b.reqs) {
      record_on(r.tensor, s, dev);
      record_on(r.output, s, dev);
    }
    return;
  }
  TORCH_CHECK(dt == 0 || dt == 1, "fusion engine: fused batches support fp32/bf16 tensors");
  const int wire = (r0.compress || dt == 1) ? 1 : 0;
  const int64_t need = total * (wire == 1 ? 2 : 4);
  ensure_stage(stage, r0.tensor, need, s, inline_mode);
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
    hip_ok(fusion_pack(tab, stage.data_ptr(), wire, pre, s), "pack");
  });
  comm_->allreduce(stage.data_ptr(), stage.data_ptr(), total, wire, r0.op, s);
  each_chunk([&](size_t first) {
    for (int k = 0; k < tab.count; ++k) tab.seg[k].ptr = b.reqs[first + k].output.data_ptr();
    hip_ok(fusion_unpack(tab, stage.data_ptr(), wire, post, s), "unpack");
  });
  for (auto& r : b.reqs) {
    record_on(r.tensor, s, dev);
    record_on(r.output, s, dev);
  }
}

void FusionEngine::single_gpu_via_host(Request& r) {
  // no RCCL communicator (ranks rehearsing on one GPU): broadcast / allgather through the CPU backend
  if (r.ready) hip_ok(hipEventSynchronize(r.ready), "wait producer");
  at::Tensor h = r.tensor.to(at::kCPU);
  py::gil_scoped_acquire g;
  if (r.type == ReqType::BROADCAST) {
    py_broadcast_(h, r.root);
    r.tensor.copy_(h);
  } else {
    at::Tensor out = at::empty(r.output.sizes(), h.options());
    py_allgather_(h, out);
    r.output.copy_(out);
  }
  hip_ok(hipDeviceSynchronize(), "host-staged collective");
}

void FusionEngine::allreduce_inline(const std::vector<at::Tensor>& tensors, int op, double prescale,
                                    double postscale, bool compress) {
  TORCH_CHECK(!tensors.empty(), "allreduce_inline: no tensors");
  TORCH_CHECK(tensors.front().is_cuda() && gpu_backend_, "allreduce_inline: GPU tensors and a GPU data plane");
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!error_.empty()) throw std::runtime_error("HorovodInternalError: " + error_);
    ++n_inline_calls_;
  }
  if (size_ == 1) return;
  std::vector<Request> reqs;
  for (const auto& t : tensors) {
    TORCH_CHECK(t.is_contiguous(), "allreduce_inline: contiguous tensors");
    Request r;
    r.type = ReqType::ALLREDUCE;
    r.tensor = t;
    r.output = t;
    r.op = op;
    r.prescale = prescale;
    r.postscale = postscale;
    r.compress = compress && t.scalar_type() == at::kFloat;
    reqs.push_back(std::move(r));
  }
  hipStream_t s = at::hip::getCurrentHIPStream(tensors.front().device().index()).stream();
  std::vector<Batch> batches = make_batches(reqs);
  for (auto& b : batches) run_allreduce_gpu(b, s, inline_fused_, true);
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
