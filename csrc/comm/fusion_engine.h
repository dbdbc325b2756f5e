// Horovod-style tensor-fusion engine (the reference's Horovod core is C++:
// background thread, ready queue, fusion buffer, timeline).  MI355X-native design:
//
//  * Requests (allreduce / broadcast / allgather on named tensors) are enqueued by the framework thread
//    and return a handle immediately.  GPU requests record a HIP event on the producer's stream, so the
//    engine never blocks the host on compute.
//  * Allreduce requests are fused into batches of up to `fusion_bytes` (default sized for xGMI, see
//    parallel/xgmi.py) with a DETERMINISTIC cut rule (cumulative bytes / op change / explicit flush at
//    synchronize) instead of Horovod's coordinator negotiation: every rank issues the same request
//    sequence (true for DistributedOptimizer's backward hooks), so every rank cuts identical batches
//    without a control-plane round trip per cycle.
//  * A background thread executes closed batches in order.  GPU backend: wait producer events on the
//    engine's high-priority comm stream -> ONE pack kernel (pre-scale, optional fp32->bf16 wire
//    compression) -> RCCL all-reduce (ncclAvg for Average) -> ONE unpack kernel (post-scale) ->
//    completion event.  Single-tensor batches without scaling/compression reduce in place (no copies).
//    CPU backend: the same batching, the collective delegated to a Python callable (gloo process group).
//  * synchronize(handle) makes the caller's stream wait on the completion event (GPU) or blocks until
//    done (CPU); failures surface as exceptions (-> hvd.HorovodInternalError in Python).
//  * Optional Chrome-trace timeline (HOROVOD_TIMELINE-compatible env var handled in Python).
#pragma once

#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "comm_manager.h"

namespace pde {

enum class ReqType { ALLREDUCE, BROADCAST, ALLGATHER };

struct Request {
  int64_t handle = 0;
  ReqType type = ReqType::ALLREDUCE;
  std::string name;
  at::Tensor tensor;   // input
  at::Tensor output;   // output (== tensor for in-place)
  int op = 1;          // 0 sum, 1 avg, 2 min, 3 max, 4 prod
  int root = 0;
  double prescale = 1.0, postscale = 1.0;
  bool compress = false;  // fp32 -> bf16 on the wire
  hipEvent_t ready = nullptr;
  double t_enqueue = 0.0;
};

struct Batch {
  std::vector<Request> reqs;
  int64_t bytes = 0;
};

struct HandleState {
  bool done = false;
  std::string error;
  at::Tensor output;
  hipEvent_t finished = nullptr;  // GPU: recorded on the comm stream after the batch
};

class FusionEngine {
 public:
  FusionEngine(int rank, int size, int64_t fusion_bytes, const std::string& timeline_path);
  ~FusionEngine();

  void set_rccl(std::shared_ptr<RcclComm> comm);
  void set_py_backend(py::object allreduce_fn, py::object broadcast_fn, py::object allgather_fn);

  int64_t allreduce(at::Tensor t, at::Tensor out, const std::string& name, int op, double prescale,
                    double postscale, bool compress);
  int64_t broadcast(at::Tensor t, int root, const std::string& name);
  int64_t allgather(at::Tensor t, const std::string& name);
  void flush();
  bool poll(int64_t h);
  at::Tensor wait(int64_t h);
  void shutdown();
  py::dict stats();
  int64_t fusion_bytes() const { return fusion_bytes_; }
  void set_fusion_bytes(int64_t b) { fusion_bytes_ = b; }

 private:
  void loop();
  void execute(Batch& b);
  void run_allreduce_gpu(Batch& b);
  void run_allreduce_cpu(Batch& b);
  void run_single_gpu(Request& r);
  void run_single_cpu(Request& r);
  void finish(Batch& b, const std::string& err, bool gpu_done);
  void close_open_locked();
  double now() const;
  void trace(const std::string& name, const std::string& phase, double t0, double t1, int64_t bytes);

  int rank_, size_;
  std::atomic<int64_t> fusion_bytes_;
  std::shared_ptr<RcclComm> comm_;
  py::object py_allreduce_, py_broadcast_, py_allgather_;
  bool gpu_backend_ = false;

  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  Batch open_;
  std::deque<Batch> closed_;
  std::map<int64_t, HandleState> handles_;
  int64_t next_handle_ = 1;
  bool stop_ = false;
  std::thread worker_;
  at::Tensor fused_;  // reusable fusion buffer (device or host)

  // stats
  int64_t n_requests_ = 0, n_batches_ = 0, n_bytes_ = 0, n_fused_requests_ = 0;

  std::mutex trace_mu_;
  std::ofstream trace_;
  bool trace_first_ = true;
  std::chrono::steady_clock::time_point t0_;
};

}  // namespace pde
