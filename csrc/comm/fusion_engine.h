// Horovod-style tensor-fusion engine (the reference's Horovod core is C++:
// background thread, coordinator negotiation, fusion buffer, timeline).  MI355X-native design:
//
//  * Requests (allreduce / broadcast / allgather on NAMED tensors) are enqueued by the framework thread
//    and return a handle immediately.  GPU requests record a HIP event on the producer's stream, so the
//    engine never blocks the host on compute.  A name may be outstanding only once per rank.
//  * Negotiation (Horovod's controller): the background thread runs a control CYCLE every
//    `cycle_ms` while anything is outstanding.  Each cycle every rank all-gathers, over a CPU (gloo)
//    control process group, the names + signatures (type, dtype, element count, op, root, scaling) of the
//    requests it enqueued since the last cycle.  Every rank then applies the SAME deterministic rule to
//    the same gathered table (a decentralised coordinator): a name is ready once all ranks announced it;
//    ready names are executed in first-announcement order (rank-major), so ranks whose hooks fire in
//    different orders still cut identical fusion batches.  A signature mismatch fails that request on
//    every rank ("mismatched ...") instead of mis-reducing.  A shutdown request from any rank ends the
//    engine on all ranks at the end of that cycle.  World size 1 skips the collective.
//  * Response cache (Horovod's): a (name, signature) that completed negotiation once gets a cache id, the
//    same on every rank (ids are assigned in the deterministic completion order).  From then on a cycle is
//    ONE small MIN all-reduce of an int32 vector [one 0/1 word per cache id, -stop, -has_uncached]: the
//    per-id minimum is the AND of "announced by this rank" (ready everywhere), the two negated flags are
//    MAXes.  The name/signature all-gathers run only in cycles where some rank announced an uncached
//    request (first step, a new tensor, a changed shape); a cached name that reappears there is evicted on
//    every rank and pending cached requests for it are re-announced through the string path, so a
//    signature change is still reported as a mismatch.  HOROVOD_CACHE_CAPACITY=0 turns the cache off.
//  * Data plane on GPUs: fused batches up to `xgmi_threshold` bytes (fp32, Sum/Average) take the one-shot
//    xGMI peer all-reduce (every rank reads all peers' staged batch over its direct links: one kernel, no
//    ring hops) when an XgmiAllreduce is attached; larger ones RCCL.  A batch whose tensors are adjacent views
//    of one buffer (the flat gradient buffer of a fused model) is reduced in place, without pack / unpack.
//    Broadcast / allgather of GPU tensors without an RCCL communicator (several ranks rehearsing on one GPU)
//    stage through the host over the CPU backend.
//  * Graph mode (`allreduce_inline`): once the response cache holds a fixed tensor set, the optimizer may
//    skip the engine thread and enqueue the SAME batches on the caller's stream -- stream-ordered, no host
//    wait, hipGraph-capturable.  Every rank must call it with the same tensors in the same order (SPMD).
//  * Ready allreduces are fused into batches of up to `fusion_bytes` (same dtype/op/scaling/compression).
//    GPU backend: wait producer events on the engine's high-priority comm stream -> ONE pack kernel
//    (pre-scale, optional fp32->bf16 wire compression) -> RCCL all-reduce (ncclAvg for Average) -> ONE
//    unpack kernel (post-scale) -> completion event.  Single-tensor batches without scaling or
//    compression reduce in place.  CPU backend: the collective is delegated to a Python callable (gloo).
//  * Failure detection: a control-plane error (dead peer: gloo connection reset / timeout) or an RCCL
//    failure puts the engine in an ERROR state: every outstanding and later request fails with an error
//    that Python raises as hvd.HorovodInternalError.  In-flight GPU batches are watched: an RCCL async
//    error or a batch older than `timeout_s` aborts the communicator (which releases hung kernels).
//    `blocking_wait` makes synchronize() poll the batch's completion on the host (elastic mode), so a
//    failure surfaces from the very synchronize() that waits on it.
//  * Optional Chrome-trace timeline (HOROVOD_TIMELINE), with NEGOTIATE / QUEUE / ALLREDUCE phases.
#pragma once

#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>

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
#include "xgmi_allreduce.h"

namespace pde {

enum class ReqType { ALLREDUCE = 0, BROADCAST = 1, ALLGATHER = 2 };

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
  std::string error;      // set when negotiation rejected it
  std::string signature() const;
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

// one in-flight GPU batch watched for completion / failure
struct Inflight {
  hipEvent_t done = nullptr;
  double t_start = 0.0;
};

// negotiation table entry (identical on every rank)
struct NegEntry {
  std::string signature;
  int count = 0;
  int64_t order = 0;
  std::string error;
  double t_first = 0;   // when the first rank announced it (stall inspector)
  bool warned = false;  // stall warning printed once
};

class FusionEngine {
 public:
  FusionEngine(int rank, int size, int64_t fusion_bytes, const std::string& timeline_path, double cycle_ms);
  ~FusionEngine();

  void set_rccl(std::shared_ptr<RcclComm> comm);
  void set_xgmi(std::shared_ptr<XgmiAllreduce> xgmi, int64_t threshold_bytes);
  // graph mode: all-reduce `tensors` (in place) as the engine would batch them, on the caller's CURRENT
  // stream, without negotiation -- the caller guarantees every rank makes the same call (cached tensor set)
  void allreduce_inline(const std::vector<at::Tensor>& tensors, int op, double prescale, double postscale,
                        bool compress);
  // graph mode on: (1) the idle loop parks on its condition variable instead of cycling the lockstep bit
  // all-reduce (the captured step bypasses the engine; every rank wakes when it enqueues again -- SPMD, as
  // allreduce_inline already requires); (2) `tensors` size the inline staging buffer ONCE, so a replayed
  // graph never points at storage a later regrow frees
  void set_graph_mode(bool on, const std::vector<at::Tensor>& tensors);
  // graph mode's health check (replays bypass the engine thread): a timed-out xGMI exchange puts the engine
  // into the error state and raises HorovodInternalError; a plain host read, no device sync
  void check_xgmi();
  bool cached(const std::string& name) {
    std::lock_guard<std::mutex> g(mu_);
    return cache_.count(name) > 0;
  }
  void set_py_backend(py::object allreduce_fn, py::object broadcast_fn, py::object allgather_fn);
  void set_control(c10::intrusive_ptr<c10d::ProcessGroup> pg);
  void set_timeout(double seconds) { timeout_s_ = seconds; }
  void set_blocking_wait(bool b) { blocking_wait_ = b; }

  int64_t allreduce(at::Tensor t, at::Tensor out, const std::string& name, int op, double prescale,
                    double postscale, bool compress);
  int64_t broadcast(at::Tensor t, int root, const std::string& name);
  int64_t allgather(at::Tensor t, const std::string& name);
  void flush();
  bool poll(int64_t h);
  at::Tensor wait(int64_t h);
  void shutdown(bool abort);
  py::dict stats();
  int64_t fusion_bytes() const { return fusion_bytes_; }
  void set_fusion_bytes(int64_t b) { fusion_bytes_ = b; }
  std::string error() {
    std::lock_guard<std::mutex> g(mu_);
    return error_;
  }
  // test hook: put the engine into the error state as a failed collective would
  void inject_error(const std::string& why);

 private:
  int64_t enqueue(Request&& r);
  void loop();
  void negotiate(std::vector<Request>& announce, std::vector<Request>& ready, bool& stop);
  void execute(Batch& b);
  // stage: the fusion buffer to use (the engine thread's fused_, or graph mode's inline_fused_, which may
  // not grow while the stream is capturing)
  void run_allreduce_gpu(Batch& b, hipStream_t s, at::Tensor& stage, bool inline_mode);
  void ensure_stage(at::Tensor& stage, const at::Tensor& like, int64_t bytes, hipStream_t s, bool inline_mode);
  void single_gpu_via_host(Request& r);
  hipStream_t engine_stream();  // the RCCL communicator's stream, else one of the engine's own
  void run_allreduce_cpu(Batch& b);
  void run_single_gpu(Request& r);
  void run_single_cpu(Request& r);
  void finish(Batch& b, const std::string& err, bool gpu_done);
  void fail_all_locked(const std::string& err);
  void set_error(const std::string& err);
  void check_inflight();
  std::string xgmi_failure();  // non-empty once the attached xGMI exchange reported a timed-out wait
  std::vector<Batch> make_batches(std::vector<Request>& ready);
  double now() const;
  void trace(const std::string& name, const std::string& phase, double t0, double t1, int64_t bytes);

  int rank_, size_;
  std::atomic<int64_t> fusion_bytes_;
  double cycle_ms_;
  double idle_ms_ = 2.0;         // lockstep back-off between idle cycles (PDE_HVD_IDLE_MS)
  double stall_warn_s_ = 60.0;   // stall inspector threshold (HOROVOD_STALL_CHECK_TIME_SECONDS)
  std::shared_ptr<RcclComm> comm_;
  std::shared_ptr<XgmiAllreduce> xgmi_;
  int64_t xgmi_threshold_ = 0;
  hipStream_t own_stream_ = nullptr;
  c10::intrusive_ptr<c10d::ProcessGroup> control_;
  py::object py_allreduce_, py_broadcast_, py_allgather_;
  bool gpu_backend_ = false;
  double timeout_s_ = 300.0;
  bool blocking_wait_ = false;

  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<Request> unannounced_;            // enqueued since the last cycle
  std::map<std::string, Request> announced_;   // announced by this rank, not yet globally ready
  std::map<std::string, NegEntry> table_;      // negotiation state (same on every rank)
  int64_t order_seq_ = 0;
  // response cache: name -> (id, signature); ids are never reused (an evicted id's word stays 0)
  struct CacheEntry {
    int id;
    std::string signature;
  };
  std::map<std::string, CacheEntry> cache_;
  std::map<int, Request> cached_pending_;  // announced through the cache, not yet ready everywhere
  int cache_ids_ = 0;
  int64_t cache_capacity_ = 1 << 16;
  std::map<int64_t, HandleState> handles_;
  int64_t next_handle_ = 1;
  bool stop_requested_ = false;
  bool stopped_ = false;
  std::string error_;
  std::thread worker_;
  at::Tensor fused_;  // reusable fusion buffer (device or host), engine thread only
  at::Tensor inline_fused_;  // graph mode's staging buffer (caller's stream), sized by set_graph_mode
  // earlier, smaller staging buffers: a graph captured against one keeps pointing at it, so it lives as long as the
  // engine (never returned to the allocator while a replay could still write it)
  std::vector<at::Tensor> retired_inline_;
  bool graph_mode_ = false;
  std::vector<Inflight> inflight_;

  // stats
  int64_t n_requests_ = 0, n_batches_ = 0, n_bytes_ = 0, n_fused_requests_ = 0, n_cycles_ = 0;
  int64_t n_xgmi_batches_ = 0, n_rccl_batches_ = 0, n_inline_calls_ = 0, n_inplace_batches_ = 0;
  int64_t n_string_gathers_ = 0, n_bit_allreduces_ = 0, n_cache_hits_ = 0, n_cache_evictions_ = 0;

  std::mutex trace_mu_;
  std::ofstream trace_;
  bool trace_first_ = true;
  std::chrono::steady_clock::time_point t0_;
};

}  // namespace pde
