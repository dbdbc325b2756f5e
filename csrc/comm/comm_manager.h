// RCCL communicator manager (SURVEY.md §2.3 B5, §5.3 re-wire, §7.4 H3/H4).
//
// One RcclComm = one ncclComm_t bound to a device and a dedicated high-priority HIP stream.  The
// unique id is created by rank 0 (get_unique_id) and distributed by the caller through the c10d store,
// so the same code path builds the initial communicator and every re-wired one after an elastic
// membership change: abort() tears a (possibly hung) communicator down without waiting for peers,
// then a fresh init() joins the new membership -- no process restart.
//
// Linked against torch's own librccl.so.1 (same soname as /opt/rocm's), so this communicator and
// torch's ProcessGroupNCCL share one RCCL instance and one HIP runtime.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <string>
#include <vector>

namespace pde {

std::string rccl_unique_id();  // ncclUniqueId as raw bytes (NCCL_UNIQUE_ID_BYTES)
int rccl_version();

class RcclComm {
 public:
  RcclComm() = default;
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  // Blocking (collective over all `size` ranks).  `blocking=false` uses a non-blocking
  // communicator config so a later abort() never waits on a dead peer.
  void init(const std::string& uid, int rank, int size, int device, bool blocking = true);
  void abort();    // ncclCommAbort: safe while collectives are hung
  // Shrink-only membership change: a communicator over `parent` minus `exclude` (parent
  // ranks).  ncclCommShrink when the loaded RCCL exports it (survivors only; `abort_parent` first aborts
  // in-flight work) -> returns 1; else ncclCommSplit (every parent rank must call, leavers get no
  // communicator) -> returns 2.  The parent stays valid (destroy/abort it separately).
  int shrink_from(RcclComm& parent, const std::vector<int>& exclude, bool abort_parent);
  static bool shrink_supported();
  // Planned membership change with every parent rank alive (elastic scale-down): ncclCommSplit over the
  // parent, collective over ALL parent ranks.  color < 0 = leaving (NCCL_SPLIT_NOCOLOR: no communicator,
  // returns false); `key` orders the ranks of the child.  No unique-id exchange, topology reused.
  // bounded: a split that does not complete within timeout_s (a member died) is aborted and throws
  bool split_from(RcclComm& parent, int color, int key, double timeout_s = 300.0);
  void destroy();  // ncclCommDestroy after a clean finish
  bool valid() const { return comm_ != nullptr; }
  int rank() const { return rank_; }
  int size() const { return size_; }
  int device() const { return device_; }
  hipStream_t stream() const { return stream_; }
  ncclComm_t raw() const { return comm_; }
  // returns ncclSuccess / ncclInProgress / an async error
  int async_error() const;
  // ncclCommCount: the number of ranks RCCL itself reports for this communicator
  int nranks() const;

  // dtype codes: 0 f32, 1 bf16, 2 f16, 3 f64, 4 i32, 5 i64, 6 u8 ; op codes: 0 sum, 1 avg, 2 min, 3 max, 4 prod
  void allreduce(const void* send, void* recv, size_t count, int dtype, int op, hipStream_t s);
  void broadcast(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t s);
  void allgather(const void* send, void* recv, size_t count_per_rank, int dtype, hipStream_t s);
  void reduce_scatter(const void* send, void* recv, size_t count_per_rank, int dtype, int op, hipStream_t s);
  void alltoall(const void* send, void* recv, size_t count_per_rank, int dtype, hipStream_t s);
  void send(const void* buf, size_t count, int dtype, int peer, hipStream_t s);
  void recv(void* buf, size_t count, int dtype, int peer, hipStream_t s);
  void group_start();
  void group_end();

 private:
  void check(ncclResult_t r, const char* what) const;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  int rank_ = -1, size_ = 0, device_ = -1;
};

size_t dtype_size(int dtype);

}  // namespace pde
