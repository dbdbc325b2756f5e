// RCCL communicator manager: see comm_manager.h.
#include "comm_manager.h"

#include <dlfcn.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace pde {

namespace {

ncclDataType_t to_nccl(int dtype) {
  switch (dtype) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclFloat64;
    case 4: return ncclInt32;
    case 5: return ncclInt64;
    case 6: return ncclUint8;
    default: throw std::invalid_argument("pde rccl: unsupported dtype code " + std::to_string(dtype));
  }
}

ncclRedOp_t to_nccl_op(int op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclAvg;
    case 2: return ncclMin;
    case 3: return ncclMax;
    case 4: return ncclProd;
    default: throw std::invalid_argument("pde rccl: unsupported reduce op " + std::to_string(op));
  }
}

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("pde rccl: ") + what + ": " + hipGetErrorString(e));
}

}  // namespace

size_t dtype_size(int dtype) {
  switch (dtype) {
    case 0: case 4: return 4;
    case 1: case 2: return 2;
    case 3: case 5: return 8;
    case 6: return 1;
    default: return 0;
  }
}

std::string rccl_unique_id() {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) throw std::runtime_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

int rccl_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

RcclComm::~RcclComm() {
  // Never block in a destructor: a communicator that was not destroyed cleanly is aborted.
  if (comm_ != nullptr) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
  // The stream is deliberately NOT destroyed: tensors used by collectives were recordStream()-ed on it,
  // and torch's caching allocator records events on every such stream when those tensors are freed --
  // possibly long after this communicator is gone (elastic re-init).  A stream per communicator
  // lifetime is a negligible leak; a destroyed one would be a use-after-free inside the allocator.
}

void RcclComm::check(ncclResult_t r, const char* what) const {
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string("pde rccl ") + what + " (rank " + std::to_string(rank_) + "/" +
                             std::to_string(size_) + "): " + ncclGetErrorString(r));
}

void RcclComm::init(const std::string& uid, int rank, int size, int device, bool blocking) {
  if (uid.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("pde rccl: bad unique id size");
  if (comm_ != nullptr) abort();
  hip_check(hipSetDevice(device), "hipSetDevice");
  if (stream_ == nullptr) {
    int lo = 0, hi = 0;
    hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "stream priority range");
    hip_check(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "comm stream");
  }
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = blocking ? 1 : 0;
  ncclResult_t r = ncclCommInitRankConfig(&comm_, size, id, rank, &cfg);
  rank_ = rank;
  size_ = size;
  device_ = device;
  if (!blocking) {
    // wait for the non-blocking init to finish (bounded: 300 s)
    auto t0 = std::chrono::steady_clock::now();
    ncclResult_t st = ncclInProgress;
    while (r == ncclInProgress || st == ncclInProgress) {
      ncclCommGetAsyncError(comm_, &st);
      if (st != ncclInProgress) break;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(300)) {
        ncclCommAbort(comm_);
        comm_ = nullptr;
        throw std::runtime_error("pde rccl: communicator init timed out");
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
      r = ncclSuccess;
    }
    check(st, "init(async)");
  } else {
    check(r, "ncclCommInitRankConfig");
  }
}

// ncclCommShrink appeared in RCCL 2.27; torch's bundled librccl (2.26.x) does not export it, and this module
// binds to the librccl torch already loaded, so the symbol is looked up at run time.
using ShrinkFn = ncclResult_t (*)(ncclComm_t, int*, int, ncclComm_t*, ncclConfig_t*, int);
static ShrinkFn shrink_fn() {
  static ShrinkFn fn = reinterpret_cast<ShrinkFn>(dlsym(RTLD_DEFAULT, "ncclCommShrink"));
  return fn;
}

bool RcclComm::shrink_supported() { return shrink_fn() != nullptr; }

int RcclComm::shrink_from(RcclComm& parent, const std::vector<int>& exclude, bool abort_parent) {
  if (parent.comm_ == nullptr) throw std::runtime_error("pde rccl: shrink from an invalid communicator");
  if (comm_ != nullptr) abort();
  hip_check(hipSetDevice(parent.device_), "hipSetDevice");
  if (stream_ == nullptr) {
    int lo = 0, hi = 0;
    hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "stream priority range");
    hip_check(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "comm stream");
  }
  std::vector<int> ex(exclude);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  ncclComm_t out = nullptr;
  if (ShrinkFn fn = shrink_fn()) {
    // survivors only: the excluded (dead) ranks do not take part; ABORT first tears down in-flight work
    check(fn(parent.comm_, ex.data(), static_cast<int>(ex.size()), &out, &cfg,
             abort_parent ? NCCL_SHRINK_ABORT : NCCL_SHRINK_DEFAULT), "ncclCommShrink");
    comm_ = out;
    device_ = parent.device_;
    check(ncclCommUserRank(comm_, &rank_), "ncclCommUserRank");
    check(ncclCommCount(comm_, &size_), "ncclCommCount");
    return 1;
  }
  // graceful shrink without ncclCommShrink (every parent rank alive and calling): the leaving ranks pass
  // NCCL_SPLIT_NOCOLOR -- a split keeps the parent's topology and skips the unique-id exchange
  bool leaving = false;
  for (int r : ex) leaving = leaving || r == parent.rank_;
  check(ncclCommSplit(parent.comm_, leaving ? NCCL_SPLIT_NOCOLOR : 0, parent.rank_, &out, &cfg), "ncclCommSplit");
  comm_ = out;
  device_ = parent.device_;
  if (comm_ != nullptr) {
    check(ncclCommUserRank(comm_, &rank_), "ncclCommUserRank");
    check(ncclCommCount(comm_, &size_), "ncclCommCount");
  }
  return 2;
}

bool RcclComm::split_from(RcclComm& parent, int color, int key, double timeout_s) {
  if (parent.comm_ == nullptr) throw std::runtime_error("pde rccl: split from an invalid communicator");
  if (comm_ != nullptr) abort();
  hip_check(hipSetDevice(parent.device_), "hipSetDevice");
  if (stream_ == nullptr) {
    int lo = 0, hi = 0;
    hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "stream priority range");
    hip_check(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "comm stream");
  }
  // non-blocking: a member that dies between the control-plane agreement and the split would otherwise
  // hang every survivor inside ncclCommSplit; here the split is polled against the round's timeout and
  // aborted on expiry (the caller turns the exception into a peer failure and re-wires)
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t out = nullptr;
  ncclResult_t r = ncclCommSplit(parent.comm_, color < 0 ? NCCL_SPLIT_NOCOLOR : color, key, &out, &cfg);
  check(r, "ncclCommSplit");
  if (out != nullptr) {
    const auto t0 = std::chrono::steady_clock::now();
    ncclResult_t st = ncclInProgress;
    for (;;) {
      ncclCommGetAsyncError(out, &st);
      if (st != ncclInProgress) break;
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
        ncclCommAbort(out);
        throw std::runtime_error("pde rccl: ncclCommSplit did not complete within " + std::to_string(timeout_s) +
                                 " s (a member is gone)");
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (st != ncclSuccess) {
      ncclCommAbort(out);
      check(st, "ncclCommSplit(async)");
    }
  }
  comm_ = out;
  device_ = parent.device_;
  if (comm_ == nullptr) return false;
  check(ncclCommUserRank(comm_, &rank_), "ncclCommUserRank");
  check(ncclCommCount(comm_, &size_), "ncclCommCount");
  return true;
}

void RcclComm::abort() {
  if (comm_ != nullptr) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

void RcclComm::destroy() {
  if (comm_ != nullptr) {
    ncclCommFinalize(comm_);
    ncclCommDestroy(comm_);
    comm_ = nullptr;
  }
}

int RcclComm::async_error() const {
  if (comm_ == nullptr) return ncclInvalidUsage;
  ncclResult_t st = ncclSuccess;
  ncclCommGetAsyncError(comm_, &st);
  return static_cast<int>(st);
}

int RcclComm::nranks() const {
  if (comm_ == nullptr) return 0;
  int n = 0;
  check(ncclCommCount(comm_, &n), "ncclCommCount");
  return n;
}

void RcclComm::allreduce(const void* send, void* recv, size_t count, int dtype, int op, hipStream_t s) {
  check(ncclAllReduce(send, recv, count, to_nccl(dtype), to_nccl_op(op), comm_, s ? s : stream_), "allreduce");
}
void RcclComm::broadcast(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t s) {
  check(ncclBroadcast(send, recv, count, to_nccl(dtype), root, comm_, s ? s : stream_), "broadcast");
}
void RcclComm::allgather(const void* send, void* recv, size_t count, int dtype, hipStream_t s) {
  check(ncclAllGather(send, recv, count, to_nccl(dtype), comm_, s ? s : stream_), "allgather");
}
void RcclComm::reduce_scatter(const void* send, void* recv, size_t count, int dtype, int op, hipStream_t s) {
  check(ncclReduceScatter(send, recv, count, to_nccl(dtype), to_nccl_op(op), comm_, s ? s : stream_),
        "reduce_scatter");
}
void RcclComm::alltoall(const void* send, void* recv, size_t count, int dtype, hipStream_t s) {
  check(ncclAllToAll(send, recv, count, to_nccl(dtype), comm_, s ? s : stream_), "alltoall");
}
void RcclComm::send(const void* buf, size_t count, int dtype, int peer, hipStream_t s) {
  check(ncclSend(buf, count, to_nccl(dtype), peer, comm_, s ? s : stream_), "send");
}
void RcclComm::recv(void* buf, size_t count, int dtype, int peer, hipStream_t s) {
  check(ncclRecv(buf, count, to_nccl(dtype), peer, comm_, s ? s : stream_), "recv");
}
void RcclComm::group_start() { check(ncclGroupStart(), "group_start"); }
void RcclComm::group_end() { check(ncclGroupEnd(), "group_end"); }

}  // namespace pde
