// Stage-to-stage P2P channel over xGMI: see p2p_ring.h for the protocol.
#include <hip/hip_runtime.h>

#include <chrono>
#include <thread>
#include <cstdlib>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>

#include "p2p_ring.h"

namespace pde {

namespace {

constexpr int kThreads = 256;
constexpr int kCtrlBytes = 4096;
constexpr int64_t kWgBytes = 32 << 10;  // bytes per workgroup before the grid widens (<= kMaxWg)
// device-local state words
constexpr int kSendSeq = 0, kRecvSeq = 1, kSendDone = 2, kRecvDone = 3, kError = 4, kStateWords = 8;

struct RingArgs {
  char* local;   // my exported allocation: ctrl | flags | slots
  char* peer;    // the peer's, mapped
  uint32_t* state;
  int64_t flag_off, slot_off, slot_bytes;
  uint64_t timeout_ticks;
};

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("p2p ring: ") + what + ": " + hipGetErrorString(e));
}

// Workgroups per message, capped at PDE_P2P_MAX_WG (default 32, <= kMaxWg; the same on both sides): a send
// that waits for credit keeps its whole grid spinning on a side stream, so the cap is also what the one-launch
// BatchNorm must leave free (P2PRing::max_wg, bn_reserve_headroom).  32 workgroups already saturate one link.
int ring_max_wg() {
  static const int w = [] {
    const char* e = std::getenv("PDE_P2P_MAX_WG");
    const int v = e ? std::atoi(e) : 32;
    return std::max(1, std::min(P2PRing::kMaxWg, v));
  }();
  return w;
}
int grid_of(int64_t bytes) {
  return static_cast<int>(std::min<int64_t>(ring_max_wg(), std::max<int64_t>(1, (bytes + kWgBytes - 1) / kWgBytes)));
}
int64_t chunk_of(int64_t bytes, int g) { return ((bytes + g - 1) / g + 15) / 16 * 16; }

// Bounded wait until *p reaches `target` (wrapping compare); false (and the error word set) on timeout.
__device__ __forceinline__ bool wait_at_least(const uint32_t* p, uint32_t target, const RingArgs& a) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (static_cast<int32_t>(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target) < 0) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
      __hip_atomic_store(a.state + kError, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

// Copy [lo, hi) bytes: 16-B vectors with 4 loads in flight per lane, then the byte tail.
__device__ __forceinline__ void copy_range(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int64_t lo,
                                           int64_t hi) {
  const int tid = threadIdx.x;
  const int64_t vend = lo + (hi - lo) / 16 * 16;
  int64_t i = lo + 16 * tid;
  for (; i + 3 * 16 * kThreads < vend; i += 4 * 16 * kThreads) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint4*>(src + i + u * 16 * kThreads);
#pragma unroll
    for (int u = 0; u < 4; ++u) *reinterpret_cast<uint4*>(dst + i + u * 16 * kThreads) = v[u];
  }
  for (; i < vend; i += 16 * kThreads) *reinterpret_cast<uint4*>(dst + i) = *reinterpret_cast<const uint4*>(src + i);
  for (int64_t j = vend + tid; j < hi; j += kThreads) dst[j] = src[j];
}

// The call's last finishing workgroup returns true (block-collective; every wave's memory ops issued
// before it are complete: the caller drained them).
__device__ __forceinline__ bool last_to_finish(uint32_t* done, int* s_last) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t n = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_last = n == gridDim.x - 1;
    if (*s_last) __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return *s_last != 0;
}

__global__ __launch_bounds__(kThreads) void k_ring_send(const uint8_t* __restrict__ src, int64_t bytes, int64_t chunk,
                                                        RingArgs a) {
  __shared__ uint32_t s_seq;
  __shared__ int s_ok, s_last;
  const int wg = blockIdx.x;
  if (threadIdx.x == 0) {
    const uint32_t seq = __hip_atomic_load(a.state + kSendSeq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_seq = seq;
    // credit: message seq - kSlots (same slot) must have been consumed by the peer (its ACK in my ctrl word)
    s_ok = seq < static_cast<uint32_t>(P2PRing::kSlots)
               ? 1
               : wait_at_least(reinterpret_cast<const uint32_t*>(a.local), seq + 1u - P2PRing::kSlots, a);
  }
  __syncthreads();
  const uint32_t seq = s_seq;
  const int slot = static_cast<int>(seq % P2PRing::kSlots);
  const int64_t lo = static_cast<int64_t>(wg) * chunk;
  const int64_t hi = lo + chunk < bytes ? lo + chunk : bytes;
  if (s_ok && lo < hi) copy_range(src, reinterpret_cast<uint8_t*>(a.peer + a.slot_off + slot * a.slot_bytes), lo, hi);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's stores into the peer's slot drained
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t* flag = reinterpret_cast<uint32_t*>(a.peer + a.flag_off) + slot * P2PRing::kMaxWg + wg;
    __hip_atomic_store(flag, seq + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (last_to_finish(a.state + kSendDone, &s_last) && threadIdx.x == 0)
    __hip_atomic_store(a.state + kSendSeq, seq + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kThreads) void k_ring_recv(uint8_t* __restrict__ dst, int64_t bytes, int64_t chunk,
                                                        RingArgs a) {
  __shared__ uint32_t s_seq;
  __shared__ int s_ok, s_last;
  const int wg = blockIdx.x;
  if (threadIdx.x == 0) {
    const uint32_t seq = __hip_atomic_load(a.state + kRecvSeq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_seq = seq;
    const int slot = static_cast<int>(seq % P2PRing::kSlots);
    const uint32_t* flag = reinterpret_cast<const uint32_t*>(a.local + a.flag_off) + slot * P2PRing::kMaxWg + wg;
    s_ok = wait_at_least(flag, seq + 1u, a);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const uint32_t seq = s_seq;
  const int slot = static_cast<int>(seq % P2PRing::kSlots);
  const int64_t lo = static_cast<int64_t>(wg) * chunk;
  const int64_t hi = lo + chunk < bytes ? lo + chunk : bytes;
  if (s_ok && lo < hi) copy_range(reinterpret_cast<const uint8_t*>(a.local + a.slot_off + slot * a.slot_bytes), dst, lo, hi);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's slot reads have completed
  if (last_to_finish(a.state + kRecvDone, &s_last) && threadIdx.x == 0) {
    __hip_atomic_store(a.state + kRecvSeq, seq + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the slot is free again: ACK in the sender's ctrl word
    __hip_atomic_store(reinterpret_cast<uint32_t*>(a.peer), seq + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace

P2PRing::P2PRing(int device, int64_t slot_bytes, double timeout_s) : device_(device) {
  if (slot_bytes < 4096) throw std::invalid_argument("p2p ring: slot_bytes >= 4096");
  slot_bytes_ = (slot_bytes + 4095) / 4096 * 4096;
  flag_bytes_ = ((static_cast<int64_t>(kSlots) * kMaxWg * 4 + 4095) / 4096) * 4096;
  timeout_ticks_ = static_cast<uint64_t>(timeout_s * 1e8);  // s_memrealtime: 100 MHz
  hip_check(hipSetDevice(device), "hipSetDevice");
  const size_t total = static_cast<size_t>(kCtrlBytes + flag_bytes_ + kSlots * slot_bytes_);
  void* p = nullptr;
  hip_check(hipExtMallocWithFlags(&p, total, hipDeviceMallocUncached), "hipExtMallocWithFlags(uncached)");
  local_ = static_cast<char*>(p);
  hip_check(hipMemset(local_, 0, kCtrlBytes + flag_bytes_), "zero ctrl/flags");
  void* st = nullptr;
  hip_check(hipMalloc(&st, kStateWords * 4), "hipMalloc state");
  state_ = static_cast<uint32_t*>(st);
  hip_check(hipMemset(state_, 0, kStateWords * 4), "zero state");
  hip_check(hipDeviceSynchronize(), "sync after init");  // zeroed before the peer can map it
}

P2PRing::~P2PRing() {
  try {
    close();
  } catch (...) {
  }
}

std::string P2PRing::ipc_handle() const {
  hipIpcMemHandle_t h;
  // (a few spaced attempts before giving up -- a host call, no GPU work; the "invalid argument" seen with several
  // processes sharing one card right after a close did not clear this way: see tests/test_xgmi_twoshot_gpu.py)
  hipError_t e = hipErrorUnknown;
  for (int attempt = 0; attempt < 4; ++attempt) {
    e = hipIpcGetMemHandle(&h, local_);
    if (e == hipSuccess) break;
    (void)hipGetLastError();
    std::this_thread::sleep_for(std::chrono::milliseconds(50 * (attempt + 1)));
  }
  hip_check(e, "hipIpcGetMemHandle");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void P2PRing::open(const std::string& peer_handle) {
  if (peer_handle.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("p2p ring: bad handle");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hipIpcMemHandle_t h;
  std::memcpy(&h, peer_handle.data(), sizeof(h));
  void* p = nullptr;
  hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  peer_ = static_cast<char*>(p);
  peer_ipc_ = true;
  opened_ = true;
}

void P2PRing::open_local(P2PRing& peer) {
  if (peer.device_ != device_ || peer.local_ == nullptr) throw std::invalid_argument("p2p ring: local peer");
  peer_ = peer.local_;
  peer_ipc_ = false;
  opened_ = true;
}

int P2PRing::max_wg() { return ring_max_wg(); }

static RingArgs args_of(char* local, char* peer, uint32_t* state, int64_t flag_bytes, int64_t slot_bytes,
                        uint64_t timeout) {
  RingArgs a{};
  a.local = local;
  a.peer = peer;
  a.state = state;
  a.flag_off = kCtrlBytes;
  a.slot_off = kCtrlBytes + flag_bytes;
  a.slot_bytes = slot_bytes;
  a.timeout_ticks = timeout;
  return a;
}

// Messages larger than a slot go as consecutive slot-sized pieces (the same cut on both sides).
void P2PRing::send(const void* src, int64_t bytes, hipStream_t s) {
  if (!opened_) throw std::runtime_error("p2p ring: peer not opened");
  if (reinterpret_cast<uintptr_t>(src) & 15) throw std::invalid_argument("p2p ring: 16-B aligned source");
  const RingArgs a = args_of(local_, peer_, state_, flag_bytes_, slot_bytes_, timeout_ticks_);
  for (int64_t off = 0; off < bytes; off += slot_bytes_) {
    const int64_t n = std::min(slot_bytes_, bytes - off);
    const int g = grid_of(n);
    hipLaunchKernelGGL(k_ring_send, dim3(g), dim3(kThreads), 0, s, static_cast<const uint8_t*>(src) + off, n,
                       chunk_of(n, g), a);
    hip_check(hipGetLastError(), "send launch");
    ++sent_;
  }
}

void P2PRing::recv(void* dst, int64_t bytes, hipStream_t s) {
  if (!opened_) throw std::runtime_error("p2p ring: peer not opened");
  if (reinterpret_cast<uintptr_t>(dst) & 15) throw std::invalid_argument("p2p ring: 16-B aligned destination");
  const RingArgs a = args_of(local_, peer_, state_, flag_bytes_, slot_bytes_, timeout_ticks_);
  for (int64_t off = 0; off < bytes; off += slot_bytes_) {
    const int64_t n = std::min(slot_bytes_, bytes - off);
    const int g = grid_of(n);
    hipLaunchKernelGGL(k_ring_recv, dim3(g), dim3(kThreads), 0, s, static_cast<uint8_t*>(dst) + off, n,
                       chunk_of(n, g), a);
    hip_check(hipGetLastError(), "recv launch");
    ++received_;
  }
}

int P2PRing::error() {
  uint32_t e = 0;
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipDeviceSynchronize(), "sync");
  hip_check(hipMemcpy(&e, state_ + kError, 4, hipMemcpyDeviceToHost), "read error word");
  return static_cast<int>(e);
}

void P2PRing::close() {
  if (local_ == nullptr) return;
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  if (peer_ != nullptr && peer_ipc_) (void)hipIpcCloseMemHandle(peer_);
  (void)hipFree(local_);
  (void)hipFree(state_);
  local_ = peer_ = nullptr;
  state_ = nullptr;
  opened_ = false;
}

}  // namespace pde
