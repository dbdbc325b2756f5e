// One-shot peer all-reduce over xGMI: see xgmi_allreduce.h for the protocol.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>

#include "xgmi_allreduce.h"

namespace pde {

namespace {

constexpr int kThreads = 256;

struct Peers {
  char* base[kXgmiMaxRanks];
};

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("xgmi allreduce: ") + what + ": " + hipGetErrorString(e));
}

__device__ __forceinline__ uint32_t load_flag(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void store_flag(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// grid = one workgroup per chunk of `chunk` elements (the same grid on every rank and every call: the
// per-workgroup epochs must advance in step across ranks).
template <int NR, bool VEC>
__global__ __launch_bounds__(kThreads) void k_xgmi_oneshot(const float* src, float* dst, int64_t n, float scale,
                                                            Peers peers, int rank, int64_t chunk,
                                                            int64_t flag_bytes, int64_t slot_bytes,
                                                            uint32_t* state, uint64_t timeout_ticks) {
  __shared__ uint32_t s_epoch;
  __shared__ int s_fail;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  if (tid == 0) {
    s_epoch = state[b] + 1u;
    s_fail = 0;
  }
  __syncthreads();
  const uint32_t epoch = s_epoch;
  const int64_t slot_off = flag_bytes + static_cast<int64_t>(epoch & 1u) * slot_bytes;
  const int64_t lo = static_cast<int64_t>(b) * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  float* mine = reinterpret_cast<float*>(peers.base[rank] + slot_off);

  // 1. stage this workgroup's chunk into my exported slot
  if (VEC) {
    for (int64_t i = lo + 4 * tid; i < hi; i += 4 * kThreads)
      *reinterpret_cast<float4*>(mine + i) = *reinterpret_cast<const float4*>(src + i);
  } else {
    for (int64_t i = lo + tid; i < hi; i += kThreads) mine[i] = src[i];
  }
  // 2. publish: every storing wave drains its stores, the workgroup meets, one lane releases at system
  //    scope, then one lane per peer raises this workgroup's flag in that peer's flag array
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (tid < NR) {
    uint32_t* f = reinterpret_cast<uint32_t*>(peers.base[tid]) + b * kXgmiMaxRanks + rank;
    store_flag(f, epoch);
  }
  // 3. wait for every rank's flag of this workgroup: one polling lane per peer, bounded by wall clock
  if (tid < NR) {
    uint32_t* f = reinterpret_cast<uint32_t*>(peers.base[rank]) + b * kXgmiMaxRanks + tid;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (static_cast<int32_t>(load_flag(f) - epoch) < 0) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        s_fail = 1;
        __hip_atomic_store(state + gridDim.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // 4. sum the chunk over all ranks' slots in rank order (bit-identical on every rank)
  if (!s_fail) {
    const float* slots[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) slots[r] = reinterpret_cast<const float*>(peers.base[r] + slot_off);
    if (VEC) {
      for (int64_t i = lo + 4 * tid; i < hi; i += 4 * kThreads) {
        float4 v[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) v[r] = *reinterpret_cast<const float4*>(slots[r] + i);
        float4 acc = v[0];
#pragma unroll
        for (int r = 1; r < NR; ++r) {
          acc.x += v[r].x;
          acc.y += v[r].y;
          acc.z += v[r].z;
          acc.w += v[r].w;
        }
        acc.x *= scale;
        acc.y *= scale;
        acc.z *= scale;
        acc.w *= scale;
        *reinterpret_cast<float4*>(dst + i) = acc;
      }
    } else {
      for (int64_t i = lo + tid; i < hi; i += kThreads) {
        float v[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) v[r] = slots[r][i];
        float acc = v[0];
#pragma unroll
        for (int r = 1; r < NR; ++r) acc += v[r];
        dst[i] = acc * scale;
      }
    }
  }
  // 5. this workgroup's epoch advances (read again by the same workgroup index next call)
  if (tid == 0) state[b] = epoch;
}

__global__ void k_scale(const float* src, float* dst, int64_t n, float scale) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    dst[i] = src[i] * scale;
}

template <int NR>
void launch(bool vec, dim3 grid, hipStream_t s, const float* src, float* dst, int64_t n, float scale,
            const Peers& p, int rank, int64_t chunk, int64_t flag_bytes, int64_t slot_bytes, uint32_t* state,
            uint64_t ticks) {
  if (vec)
    hipLaunchKernelGGL((k_xgmi_oneshot<NR, true>), grid, dim3(kThreads), 0, s, src, dst, n, scale, p, rank, chunk,
                       flag_bytes, slot_bytes, state, ticks);
  else
    hipLaunchKernelGGL((k_xgmi_oneshot<NR, false>), grid, dim3(kThreads), 0, s, src, dst, n, scale, p, rank, chunk,
                       flag_bytes, slot_bytes, state, ticks);
}

}  // namespace

XgmiAllreduce::XgmiAllreduce(int rank, int size, int device, int64_t max_bytes, int blocks, double timeout_s)
    : rank_(rank), size_(size), device_(device), blocks_(blocks), max_bytes_(max_bytes) {
  if (size < 1 || size > kXgmiMaxRanks) throw std::invalid_argument("xgmi allreduce: 1..8 ranks");
  if (blocks < 1 || blocks > 1024) throw std::invalid_argument("xgmi allreduce: 1..1024 workgroups");
  slot_bytes_ = ((max_bytes + 4095) / 4096) * 4096;
  flag_bytes_ = ((static_cast<int64_t>(blocks) * kXgmiMaxRanks * 4 + 4095) / 4096) * 4096;
  timeout_ticks_ = static_cast<uint64_t>(timeout_s * 1e8);  // s_memrealtime runs at 100 MHz
  hip_check(hipSetDevice(device), "hipSetDevice");
  const size_t bytes = static_cast<size_t>(flag_bytes_ + 2 * slot_bytes_);
  void* p = nullptr;
  hip_check(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached), "hipExtMallocWithFlags(uncached)");
  local_ = static_cast<char*>(p);
  hip_check(hipMemset(local_, 0, bytes), "zero flags");
  void* st = nullptr;
  hip_check(hipMalloc(&st, static_cast<size_t>(blocks + 1) * 4), "hipMalloc state");
  state_ = static_cast<uint32_t*>(st);
  hip_check(hipMemset(state_, 0, static_cast<size_t>(blocks + 1) * 4), "zero state");
  hip_check(hipDeviceSynchronize(), "sync after init");  // flags are zero before any peer can map them
  peers_.assign(size, nullptr);
  peers_[rank] = local_;
}

XgmiAllreduce::~XgmiAllreduce() {
  try {
    close();
  } catch (...) {
  }
}

std::string XgmiAllreduce::ipc_handle() const {
  hipIpcMemHandle_t h;
  hip_check(hipIpcGetMemHandle(&h, local_), "hipIpcGetMemHandle");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void XgmiAllreduce::open(const std::vector<std::string>& handles) {
  if (static_cast<int>(handles.size()) != size_) throw std::invalid_argument("xgmi allreduce: one handle per rank");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  for (int r = 0; r < size_; ++r) {
    if (r == rank_) continue;
    if (handles[r].size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("xgmi allreduce: bad handle");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[r].data(), sizeof(h));
    void* p = nullptr;
    hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    peers_[r] = static_cast<char*>(p);
  }
  opened_ = true;
}

void XgmiAllreduce::allreduce(const float* src, float* dst, int64_t n, float scale, hipStream_t s) {
  if (n <= 0) return;
  if (n * 4 > max_bytes_) throw std::invalid_argument("xgmi allreduce: bucket exceeds max_bytes");
  if (size_ == 1) {
    const int g = static_cast<int>(std::min<int64_t>(1024, (n + kThreads - 1) / kThreads));
    hipLaunchKernelGGL(k_scale, dim3(g), dim3(kThreads), 0, s, src, dst, n, scale);
    hip_check(hipGetLastError(), "scale launch");
    return;
  }
  if (!opened_) throw std::runtime_error("xgmi allreduce: peers not opened");
  Peers p{};
  for (int r = 0; r < size_; ++r) p.base[r] = peers_[r];
  // chunk per workgroup, a multiple of 64 floats (256 B rows) so float4 lanes stay aligned
  int64_t chunk = (n + blocks_ - 1) / blocks_;
  chunk = ((chunk + 63) / 64) * 64;
  const bool vec = (n % 4 == 0) && (reinterpret_cast<uintptr_t>(src) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(dst) % 16 == 0);
  const dim3 grid(blocks_);
  switch (size_) {
    case 2: launch<2>(vec, grid, s, src, dst, n, scale, p, rank_, chunk, flag_bytes_, slot_bytes_, state_, timeout_ticks_); break;
    case 3: launch<3>(vec, grid, s, src, dst, n, scale, p, rank_, chunk, flag_bytes_, slot_bytes_, state_, timeout_ticks_); break;
    case 4: launch<4>(vec, grid, s, src, dst, n, scale, p, rank_, chunk, flag_bytes_, slot_bytes_, state_, timeout_ticks_); break;
    case 5: launch<5>(vec, grid, s, src, dst, n, scale, p, rank_, chunk, flag_bytes_, slot_bytes_, state_, timeout_ticks_); break;
    case 6: launch<6>(vec, grid, s, src, dst, n, scale, p, rank_, chunk, flag_bytes_, slot_bytes_, state_, timeout_ticks_); break;
    case 7: launch<7>(vec, grid, s, src, dst, n, scale, p, rank_, chunk, flag_bytes_, slot_bytes_, state_, timeout_ticks_); break;
    default: launch<8>(vec, grid, s, src, dst, n, scale, p, rank_, chunk, flag_bytes_, slot_bytes_, state_, timeout_ticks_); break;
  }
  hip_check(hipGetLastError(), "oneshot launch");
  ++calls_;
}

int XgmiAllreduce::error() {
  uint32_t e = 0;
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipDeviceSynchronize(), "sync");
  hip_check(hipMemcpy(&e, state_ + blocks_, 4, hipMemcpyDeviceToHost), "read error word");
  return static_cast<int>(e);
}

void XgmiAllreduce::close() {
  if (local_ == nullptr) return;
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  for (int r = 0; r < size_; ++r)
    if (r != rank_ && peers_[r] != nullptr) (void)hipIpcCloseMemHandle(peers_[r]);
  peers_.clear();
  (void)hipFree(local_);
  (void)hipFree(state_);
  local_ = nullptr;
  state_ = nullptr;
  opened_ = false;
}

}  // namespace pde
