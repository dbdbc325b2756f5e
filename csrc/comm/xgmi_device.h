// Device side of the one-shot xGMI peer exchange (protocol: xgmi_allreduce.h), shared by the stand-alone
// all-reduce kernel (xgmi_allreduce.hip) and kernels that fold the exchange into their own epilogue (the
// fused CNN's gradient reduction, cnn_fused.hip): such a kernel stages its output chunk into its slot,
// calls xgmi_publish_and_wait, and reads every rank's chunk back from the peers' slots in rank order.
//
// XgmiView (xgmi_view.h) is plain data filled by XgmiAllreduce::view(); a kernel takes it by value.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "xgmi_view.h"

namespace pde {

// This call's epoch (block-collective: every thread gets it through LDS).  ONE epoch per call for all
// workgroups -- whatever the grid size -- so the staging-slot parity is the same for every byte of a call:
// consecutive calls with different sizes (or kernels sharing the instance) never hand the same slot range
// to two calls in flight.  Why that is enough: rank A can write slot (e & 1) of call e + 2 only after its
// call e + 1 saw every peer's flags of e + 1, i.e. after every peer LAUNCHED call e + 1, which on a peer's
// stream starts only when its call e -- all of its reads of slot (e & 1) -- has completed.
__device__ __forceinline__ uint32_t xgmi_epoch(const XgmiView& v, int b, uint32_t* s_epoch) {
  (void)b;
  if (threadIdx.x == 0)
    *s_epoch = __hip_atomic_load(v.state + kXgmiStateEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  return *s_epoch;
}

// Rank r's staging slot for this epoch (two slots alternate: a peer is at most one call ahead).
__device__ __forceinline__ float* xgmi_slot(const XgmiView& v, int r, uint32_t epoch) {
  return reinterpret_cast<float*>(v.base[r] + v.flag_bytes + static_cast<int64_t>(epoch & 1u) * v.slot_bytes);
}

// Block-collective, after every thread issued its stores into xgmi_slot(v, v.rank, epoch):
//   every storing wave drains, the workgroup meets, one lane releases at system scope, one lane per rank
//   raises flag (b, my rank) in that rank's flag array; one lane per rank polls my flag (b, r) until it
//   reaches the epoch (bounded by wall clock or the host's abort word: a timeout sets the error words -- the
//   device one for fail-fast, the host-mapped one the host polls without a sync -- and the result is dropped),
//   then one lane acquires at system scope and the workgroup meets again.
// Returns true when every rank's chunk of workgroup b may be read.
__device__ __forceinline__ bool xgmi_publish_and_wait(const XgmiView& v, int b, uint32_t epoch, int* s_fail) {
  const int tid = threadIdx.x;
  if (tid == 0) *s_fail = 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (tid < v.size) {
    uint32_t* f = reinterpret_cast<uint32_t*>(v.base[tid]) + b * kXgmiMaxRanks + v.rank;
    __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = reinterpret_cast<uint32_t*>(v.base[v.rank]) + b * kXgmiMaxRanks + tid;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t polls = 0;
    while (static_cast<int32_t>(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      // Give up on: the wall-clock bound; an earlier timed-out wait of this instance (fail fast: a dead peer
      // costs ONE timeout, not one per queued call of a graph replay -- the word is cleared by the host's
      // check at its next sync point, XgmiAllreduce::clear_error); or the host's abort word (an elastic
      // driver published a new round / the engine failed), polled over PCIe every 64th spin.
      bool give_up = __builtin_amdgcn_s_memrealtime() - t0 > v.timeout_ticks ||
                     __hip_atomic_load(v.state + kXgmiStateError, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
      if (!give_up && v.host != nullptr && (++polls & 63u) == 0u)
        give_up = __hip_atomic_load(v.host + kXgmiHostAbort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
      if (give_up) {
        *s_fail = 1;
        __hip_atomic_store(v.state + kXgmiStateError, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // (a plain system-scope store, not an atomic: PCIe atomics to host memory are not assumed)
        if (v.host != nullptr) __hip_atomic_store(v.host + kXgmiHostError, epoch + 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_SYSTEM);
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
  return *s_fail == 0;
}

// Test hook: hold this workgroup between the flag wait and its peer reads (a slow reader).
__device__ __forceinline__ void xgmi_read_delay(const XgmiView& v) {
  if (v.read_delay_ticks == 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < v.read_delay_ticks) __builtin_amdgcn_s_sleep(8);
}

// Block-collective, once per workgroup after its last peer read: the workgroup that finishes last advances
// the call's epoch (the next kernel using the view reads it; kernel boundaries order the store).
__device__ __forceinline__ void xgmi_finish(const XgmiView& v, int b, uint32_t epoch) {
  (void)b;
  __syncthreads();  // every wave's peer reads are issued before the workgroup counts itself done
  if (threadIdx.x == 0) {
    const uint32_t n = __hip_atomic_fetch_add(v.state + kXgmiStateDone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (n == gridDim.x - 1) {
      __hip_atomic_store(v.state + kXgmiStateDone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(v.state + kXgmiStateEpoch, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace pde
