// Fused multi-tensor optimisers (gfx950): SGD (+momentum), Adam, AdamW over ALL parameter tensors
// of a model in ONE launch ("one fused multi-tensor Adam kernel").
//
// The parameter set is described by a device-resident table (built once by the caller); each
// block walks fixed-size chunks of the concatenated element space and finds its tensor by binary
// search over the prefix offsets.  Hyper-parameters and the step counter live in device memory so
// the update can be replayed inside a hipGraph while the LR changes between replays (elastic LR
// rescale, horovod_mnist_elastic.py:80-82).  fp32 master weights; optionally also writes a bf16
// copy of the updated weight (the compute copy consumed by the MFMA kernels).  The step counter is
// int32[2] = {steps taken, arrival counter}: the last block to finish advances it, so one launch per
// step (no separate increment kernel).
#include "common.cuh"
#include "pde_kernels.h"

namespace pde {

namespace {

// Element space: every tensor starts at a multiple of 4 (offsets padded by optim_table), so a thread's
// group of 4 consecutive elements never straddles two tensors.  A block iteration covers kChunk
// elements = 256 threads x kGroups groups of 4 (independent loads in flight per thread).
constexpr int kThreads = 256;
constexpr int kGroups = 2;
constexpr int kChunk = kThreads * 4 * kGroups;
constexpr int kLdsTab = 2048;  // tensor offsets searched in LDS up to this many tensors

__device__ __forceinline__ int find_tensor(const long* off, int n, long e) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= e) lo = mid; else hi = mid - 1;
  }
  return lo;
}
__device__ __forceinline__ int find_tensor_g(const OptimEntry* tab, int n, long e) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].offset <= e) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

struct Hyper {
  float lr, b1, b2, eps, wd, mom, gscale, step_size, inv_sqrt_bc2;
  int step;
};

template <int MODE>
__device__ __forceinline__ void update(const Hyper& h, float& p, float g, float& m, float& v) {
  g *= h.gscale;
  if (MODE == 0) {  // SGD (+momentum, +L2)
    if (h.wd != 0.f) g += h.wd * p;
    if (h.mom != 0.f) {
      m = (h.step == 1) ? g : h.mom * m + g;
      g = m;
    }
    p -= h.lr * g;
  } else {
    if (MODE == 1) {
      if (h.wd != 0.f) g += h.wd * p;
    } else {
      p *= 1.f - h.lr * h.wd;
    }
    m = h.b1 * m + (1.f - h.b1) * g;
    v = h.b2 * v + (1.f - h.b2) * g * g;
    p -= h.step_size * m / (sqrtf(v) * h.inv_sqrt_bc2 + h.eps);
  }
}

template <int MODE>
__global__ __launch_bounds__(kThreads) void k_optim(const OptimEntry* __restrict__ tab, int ntensors, long total,
                                                    const float* __restrict__ hp, int* __restrict__ step_ptr) {
  __shared__ long s_off[kLdsTab];
  __shared__ int s_step;
  if (threadIdx.x == 0) s_step = step_ptr[0] + 1;  // step being taken (1-based)
  const bool lds_tab = ntensors <= kLdsTab;
  if (lds_tab)
    for (int i = threadIdx.x; i < ntensors; i += kThreads) s_off[i] = tab[i].offset;
  __syncthreads();
  Hyper h;
  h.lr = hp[HP_LR]; h.b1 = hp[HP_BETA1]; h.b2 = hp[HP_BETA2]; h.eps = hp[HP_EPS];
  h.wd = hp[HP_WD]; h.mom = hp[HP_MOMENTUM]; h.gscale = hp[HP_GRAD_SCALE];
  h.step = s_step;
  if (MODE != 0) {
    const float bc1 = 1.f - __powf(h.b1, static_cast<float>(h.step));
    const float bc2 = 1.f - __powf(h.b2, static_cast<float>(h.step));
    h.step_size = h.lr / bc1;
    h.inv_sqrt_bc2 = rsqrtf(bc2);
  }

  for (long base = static_cast<long>(blockIdx.x) * kChunk; base < total;
       base += static_cast<long>(gridDim.x) * kChunk) {
#pragma unroll
    for (int u = 0; u < kGroups; ++u) {
      const long e0 = base + (static_cast<long>(u) * kThreads + threadIdx.x) * 4;
      if (e0 >= total) continue;
      const int ti = lds_tab ? find_tensor(s_off, ntensors, e0) : find_tensor_g(tab, ntensors, e0);
      const OptimEntry te = tab[ti];
      const long i = e0 - te.offset;
      if (i >= te.size) continue;  // padding between tensors
      const int cnt = te.size - i < 4 ? static_cast<int>(te.size - i) : 4;
      const bool use_m = MODE != 0 || h.mom != 0.f;
      const bool vec = cnt == 4 && al16(te.param + i) && (te.grad == nullptr || al16(te.grad + i)) &&
                       (!use_m || al16(te.exp_avg + i)) && (MODE == 0 || al16(te.exp_avg_sq + i));
      float p[4], g[4] = {0.f, 0.f, 0.f, 0.f}, m[4] = {0.f, 0.f, 0.f, 0.f}, v[4] = {0.f, 0.f, 0.f, 0.f};
      if (vec) {
        const f32x4 pv = *reinterpret_cast<const f32x4*>(te.param + i);
        p[0] = pv[0]; p[1] = pv[1]; p[2] = pv[2]; p[3] = pv[3];
        if (te.grad) {
          const f32x4 gv = *reinterpret_cast<const f32x4*>(te.grad + i);
          g[0] = gv[0]; g[1] = gv[1]; g[2] = gv[2]; g[3] = gv[3];
        }
        if (use_m) {
          const f32x4 mv = *reinterpret_cast<const f32x4*>(te.exp_avg + i);
          m[0] = mv[0]; m[1] = mv[1]; m[2] = mv[2]; m[3] = mv[3];
        }
        if (MODE != 0) {
          const f32x4 vv = *reinterpret_cast<const f32x4*>(te.exp_avg_sq + i);
          v[0] = vv[0]; v[1] = vv[1]; v[2] = vv[2]; v[3] = vv[3];
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k < cnt) {
            p[k] = te.param[i + k];
            if (te.grad) g[k] = te.grad[i + k];
            if (use_m) m[k] = te.exp_avg[i + k];
            if (MODE != 0) v[k] = te.exp_avg_sq[i + k];
          } else {
            p[k] = 0.f;
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) update<MODE>(h, p[k], g[k], m[k], v[k]);
      if (vec) {
        *reinterpret_cast<f32x4*>(te.param + i) = f32x4{p[0], p[1], p[2], p[3]};
        if (use_m) *reinterpret_cast<f32x4*>(te.exp_avg + i) = f32x4{m[0], m[1], m[2], m[3]};
        if (MODE != 0) *reinterpret_cast<f32x4*>(te.exp_avg_sq + i) = f32x4{v[0], v[1], v[2], v[3]};
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k < cnt) {
            te.param[i + k] = p[k];
            if (use_m) te.exp_avg[i + k] = m[k];
            if (MODE != 0) te.exp_avg_sq[i + k] = v[k];
          }
        }
      }
      if (te.bf16_copy) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (k < cnt) te.bf16_copy[i + k] = f2bf(p[k]);
      }
    }
  }
  // the last block to finish publishes the new step count (every block read it before arriving here)
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const int prev = atomicAdd(step_ptr + 1, 1);
    if (prev == static_cast<int>(gridDim.x) - 1) {
      step_ptr[0] = s_step;
      step_ptr[1] = 0;
      __threadfence();
    }
  }
}

}  // namespace

hipError_t multi_tensor_optim(int mode, const OptimEntry* dev_table, int ntensors, long total_elems,
                              const float* dev_hparams, int* dev_step, hipStream_t s) {
  if (ntensors <= 0 || total_elems <= 0) return hipSuccess;
  long blocks = (total_elems + kChunk - 1) / kChunk;
  if (blocks > 4096) blocks = 4096;
  dim3 grid(static_cast<unsigned>(blocks));
  if (mode == 0)
    hipLaunchKernelGGL(k_optim<0>, grid, dim3(kThreads), 0, s, dev_table, ntensors, total_elems, dev_hparams, dev_step);
  else if (mode == 1)
    hipLaunchKernelGGL(k_optim<1>, grid, dim3(kThreads), 0, s, dev_table, ntensors, total_elems, dev_hparams, dev_step);
  else
    hipLaunchKernelGGL(k_optim<2>, grid, dim3(kThreads), 0, s, dev_table, ntensors, total_elems, dev_hparams, dev_step);
  return hipGetLastError();
}

}  // namespace pde
