// Fused multi-tensor optimisers (gfx950): SGD (+momentum), Adam, AdamW over ALL parameter tensors
// of a model in ONE launch ("one fused multi-tensor Adam kernel").
//
// The parameter set is described by a device-resident table (built once by the caller); each
// block walks fixed-size chunks of the concatenated element space and finds its tensor by binary
// search over the prefix offsets.  Hyper-parameters and the step counter live in device memory so
// the update can be replayed inside a hipGraph while the LR changes between replays (elastic LR
// rescale, horovod_mnist_elastic.py:80-82).  fp32 master weights; optionally also writes a bf16
// copy of the updated weight (the compute copy consumed by the MFMA kernels).
#include "common.cuh"
#include "pde_kernels.h"

namespace pde {

namespace {

constexpr int kChunk = 4096;  // elements per block iteration (256 threads x 4 x f32x4)

__device__ __forceinline__ int find_tensor(const OptimEntry* tab, int n, long e) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].offset <= e) lo = mid; else hi = mid - 1;
  }
  return lo;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_optim(const OptimEntry* __restrict__ tab, int ntensors, long total,
                                               const float* __restrict__ hp, const int* __restrict__ step_ptr) {
  const float lr = hp[HP_LR], b1 = hp[HP_BETA1], b2 = hp[HP_BETA2], eps = hp[HP_EPS];
  const float wd = hp[HP_WD], mom = hp[HP_MOMENTUM], gscale = hp[HP_GRAD_SCALE];
  const int step = step_ptr[0] + 1;  // step being taken (1-based), incremented by k_step_inc
  const float bc1 = 1.f - __powf(b1, static_cast<float>(step));
  const float bc2 = 1.f - __powf(b2, static_cast<float>(step));
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = rsqrtf(bc2);

  for (long c0 = static_cast<long>(blockIdx.x) * kChunk; c0 < total; c0 += static_cast<long>(gridDim.x) * kChunk) {
    int t = find_tensor(tab, ntensors, c0);
    for (int it = 0; it < kChunk / 256; ++it) {
      const long e = c0 + it * 256 + threadIdx.x;
      if (e >= total) break;
      while (t + 1 < ntensors && tab[t + 1].offset <= e) ++t;
      const OptimEntry& te = tab[t];
      const long i = e - te.offset;
      float p = te.param[i];
      float g = te.grad ? te.grad[i] * gscale : 0.f;
      if (MODE == 0) {  // SGD
        if (wd != 0.f) g += wd * p;
        if (mom != 0.f) {
          float buf = te.exp_avg[i];
          buf = (step == 1) ? g : mom * buf + g;
          te.exp_avg[i] = buf;
          g = buf;
        }
        p -= lr * g;
      } else {
        if (MODE == 1) {
          if (wd != 0.f) g += wd * p;
        } else {
          p *= 1.f - lr * wd;
        }
        float m = te.exp_avg[i], v = te.exp_avg_sq[i];
        m = b1 * m + (1.f - b1) * g;
        v = b2 * v + (1.f - b2) * g * g;
        te.exp_avg[i] = m;
        te.exp_avg_sq[i] = v;
        const float denom = sqrtf(v) * inv_sqrt_bc2 + eps;
        p -= step_size * m / denom;
      }
      te.param[i] = p;
      if (te.bf16_copy) te.bf16_copy[i] = f2bf(p);
    }
  }
}

__global__ void k_step_inc(int* step) { step[0] += 1; }

}  // namespace

hipError_t multi_tensor_optim(int mode, const OptimEntry* dev_table, int ntensors, long total_elems,
                              const float* dev_hparams, int* dev_step, hipStream_t s) {
  if (ntensors <= 0 || total_elems <= 0) return hipSuccess;
  long blocks = (total_elems + kChunk - 1) / kChunk;
  if (blocks > 2048) blocks = 2048;
  dim3 grid(static_cast<unsigned>(blocks));
  if (mode == 0)
    hipLaunchKernelGGL(k_optim<0>, grid, dim3(256), 0, s, dev_table, ntensors, total_elems, dev_hparams, dev_step);
  else if (mode == 1)
    hipLaunchKernelGGL(k_optim<1>, grid, dim3(256), 0, s, dev_table, ntensors, total_elems, dev_hparams, dev_step);
  else
    hipLaunchKernelGGL(k_optim<2>, grid, dim3(256), 0, s, dev_table, ntensors, total_elems, dev_hparams, dev_step);
  hipLaunchKernelGGL(k_step_inc, dim3(1), dim3(1), 0, s, dev_step);
  return hipGetLastError();
}

}  // namespace pde
