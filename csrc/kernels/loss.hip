// Loss kernels (gfx950): fused log-softmax + NLL (cross-entropy) forward / backward, log_softmax
// forward / backward, NLL forward / backward and MSE forward / backward.
//
// The batch reductions are done by ONE workgroup of 1024 threads with a fixed-order LDS tree, so
// the loss value is bitwise reproducible from run to run (no float atomics).  For the class counts
// of this suite (10 for MNIST, 8 for the EmbeddingBag hybrid, 1000 for ResNet-50 MSE) a row fits
// one lane (V <= 64) or one wave.
#include "common.cuh"
#include "pde_kernels.h"

namespace pde {

namespace {

constexpr int kLossThreads = 1024;

__device__ __forceinline__ float ld(const void* p, int f32, long i) {
  return f32 ? static_cast<const float*>(p)[i] : bf2f(static_cast<const uint16_t*>(p)[i]);
}

// Block-wide fixed-order sum; result valid in every thread.
__device__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x < 64) {
    t = threadIdx.x < (blockDim.x >> 6) ? red[threadIdx.x] : 0.f;
    t = wave_sum(t);
    if (threadIdx.x == 0) red[0] = t;
  }
  __syncthreads();
  t = red[0];
  __syncthreads();
  return t;
}

// Row log-sum-exp of row b (thread-per-row variant).
__device__ __forceinline__ float row_lse(const void* x, int f32, long base, int V) {
  float m = -INFINITY;
  for (int v = 0; v < V; ++v) m = fmaxf(m, ld(x, f32, base + v));
  float s = 0.f;
  for (int v = 0; v < V; ++v) s += __expf(ld(x, f32, base + v) - m);
  return m + __logf(s);
}

// mode 0: cross-entropy on logits; mode 1: NLL on log-probabilities.
__global__ void __launch_bounds__(kLossThreads)
k_ce_fwd(const void* x, int f32, const int64_t* __restrict__ tgt, int B, int V, int mode,
         float* __restrict__ loss, float* __restrict__ lse_out) {
  __shared__ float red[16];
  float acc = 0.f;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const long base = static_cast<long>(b) * V;
    const int t = static_cast<int>(tgt[b]);
    if (mode == 0) {
      const float l = row_lse(x, f32, base, V);
      if (lse_out) lse_out[b] = l;
      acc += l - ld(x, f32, base + t);
    } else {
      acc -= ld(x, f32, base + t);
    }
  }
  const float tot = block_sum(acc, red);
  if (threadIdx.x == 0) loss[0] = tot / static_cast<float>(B);
}

// dx[b, v] = (softmax - onehot) * g / B   (mode 0, uses lse)   |   -onehot * g / B  (mode 1)
__global__ void k_ce_bwd(const void* x, int f32, const int64_t* __restrict__ tgt, const float* __restrict__ lse,
                         const float* __restrict__ gout, int B, int V, int mode, void* dx, int dx_f32) {
  const float g = gout[0] / static_cast<float>(B);
  const long total = static_cast<long>(B) * V;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int b = static_cast<int>(i / V);
    const int v = static_cast<int>(i - static_cast<long>(b) * V);
    const float oh = (v == static_cast<int>(tgt[b])) ? 1.f : 0.f;
    float d = mode == 0 ? (__expf(ld(x, f32, i) - lse[b]) - oh) * g : -oh * g;
    if (dx_f32) static_cast<float*>(dx)[i] = d;
    else static_cast<uint16_t*>(dx)[i] = f2bf(d);
  }
}

// Fused mean cross-entropy forward + backward (one block; thread per row)
__global__ void k_ce_fused(const void* x, int f32, const int64_t* __restrict__ tgt, int B, int V,
                           float* __restrict__ loss, uint16_t* __restrict__ dx, int ldx) {
  __shared__ float red[16];
  const float inv_b = 1.f / static_cast<float>(B);
  float acc = 0.f;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const long base = static_cast<long>(b) * V;
    const int t = static_cast<int>(tgt[b]);
    uint16_t* drow = dx + static_cast<long>(b) * ldx;  // (row pitch ldx >= V: columns past V are untouched)
    if (V <= 16) {  // the row in registers: one round of loads, the target logit selected, not re-read
      float r[16];
#pragma unroll
      for (int v = 0; v < 16; ++v) r[v] = v < V ? ld(x, f32, base + v) : -INFINITY;
      float m = r[0], xt = 0.f;
#pragma unroll
      for (int v = 1; v < 16; ++v) m = fmaxf(m, r[v]);
      float sum = 0.f;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        sum += v < V ? __expf(r[v] - m) : 0.f;
        xt = v == t ? r[v] : xt;
      }
      const float l = m + __logf(sum);
      acc += l - xt;
#pragma unroll
      for (int v = 0; v < 16; ++v)
        if (v < V) drow[v] = f2bf((__expf(r[v] - l) - (v == t ? 1.f : 0.f)) * inv_b);
    } else {
      const float l = row_lse(x, f32, base, V);
      acc += l - ld(x, f32, base + t);
      for (int v = 0; v < V; ++v) drow[v] = f2bf((__expf(ld(x, f32, base + v) - l) - (v == t ? 1.f : 0.f)) * inv_b);
    }
  }
  const float tot = block_sum(acc, red);
  if (threadIdx.x == 0) loss[0] = tot * inv_b;
}

// log_softmax over rows (thread per row for V <= 64; wave per row otherwise)
__global__ void k_log_softmax_fwd(const void* x, int f32, int B, int V, float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  if (V <= 64) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const long base = static_cast<long>(b) * V;
    const float l = row_lse(x, f32, base, V);
    for (int v = 0; v < V; ++v) y[base + v] = ld(x, f32, base + v) - l;
    return;
  }
  const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (b >= B) return;
  const long base = static_cast<long>(b) * V;
  float m = -INFINITY;
  for (int v = lane; v < V; v += 64) m = fmaxf(m, ld(x, f32, base + v));
  m = wave_max(m);
  float s = 0.f;
  for (int v = lane; v < V; v += 64) s += __expf(ld(x, f32, base + v) - m);
  s = wave_sum(s);
  const float l = m + __logf(s);
  for (int v = lane; v < V; v += 64) y[base + v] = ld(x, f32, base + v) - l;
}

// dx = dy - exp(y) * rowsum(dy)
__global__ void k_log_softmax_bwd(const float* __restrict__ dy, const float* __restrict__ y, int B, int V,
                                  void* dx, int dx_f32) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long base = static_cast<long>(b) * V;
  float s = 0.f;
  for (int v = 0; v < V; ++v) s += dy[base + v];
  for (int v = 0; v < V; ++v) {
    const float d = dy[base + v] - __expf(y[base + v]) * s;
    if (dx_f32) static_cast<float*>(dx)[base + v] = d;
    else static_cast<uint16_t*>(dx)[base + v] = f2bf(d);
  }
}

__global__ void __launch_bounds__(kLossThreads)
k_mse_fwd(const void* p, int f32, const float* __restrict__ t, long n, float* __restrict__ loss) {
  __shared__ float red[16];
  // 8 element pairs per thread in flight per trip (one block: the trip count, not bandwidth, sets the time)
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const long st = blockDim.x;
  long i = threadIdx.x;
  for (; i + 7 * st < n; i += 8 * st) {
    float a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a[u] = ld(p, f32, i + u * st);
      b[u] = t[i + u * st];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float d = a[u] - b[u];
      acc[u & 3] += d * d;
    }
  }
  for (; i < n; i += st) {
    const float d = ld(p, f32, i) - t[i];
    acc[0] += d * d;
  }
  const float tot = block_sum((acc[0] + acc[1]) + (acc[2] + acc[3]), red);
  if (threadIdx.x == 0) loss[0] = tot / static_cast<float>(n);
}

__global__ void k_mse_bwd(const void* p, int f32, const float* __restrict__ t, const float* __restrict__ gout,
                          long n, void* dx, int dx_f32) {
  const float g = 2.f * gout[0] / static_cast<float>(n);
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const float d = (ld(p, f32, i) - t[i]) * g;
    if (dx_f32) static_cast<float*>(dx)[i] = d;
    else static_cast<uint16_t*>(dx)[i] = f2bf(d);
  }
}

}  // namespace

hipError_t ce_fwd(const void* x, int f32, const int64_t* tgt, int B, int V, int mode, float* loss, float* lse,
                  hipStream_t s) {
  hipLaunchKernelGGL(k_ce_fwd, dim3(1), dim3(kLossThreads), 0, s, x, f32, tgt, B, V, mode, loss, lse);
  return hipGetLastError();
}
hipError_t ce_bwd(const void* x, int f32, const int64_t* tgt, const float* lse, const float* gout, int B, int V,
                  int mode, void* dx, int dx_f32, hipStream_t s) {
  const long total = static_cast<long>(B) * V;
  hipLaunchKernelGGL(k_ce_bwd, dim3(stream_grid(total, 256)), dim3(256), 0, s, x, f32, tgt, lse, gout, B, V,
                     mode, dx, dx_f32);
  return hipGetLastError();
}
hipError_t ce_fused(const void* x, int f32, const int64_t* tgt, int B, int V, float* loss, uint16_t* dx, int ldx,
                    hipStream_t s) {
  hipLaunchKernelGGL(k_ce_fused, dim3(1), dim3(kLossThreads), 0, s, x, f32, tgt, B, V, loss, dx, ldx);
  return hipGetLastError();
}
hipError_t log_softmax_fwd(const void* x, int f32, int B, int V, float* y, hipStream_t s) {
  if (V <= 64)
    hipLaunchKernelGGL(k_log_softmax_fwd, dim3(ceil_div(B, 256)), dim3(256), 0, s, x, f32, B, V, y);
  else
    hipLaunchKernelGGL(k_log_softmax_fwd, dim3(ceil_div(B, 4)), dim3(256), 0, s, x, f32, B, V, y);
  return hipGetLastError();
}
hipError_t log_softmax_bwd(const float* dy, const float* y, int B, int V, void* dx, int dx_f32, hipStream_t s) {
  hipLaunchKernelGGL(k_log_softmax_bwd, dim3(ceil_div(B, 256)), dim3(256), 0, s, dy, y, B, V, dx, dx_f32);
  return hipGetLastError();
}
hipError_t mse_fwd(const void* p, int f32, const float* t, long n, float* loss, hipStream_t s) {
  hipLaunchKernelGGL(k_mse_fwd, dim3(1), dim3(kLossThreads), 0, s, p, f32, t, n, loss);
  return hipGetLastError();
}
hipError_t mse_bwd(const void* p, int f32, const float* t, const float* gout, long n, void* dx, int dx_f32,
                   hipStream_t s) {
  hipLaunchKernelGGL(k_mse_bwd, dim3(stream_grid(n, 256)), dim3(256), 0, s, p, f32, t, gout, n, dx, dx_f32);
  return hipGetLastError();
}

}  // namespace pde
