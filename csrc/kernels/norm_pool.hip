// BatchNorm (training, NHWC bf16), max/avg pooling, dropout and EmbeddingBag kernels (gfx950).
//
// BatchNorm follows SURVEY.md §2.5 / §7.4 H2: per-micro-batch batch statistics in fp32, bf16
// activations.  Forward = shifted-sum partials per block -> per-channel finalize (fixed order,
// deterministic; running-stat update with unbiased variance) -> fused normalize(+residual)(+ReLU).
// Backward = partials of (sum dy, sum dy*xhat) with the ReLU mask applied on the fly -> finalize ->
// fused dx (+ residual grad).  Every pass streams 16 B (8 channels) per lane.
#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "common.cuh"
#include "pde_kernels.h"

namespace pde {

namespace {

// Thread -> (row-in-iteration, 8-channel group) mapping for [P][C] streaming reductions.
struct RowGroupMap {
  int G, rows_per_iter, r, g;
  bool active;
  __device__ RowGroupMap(int C) {
    G = C / 8;
    const int gg = G < 256 ? G : 256;
    rows_per_iter = 256 / gg;
    r = threadIdx.x / gg;
    g = threadIdx.x % gg;
    active = r < rows_per_iter;
  }
};

__device__ __forceinline__ void load8(const uint16_t* p, float (&v)[8]) {
  const u16x8 u = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf2f(u[j]);
}

// Partial shifted sums: ws[blk][0][c] = sum(x - K_c), ws[blk][1][c] = sum((x - K_c)^2), K_c = x[0][c].
__global__ __launch_bounds__(256) void k_bn_stats(const uint16_t* __restrict__ x, int P, int C, int rows_per_block,
                                                  float* __restrict__ ws) {
  const RowGroupMap mp(C);
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(P, r0 + rows_per_block);
  for (int gbase = 0; gbase < mp.G; gbase += 256 / mp.rows_per_iter) {
    const int g = gbase + mp.g;
    float s1[8], s2[8], piv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
    const bool ok = mp.active && g < mp.G;
    if (ok) {
      load8(x + g * 8, piv);
      const int st = mp.rows_per_iter;
      int r = r0 + mp.r;
      // 4 rows per trip, all loads issued before the math (4 x 16 B in flight per lane)
      for (; r + 3 * st < r1; r += 4 * st) {
        u16x8 u[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) u[q] = *reinterpret_cast<const u16x8*>(x + static_cast<long>(r + q * st) * C + g * 8);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int j = 0; j < 8; ++j) { const float d = bf2f(u[q][j]) - piv[j]; s1[j] += d; s2[j] += d * d; }
      }
      for (; r < r1; r += st) {
        float v[8];
        load8(x + static_cast<long>(r) * C + g * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = v[j] - piv[j]; s1[j] += d; s2[j] += d * d; }
      }
    }
    // reduce over the rows_per_iter threads sharing g via LDS
    __shared__ float red[2][256][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { red[0][threadIdx.x][j] = s1[j]; red[1][threadIdx.x][j] = s2[j]; }
    __syncthreads();
    if (mp.r == 0 && ok) {
      const int gg = 256 / mp.rows_per_iter;
      for (int rr = 1; rr < mp.rows_per_iter; ++rr) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { s1[j] += red[0][rr * gg + mp.g][j]; s2[j] += red[1][rr * gg + mp.g][j]; }
      }
      float* o = ws + static_cast<long>(blockIdx.x) * 2 * C;
#pragma unroll
      for (int j = 0; j < 8; ++j) { o[g * 8 + j] = s1[j]; o[C + g * 8 + j] = s2[j]; }
    }
    __syncthreads();
  }
}

// Per channel: combine partials -> mean, invstd, scale/shift; update running stats.
__global__ void k_bn_finalize(const uint16_t* __restrict__ x, const float* __restrict__ ws, int nblk, int P, int C,
                              const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                              float momentum, float* __restrict__ running_mean, float* __restrict__ running_var,
                              float* __restrict__ save_mean, float* __restrict__ save_invstd,
                              float* __restrict__ scale, float* __restrict__ shift) {
  // one wave per channel: lanes stride the block partials (fixed order -> deterministic)
  const int c = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= C) return;
  float p1 = 0.f, p2 = 0.f;
  for (int b = lane; b < nblk; b += 64) {
    p1 += ws[static_cast<long>(b) * 2 * C + c];
    p2 += ws[static_cast<long>(b) * 2 * C + C + c];
  }
  const double s1 = wave_sum(p1), s2 = wave_sum(p2);
  if (lane != 0) return;
  const float piv = bf2f(x[c]);
  const double n = static_cast<double>(P);
  const double mean_s = s1 / n;
  double var = s2 / n - mean_s * mean_s;
  if (var < 0.0) var = 0.0;
  const float mean = static_cast<float>(mean_s) + piv;
  const float invstd = rsqrtf(static_cast<float>(var) + eps);
  save_mean[c] = mean;
  save_invstd[c] = invstd;
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  scale[c] = g * invstd;
  shift[c] = b - mean * g * invstd;
  if (running_mean) {
    const float unbiased = P > 1 ? static_cast<float>(var * n / (n - 1.0)) : static_cast<float>(var);
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
  }
}

// y = x * scale + shift (+ res) (relu) ; bf16 out
__global__ void k_bn_apply(const uint16_t* __restrict__ x, const float* __restrict__ scale,
                           const float* __restrict__ shift, const uint16_t* __restrict__ res, uint16_t* __restrict__ y,
                           long nvec, int C, int relu) {
  const int G = C / 8;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < nvec;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int g = static_cast<int>(i % G);
    float v[8];
    load8(x + i * 8, v);
    float rv[8];
    if (res) load8(res + i * 8, rv);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = v[j] * scale[g * 8 + j] + shift[g * 8 + j];
      if (res) t += rv[j];
      if (relu) t = fmaxf(t, 0.f);
      o[j] = f2bf(t);
    }
    reinterpret_cast<u16x8*>(y)[i] = o;
  }
}

// Backward partials: ws[blk][0][c] = sum dyr, ws[blk][1][c] = sum dyr * (x - mean) * invstd,
// dyr = dy * (relu ? y > 0 : 1)
__global__ __launch_bounds__(256) void k_bn_bwd_reduce(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                       const uint16_t* __restrict__ y, const float* __restrict__ mean,
                                                       const float* __restrict__ invstd, int P, int C,
                                                       int rows_per_block, int relu, float* __restrict__ ws) {
  const RowGroupMap mp(C);
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(P, r0 + rows_per_block);
  for (int gbase = 0; gbase < mp.G; gbase += 256 / mp.rows_per_iter) {
    const int g = gbase + mp.g;
    float s1[8], s2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
    const bool ok = mp.active && g < mp.G;
    if (ok) {
      float mu[8], is[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { mu[j] = mean[g * 8 + j]; is[j] = invstd[g * 8 + j]; }
      const int st = mp.rows_per_iter;
      int r = r0 + mp.r;
      // 2 rows per trip with every load (dy, x, y of both rows) issued before the math
      for (; r + st < r1; r += 2 * st) {
        u16x8 ud[2], ux[2], uy[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const long off = static_cast<long>(r + q * st) * C + g * 8;
          ud[q] = *reinterpret_cast<const u16x8*>(dy + off);
          ux[q] = *reinterpret_cast<const u16x8*>(x + off);
          if (relu) uy[q] = *reinterpret_cast<const u16x8*>(y + off);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float d = bf2f(ud[q][j]);
            if (relu && !(bf2f(uy[q][j]) > 0.f)) d = 0.f;
            s1[j] += d;
            s2[j] += d * (bf2f(ux[q][j]) - mu[j]) * is[j];
          }
      }
      for (; r < r1; r += st) {
        const long off = static_cast<long>(r) * C + g * 8;
        float d[8], xv[8];
        load8(dy + off, d);
        load8(x + off, xv);
        if (relu) {
          float yv[8];
          load8(y + off, yv);
#pragma unroll
          for (int j = 0; j < 8; ++j) d[j] = yv[j] > 0.f ? d[j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) { s1[j] += d[j]; s2[j] += d[j] * (xv[j] - mu[j]) * is[j]; }
      }
    }
    __shared__ float red[2][256][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { red[0][threadIdx.x][j] = s1[j]; red[1][threadIdx.x][j] = s2[j]; }
    __syncthreads();
    if (mp.r == 0 && ok) {
      const int gg = 256 / mp.rows_per_iter;
      for (int rr = 1; rr < mp.rows_per_iter; ++rr) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { s1[j] += red[0][rr * gg + mp.g][j]; s2[j] += red[1][rr * gg + mp.g][j]; }
      }
      float* o = ws + static_cast<long>(blockIdx.x) * 2 * C;
#pragma unroll
      for (int j = 0; j < 8; ++j) { o[g * 8 + j] = s1[j]; o[C + g * 8 + j] = s2[j]; }
    }
    __syncthreads();
  }
}

// Per channel: dgamma, dbeta (written / accumulated) and the dx coefficients.
__global__ void k_bn_bwd_finalize(const float* __restrict__ ws, int nblk, int P, int C, const float* __restrict__ gamma,
                                  const float* __restrict__ invstd, float* __restrict__ dgamma, float* __restrict__ dbeta,
                                  int accum, float* __restrict__ coef) {
  const int c = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= C) return;
  float p1 = 0.f, p2 = 0.f;
  for (int b = lane; b < nblk; b += 64) {
    p1 += ws[static_cast<long>(b) * 2 * C + c];
    p2 += ws[static_cast<long>(b) * 2 * C + C + c];
  }
  const float s1 = wave_sum(p1), s2 = wave_sum(p2);
  if (lane != 0) return;
  if (dgamma) dgamma[c] = accum ? dgamma[c] + s2 : s2;
  if (dbeta) dbeta[c] = accum ? dbeta[c] + s1 : s1;
  const float a = (gamma ? gamma[c] : 1.f) * invstd[c];
  coef[c] = a;                                   // a
  coef[C + c] = a * s1 / static_cast<float>(P);  // b
  coef[2 * C + c] = a * s2 / static_cast<float>(P);  // c
}

// dx = a*dyr - b - c*xhat ; dres = dyr (if requested)
__global__ void k_bn_bwd_apply(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                               const uint16_t* __restrict__ y, const float* __restrict__ mean,
                               const float* __restrict__ invstd, const float* __restrict__ coef, long nvec, int C,
                               int relu, uint16_t* __restrict__ dx, uint16_t* __restrict__ dres) {
  const int G = C / 8;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < nvec;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int g = static_cast<int>(i % G);
    float d[8], xv[8];
    load8(dy + i * 8, d);
    load8(x + i * 8, xv);
    if (relu) {
      float yv[8];
      load8(y + i * 8, yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = yv[j] > 0.f ? d[j] : 0.f;
    }
    u16x8 o, orr;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = g * 8 + j;
      const float xh = (xv[j] - mean[c]) * invstd[c];
      o[j] = f2bf(coef[c] * d[j] - coef[C + c] - coef[2 * C + c] * xh);
      orr[j] = f2bf(d[j]);
    }
    reinterpret_cast<u16x8*>(dx)[i] = o;
    if (dres) reinterpret_cast<u16x8*>(dres)[i] = orr;
  }
}

// ---------------------------------------------------------------------------------------------
// Two-kernel BatchNorm: the statistics pass finalizes in the same launch.  Grid = (row chunks) x (64-channel
// groups); every block stores its partials write-through (sc1), drains, and takes a per-channel-group ticket;
// the block that draws the last ticket acquires (agent scope) and combines that group's partials in fixed
// row-chunk order (deterministic) -- cdna_hip_programming.md §6 Guideline 16, recipe R1 in counter form.
// Saves the separate finalize launch in both directions (6 -> 4 kernels per BatchNorm layer).
constexpr int kBnCG = 64;       // channels per group: 8 channel-vector lanes x 8 channels
constexpr int kBnThreads = 512;  // 64 row lanes x 8 channel-vector lanes
constexpr int kBnRows = kBnThreads / 8;
constexpr int kBnQ = kBnThreads / kBnCG;  // lanes per (channel) in the finalizing combine
constexpr int kBnUnroll = 8;     // rows per lane per trip, all loads issued before the math

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// lite: an agent-coherent load (sc1) of data another block stored with st_sc1, instead of a plain load behind an
// agent acquire (buffer_inv sc1: the XCD's L1/L2 invalidated once per reading block)
__device__ __forceinline__ float ld_coh(const float* p, int lite) {
  return lite ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
}

// Block-collective tail shared by both passes: partial (s1, s2)[64] -> ws, ticket, and on the last arrival
// the per-channel totals over all row chunks in fixed order into tot1/tot2 (LDS).  Returns true on the block
// that finalizes.
// (1) the block's partial (s1, s2)[64] -> ws (write-through), every storing wave drained, barrier.
__device__ __forceinline__ void bn_store_partials(const float (&s1)[8], const float (&s2)[8], float* ws, int C,
                                                  float (*red)[kBnRows][kBnCG + 1]) {
  const int tid = threadIdx.x, tv = tid & 7, tr = tid >> 3;
  const int rb = blockIdx.x, cbase = blockIdx.y * kBnCG;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][tr][tv * 8 + j] = s1[j];
    red[1][tr][tv * 8 + j] = s2[j];
  }
  __syncthreads();
  if (tid < 2 * kBnCG) {
    const int which = tid / kBnCG, ch = tid % kBnCG;
    float v = 0.f;
    for (int r = 0; r < kBnRows; ++r) v += red[which][r][ch];
    if (cbase + ch < C) st_sc1(ws + (static_cast<long>(rb) * 2 + which) * C + cbase + ch, v);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// (2) the per-channel totals over all gridDim.x row chunks in fixed order -> tot1/tot2 (LDS; written by the
// first kBnCG threads, the caller synchronises).
__device__ __forceinline__ void bn_load_totals(const float* ws, int C, float (*red)[kBnRows][kBnCG + 1], float* tot1,
                                               float* tot2, int lite) {
  const int tid = threadIdx.x, nrb = gridDim.x, cbase = blockIdx.y * kBnCG;
  // kBnQ lanes per (which, channel) over the row chunks, combined in lane order
  {
    const int q = tid >> 6, ch = tid & 63;
    float a1 = 0.f, a2 = 0.f;
    if (cbase + ch < C) {
      // KT chunks per trip with all 2 KT loads issued before the adds (the tail is latency-bound): up to 256
      // chunks (kBnQ = 8 lanes per channel) in ONE round trip
      constexpr int KT = 32;
      int b = q;
      for (; b + (KT - 1) * kBnQ < nrb; b += KT * kBnQ) {
        float u1[KT], u2[KT];
#pragma unroll
        for (int k = 0; k < KT; ++k) {
          u1[k] = ld_coh(ws + (static_cast<long>(b + kBnQ * k) * 2) * C + cbase + ch, lite);
          u2[k] = ld_coh(ws + (static_cast<long>(b + kBnQ * k) * 2 + 1) * C + cbase + ch, lite);
        }
#pragma unroll
        for (int k = 0; k < KT; ++k) {
          a1 += u1[k];
          a2 += u2[k];
        }
      }
      for (; b + 7 * kBnQ < nrb; b += 8 * kBnQ) {
        float u1[8], u2[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          u1[k] = ld_coh(ws + (static_cast<long>(b + kBnQ * k) * 2) * C + cbase + ch, lite);
          u2[k] = ld_coh(ws + (static_cast<long>(b + kBnQ * k) * 2 + 1) * C + cbase + ch, lite);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          a1 += u1[k];
          a2 += u2[k];
        }
      }
      for (; b < nrb; b += kBnQ) {
        a1 += ld_coh(ws + (static_cast<long>(b) * 2) * C + cbase + ch, lite);
        a2 += ld_coh(ws + (static_cast<long>(b) * 2 + 1) * C + cbase + ch, lite);
      }
    }
    red[0][q][ch] = a1;
    red[1][q][ch] = a2;
  }
  __syncthreads();
  if (tid < kBnCG) {
    float v1 = red[0][0][tid], v2 = red[1][0][tid];
#pragma unroll
    for (int q = 1; q < kBnQ; ++q) {
      v1 += red[0][q][tid];
      v2 += red[1][q][tid];
    }
    tot1[tid] = v1;
    tot2[tid] = v2;
  }
}

// Block-collective tail shared by both passes: partials -> ws, ticket, and on the last arrival the per-channel
// totals over all row chunks in fixed order into tot1/tot2 (LDS).  Returns true on the block that finalizes.
__device__ __forceinline__ bool bn_partials_and_ticket(const float (&s1)[8], const float (&s2)[8], float* ws, int C,
                                                       int* ticket, float (*red)[kBnRows][kBnCG + 1], float* tot1,
                                                       float* tot2, int* s_last, int lite = 0) {
  const int tid = threadIdx.x, nrb = gridDim.x;
  bn_store_partials(s1, s2, ws, C, red);
  if (tid == 0) *s_last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nrb - 1;
  __syncthreads();
  if (!*s_last) return false;
  if (tid == 0) {
    if (!lite) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  bn_load_totals(ws, C, red, tot1, tot2, lite);
  if (tid == 0) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
  __syncthreads();
  return true;
}

__global__ __launch_bounds__(kBnThreads) void k_bn_stats_fin(const uint16_t* __restrict__ x, int P, int C, int rpb,
                                                      float* __restrict__ ws, int* __restrict__ tickets,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      float eps, float momentum, float* __restrict__ running_mean,
                                                      float* __restrict__ running_var, float* __restrict__ save_mean,
                                                      float* __restrict__ save_invstd, float* __restrict__ scale,
                                                      float* __restrict__ shift) {
  __shared__ float red[2][kBnRows][kBnCG + 1];
  __shared__ float tot1[kBnCG], tot2[kBnCG];
  __shared__ int s_last;
  const int tid = threadIdx.x, tv = tid & 7, tr = tid >> 3;
  const int c0 = blockIdx.y * kBnCG + tv * 8;
  const bool cok = c0 < C;
  float s1[8], s2[8], piv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = piv[j] = 0.f;
  if (cok) {
    load8(x + c0, piv);  // shift by row 0 (same pivot in every block)
    const int r1 = min(P, (blockIdx.x + 1) * rpb);
    int r = blockIdx.x * rpb + tr;
    constexpr int U = kBnUnroll;
    for (; r + (U - 1) * kBnRows < r1; r += U * kBnRows) {
      u16x8 u[U];
#pragma unroll
      for (int q = 0; q < U; ++q)
        u[q] = *reinterpret_cast<const u16x8*>(x + static_cast<long>(r + kBnRows * q) * C + c0);
#pragma unroll
      for (int q = 0; q < U; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = bf2f(u[q][j]) - piv[j]; s1[j] += d; s2[j] += d * d; }
    }
    for (; r < r1; r += kBnRows) {
      float v[8];
      load8(x + static_cast<long>(r) * C + c0, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[j] - piv[j]; s1[j] += d; s2[j] += d * d; }
    }
  }
  if (!bn_partials_and_ticket(s1, s2, ws, C, tickets + blockIdx.y, red, tot1, tot2, &s_last)) return;
  if (tid < kBnCG && blockIdx.y * kBnCG + tid < C) {
    const int c = blockIdx.y * kBnCG + tid;
    const double n = static_cast<double>(P);
    const double mean_s = static_cast<double>(tot1[tid]) / n;
    double var = static_cast<double>(tot2[tid]) / n - mean_s * mean_s;
    if (var < 0.0) var = 0.0;
    const float mean = static_cast<float>(mean_s) + bf2f(x[c]);
    const float invstd = rsqrtf(static_cast<float>(var) + eps);
    save_mean[c] = mean;
    save_invstd[c] = invstd;
    const float g = gamma ? gamma[c] : 1.f;
    const float b = beta ? beta[c] : 0.f;
    scale[c] = g * invstd;
    shift[c] = b - mean * g * invstd;
    if (running_mean) {
      const float unbiased = P > 1 ? static_cast<float>(var * n / (n - 1.0)) : static_cast<float>(var);
      running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
      running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
    }
  }
}

__global__ __launch_bounds__(kBnThreads) void k_bn_bwd_reduce_fin(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, const uint16_t* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, int P, int C, int rpb, int relu,
    float* __restrict__ ws, int* __restrict__ tickets, const float* __restrict__ gamma, float* __restrict__ dgamma,
    float* __restrict__ dbeta, int accum, float* __restrict__ coef) {
  __shared__ float red[2][kBnRows][kBnCG + 1];
  __shared__ float tot1[kBnCG], tot2[kBnCG];
  __shared__ int s_last;
  const int tid = threadIdx.x, tv = tid & 7, tr = tid >> 3;
  const int c0 = blockIdx.y * kBnCG + tv * 8;
  const bool cok = c0 < C;
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  if (cok) {
    float mu[8], is[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { mu[j] = mean[c0 + j]; is[j] = invstd[c0 + j]; }
    const int r1 = min(P, (blockIdx.x + 1) * rpb);
    int r = blockIdx.x * rpb + tr;
    constexpr int U = kBnUnroll / 2;  // 3 tensors per row: 12 x 16-B loads in flight per lane
    for (; r + (U - 1) * kBnRows < r1; r += U * kBnRows) {
      u16x8 ud[U], ux[U], uy[U];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const long off = static_cast<long>(r + kBnRows * q) * C + c0;
        ud[q] = *reinterpret_cast<const u16x8*>(dy + off);
        ux[q] = *reinterpret_cast<const u16x8*>(x + off);
        if (relu) uy[q] = *reinterpret_cast<const u16x8*>(y + off);
      }
#pragma unroll
      for (int q = 0; q < U; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float d = bf2f(ud[q][j]);
          if (relu && !(bf2f(uy[q][j]) > 0.f)) d = 0.f;
          s1[j] += d;
          s2[j] += d * (bf2f(ux[q][j]) - mu[j]) * is[j];
        }
    }
    for (; r < r1; r += kBnRows) {
      const long off = static_cast<long>(r) * C + c0;
      float d[8], xv[8];
      load8(dy + off, d);
      load8(x + off, xv);
      if (relu) {
        float yv[8];
        load8(y + off, yv);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = yv[j] > 0.f ? d[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) { s1[j] += d[j]; s2[j] += d[j] * (xv[j] - mu[j]) * is[j]; }
    }
  }
  if (!bn_partials_and_ticket(s1, s2, ws, C, tickets + blockIdx.y, red, tot1, tot2, &s_last)) return;
  if (tid < kBnCG && blockIdx.y * kBnCG + tid < C) {
    const int c = blockIdx.y * kBnCG + tid;
    const float t1 = tot1[tid], t2 = tot2[tid];
    if (dgamma) dgamma[c] = accum ? dgamma[c] + t2 : t2;
    if (dbeta) dbeta[c] = accum ? dbeta[c] + t1 : t1;
    const float a = (gamma ? gamma[c] : 1.f) * invstd[c];
    coef[c] = a;
    coef[C + c] = a * t1 / static_cast<float>(P);
    coef[2 * C + c] = a * t2 / static_cast<float>(P);
  }
}

// ---------------------------------------------------------------------------------------------
// ONE-launch BatchNorm (forward and backward): statistics pass -> per-channel-group ticket -> the group's
// last arriver finalizes and raises the group's generation flag -> every block of the group waits for the
// flag and applies the normalization (forward: y = relu?(x*scale + shift + res); backward: dx, dres) to its
// own row chunk.  Halves the BatchNorm launches of a ResNet-50 step (4 -> 2 per layer) and the apply pass
// re-reads a chunk its block has just streamed (L2).
//
// Co-residency: the grid is <= 256 blocks of 512 threads (bn_fin_grid) and the host caps it at 2 x CUs,
// one-per-CU capacity being ~4 blocks; a kernel on a stream starts only once its predecessor finished, so
// every block of the grid is resident and the waits complete.  Hand-off (cdna_hip_programming.md §6
// Guideline 16): finalizer plain stores -> every storing wave s_waitcnt vmcnt(0) -> barrier -> lane-0
// agent release -> s_waitcnt vmcnt(0) -> relaxed flag store; waiters: relaxed poll of the flag -> ONE agent
// acquire -> s_waitcnt vmcnt(0) -> barrier -> plain loads.  Flags are generation counters (read at kernel
// start, before the block's own ticket, hence before any increment of this launch), so they need no reset
// and hipGraph replays just count up.  Spins are bounded (2 s): a timeout sets the BatchNorm error word.
constexpr uint64_t kBnWaitTicks = 200000000ull;  // s_memrealtime 100 MHz: 2 s

// Lane 0 reads the group's generation at kernel start (the block reads s_gen after the next barrier).
__device__ __forceinline__ void bn_gen_start(const uint32_t* flag, uint32_t* s_gen) {
  if (threadIdx.x == 0) *s_gen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The finalizing block, after its threads stored the group's coefficients: publish generation gen + 1.
// lite: the hand-off data was stored write-through (st_sc1) and is read with agent-coherent loads (ld_sc1), so
// neither the L2 write-back (release) nor the L2 invalidate (acquire, one per waiting block) is issued.
__device__ __forceinline__ void bn_publish(uint32_t* flag, uint32_t gen, int lite) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (!lite) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(flag, gen + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Every other block of the group: wait (bounded) for generation gen + 1, then acquire.
__device__ __forceinline__ void bn_wait(const uint32_t* flag, uint32_t gen, int* err, int lite) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > kBnWaitTicks) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!lite) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}


// 8 consecutive channels of one row of the sum over z of fp32 slabs [splits][P*C] (z order).
__device__ __forceinline__ void slab_row8(const float* __restrict__ slabs, long zs, int splits, long off,
                                          float (&v)[8]) {
  const f32x4* p = reinterpret_cast<const f32x4*>(slabs + off);
  f32x4 a = p[0], b = p[1];
  // 4 slabs' loads in flight per trip, summed in slab order (a loop of one load pair per trip waited for each
  // pair in turn: `splits` dependent L2 round trips -- a 128 x 512 layer-4 BatchNorm reading 16 slabs took
  // 16.4 us at m = 8, r6e_prof_s2)
  int z = 1;
  for (; z + 3 < splits; z += 4) {
    f32x4 q[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4* r = reinterpret_cast<const f32x4*>(slabs + (z + u) * zs + off);
      q[u][0] = r[0];
      q[u][1] = r[1];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a += q[u][0];
      b += q[u][1];
    }
  }
  {  // the last 0..3 slabs: their loads issued together too (one more round trip, not up to three)
    const int rem = splits - z;
    f32x4 q[3][2];
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (u < rem) {
        const f32x4* r = reinterpret_cast<const f32x4*>(slabs + (z + u) * zs + off);
        q[u][0] = r[0];
        q[u][1] = r[1];
      }
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (u < rem) {
        a += q[u][0];
        b += q[u][1];
      }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = a[j];
    v[4 + j] = b[j];
  }
}

// Two rows' slab sums (the pivot row and a thread's first row) with both rows' loads of every 4-slab trip issued
// together: one chain of ceil(splits / 4) round trips instead of two.  Same slab order as slab_row8 (bitwise).
__device__ __forceinline__ void slab_2rows8(const float* __restrict__ slabs, long zs, int splits, long off0,
                                            long off1, bool ok1, float (&v0)[8], float (&v1)[8]) {
  const f32x4* p0 = reinterpret_cast<const f32x4*>(slabs + off0);
  const f32x4* p1 = reinterpret_cast<const f32x4*>(slabs + (ok1 ? off1 : off0));
  f32x4 a0 = p0[0], b0 = p0[1], a1 = p1[0], b1 = p1[1];
  int z = 1;
  for (; z + 3 < splits; z += 4) {
    f32x4 q[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4* r0 = reinterpret_cast<const f32x4*>(slabs + (z + u) * zs + off0);
      const f32x4* r1 = reinterpret_cast<const f32x4*>(slabs + (z + u) * zs + (ok1 ? off1 : off0));
      q[u][0] = r0[0];
      q[u][1] = r0[1];
      q[u][2] = r1[0];
      q[u][3] = r1[1];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a0 += q[u][0];
      b0 += q[u][1];
      a1 += q[u][2];
      b1 += q[u][3];
    }
  }
  {  // the last 0..3 slabs of both rows in one more round trip
    const int rem = splits - z;
    f32x4 q[3][4];
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (u < rem) {
        const f32x4* r0 = reinterpret_cast<const f32x4*>(slabs + (z + u) * zs + off0);
        const f32x4* r1 = reinterpret_cast<const f32x4*>(slabs + (z + u) * zs + (ok1 ? off1 : off0));
        q[u][0] = r0[0];
        q[u][1] = r0[1];
        q[u][2] = r1[0];
        q[u][3] = r1[1];
      }
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (u < rem) {
        a0 += q[u][0];
        b0 += q[u][1];
        a1 += q[u][2];
        b1 += q[u][3];
      }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v0[j] = a0[j];
    v0[4 + j] = b0[j];
    v1[j] = a1[j];
    v1[4 + j] = b1[j];
  }
}

// All-finalize variant of the hand-off (allfin): the last arrival at the ticket publishes the generation flag at
// once, and EVERY block then reads the chunk partials (agent-coherent loads) and derives the coefficients of its
// channel group itself, in the same fixed order -- identical values in every block.  The serial chain per launch
// is ticket -> flag -> partial loads instead of ticket -> partial loads -> coefficient stores (drained) -> flag ->
// coefficient loads.  Returns true on the last arrival, which writes the launch's global outputs.
__device__ __forceinline__ bool bn_partials_all(const float (&s1)[8], const float (&s2)[8], float* ws, int C,
                                                int* ticket, uint32_t* flag, uint32_t gen, int* err,
                                                float (*red)[kBnRows][kBnCG + 1], float* tot1, float* tot2,
                                                int* s_last) {
  const int tid = threadIdx.x, nrb = gridDim.x;
  bn_store_partials(s1, s2, ws, C, red);
  if (tid == 0) {
    const bool last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nrb - 1;
    if (last) {
      __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
      __hip_atomic_store(flag, gen + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > kBnWaitTicks) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *s_last = last ? 1 : 0;
  }
  __syncthreads();
  bn_load_totals(ws, C, red, tot1, tot2, 1);
  __syncthreads();
  return *s_last != 0;
}

// Tagged hand-off (mode bit 4): no ticket, no flag wait.  Every block stores its chunk partials as 64-bit words
// {value, tag = epoch + 1} (one single-copy-atomic store each, no drain) into the (group, channel group)'s own
// fixed region, and every block polls the region until all nrb x 2 x 64 words carry the tag -- the serial chain
// is one store + one load round trip.  epoch = the region's header word, read at kernel start; block 0, having
// seen every block's tagged partials (so every block has read the header), stores header = epoch + 1.  A region
// and its header are only ever written by launches that hold that slot, so every stale tag in it is <= the
// header: a tag equal to header + 1 is always this launch's.  Returns true on block 0 (the writer).
constexpr int kBnTagChunks = 128;                        // row chunks per region (nrb cap of the tagged mode)
constexpr int kBnTagWords = kBnTagChunks * 2 * kBnCG;    // 64-bit words per region

__device__ __forceinline__ uint64_t bn_tag_pack(float v, uint32_t tag) {
  return (static_cast<uint64_t>(tag) << 32) | __float_as_uint(v);
}

__device__ __forceinline__ bool bn_partials_tagged(const float (&s1)[8], const float (&s2)[8], uint64_t* parts, int C,
                                                   uint32_t* hdr, const uint32_t* s_epoch, int* err,
                                                   float (*red)[kBnRows][kBnCG + 1], float* tot1, float* tot2) {
  const int tid = threadIdx.x, tv = tid & 7, tr = tid >> 3;
  const int rb = blockIdx.x, nrb = gridDim.x, cbase = blockIdx.y * kBnCG;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][tr][tv * 8 + j] = s1[j];
    red[1][tr][tv * 8 + j] = s2[j];
  }
  __syncthreads();  // also publishes the epoch (bn_gen_start) to the block
  const uint32_t tag = *s_epoch + 1u;
  if (nrb == 1) {  // one row chunk (small tensors, bn_fin_grid): the block's own sums ARE the totals -- no hand-off
    if (tid < 2 * kBnCG) {
      const int which = tid / kBnCG, ch = tid % kBnCG;
      float v = 0.f;
      for (int r = 0; r < kBnRows; ++r) v += red[which][r][ch];
      (which ? tot2 : tot1)[ch] = v;
    }
    if (tid == 0) __hip_atomic_store(hdr, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    return true;
  }
  if (tid < 2 * kBnCG) {
    const int which = tid / kBnCG, ch = tid % kBnCG;
    float v = 0.f;
    for (int r = 0; r < kBnRows; ++r) v += red[which][r][ch];
    __hip_atomic_store(parts + (rb * 2 + which) * kBnCG + ch, bn_tag_pack(v, tag), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();  // red is reused below
  const int q = tid >> 6, ch = tid & 63;
  float a1 = 0.f, a2 = 0.f;
  if (cbase + ch < C) {
    constexpr int KT = 64 / kBnQ;  // 64 chunks per trip (one trip up to 64 chunks)
    const uint64_t pad = bn_tag_pack(0.f, tag);
    for (int b0 = q; b0 < nrb; b0 += KT * kBnQ) {
      uint64_t u1[KT], u2[KT];
#pragma unroll
      for (int k = 0; k < KT; ++k) {
        const int b = b0 + k * kBnQ;
        u1[k] = b < nrb ? __hip_atomic_load(parts + (b * 2) * kBnCG + ch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : pad;
        u2[k] = b < nrb ? __hip_atomic_load(parts + (b * 2 + 1) * kBnCG + ch, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT)
                        : pad;
      }
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        bool ok = true;
#pragma unroll
        for (int k = 0; k < KT; ++k) ok = ok && (u1[k] >> 32) == tag && (u2[k] >> 32) == tag;
        if (ok) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kBnWaitTicks) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int k = 0; k < KT; ++k) {
          const int b = b0 + k * kBnQ;
          if ((u1[k] >> 32) != tag)
            u1[k] = __hip_atomic_load(parts + (b * 2) * kBnCG + ch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((u2[k] >> 32) != tag)
            u2[k] = __hip_atomic_load(parts + (b * 2 + 1) * kBnCG + ch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
#pragma unroll
      for (int k = 0; k < KT; ++k) {
        a1 += __uint_as_float(static_cast<uint32_t>(u1[k]));
        a2 += __uint_as_float(static_cast<uint32_t>(u2[k]));
      }
    }
  }
  red[0][q][ch] = a1;
  red[1][q][ch] = a2;
  __syncthreads();
  if (tid < kBnCG) {
    float v1 = red[0][0][tid], v2 = red[1][0][tid];
#pragma unroll
    for (int qq = 1; qq < kBnQ; ++qq) {
      v1 += red[0][qq][tid];
      v2 += red[1][qq][tid];
    }
    tot1[tid] = v1;
    tot2[tid] = v2;
  }
  if (rb == 0 && tid == 0) __hip_atomic_store(hdr, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  return rb == 0;
}

// Grouped BatchNorm (blockIdx.z = group: the rows of G equal, contiguous micro-batches normalised with
// their OWN statistics in one launch -- a pipeline stage running several micro-batches per launch keeps the
// reference's per-micro-batch BatchNorm semantics, quirk Q17).  Quantities that combine the groups IN ORDER
// (running statistics: G sequential momentum updates; dgamma / dbeta: sum over groups) are finished by the
// last group's finalizer of each channel group: finalizer stores -> vmcnt(0) -> barrier -> lane-0 agent
// release + ticket; the last arrival acquires, resets the ticket and combines.  Returns true on that block.
__device__ __forceinline__ bool bn_group_last(int* gticket, int G, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const bool last = __hip_atomic_fetch_add(gticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(gticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    }
    *s_flag = last ? 1 : 0;
  }
  __syncthreads();
  return *s_flag != 0;
}

// RC > 0: a thread's rows of the chunk (<= RC of them) stay in registers from the statistics pass to the apply
// pass, and the residual rows are requested before the finalize wait (micro-batch sized tensors).
template <int RC>
__global__ __launch_bounds__(kBnThreads) void k_bn_fwd_fused(
    uint16_t* x, int P, int C, int rpb, float* __restrict__ ws, int* __restrict__ tickets,
    uint32_t* __restrict__ flags, int* __restrict__ err, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float momentum, float* __restrict__ running_mean,
    float* __restrict__ running_var, float* __restrict__ save_mean, float* __restrict__ save_invstd,
    float* __restrict__ scale, float* __restrict__ shift, const uint16_t* __restrict__ res, int relu,
    uint16_t* __restrict__ y, const float* __restrict__ slabs, int splits, long slab_zs,
    float* __restrict__ gvar, int* __restrict__ gtickets, int lite, uint64_t* __restrict__ parts) {
  __shared__ float red[2][kBnRows][kBnCG + 1];
  __shared__ float tot1[kBnCG], tot2[kBnCG], s_coef[2][kBnCG];
  __shared__ int s_last;
  __shared__ uint32_t s_gen;
  const int tid = threadIdx.x, tv = tid & 7, tr = tid >> 3;
  const int c0 = blockIdx.y * kBnCG + tv * 8;
  const bool cok = c0 < C;
  // group z: rows [z P, (z + 1) P) of x / res / y / slabs, its own partials, tickets, flags and statistics
  const int gz = blockIdx.z, G = gridDim.z;
  const float* save_mean_all = save_mean;
  {
    const long xo = static_cast<long>(gz) * P * C;
    x += xo;
    y += xo;
    if (res) res += xo;
    if (slabs) slabs += xo;
    ws += static_cast<long>(gz) * gridDim.x * 2 * C;
    tickets += gz * gridDim.y;
    flags += gz * gridDim.y;
    save_mean += gz * C;
    save_invstd += gz * C;
    scale += gz * 2 * C;
    shift += gz * 2 * C;
  }
  bn_gen_start(flags + blockIdx.y, &s_gen);
  const int r1 = min(P, (blockIdx.x + 1) * rpb);
  const int r0 = blockIdx.x * rpb + tr;
  float s1[8], s2[8], piv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = piv[j] = 0.f;
  u16x8 cx[RC > 0 ? RC : 1], cq[RC > 0 ? RC : 1];  // RC: the thread's x rows / residual rows
  if constexpr (RC > 0) {
    if (cok && slabs != nullptr) {
      float v0[8];  // the pivot (row 0) and the thread's first row: one batched chain of slab loads
      slab_2rows8(slabs, slab_zs, splits, c0, static_cast<long>(r0) * C + c0, r0 < r1, piv, v0);
#pragma unroll
      for (int j = 0; j < 8; ++j) piv[j] = bf2f(f2bf(piv[j]));
#pragma unroll
      for (int k = 0; k < RC; ++k) {
        const int r = r0 + k * kBnRows;
        if (r < r1) {
          float v[8];
          if (k == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = v0[j];
          } else {
            slab_row8(slabs, slab_zs, splits, static_cast<long>(r) * C + c0, v);
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            cx[k][j] = f2bf(v[j]);
            const float d = bf2f(cx[k][j]) - piv[j];
            s1[j] += d;
            s2[j] += d * d;
          }
          *reinterpret_cast<u16x8*>(x + static_cast<long>(r) * C + c0) = cx[k];
        }
      }
    } else if (cok) {
      load8(x + c0, piv);
#pragma unroll
      for (int k = 0; k < RC; ++k) {  // every load in flight, then the sums
        const int r = r0 + k * kBnRows;
        if (r < r1) cx[k] = *reinterpret_cast<const u16x8*>(x + static_cast<long>(r) * C + c0);
      }
#pragma unroll
      for (int k = 0; k < RC; ++k)
        if (r0 + k * kBnRows < r1)
#pragma unroll
          for (int j = 0; j < 8; ++j) { const float d = bf2f(cx[k][j]) - piv[j]; s1[j] += d; s2[j] += d * d; }
    }
    if (cok && res != nullptr) {  // independent of the statistics: requested before the finalize wait
#pragma unroll
      for (int k = 0; k < RC; ++k) {
        const int r = r0 + k * kBnRows;
        if (r < r1) cq[k] = *reinterpret_cast<const u16x8*>(res + static_cast<long>(r) * C + c0);
      }
    }
  } else if (cok && slabs != nullptr) {
    // x = bf16(sum_z slab_z) in z order (== the GEMM's own reduction), written here, its statistics taken
    // from the rounded values; the pivot (row 0) is recomputed from the slabs by every block
    const long zs = slab_zs;
    slab_row8(slabs, zs, splits, c0, piv);
#pragma unroll
    for (int j = 0; j < 8; ++j) piv[j] = bf2f(f2bf(piv[j]));  // the ROUNDED row 0, as the finalize uses it
    for (int r = blockIdx.x * rpb + tr; r < r1; r += kBnRows) {
      float v[8];
      slab_row8(slabs, zs, splits, static_cast<long>(r) * C + c0, v);
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = f2bf(v[j]);
        const float d = bf2f(o[j]) - piv[j];
        s1[j] += d;
        s2[j] += d * d;
      }
      *reinterpret_cast<u16x8*>(x + static_cast<long>(r) * C + c0) = o;  // x: written here, re-read below
    }
  } else if (cok) {
    load8(x + c0, piv);  // shift by row 0 (same pivot in every block)
    int r = blockIdx.x * rpb + tr;
    constexpr int U = kBnUnroll;
    for (; r + (U - 1) * kBnRows < r1; r += U * kBnRows) {
      u16x8 u[U];
#pragma unroll
      for (int q = 0; q < U; ++q) u[q] = *reinterpret_cast<const u16x8*>(x + static_cast<long>(r + kBnRows * q) * C + c0);
#pragma unroll
      for (int q = 0; q < U; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = bf2f(u[q][j]) - piv[j]; s1[j] += d; s2[j] += d * d; }
    }
    for (; r < r1; r += kBnRows) {
      float v[8];
      load8(x + static_cast<long>(r) * C + c0, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[j] - piv[j]; s1[j] += d; s2[j] += d * d; }
    }
  }
  // (bn_partials_and_ticket's first barrier also publishes s_gen to the block)
  // lite bit 0: fence-free hand-off; bit 1: every block finalizes its channel group (bn_partials_all); bit 2:
  // tagged partials (bn_partials_tagged, implies 1 and 2); bit 3: write-through outputs (st_vec)
  const bool tagged = (lite & 4) != 0, allfin = (lite & 2) != 0, wt = (lite & 8) != 0;
  lite &= 1;
  const bool writer =
      tagged ? bn_partials_tagged(s1, s2, parts + static_cast<long>(gz * gridDim.y + blockIdx.y) * kBnTagWords, C,
                                  flags + blockIdx.y, &s_gen, err, red, tot1, tot2)
      : allfin ? bn_partials_all(s1, s2, ws, C, tickets + blockIdx.y, flags + blockIdx.y, s_gen, err, red, tot1, tot2,
                                 &s_last)
               : bn_partials_and_ticket(s1, s2, ws, C, tickets + blockIdx.y, red, tot1, tot2, &s_last, lite);
  if (writer || allfin) {
    if (tid < kBnCG && blockIdx.y * kBnCG + tid < C) {
      const int c = blockIdx.y * kBnCG + tid;
      const double n = static_cast<double>(P);
      const double mean_s = static_cast<double>(tot1[tid]) / n;
      double var = static_cast<double>(tot2[tid]) / n - mean_s * mean_s;
      if (var < 0.0) var = 0.0;
      float pv;
      if (slabs != nullptr) {  // the pivot row of another block may not be visible yet: from the slabs
        float a = slabs[c];
        for (int z = 1; z < splits; ++z) a += slabs[z * slab_zs + c];
        pv = bf2f(f2bf(a));
      } else {
        pv = bf2f(x[c]);
      }
      const float mean = static_cast<float>(mean_s) + pv;
      const float invstd = rsqrtf(static_cast<float>(var) + eps);
      const float g = gamma ? gamma[c] : 1.f;
      const float b = beta ? beta[c] : 0.f;
      const float a_sc = g * invstd, a_sh = b - mean * g * invstd;
      s_coef[0][tid] = a_sc;
      s_coef[1][tid] = a_sh;
      if (writer) {  // the launch's global outputs: one block per (group, channel group)
        save_mean[c] = mean;
        save_invstd[c] = invstd;
        st_sc1(scale + c, a_sc);
        st_sc1(shift + c, a_sh);
        if (running_mean) {
          const float unbiased = P > 1 ? static_cast<float>(var * n / (n - 1.0)) : static_cast<float>(var);
          if (G == 1) {
            running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
            running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
          } else {
            gvar[gz * C + c] = unbiased;
          }
        }
      }
    }
    if (writer) {
      if (!allfin) bn_publish(flags + blockIdx.y, s_gen, lite);
      __syncthreads();
      // grouped: the last group's finalizer applies the G momentum updates in micro-batch order
      if (G > 1 && running_mean != nullptr && bn_group_last(gtickets + blockIdx.y, G, &s_last)) {
        if (tid < kBnCG && blockIdx.y * kBnCG + tid < C) {
          const int c = blockIdx.y * kBnCG + tid;
          float rm = running_mean[c], rv = running_var[c];
          for (int g = 0; g < G; ++g) {
            rm = (1.f - momentum) * rm + momentum * save_mean_all[g * C + c];
            rv = (1.f - momentum) * rv + momentum * gvar[g * C + c];
          }
          running_mean[c] = rm;
          running_var[c] = rv;
        }
      }
    }
    if (allfin) __syncthreads();  // s_coef
  } else {
    bn_wait(flags + blockIdx.y, s_gen, err, lite);
  }
  if (!cok) return;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = allfin ? s_coef[0][tv * 8 + j] : ld_coh(scale + c0 + j, lite);
    sh[j] = allfin ? s_coef[1][tv * 8 + j] : ld_coh(shift + c0 + j, lite);
  }
  if constexpr (RC > 0) {
#pragma unroll
    for (int k = 0; k < RC; ++k) {
      const int r = r0 + k * kBnRows;
      if (r < r1) {
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = bf2f(cx[k][j]) * sc[j] + sh[j];
          if (res) t += bf2f(cq[k][j]);
          if (relu) t = fmaxf(t, 0.f);
          o[j] = f2bf(t);
        }
        st_vec(reinterpret_cast<u16x8*>(y + static_cast<long>(r) * C + c0), o, wt);
      }
    }
    return;
  }
  int r = r0;
  constexpr int U = 4;
  for (; r + (U - 1) * kBnRows < r1; r += U * kBnRows) {
    u16x8 u[U], q[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long off = static_cast<long>(r + kBnRows * k) * C + c0;
      u[k] = *reinterpret_cast<const u16x8*>(x + off);
      if (res) q[k] = *reinterpret_cast<const u16x8*>(res + off);
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = bf2f(u[k][j]) * sc[j] + sh[j];
        if (res) t += bf2f(q[k][j]);
        if (relu) t = fmaxf(t, 0.f);
        o[j] = f2bf(t);
      }
      st_vec(reinterpret_cast<u16x8*>(y + static_cast<long>(r + kBnRows * k) * C + c0), o, wt);
    }
  }
  for (; r < r1; r += kBnRows) {
    const long off = static_cast<long>(r) * C + c0;
    float v[8], rv[8];
    load8(x + off, v);
    if (res) load8(res + off, rv);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = v[j] * sc[j] + sh[j];
      if (res) t += rv[j];
      if (relu) t = fmaxf(t, 0.f);
      o[j] = f2bf(t);
    }
    st_vec(reinterpret_cast<u16x8*>(y + off), o, wt);
  }
}

// ReLU mask of a BatchNorm output, recomputed from its INPUT when the forward had no residual: relu(x*sc+sh)
// > 0 <=> x*sc + sh > 0 with the forward's own fp32 scale/shift (ss) -- the backward then streams dy and x
// only, not y.  With a residual (the block's last BN) the saved y decides.
__device__ __forceinline__ void bn_relu_mask(const u16x8& ux, const uint16_t* __restrict__ y, long off,
                                             const float (&sc)[8], const float (&sh)[8], bool from_x,
                                             float (&d)[8]) {
  if (from_x) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (!(bf2f(ux[j]) * sc[j] + sh[j] > 0.f)) d[j] = 0.f;
  } else {
    const u16x8 uy = *reinterpret_cast<const u16x8*>(y + off);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (!(bf2f(uy[j]) > 0.f)) d[j] = 0.f;
  }
}

// RC > 0: a thread's rows of the chunk (<= RC of them) stay in registers between the statistics pass and the
// apply pass (micro-batch sized tensors), else the apply pass re-reads them (L2).
template <int RC>
__global__ __launch_bounds__(kBnThreads) void k_bn_bwd_fused(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, const uint16_t* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, int P, int C, int rpb, int relu,
    float* __restrict__ ws, int* __restrict__ tickets, uint32_t* __restrict__ flags, int* __restrict__ err,
    const float* __restrict__ gamma, float* __restrict__ dgamma, float* __restrict__ dbeta, int accum,
    float* __restrict__ coef, uint16_t* __restrict__ dx, uint16_t* __restrict__ dres,
    const float* __restrict__ ss, float* __restrict__ gdgb, int* __restrict__ gtickets, int lite,
    uint64_t* __restrict__ parts, const float* __restrict__ dys, int dysplits, long dyzs) {
  __shared__ float red[2][kBnRows][kBnCG + 1];
  __shared__ float tot1[kBnCG], tot2[kBnCG], s_coef[3][kBnCG];
  __shared__ int s_last;
  __shared__ uint32_t s_gen;
  const int tid = threadIdx.x, tv = tid & 7, tr = tid >> 3;
  const int c0 = blockIdx.y * kBnCG + tv * 8;
  const bool cok = c0 < C;
  const bool from_x = relu && ss != nullptr;
  // dys (RC > 0 only, host-checked): dy is the unreduced split-K slabs of the conv dgrad that produced it; the
  // thread's rows are summed here in slab order and rounded to bf16, the value the slab reduction would store
  const int gz = blockIdx.z, G = gridDim.z;  // group (see bn_group_last)
  {
    const long xo = static_cast<long>(gz) * P * C;
    dy += xo;
    if (dys) dys += xo;
    x += xo;
    if (y) y += xo;
    dx += xo;
    if (dres) dres += xo;
    mean += gz * C;
    invstd += gz * C;
    if (ss) ss += gz * 2 * C;
    ws += static_cast<long>(gz) * gridDim.x * 2 * C;
    tickets += gz * gridDim.y;
    flags += gz * gridDim.y;
    coef += gz * 3 * C;
  }
  bn_gen_start(flags + blockIdx.y, &s_gen);
  const int r0 = blockIdx.x * rpb + tr;
  const int r1 = min(P, (blockIdx.x + 1) * rpb);
  float s1[8], s2[8], mu[8], is[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = mu[j] = is[j] = sc[j] = sh[j] = 0.f;
  u16x8 cd[RC > 0 ? RC : 1], cx[RC > 0 ? RC : 1];
  if (cok) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { mu[j] = mean[c0 + j]; is[j] = invstd[c0 + j]; }
    if (from_x) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { sc[j] = ss[c0 + j]; sh[j] = ss[C + c0 + j]; }
    }
    if constexpr (RC > 0) {
#pragma unroll
      for (int k = 0; k < RC; ++k) {  // all of the thread's loads in flight, kept for the apply pass
        const int r = r0 + k * kBnRows;
        if (r < r1) {
          const long off = static_cast<long>(r) * C + c0;
          if (dys == nullptr) cd[k] = *reinterpret_cast<const u16x8*>(dy + off);
          cx[k] = *reinterpret_cast<const u16x8*>(x + off);
        }
      }
      if (dys != nullptr) {
#pragma unroll
        for (int k = 0; k < RC; ++k) {
          const int r = r0 + k * kBnRows;
          if (r < r1) {
            float v[8];
            slab_row8(dys, dyzs, dysplits, static_cast<long>(r) * C + c0, v);
#pragma unroll
            for (int j = 0; j < 8; ++j) cd[k][j] = f2bf(v[j]);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < RC; ++k) {
        const int r = r0 + k * kBnRows;
        if (r < r1) {
          float d[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) d[j] = bf2f(cd[k][j]);
          if (relu) bn_relu_mask(cx[k], y, static_cast<long>(r) * C + c0, sc, sh, from_x, d);
#pragma unroll
          for (int j = 0; j < 8; ++j) { s1[j] += d[j]; s2[j] += d[j] * (bf2f(cx[k][j]) - mu[j]) * is[j]; }
        }
      }
    } else {
      int r = r0;
      constexpr int U = kBnUnroll / 2;
      for (; r + (U - 1) * kBnRows < r1; r += U * kBnRows) {
        u16x8 ud[U], ux[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {
          const long off = static_cast<long>(r + kBnRows * q) * C + c0;
          ud[q] = *reinterpret_cast<const u16x8*>(dy + off);
          ux[q] = *reinterpret_cast<const u16x8*>(x + off);
        }
#pragma unroll
        for (int q = 0; q < U; ++q) {
          float d[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) d[j] = bf2f(ud[q][j]);
          if (relu) bn_relu_mask(ux[q], y, static_cast<long>(r + kBnRows * q) * C + c0, sc, sh, from_x, d);
#pragma unroll
          for (int j = 0; j < 8; ++j) { s1[j] += d[j]; s2[j] += d[j] * (bf2f(ux[q][j]) - mu[j]) * is[j]; }
        }
      }
      for (; r < r1; r += kBnRows) {
        const long off = static_cast<long>(r) * C + c0;
        const u16x8 ud = *reinterpret_cast<const u16x8*>(dy + off);
        const u16x8 ux = *reinterpret_cast<const u16x8*>(x + off);
        float d[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = bf2f(ud[j]);
        if (relu) bn_relu_mask(ux, y, off, sc, sh, from_x, d);
#pragma unroll
        for (int j = 0; j < 8; ++j) { s1[j] += d[j]; s2[j] += d[j] * (bf2f(ux[j]) - mu[j]) * is[j]; }
      }
    }
  }
  // lite bit 0: fence-free hand-off; bit 1: every block finalizes its channel group (bn_partials_all); bit 2:
  // tagged partials (bn_partials_tagged, implies 1 and 2); bit 3: write-through outputs (st_vec)
  const bool tagged = (lite & 4) != 0, allfin = (lite & 2) != 0, wt = (lite & 8) != 0;
  lite &= 1;
  const bool writer =
      tagged ? bn_partials_tagged(s1, s2, parts + static_cast<long>(gz * gridDim.y + blockIdx.y) * kBnTagWords, C,
                                  flags + blockIdx.y, &s_gen, err, red, tot1, tot2)
      : allfin ? bn_partials_all(s1, s2, ws, C, tickets + blockIdx.y, flags + blockIdx.y, s_gen, err, red, tot1, tot2,
                                 &s_last)
               : bn_partials_and_ticket(s1, s2, ws, C, tickets + blockIdx.y, red, tot1, tot2, &s_last, lite);
  if (writer || allfin) {
    if (tid < kBnCG && blockIdx.y * kBnCG + tid < C) {
      const int c = blockIdx.y * kBnCG + tid;
      const float t1 = tot1[tid], t2 = tot2[tid];
      const float a = (gamma ? gamma[c] : 1.f) * invstd[c];
      const float a1 = a * t1 / static_cast<float>(P), a2 = a * t2 / static_cast<float>(P);
      s_coef[0][tid] = a;
      s_coef[1][tid] = a1;
      s_coef[2][tid] = a2;
      if (writer) {  // the launch's global outputs: one block per (group, channel group)
        if (G == 1) {
          if (dgamma) dgamma[c] = accum ? dgamma[c] + t2 : t2;
          if (dbeta) dbeta[c] = accum ? dbeta[c] + t1 : t1;
        } else {
          gdgb[gz * 2 * C + c] = t2;
          gdgb[gz * 2 * C + C + c] = t1;
        }
        st_sc1(coef + c, a);
        st_sc1(coef + C + c, a1);
        st_sc1(coef + 2 * C + c, a2);
      }
    }
    if (writer) {
      if (!allfin) bn_publish(flags + blockIdx.y, s_gen, lite);
      __syncthreads();
      // grouped: dgamma / dbeta = sum over the groups in group order, by the last group's finalizer
      if (G > 1 && bn_group_last(gtickets + blockIdx.y, G, &s_last)) {
        if (tid < kBnCG && blockIdx.y * kBnCG + tid < C) {
          const int c = blockIdx.y * kBnCG + tid;
          float t2 = 0.f, t1 = 0.f;
          for (int g = 0; g < G; ++g) {
            t2 += gdgb[g * 2 * C + c];
            t1 += gdgb[g * 2 * C + C + c];
          }
          if (dgamma) dgamma[c] = accum ? dgamma[c] + t2 : t2;
          if (dbeta) dbeta[c] = accum ? dbeta[c] + t1 : t1;
        }
      }
    }
    if (allfin) __syncthreads();  // s_coef
  } else {
    bn_wait(flags + blockIdx.y, s_gen, err, lite);
  }
  if (!cok) return;
  float ca[8], cb[8], cc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ca[j] = allfin ? s_coef[0][tv * 8 + j] : ld_coh(coef + c0 + j, lite);
    cb[j] = allfin ? s_coef[1][tv * 8 + j] : ld_coh(coef + C + c0 + j, lite);
    cc[j] = allfin ? s_coef[2][tv * 8 + j] : ld_coh(coef + 2 * C + c0 + j, lite);
  }
  auto apply = [&](const u16x8& ud, const u16x8& ux, long off) {
    float d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = bf2f(ud[j]);
    if (relu) bn_relu_mask(ux, y, off, sc, sh, from_x, d);
    u16x8 o, orr;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xh = (bf2f(ux[j]) - mu[j]) * is[j];
      o[j] = f2bf(ca[j] * d[j] - cb[j] - cc[j] * xh);
      orr[j] = f2bf(d[j]);
    }
    st_vec(reinterpret_cast<u16x8*>(dx + off), o, wt);
    if (dres) st_vec(reinterpret_cast<u16x8*>(dres + off), orr, wt);
  };
  if constexpr (RC > 0) {
#pragma unroll
    for (int k = 0; k < RC; ++k) {
      const int r = r0 + k * kBnRows;
      if (r < r1) apply(cd[k], cx[k], static_cast<long>(r) * C + c0);
    }
  } else {
    for (int r = r0; r < r1; r += kBnRows) {
      const long off = static_cast<long>(r) * C + c0;
      apply(*reinterpret_cast<const u16x8*>(dy + off), *reinterpret_cast<const u16x8*>(x + off), off);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Max pooling, NHWC, any C (scalar channel loop for C % 8 != 0, the MNIST CNN's 10 / 20 channels).
// Saves the argmax window index (uint8) for the backward gather.
__global__ void k_maxpool_fwd(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, uint8_t* __restrict__ idx,
                              int N, int H, int W, int C, int Ho, int Wo, int k, int s, int p, int relu) {
  const long total = static_cast<long>(N) * Ho * Wo * C;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(i % C);
    long t = i / C;
    const int ox = static_cast<int>(t % Wo);
    t /= Wo;
    const int oy = static_cast<int>(t % Ho);
    const int n = static_cast<int>(t / Ho);
    float best = -INFINITY;
    int bi = 0;
    for (int ky = 0; ky < k; ++ky) {
      const int iy = oy * s - p + ky;
      if (iy < 0 || iy >= H) continue;
      for (int kx = 0; kx < k; ++kx) {
        const int ix = ox * s - p + kx;
        if (ix < 0 || ix >= W) continue;
        const float v = bf2f(x[((static_cast<long>(n) * H + iy) * W + ix) * C + c]);
        if (v > best) { best = v; bi = ky * k + kx; }
      }
    }
    if (relu) best = fmaxf(best, 0.f);
    y[i] = f2bf(best);
    idx[i] = static_cast<uint8_t>(bi);
  }
}

// 8-channel forms (C % 8 == 0, every ResNet pooling): one thread per (pixel, 8-channel group) with 16-byte
// activation and 8-byte argmax accesses; same window order and tie rule as the scalar kernels.
__global__ void k_maxpool_fwd8(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, uint8_t* __restrict__ idx,
                               int N, int H, int W, int C, int Ho, int Wo, int k, int s, int p, int relu) {
  const int G = C / 8;
  const long total = static_cast<long>(N) * Ho * Wo * G;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int g = static_cast<int>(i % G);
    long t = i / G;
    const int ox = static_cast<int>(t % Wo);
    t /= Wo;
    const int oy = static_cast<int>(t % Ho);
    const int n = static_cast<int>(t / Ho);
    float best[8];
    int bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    for (int ky = 0; ky < k; ++ky) {
      const int iy = oy * s - p + ky;
      if (iy < 0 || iy >= H) continue;
      for (int kx = 0; kx < k; ++kx) {
        const int ix = ox * s - p + kx;
        if (ix < 0 || ix >= W) continue;
        const u16x8 u = *reinterpret_cast<const u16x8*>(x + ((static_cast<long>(n) * H + iy) * W + ix) * C + g * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = bf2f(u[j]);
          if (v > best[j]) { best[j] = v; bi[j] = ky * k + kx; }
        }
      }
    }
    u16x8 o;
    unsigned long long packed = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = f2bf(relu ? fmaxf(best[j], 0.f) : best[j]);
      packed |= static_cast<unsigned long long>(bi[j] & 0xff) << (8 * j);
    }
    reinterpret_cast<u16x8*>(y)[i] = o;
    reinterpret_cast<unsigned long long*>(idx)[i] = packed;
  }
}

__global__ void k_maxpool_bwd8(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
                               const uint8_t* __restrict__ idx, uint16_t* __restrict__ dx, int N, int H, int W, int C,
                               int Ho, int Wo, int k, int s, int p, int relu) {
  const int G = C / 8;
  const long total = static_cast<long>(N) * H * W * G;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int g = static_cast<int>(i % G);
    long t = i / G;
    const int ix = static_cast<int>(t % W);
    t /= W;
    const int iy = static_cast<int>(t % H);
    const int n = static_cast<int>(t / H);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    const int oy_lo = max(0, (iy + p - k + s) / s), oy_hi = min(Ho - 1, (iy + p) / s);
    const int ox_lo = max(0, (ix + p - k + s) / s), ox_hi = min(Wo - 1, (ix + p) / s);
    for (int oy = oy_lo; oy <= oy_hi; ++oy) {
      const int ky = iy + p - oy * s;
      if (ky < 0 || ky >= k) continue;
      for (int ox = ox_lo; ox <= ox_hi; ++ox) {
        const int kx = ix + p - ox * s;
        if (kx < 0 || kx >= k) continue;
        const long o8 = ((static_cast<long>(n) * Ho + oy) * Wo + ox) * G + g;  // 8-channel group index
        const unsigned long long id = reinterpret_cast<const unsigned long long*>(idx)[o8];
        const u16x8 d = reinterpret_cast<const u16x8*>(dy)[o8];
        u16x8 yv;
        if (relu) yv = reinterpret_cast<const u16x8*>(y)[o8];
        const unsigned int tap = static_cast<unsigned int>(ky * k + kx);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (((id >> (8 * j)) & 0xff) == tap && (!relu || bf2f(yv[j]) > 0.f)) acc[j] += bf2f(d[j]);
        }
      }
    }
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
    reinterpret_cast<u16x8*>(dx)[i] = o;
  }
}

// Gather form: each input element sums the grads of the outputs whose argmax it is (deterministic).
__global__ void k_maxpool_bwd(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
                              const uint8_t* __restrict__ idx, uint16_t* __restrict__ dx, int N, int H, int W, int C,
                              int Ho, int Wo, int k, int s, int p, int relu) {
  const long total = static_cast<long>(N) * H * W * C;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(i % C);
    long t = i / C;
    const int ix = static_cast<int>(t % W);
    t /= W;
    const int iy = static_cast<int>(t % H);
    const int n = static_cast<int>(t / H);
    float acc = 0.f;
    // outputs oy with oy*s - p <= iy <= oy*s - p + k - 1
    const int oy_lo = max(0, (iy + p - k + s) / s), oy_hi = min(Ho - 1, (iy + p) / s);
    const int ox_lo = max(0, (ix + p - k + s) / s), ox_hi = min(Wo - 1, (ix + p) / s);
    for (int oy = oy_lo; oy <= oy_hi; ++oy) {
      const int ky = iy + p - oy * s;
      if (ky < 0 || ky >= k) continue;
      for (int ox = ox_lo; ox <= ox_hi; ++ox) {
        const int kx = ix + p - ox * s;
        if (kx < 0 || kx >= k) continue;
        const long o = ((static_cast<long>(n) * Ho + oy) * Wo + ox) * C + c;
        if (idx[o] == ky * k + kx) {
          if (!relu || bf2f(y[o]) > 0.f) acc += bf2f(dy[o]);
        }
      }
    }
    dx[i] = f2bf(acc);
  }
}

// Global average pool NHWC [N][HW][C] -> [N][C] (bf16 out), one thread per (n, c-group of 8).
__global__ void k_avgpool_fwd(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int N, int HW, int C) {
  const int G = C / 8;
  const long total = static_cast<long>(N) * G;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int g = static_cast<int>(i % G);
    const int n = static_cast<int>(i / G);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int q = 0; q < HW; ++q) {
      float v[8];
      load8(x + (static_cast<long>(n) * HW + q) * C + g * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
    u16x8 o;
    const float inv = 1.f / static_cast<float>(HW);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j] * inv);
    reinterpret_cast<u16x8*>(y)[i] = o;
  }
}

__global__ void k_avgpool_bwd(const uint16_t* __restrict__ dy, uint16_t* __restrict__ dx, int N, int HW, int C) {
  const int G = C / 8;
  const long total = static_cast<long>(N) * HW * G;
  const float inv = 1.f / static_cast<float>(HW);
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int g = static_cast<int>(i % G);
    const int n = static_cast<int>(i / (static_cast<long>(HW) * G));
    float v[8];
    load8(dy + static_cast<long>(n) * C + g * 8, v);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j] * inv);
    reinterpret_cast<u16x8*>(dx)[i] = o;
  }
}

// ---------------------------------------------------------------------------------------------
// Dropout.  Counter-based hash RNG (splitmix64 of seed ^ element id): deterministic for a given
// (seed, offset), no state.  Channel mode (Dropout2d): one draw per (n, c) of an NHWC tensor.
__device__ __forceinline__ float uniform01(unsigned long long seed, unsigned long long id) {
  unsigned long long z = seed + 0x9E3779B97F4A7C15ULL * (id + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return static_cast<float>(z >> 40) * (1.0f / 16777216.0f);
}

// mode 0: elementwise on [n_elems]; mode 1: channel mask over NHWC with (HW, C).
// mask out (uint8) is written so backward is a pure multiply.  The seed is (*counter, salt): the
// counter lives in device memory and is advanced by k_rng_advance after every call, so a captured
// hipGraph draws fresh masks on every replay.
__global__ void k_dropout_fwd(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, uint8_t* __restrict__ mask,
                              long n, int mode, int HW, int C, float p, const unsigned long long* counter,
                              unsigned long long salt) {
  const unsigned long long seed = counter[0] * 0xD1B54A32D192ED03ULL + salt;
  const float scale = 1.f / (1.f - p);
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    unsigned long long id;
    if (mode == 0) {
      id = static_cast<unsigned long long>(i);
    } else {
      const long c = i % C;
      const long nimg = i / (static_cast<long>(HW) * C);
      id = static_cast<unsigned long long>(nimg * C + c);
    }
    const bool keep = uniform01(seed, id) >= p;
    mask[i] = keep ? 1 : 0;
    y[i] = keep ? f2bf(bf2f(x[i]) * scale) : uint16_t(0);
  }
}

__global__ void k_rng_advance(unsigned long long* counter) { counter[0] += 1; }

__global__ void k_dropout_bwd(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ mask,
                              uint16_t* __restrict__ dx, long n, float p) {
  const float scale = 1.f / (1.f - p);
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<long>(gridDim.x) * blockDim.x)
    dx[i] = mask[i] ? f2bf(bf2f(dy[i]) * scale) : uint16_t(0);
}

// ---------------------------------------------------------------------------------------------
// EmbeddingBag (mode=sum): one wave per bag, lanes over the embedding dim.
// EmbeddingBag (sum mode), one wave per bag.  For D <= 32 the wave splits into G = 64 / Dp lane groups
// (Dp = D rounded up to a power of two): group g sums indices s+g, s+g+G, ... and the groups are combined
// with a fixed xor-shuffle tree, so every lane works and the result is deterministic.
__global__ void k_embbag_fwd(const float* __restrict__ w, const int64_t* __restrict__ idx,
                             const int64_t* __restrict__ off, int B, long L, int D, int Dp,
                             float* __restrict__ out) {
  const int bag = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (bag >= B) return;  // wave-uniform
  const long s = off[bag];
  const long e = bag + 1 < B ? off[bag + 1] : L;
  if (Dp <= 32) {
    const int G = 64 / Dp, g = lane / Dp, d = lane % Dp;
    float acc = 0.f;
    if (d < D)
      for (long j = s + g; j < e; j += G) acc += w[idx[j] * D + d];
    for (int m = Dp; m < 64; m <<= 1) acc += __shfl_xor(acc, m);
    if (g == 0 && d < D) out[static_cast<long>(bag) * D + d] = acc;
    return;
  }
  for (int d = lane; d < D; d += 64) {
    float acc = 0.f;
    for (long j = s; j < e; ++j) acc += w[idx[j] * D + d];
    out[static_cast<long>(bag) * D + d] = acc;
  }
}

// dW[r, :] += sum over positions j with idx[j] == r (increasing j) of dy[bag(j), :] -- deterministic: one
// wave owns table row r, ballots the matching positions 64 at a time and adds them in index order (the bag
// of a position by binary search over the offsets).  O(rows x L) scanning: used for parameter-server-sized
// tables (host picks k_embbag_bwd_atomic beyond that).
__global__ void k_embbag_bwd_det(const float* __restrict__ dy, const int64_t* __restrict__ idx,
                                 const int64_t* __restrict__ off, int B, long L, int D, long rows,
                                 float* __restrict__ dw) {
  const long row = static_cast<long>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;  // wave-uniform
  float acc[4] = {0.f, 0.f, 0.f, 0.f};  // D <= 256: lane d, d + 64, d + 128, d + 192
  for (long base = 0; base < L; base += 64) {
    const long j = base + lane;
    unsigned long long m = __ballot(j < L && idx[j] == row);
    while (m) {
      const int bit = __ffsll(static_cast<long long>(m)) - 1;
      m &= m - 1;
      const long jj = base + bit;
      int lo = 0, hi = B - 1;  // last bag with off[bag] <= jj
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= jj) lo = mid;
        else hi = mid - 1;
      }
      const float* src = dy + static_cast<long>(lo) * D;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (lane + 64 * q < D) acc[q] += src[lane + 64 * q];
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (lane + 64 * q < D) dw[row * D + lane + 64 * q] += acc[q];
}

// Large tables: dW[idx[j], :] += dy[bag(j), :] with fp32 atomics (order-dependent rounding).
__global__ void k_embbag_bwd_atomic(const float* __restrict__ dy, const int64_t* __restrict__ idx,
                                    const int64_t* __restrict__ off, int B, long L, int D, float* __restrict__ dw) {
  const int bag = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (bag >= B) return;
  const long s = off[bag];
  const long e = bag + 1 < B ? off[bag + 1] : L;
  for (long j = s; j < e; ++j)
    for (int d = lane; d < D; d += 64) atomicAdd(dw + idx[j] * D + d, dy[static_cast<long>(bag) * D + d]);
}

int bn_blocks(int P, int C, int& rows_per_block) {
  const int G = C / 8;
  // ~8 16-byte vectors per thread (enough loads in flight per lane with the unrolled loops), at most
  // 1024 blocks (4 per CU); the fp32 partials stay <= C/4096 of the activation bytes
  const long vecs = static_cast<long>(P) * G;
  long nb = (vecs + 256L * 8 - 1) / (256L * 8);
  if (nb > 1024) nb = 1024;
  if (nb > P) nb = P;
  int nblk = static_cast<int>(nb);
  if (nblk < 1) nblk = 1;
  rows_per_block = ceil_div(P, nblk);
  nblk = ceil_div(P, rows_per_block);
  return nblk;
}

}  // namespace

// Fused-finalize grid: row chunks x 64-channel groups, ~256 blocks of 512 threads, >= 64 rows per chunk, <= 64 chunks (r2i: 128 chunks
// made the finalizing tail 0.14 ms/step slower; 64 chunks measure level with the 3-pass form at 106 fewer
// launches per step)
// (the finalizing block reads chunks x 2 x 64 partials).
int bn_resident_cap();
int bn_fin_grid(int P, int C, int& rpb, int groups = 1) {
  const int ncg = (C + kBnCG - 1) / kBnCG;
  // r3af (tagged hand-off): 64 -> 128 chunks, ResNet-50 3.328 -> 3.284 ms (the C <= 128 layers get 128-256 blocks)
  static const int kChunks = std::getenv("PDE_BN_CHUNKS") ? std::atoi(std::getenv("PDE_BN_CHUNKS")) : 128;
  // r2m sweep at 512 threads per block: 256 blocks (one per CU, 8 waves) 3.83 -> 3.79 ms/step
  static const int kBlocks = std::getenv("PDE_BN_BLOCKS") ? std::atoi(std::getenv("PDE_BN_BLOCKS")) : 256;
  const int target = std::min(bn_resident_cap(), kBlocks);  // (side-stream headroom may change at run time)
  int nrb = std::max(1, std::min(kChunks, target / (ncg * groups)));
  nrb = std::min(nrb, std::max(1, P / kBnRows));
  // r5 (opt-in): tensors of <= PDE_BN_SINGLE_ROWS rows per group take ONE row chunk per channel group -- the block
  // reads all rows of its 64 channels and needs no cross-block exchange.  Measured slower at every threshold
  // (profiles/r5m_bench.jsonl: 512 / 1024 / 2048 rows, ResNet-50 3.227 -> 3.31 / 3.31 / 4.30 ms, stage 2 at m = 8
  // 1.497 -> 1.77 ms): the exchange of 16-128 blocks is cheaper than one block streaming every row.  Default off.
  static const int kSingleRows = std::getenv("PDE_BN_SINGLE_ROWS") ? std::atoi(std::getenv("PDE_BN_SINGLE_ROWS")) : 0;
  if (P <= kSingleRows) nrb = 1;
  rpb = ceil_div(P, nrb);
  return ceil_div(P, rpb);
}

// Per-channel-group arrival counters: one zeroed array per device, handed out in a rolling window (each
// launch leaves its counters at 0).  Allocated on the first call outside a graph capture; until then (or
// with PDE_BN_3PASS=1) BatchNorm uses the separate finalize kernels.
int* bn_ticket_base(hipStream_t s, int** err) {
  constexpr int kSlots = 1 << 20;
  static int* base[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (base[dev] == nullptr) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return nullptr;
    void* p = nullptr;
    const size_t bytes = sizeof(int) * (kSlots + 64);  // + the error word of the one-launch kernels
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(p);
      return nullptr;
    }
    base[dev] = static_cast<int*>(p);
  }
  if (err != nullptr) *err = base[dev] + kSlots;
  return base[dev];
}

// Rolling windows over the zeroed array: [0, kHalf) arrival tickets (every launch leaves them at 0), [kHalf,
// kSlots) generation flags of the one-launch kernels (any value; never handed out as tickets).
int* bn_window(int n, hipStream_t s, int which) {
  constexpr int kSlots = 1 << 20, kHalf = kSlots / 2;
  static int next[64][2] = {};
  static const bool off = std::getenv("PDE_BN_3PASS") != nullptr;
  if (off || n > kHalf) return nullptr;
  int* base = bn_ticket_base(s, nullptr);
  if (base == nullptr) return nullptr;
  int dev = 0;
  (void)hipGetDevice(&dev);
  int& nx = next[dev][which];
  if (nx + n > kHalf) nx = 0;
  int* t = base + which * kHalf + nx;
  nx += n;
  return t;
}
// Tagged hand-off regions (bn_partials_tagged): kBnTagSlots fixed (header, region) pairs, zeroed once, handed
// out in a rolling window of n consecutive slots.  A slot's region is only written by launches holding that slot.
constexpr int kBnTagSlots = 2048;  // x 128 KB
uint64_t* bn_tag_slots(int n, hipStream_t s, uint32_t** hdr) {
  static uint64_t* parts[64] = {};
  static uint32_t* hdrs[64] = {};
  static int next[64] = {};
  int dev = 0;
  if (n > kBnTagSlots || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (parts[dev] == nullptr) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return nullptr;
    const size_t pb = sizeof(uint64_t) * kBnTagWords * kBnTagSlots, hb = sizeof(uint32_t) * kBnTagSlots;
    void* p = nullptr;
    void* h = nullptr;
    if (hipMalloc(&p, pb) != hipSuccess) return nullptr;
    if (hipMalloc(&h, hb) != hipSuccess || hipMemset(p, 0, pb) != hipSuccess || hipMemset(h, 0, hb) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(p);
      if (h != nullptr) (void)hipFree(h);
      return nullptr;
    }
    parts[dev] = static_cast<uint64_t*>(p);
    hdrs[dev] = static_cast<uint32_t*>(h);
  }
  int& nx = next[dev];
  if (nx + n > kBnTagSlots) nx = 0;
  *hdr = hdrs[dev] + nx;
  uint64_t* r = parts[dev] + static_cast<long>(nx) * kBnTagWords;
  nx += n;
  return r;
}

int* bn_tickets(int n, hipStream_t s) { return bn_window(n, s, 0); }
uint32_t* bn_flags(int n, hipStream_t s) { return reinterpret_cast<uint32_t*>(bn_window(n, s, 1)); }

// One-launch BatchNorm (k_bn_fwd_fused / k_bn_bwd_fused): on unless PDE_BN_FUSED=0, and only for grids the
// chip holds at once (every block must be resident for the flag waits).  The cap is measured, not assumed:
// the smallest hipOccupancyMaxActiveBlocksPerMultiprocessor over every k_bn_*_fused<RC> instantiation (the
// register-resident RC = 4 / 8 / 16 variants hold 169-256 VGPRs: ONE 512-thread block per CU) times the CU
// count, minus PDE_BN_HEADROOM blocks (default 0) left for kernels that other streams keep spinning (ring
// sends waiting for credit, an overlapped RCCL all-reduce).  A hand-off that still times out sets the error
// word, which every sync point reads (ops.functional.check_device_errors) and raises on.
// Blocks that kernels on OTHER streams of this process may keep resident while a one-launch BatchNorm runs --
// spinning side-stream kernels (a pipeline's ring sends waiting for credit, an overlapped RCCL all-reduce,
// bn_reserve_headroom) -- subtracted from the resident cap, so the BatchNorm grid shrinks (more rows per block)
// instead of waiting on blocks that cannot be placed.
std::atomic<int> g_bn_headroom{0};
std::atomic<long> g_bn_one_launches{0}, g_bn_multi_launches{0};
std::atomic<int> g_bn_last_grid{0};

int bn_resident_base() {
  static int base = -1;
  if (base < 0) {
    int dev = 0, cus = 1;
    hipDeviceProp_t prop{};
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      cus = prop.multiProcessorCount;
    int occ = 1 << 20;
    auto q = [&occ](const void* fn) {
      int n = 0;
      occ = (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kBnThreads, 0) == hipSuccess)
                ? std::min(occ, n) : std::min(occ, 1);
    };
    q(reinterpret_cast<const void*>(&k_bn_fwd_fused<0>));
    q(reinterpret_cast<const void*>(&k_bn_fwd_fused<4>));
    q(reinterpret_cast<const void*>(&k_bn_fwd_fused<8>));
    q(reinterpret_cast<const void*>(&k_bn_fwd_fused<16>));
    q(reinterpret_cast<const void*>(&k_bn_bwd_fused<0>));
    q(reinterpret_cast<const void*>(&k_bn_bwd_fused<4>));
    q(reinterpret_cast<const void*>(&k_bn_bwd_fused<8>));
    q(reinterpret_cast<const void*>(&k_bn_bwd_fused<16>));
    const int headroom = std::getenv("PDE_BN_HEADROOM") ? std::max(0, std::atoi(std::getenv("PDE_BN_HEADROOM"))) : 0;
    base = std::max(1, std::max(1, occ) * cus - headroom);
  }
  return base;
}
int bn_resident_cap() { return std::max(0, bn_resident_base() - g_bn_headroom.load()); }

bool bn_one_launch(int blocks) {
  static const bool off = std::getenv("PDE_BN_FUSED") != nullptr && std::getenv("PDE_BN_FUSED")[0] == '0';
  // refused up front when the grid cannot be resident beside the reserved side-stream blocks: the caller runs
  // the multi-launch BatchNorm instead of a flag wait that would time out
  const bool ok = !off && blocks <= bn_resident_cap();
  if (ok) {
    ++g_bn_one_launches;
    g_bn_last_grid = blocks;
  } else {
    ++g_bn_multi_launches;
  }
  return ok;
}

// flag hand-off without the agent-scope L2 write-back / invalidate (see bn_publish); r3w: ResNet-50
// 3.875 -> 3.760 ms/step.  PDE_BN_LITE=0: the fenced hand-off.
// Every block finalizes its channel group (bn_partials_all), r3y: 3.77 -> 3.50 ms/step; PDE_BN_ALLFIN=0: one
// finalizing block per channel group publishing the coefficients.
int bn_lite_sync() {
  static const int lite = !(std::getenv("PDE_BN_LITE") != nullptr && std::getenv("PDE_BN_LITE")[0] == '0');
  static const int allfin = !(std::getenv("PDE_BN_ALLFIN") != nullptr && std::getenv("PDE_BN_ALLFIN")[0] == '0');
  // bit 3: the normalised outputs / data gradients stored write-through (PDE_BN_WT=0 off) -- r4m: level; r5z, three
  // alternating pairs: ResNet-50 3.131 -> 3.124 ms, stage 1 g4 1.545 -> 1.516 ms, stage 2 g4 level, stage 2 m8
  // 1.352 -> 1.359 ms (profiles/r5z_bn_writethrough_ab.txt)
  static const int wt = !(std::getenv("PDE_BN_WT") != nullptr && std::getenv("PDE_BN_WT")[0] == '0');
  return (lite ? (allfin ? 3 : 1) : 0) | (wt ? 8 : 0);
}
// Chunks of 5..8 rows per thread also stay in registers between the passes (RC = 8), r3ac: ResNet-50
// 3.337 -> 3.319 ms/step (3 of 3 pairs); PDE_BN_RC8=0: off.
bool bn_rc8_on() {
  static const bool on = !(std::getenv("PDE_BN_RC8") != nullptr && std::getenv("PDE_BN_RC8")[0] == '0');
  return on;
}
// PDE_BN_RC16=1: chunks of 9..16 rows per thread in registers too (the stem's BatchNorm at batch 32); r3al:
// level or slightly slower (3.251 -> 3.260 ms), so off by default
bool bn_rc16_on() {
  static const bool on = std::getenv("PDE_BN_RC16") != nullptr && std::getenv("PDE_BN_RC16")[0] == '1';
  return on;
}
// Tagged partials (bn_partials_tagged) where the grid allows (<= kBnTagChunks row chunks), r3aa: ResNet-50
// 3.52 -> 3.34 ms/step; PDE_BN_TAGGED=0: the ticket + flag hand-off.
bool bn_tagged_on() {
  static const bool on = !(std::getenv("PDE_BN_TAGGED") != nullptr && std::getenv("PDE_BN_TAGGED")[0] == '0');
  return on;
}

const long kBnApplyCap = std::getenv("PDE_BN_APPLY_CAP") ? std::atol(std::getenv("PDE_BN_APPLY_CAP")) : 2048;

int bn_workspace_blocks(int P, int C, int groups) {
  int rpb;
  const int one = std::max(bn_blocks(P, C, rpb), bn_fin_grid(P, C, rpb));
  if (groups <= 1 || P % groups != 0) return one;
  const int Pg = P / groups;
  return std::max({one, groups * bn_fin_grid(Pg, C, rpb, groups), bn_blocks(Pg, C, rpb), bn_fin_grid(Pg, C, rpb)});
}

hipError_t bn_fwd_train(const uint16_t* x, int P, int C, const float* gamma, const float* beta, float eps,
                        float momentum, float* running_mean, float* running_var, float* save_mean,
                        float* save_invstd, float* scale_shift, float* ws, const uint16_t* res, int relu,
                        uint16_t* y, hipStream_t s, const float* slabs, int splits, int groups, float* gscratch) {
  int rpb;
  const int ncg = ceil_div(C, kBnCG);
  int* err = nullptr;
  if (groups < 1 || P % groups != 0) return hipErrorInvalidValue;
  const int Pg = P / groups;  // rows per group (micro-batch)
  const int nrb1 = bn_fin_grid(Pg, C, rpb, groups);
  if (splits <= 1) slabs = nullptr;
  if (bn_one_launch(nrb1 * ncg * groups) && bn_ticket_base(s, &err) != nullptr) {
    int* tk = bn_tickets(ncg * groups, s);
    uint32_t* fl = bn_flags(ncg * groups, s);  // generation flags of the (group, channel group)s
    int* gt = groups > 1 ? bn_tickets(ncg, s) : nullptr;
    int mode = bn_lite_sync();
    uint64_t* parts = nullptr;
    if ((mode & 7) == 3 && bn_tagged_on() && nrb1 <= kBnTagChunks) {
      uint32_t* hdr = nullptr;
      parts = bn_tag_slots(ncg * groups, s, &hdr);
      if (parts != nullptr) {
        fl = hdr;  // the slots' headers are the epochs
        mode = 7 | (mode & 8);
      }
    }
    if (tk != nullptr && fl != nullptr && (groups == 1 || (gt != nullptr && gscratch != nullptr))) {
      // rows per thread of a chunk: few enough -> kept in registers for the apply pass (PDE_BN_FWD_RC=0: off)
      static const bool rc_on = !(std::getenv("PDE_BN_FWD_RC") && std::getenv("PDE_BN_FWD_RC")[0] == '0');
      if (rc_on && ceil_div(rpb, kBnRows) <= 4)
        hipLaunchKernelGGL(k_bn_fwd_fused<4>, dim3(nrb1, ncg, groups), dim3(kBnThreads), 0, s,
                           const_cast<uint16_t*>(x), Pg, C, rpb, ws, tk, fl, err, gamma, beta, eps, momentum,
                           running_mean, running_var, save_mean, save_invstd, scale_shift, scale_shift + C, res,
                           relu, y, slabs, splits, static_cast<long>(P) * C, gscratch, gt, mode, parts);
      else if (rc_on && bn_rc8_on() && ceil_div(rpb, kBnRows) <= 8)
        hipLaunchKernelGGL(k_bn_fwd_fused<8>, dim3(nrb1, ncg, groups), dim3(kBnThreads), 0, s,
                           const_cast<uint16_t*>(x), Pg, C, rpb, ws, tk, fl, err, gamma, beta, eps, momentum,
                           running_mean, running_var, save_mean, save_invstd, scale_shift, scale_shift + C, res,
                           relu, y, slabs, splits, static_cast<long>(P) * C, gscratch, gt, mode, parts);
      else if (rc_on && bn_rc16_on() && ceil_div(rpb, kBnRows) <= 16)
        hipLaunchKernelGGL(k_bn_fwd_fused<16>, dim3(nrb1, ncg, groups), dim3(kBnThreads), 0, s,
                           const_cast<uint16_t*>(x), Pg, C, rpb, ws, tk, fl, err, gamma, beta, eps, momentum,
                           running_mean, running_var, save_mean, save_invstd, scale_shift, scale_shift + C, res,
                           relu, y, slabs, splits, static_cast<long>(P) * C, gscratch, gt, mode, parts);
      else
        hipLaunchKernelGGL(k_bn_fwd_fused<0>, dim3(nrb1, ncg, groups), dim3(kBnThreads), 0, s,
                           const_cast<uint16_t*>(x), Pg, C, rpb, ws, tk, fl, err, gamma, beta, eps, momentum,
                           running_mean, running_var, save_mean, save_invstd, scale_shift, scale_shift + C, res,
                           relu, y, slabs, splits, static_cast<long>(P) * C, gscratch, gt, mode, parts);
      return hipGetLastError();
    }
  }
  if (slabs != nullptr) {  // multi-launch BatchNorm: reduce the conv's slabs into x first
    const hipError_t e = gemm_reduce_slabs_bf16(const_cast<float*>(slabs), splits, P, C, const_cast<uint16_t*>(x), s);
    if (e != hipSuccess) return e;
  }
  if (groups > 1) {  // grouped, multi-launch: one BatchNorm per group in order (running stats sequential)
    for (int g = 0; g < groups; ++g) {
      const long xo = static_cast<long>(g) * Pg * C;
      const hipError_t e = bn_fwd_train(x + xo, Pg, C, gamma, beta, eps, momentum, running_mean, running_var,
                                        save_mean + g * C, save_invstd + g * C, scale_shift + 2 * g * C, ws,
                                        res ? res + xo : nullptr, relu, y + xo, s, nullptr, 1, 1, nullptr);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  int* tk = bn_tickets(ncg, s);
  if (tk != nullptr) {
    const int nrb = bn_fin_grid(P, C, rpb);
    hipLaunchKernelGGL(k_bn_stats_fin, dim3(nrb, ncg), dim3(kBnThreads), 0, s, x, P, C, rpb, ws, tk, gamma,
                       beta, eps, momentum, running_mean, running_var, save_mean, save_invstd, scale_shift,
                       scale_shift + C);
  } else {
    const int nblk = bn_blocks(P, C, rpb);
    hipLaunchKernelGGL(k_bn_stats, dim3(nblk), dim3(256), 0, s, x, P, C, rpb, ws);
    hipLaunchKernelGGL(k_bn_finalize, dim3(ceil_div(C, 4)), dim3(256), 0, s, x, ws, nblk, P, C, gamma, beta, eps,
                       momentum, running_mean, running_var, save_mean, save_invstd, scale_shift, scale_shift + C);
  }
  const long nvec = static_cast<long>(P) * C / 8;
  // (grid cap swept 2048 / 4096 / 8192 blocks: level, r2m)
  hipLaunchKernelGGL(k_bn_apply, dim3(stream_grid(nvec, 256, 1, kBnApplyCap)), dim3(256), 0, s, x, scale_shift,
                     scale_shift + C, res, y, nvec, C, relu);
  return hipGetLastError();
}

int bn_error(int reset) {
  int* err = nullptr;
  if (bn_ticket_base(nullptr, &err) == nullptr || err == nullptr) return 0;
  int v = 0;
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&v, err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  if (reset && v != 0) (void)hipMemset(err, 0, sizeof(int));
  return v;
}

hipError_t bn_apply(const uint16_t* x, int P, int C, const float* scale, const float* shift, const uint16_t* res,
                    int relu, uint16_t* y, hipStream_t s) {
  const long nvec = static_cast<long>(P) * C / 8;
  hipLaunchKernelGGL(k_bn_apply, dim3(stream_grid(nvec, 256)), dim3(256), 0, s, x, scale, shift, res, y, nvec, C,
                     relu);
  return hipGetLastError();
}

hipError_t bn_bwd(const uint16_t* dy, const uint16_t* x, const uint16_t* y, const float* mean, const float* invstd,
                  const float* gamma, int P, int C, int relu, float* dgamma, float* dbeta, int accum_params, float* ws,
                  float* coef, uint16_t* dx, uint16_t* dres, hipStream_t s, const float* ss, int groups,
                  float* gscratch, const float* dys, int dysplits) {
  int rpb;
  const int ncg = ceil_div(C, kBnCG);
  int* err = nullptr;
  if (groups < 1 || P % groups != 0) return hipErrorInvalidValue;
  const int Pg = P / groups;
  const int nrb1 = bn_fin_grid(Pg, C, rpb, groups);
  if (dysplits <= 1) dys = nullptr;
  const bool one = bn_one_launch(nrb1 * ncg * groups) && bn_ticket_base(s, &err) != nullptr;
  if (dys != nullptr && !(one && ceil_div(rpb, kBnRows) <= 4)) {
    // only the register-resident one-launch kernel sums dy from the slabs: reduce them into dy first
    const hipError_t e = gemm_reduce_slabs_bf16(const_cast<float*>(dys), dysplits, P, C, const_cast<uint16_t*>(dy), s);
    if (e != hipSuccess) return e;
    dys = nullptr;
  }
  if (one) {
    int* tk = bn_tickets(ncg * groups, s);
    uint32_t* fl = bn_flags(ncg * groups, s);
    int* gt = groups > 1 ? bn_tickets(ncg, s) : nullptr;
    int mode = bn_lite_sync();
    uint64_t* parts = nullptr;
    if ((mode & 7) == 3 && bn_tagged_on() && nrb1 <= kBnTagChunks) {
      uint32_t* hdr = nullptr;
      parts = bn_tag_slots(ncg * groups, s, &hdr);
      if (parts != nullptr) {
        fl = hdr;
        mode = 7 | (mode & 8);
      }
    }
    if (tk != nullptr && fl != nullptr && (groups == 1 || (gt != nullptr && gscratch != nullptr))) {
      const dim3 grid(nrb1, ncg, groups);
      // rows per thread of a chunk: small enough -> kept in registers for the apply pass
      if (ceil_div(rpb, kBnRows) <= 4)
        hipLaunchKernelGGL(k_bn_bwd_fused<4>, grid, dim3(kBnThreads), 0, s, dy, x, y, mean, invstd, Pg, C, rpb, relu,
                           ws, tk, fl, err, gamma, dgamma, dbeta, accum_params, coef, dx, dres, ss, gscratch, gt, mode, parts,
                           dys, dysplits, static_cast<long>(P) * C);
      else if (bn_rc8_on() && ceil_div(rpb, kBnRows) <= 8)
        hipLaunchKernelGGL(k_bn_bwd_fused<8>, grid, dim3(kBnThreads), 0, s, dy, x, y, mean, invstd, Pg, C, rpb, relu,
                           ws, tk, fl, err, gamma, dgamma, dbeta, accum_params, coef, dx, dres, ss, gscratch, gt, mode, parts,
                           nullptr, 1, 0L);
      else if (bn_rc16_on() && ceil_div(rpb, kBnRows) <= 16)
        hipLaunchKernelGGL(k_bn_bwd_fused<16>, grid, dim3(kBnThreads), 0, s, dy, x, y, mean, invstd, Pg, C, rpb, relu,
                           ws, tk, fl, err, gamma, dgamma, dbeta, accum_params, coef, dx, dres, ss, gscratch, gt, mode, parts,
                           nullptr, 1, 0L);
      else
        hipLaunchKernelGGL(k_bn_bwd_fused<0>, grid, dim3(kBnThreads), 0, s, dy, x, y, mean, invstd, Pg, C, rpb, relu,
                           ws, tk, fl, err, gamma, dgamma, dbeta, accum_params, coef, dx, dres, ss, gscratch, gt, mode, parts,
                           nullptr, 1, 0L);
      return hipGetLastError();
    }
  }
  if (dys != nullptr) {  // (the one-launch kernel could not be launched after all)
    const hipError_t e = gemm_reduce_slabs_bf16(const_cast<float*>(dys), dysplits, P, C, const_cast<uint16_t*>(dy), s);
    if (e != hipSuccess) return e;
    dys = nullptr;
  }
  if (groups > 1) {  // grouped, multi-launch: group 0 writes / adds the parameter gradients, the rest add
    for (int g = 0; g < groups; ++g) {
      const long xo = static_cast<long>(g) * Pg * C;
      const hipError_t e = bn_bwd(dy + xo, x + xo, y ? y + xo : nullptr, mean + g * C, invstd + g * C, gamma, Pg, C,
                                  relu, dgamma, dbeta, g > 0 ? 1 : accum_params, ws, coef + 3 * g * C, dx + xo,
                                  dres ? dres + xo : nullptr, s, ss ? ss + 2 * g * C : nullptr, 1, nullptr);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  int* tk = bn_tickets(ncg, s);
  if (tk != nullptr) {
    const int nrb = bn_fin_grid(P, C, rpb);
    hipLaunchKernelGGL(k_bn_bwd_reduce_fin, dim3(nrb, ncg), dim3(kBnThreads), 0, s, dy, x, y, mean, invstd,
                       P, C, rpb, relu, ws, tk, gamma, dgamma, dbeta, accum_params, coef);
  } else {
    const int nblk = bn_blocks(P, C, rpb);
    hipLaunchKernelGGL(k_bn_bwd_reduce, dim3(nblk), dim3(256), 0, s, dy, x, y, mean, invstd, P, C, rpb, relu, ws);
    hipLaunchKernelGGL(k_bn_bwd_finalize, dim3(ceil_div(C, 4)), dim3(256), 0, s, ws, nblk, P, C, gamma, invstd,
                       dgamma, dbeta, accum_params, coef);
  }
  const long nvec = static_cast<long>(P) * C / 8;
  hipLaunchKernelGGL(k_bn_bwd_apply, dim3(stream_grid(nvec, 256, 1, kBnApplyCap)), dim3(256), 0, s, dy, x, y, mean,
                     invstd, coef, nvec, C, relu, dx, dres);
  return hipGetLastError();
}

hipError_t maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo,
                       int k, int st, int p, int relu, hipStream_t s) {
  const long total = static_cast<long>(N) * Ho * Wo * C;
  if (C % 8 == 0 && k * k <= 256) {
    hipLaunchKernelGGL(k_maxpool_fwd8, dim3(stream_grid(total / 8, 256)), dim3(256), 0, s, x, y, idx, N, H, W, C, Ho,
                       Wo, k, st, p, relu);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_maxpool_fwd, dim3(stream_grid(total, 256)), dim3(256), 0, s, x, y, idx, N, H, W, C, Ho, Wo,
                     k, st, p, relu);
  return hipGetLastError();
}
hipError_t maxpool_bwd(const uint16_t* dy, const uint16_t* y, const uint8_t* idx, uint16_t* dx, int N, int H, int W,
                       int C, int Ho, int Wo, int k, int st, int p, int relu, hipStream_t s) {
  const long total = static_cast<long>(N) * H * W * C;
  if (C % 8 == 0 && k * k <= 256) {
    hipLaunchKernelGGL(k_maxpool_bwd8, dim3(stream_grid(total / 8, 256)), dim3(256), 0, s, dy, y, idx, dx, N, H, W,
                       C, Ho, Wo, k, st, p, relu);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_maxpool_bwd, dim3(stream_grid(total, 256)), dim3(256), 0, s, dy, y, idx, dx, N, H, W, C, Ho,
                     Wo, k, st, p, relu);
  return hipGetLastError();
}
hipError_t avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t s) {
  const long total = static_cast<long>(N) * (C / 8);
  hipLaunchKernelGGL(k_avgpool_fwd, dim3(stream_grid(total, 256)), dim3(256), 0, s, x, y, N, HW, C);
  return hipGetLastError();
}
hipError_t avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t s) {
  const long total = static_cast<long>(N) * HW * (C / 8);
  hipLaunchKernelGGL(k_avgpool_bwd, dim3(stream_grid(total, 256)), dim3(256), 0, s, dy, dx, N, HW, C);
  return hipGetLastError();
}
hipError_t dropout_fwd(const uint16_t* x, uint16_t* y, uint8_t* mask, long n, int mode, int HW, int C, float p,
                       unsigned long long* counter, unsigned long long salt, hipStream_t s) {
  hipLaunchKernelGGL(k_dropout_fwd, dim3(stream_grid(n, 256)), dim3(256), 0, s, x, y, mask, n, mode, HW, C, p,
                     counter, salt);
  hipLaunchKernelGGL(k_rng_advance, dim3(1), dim3(1), 0, s, counter);
  return hipGetLastError();
}
hipError_t dropout_bwd(const uint16_t* dy, const uint8_t* mask, uint16_t* dx, long n, float p, hipStream_t s) {
  hipLaunchKernelGGL(k_dropout_bwd, dim3(stream_grid(n, 256)), dim3(256), 0, s, dy, mask, dx, n, p);
  return hipGetLastError();
}
hipError_t embbag_fwd(const float* w, const int64_t* idx, const int64_t* off, int B, long L, int D, float* out,
                      hipStream_t s) {
  int Dp = 1;
  while (Dp < D) Dp <<= 1;
  hipLaunchKernelGGL(k_embbag_fwd, dim3(ceil_div(B, 4)), dim3(256), 0, s, w, idx, off, B, L, D, Dp, out);
  return hipGetLastError();
}
hipError_t embbag_bwd(const float* dy, const int64_t* idx, const int64_t* off, int B, long L, int D, float* dw,
                      long rows, hipStream_t s) {
  if (D <= 256 && rows > 0 && rows * L <= (1L << 26)) {  // deterministic row-owner scan
    hipLaunchKernelGGL(k_embbag_bwd_det, dim3(static_cast<unsigned>((rows + 3) / 4)), dim3(256), 0, s, dy, idx, off,
                       B, L, D, rows, dw);
  } else {
    hipLaunchKernelGGL(k_embbag_bwd_atomic, dim3(ceil_div(B, 4)), dim3(256), 0, s, dy, idx, off, B, L, D, dw);
  }
  return hipGetLastError();
}

int bn_reserve_headroom(int blocks) {
  const int v = g_bn_headroom.fetch_add(blocks) + blocks;
  if (v < 0) g_bn_headroom = 0;
  return bn_resident_cap();
}

int bn_headroom_reserved() { return g_bn_headroom.load(); }

void bn_launch_stats(long* one, long* multi, int* last_grid, int* cap) {
  *one = g_bn_one_launches.load();
  *multi = g_bn_multi_launches.load();
  *last_grid = g_bn_last_grid.load();
  *cap = bn_resident_cap();
}

}  // namespace pde
