// Memory-bound layout / cast / reduction kernels (gfx950).  All loads are vectorised (8 x bf16 or
// 4 x f32 per lane, cdna_hip_programming.md Guideline 13) and grids are capped grid-stride loops
// (Guideline 11).
#include <algorithm>

#include "common.cuh"
#include "pde_kernels.h"

namespace pde {

namespace {

// Strided row cast with an optional trailing ones column (element (r, cols)).
__global__ void k_cast_rows_bf16(const float* __restrict__ in, int rows, int cols, uint16_t* __restrict__ out,
                                 int ldo, int ones) {
  const long n = static_cast<long>(rows) * (cols + 1);
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int r = static_cast<int>(i / (cols + 1)), c = static_cast<int>(i - static_cast<long>(r) * (cols + 1));
    if (c < cols) out[static_cast<long>(r) * ldo + c] = f2bf(in[static_cast<long>(r) * cols + c]);
    else if (ones) out[static_cast<long>(r) * ldo + c] = f2bf(1.f);
  }
}

__global__ void k_cast_f32_bf16(const float* __restrict__ in, uint16_t* __restrict__ out, long n) {
  const long nv = n / 8;
  const long stride = static_cast<long>(gridDim.x) * blockDim.x;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < nv; i += stride) {
    const f32x4 a = reinterpret_cast<const f32x4*>(in)[2 * i];
    const f32x4 b = reinterpret_cast<const f32x4*>(in)[2 * i + 1];
    u16x8 o;
    o[0] = f2bf(a[0]); o[1] = f2bf(a[1]); o[2] = f2bf(a[2]); o[3] = f2bf(a[3]);
    o[4] = f2bf(b[0]); o[5] = f2bf(b[1]); o[6] = f2bf(b[2]); o[7] = f2bf(b[3]);
    reinterpret_cast<u16x8*>(out)[i] = o;
  }
  for (long i = nv * 8 + blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < n; i += stride)
    out[i] = f2bf(in[i]);
}

__global__ void k_cast_bf16_f32(const uint16_t* __restrict__ in, float* __restrict__ out, long n) {
  const long nv = n / 8;
  const long stride = static_cast<long>(gridDim.x) * blockDim.x;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < nv; i += stride) {
    const u16x8 v = reinterpret_cast<const u16x8*>(in)[i];
    f32x4 a, b;
    a[0] = bf2f(v[0]); a[1] = bf2f(v[1]); a[2] = bf2f(v[2]); a[3] = bf2f(v[3]);
    b[0] = bf2f(v[4]); b[1] = bf2f(v[5]); b[2] = bf2f(v[6]); b[3] = bf2f(v[7]);
    reinterpret_cast<f32x4*>(out)[2 * i] = a;
    reinterpret_cast<f32x4*>(out)[2 * i + 1] = b;
  }
  for (long i = nv * 8 + blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < n; i += stride)
    out[i] = bf2f(in[i]);
}

// One thread per output 8-channel group of one pixel.
__global__ void k_nchw_to_nhwc(const float* __restrict__ in, uint16_t* __restrict__ out, int N, int C,
                               int H, int W, int Cp) {
  const int groups = Cp / 8;
  const long total = static_cast<long>(N) * H * W * groups;
  const long HW = static_cast<long>(H) * W;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int g = static_cast<int>(i % groups);
    const long pix = i / groups;
    const int n = static_cast<int>(pix / HW);
    const long hw = pix - n * HW;
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = g * 8 + j;
      o[j] = c < C ? f2bf(in[(static_cast<long>(n) * C + c) * HW + hw]) : uint16_t(0);
    }
    reinterpret_cast<u16x8*>(out)[i] = o;
  }
}

__global__ void k_conv_w_fwd(const float* __restrict__ w, uint16_t* __restrict__ out, int Co, int Ci,
                             int R, int S, int Cp, int Cop) {
  const long total = static_cast<long>(Cop) * R * S * Cp;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(i % Cp);
    long t = i / Cp;
    const int s = static_cast<int>(t % S);
    t /= S;
    const int r = static_cast<int>(t % R);
    const int co = static_cast<int>(t / R);
    out[i] = (c < Ci && co < Co) ? f2bf(w[((static_cast<long>(co) * Ci + c) * R + r) * S + s]) : uint16_t(0);
  }
}

// out[ci][r][s][co] = w[co][ci][r][s]   (padded to [Cip][R][S][Cop] with zeros)
__global__ void k_conv_w_dgrad(const float* __restrict__ w, uint16_t* __restrict__ out, int Co, int Ci,
                               int R, int S, int Cip, int Cop) {
  const long total = static_cast<long>(Cop) * R * S * Cip;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int co = static_cast<int>(i % Cop);
    long t = i / Cop;
    const int s = static_cast<int>(t % S);
    t /= S;
    const int r = static_cast<int>(t % R);
    const int ci = static_cast<int>(t / R);
    out[i] = (co < Co && ci < Ci) ? f2bf(w[((static_cast<long>(co) * Ci + ci) * R + r) * S + s]) : uint16_t(0);
  }
}

// Multi-tensor form of k_conv_w_fwd + k_conv_w_dgrad: blockIdx.y = table entry (block-uniform), the x
// blocks grid-stride over (co, ci) pairs; each thread walks the pair's R*S taps (one contiguous run of
// the OIHW source).  The forward pass puts ci on consecutive lanes, the dgrad pass co, so both passes store
// 2-byte elements that are contiguous across the wave (the second pass re-reads the source from L2).
// One (co, ci) pair: all RS taps loaded before any store (RS_T = 9: the 3x3 fast path, 0: runtime RS).
template <int RS_T>
__device__ __forceinline__ void conv_w_pair(const float* __restrict__ src, uint16_t* __restrict__ dst, long dstride,
                                            int RS, bool ok) {
  if constexpr (RS_T > 0) {
    float v[RS_T];
#pragma unroll
    for (int t = 0; t < RS_T; ++t) v[t] = ok ? src[t] : 0.f;
#pragma unroll
    for (int t = 0; t < RS_T; ++t) dst[t * dstride] = f2bf(v[t]);
  } else {
    for (int t = 0; t < RS; ++t) dst[t * dstride] = ok ? f2bf(src[t]) : uint16_t(0);
  }
}

template <int RS_T>
__device__ __forceinline__ void conv_w_layouts_entry(const ConvLayoutEntry& e) {
  const int RS = e.R * e.S;
  const long pairs = static_cast<long>(e.Cop) * e.Cp;
  const long start = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x;
  const long stride = static_cast<long>(gridDim.x) * blockDim.x;
  for (long i = start; i < pairs; i += stride) {  // fwd [co][r][s][ci]: ci fastest
    const int ci = static_cast<int>(i % e.Cp), co = static_cast<int>(i / e.Cp);
    const bool ok = ci < e.Ci && co < e.Co;
    conv_w_pair<RS_T>(e.w + (static_cast<long>(co) * e.Ci + ci) * RS, e.fwd + static_cast<long>(co) * RS * e.Cp + ci,
                      e.Cp, RS, ok);
  }
  for (long i = start; i < pairs; i += stride) {  // dgrad [ci][r][s][co]: co fastest
    const int co = static_cast<int>(i % e.Cop), ci = static_cast<int>(i / e.Cop);
    const bool ok = ci < e.Ci && co < e.Co;
    conv_w_pair<RS_T>(e.w + (static_cast<long>(co) * e.Ci + ci) * RS,
                      e.dgrad + static_cast<long>(ci) * RS * e.Cop + co, e.Cop, RS, ok);
  }
}

// 3x3 fast path: a (32 co x 32 ci) tile of one weight is transposed through LDS.  The fp32 source rows
// (ci, r, s contiguous per co) are read coalesced; both bf16 layouts are written as 64-byte runs
// (fwd: ci contiguous, dgrad: co contiguous).  Padded channels come out as zeros.
constexpr int kCwTile = 32;
__device__ __forceinline__ void conv_w_layouts_tiled3x3(const ConvLayoutEntry& e) {
  constexpr int RS = 9;
  __shared__ float tile[RS][kCwTile][kCwTile + 1];
  const int tco = (e.Cop + kCwTile - 1) / kCwTile, tci = (e.Cp + kCwTile - 1) / kCwTile;
  for (int t = blockIdx.x; t < tco * tci; t += gridDim.x) {
    const int co0 = (t / tci) * kCwTile, ci0 = (t % tci) * kCwTile;
    // all 36 loads of a thread in flight before the LDS stores (a rolled loop waited one global round trip
    // per element: ~50 us per ResNet-50 step for this kernel)
    constexpr int kPer = kCwTile * kCwTile * RS / 256;
    static_assert(kCwTile * kCwTile * RS % 256 == 0, "whole loads per thread at 256 threads");
    float v[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int q = threadIdx.x + u * 256;
      const int col = q / (kCwTile * RS), rem = q - col * (kCwTile * RS);
      const int cil = rem / RS, tap = rem - cil * RS;
      const int co = co0 + col, ci = ci0 + cil;
      v[u] = (co < e.Co && ci < e.Ci) ? e.w[(static_cast<long>(co) * e.Ci + ci) * RS + tap] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int q = threadIdx.x + u * 256;
      const int col = q / (kCwTile * RS), rem = q - col * (kCwTile * RS);
      const int cil = rem / RS, tap = rem - cil * RS;
      tile[tap][col][cil] = v[u];
    }
    __syncthreads();
    // 4 consecutive channels per 8-byte store (Cp, Cop are multiples of 8: a group never straddles the edge)
    constexpr int kQ4 = kCwTile * RS * kCwTile / 4;
    for (int q = threadIdx.x; q < kQ4; q += blockDim.x) {  // fwd [co][tap][ci]
      const int col = q / (RS * kCwTile / 4), rem = q - col * (RS * kCwTile / 4);
      const int tap = rem / (kCwTile / 4), cil = (rem - tap * (kCwTile / 4)) * 4;
      const int co = co0 + col, ci = ci0 + cil;
      if (co < e.Cop && ci < e.Cp)
        *reinterpret_cast<u16x4*>(e.fwd + (static_cast<long>(co) * RS + tap) * e.Cp + ci) =
            u16x4{f2bf(tile[tap][col][cil]), f2bf(tile[tap][col][cil + 1]), f2bf(tile[tap][col][cil + 2]),
                  f2bf(tile[tap][col][cil + 3])};
    }
    for (int q = threadIdx.x; q < kQ4; q += blockDim.x) {  // dgrad [ci][tap][co]
      const int cil = q / (RS * kCwTile / 4), rem = q - cil * (RS * kCwTile / 4);
      const int tap = rem / (kCwTile / 4), col = (rem - tap * (kCwTile / 4)) * 4;
      const int co = co0 + col, ci = ci0 + cil;
      if (co < e.Cop && ci < e.Cp)
        *reinterpret_cast<u16x4*>(e.dgrad + (static_cast<long>(ci) * RS + tap) * e.Cop + co) =
            u16x4{f2bf(tile[tap][col][cil]), f2bf(tile[tap][col + 1][cil]), f2bf(tile[tap][col + 2][cil]),
                  f2bf(tile[tap][col + 3][cil])};
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_conv_w_layouts_multi(const ConvLayoutEntry* __restrict__ table) {
  const ConvLayoutEntry e = table[blockIdx.y];
  if (e.R * e.S == 9)
    conv_w_layouts_tiled3x3(e);
  else
    conv_w_layouts_entry<0>(e);
}

__global__ void k_wgrad_to_oihw(const float* __restrict__ in, float* __restrict__ out, int Co, int Ci,
                                int R, int S, int Cp, int accum) {
  const long total = static_cast<long>(Co) * Ci * R * S;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int s = static_cast<int>(i % S);
    long t = i / S;
    const int r = static_cast<int>(t % R);
    t /= R;
    const int ci = static_cast<int>(t % Ci);
    const int co = static_cast<int>(t / Ci);
    const float v = in[((static_cast<long>(co) * R + r) * S + s) * Cp + ci];
    out[i] = accum ? out[i] + v : v;
  }
}

// Column sums of bf16 [M, N] (bias gradient): each block owns a strip of 64 columns x
// (M / gridDim.y) rows; 4 waves stride the rows, partials meet in LDS, then one fp32 atomic per
// column per block (or a plain store when a single block covers all rows).
__global__ void k_colsum_bf16(const uint16_t* __restrict__ x, float* __restrict__ out, int M, int N,
                              int rows_per_block, int accum) {
  __shared__ float part[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int wid = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  float acc = 0.f;
  if (col < N)
    for (int r = r0 + wid; r < r1; r += 4) acc += bf2f(x[static_cast<long>(r) * N + col]);
  part[wid][threadIdx.x & 63] = acc;
  __syncthreads();
  if (wid == 0 && col < N) {
    const float v = part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x];
    if (gridDim.y == 1)
      out[col] = accum ? out[col] + v : v;
    else
      atomicAdd(out + col, v);
  }
}

// Narrow-matrix column sums (N % 8 == 0): thread = (row-in-iteration, 8-column group), 16-byte loads,
// fixed-order partials per block -> ws[blk][N], summed by k_colsum_final.  Deterministic.
__global__ __launch_bounds__(256) void k_colsum_vec(const uint16_t* __restrict__ x, int M, int N, int rows_per_block,
                                                    float* __restrict__ ws) {
  const int G = N / 8;
  const int gg = G < 256 ? G : 256;
  const int rpi = 256 / gg;
  const int rr = threadIdx.x / gg, g0 = threadIdx.x % gg;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  __shared__ float red[256][8];
  for (int gb = 0; gb < G; gb += gg) {
    const int g = gb + g0;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (rr < rpi && g < G)
      for (int r = r0 + rr; r < r1; r += rpi) {
        const u16x8 v = *reinterpret_cast<const u16x8*>(x + static_cast<long>(r) * N + g * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
      }
#pragma unroll
    for (int j = 0; j < 8; ++j) red[threadIdx.x][j] = acc[j];
    __syncthreads();
    if (rr == 0 && g < G) {
      for (int q = 1; q < rpi; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += red[q * gg + g0][j];
#pragma unroll
      for (int j = 0; j < 8; ++j) ws[static_cast<long>(blockIdx.x) * N + g * 8 + j] = acc[j];
    }
    __syncthreads();
  }
}

// One wave per column: lanes stride the block partials, then a wave reduction.
// Short inputs (M <= 1024 rows: the MLP's bias gradients at batch 128): one launch, no workspace.  A block
// owns 64 columns (8 groups of 8); its 32 row-lanes per group each sum every 32nd row with 16-byte loads,
// then lane 0 of the group adds the 32 partials in a fixed order (deterministic) and writes / accumulates.
__global__ __launch_bounds__(256) void k_colsum_cols(const uint16_t* __restrict__ x, int M, int N,
                                                     float* __restrict__ out, int accum) {
  const int G = N / 8;
  const int gl = threadIdx.x & 7, rl = threadIdx.x >> 3;  // 8 groups x 32 row-lanes
  const int g = blockIdx.x * 8 + gl;
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  if (g < G) {
    for (int r = rl; r < M; r += 32) {
      const u16x8 u = *reinterpret_cast<const u16x8*>(x + static_cast<long>(r) * N + g * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += bf2f(u[j]);
    }
  }
  __shared__ float part[32][8][9];
#pragma unroll
  for (int j = 0; j < 8; ++j) part[rl][gl][j] = s[j];
  __syncthreads();
  if (threadIdx.x < 64) {  // (group, column) per thread
    const int gq = threadIdx.x >> 3, j = threadIdx.x & 7;
    const int gc = blockIdx.x * 8 + gq;
    if (gc < G) {
      float t = 0.f;
      for (int k = 0; k < 32; ++k) t += part[k][gq][j];
      const int col = gc * 8 + j;
      out[col] = accum ? out[col] + t : t;
    }
  }
}

__global__ void k_colsum_final(const float* __restrict__ ws, int nblk, int N, float* __restrict__ out, int accum) {
  const int col = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (col >= N) return;
  float v = 0.f;
  for (int b = lane; b < nblk; b += 64) v += ws[static_cast<long>(b) * N + col];
  v = wave_sum(v);
  if (lane == 0) out[col] = accum ? out[col] + v : v;
}

__global__ void k_relu_bwd(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
                           uint16_t* __restrict__ dx, long n) {
  const long nv = n / 8;
  const long stride = static_cast<long>(gridDim.x) * blockDim.x;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < nv; i += stride) {
    const u16x8 g = reinterpret_cast<const u16x8*>(dy)[i];
    const u16x8 a = reinterpret_cast<const u16x8*>(y)[i];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = bf2f(a[j]) > 0.f ? g[j] : uint16_t(0);
    reinterpret_cast<u16x8*>(dx)[i] = o;
  }
  for (long i = nv * 8 + blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < n; i += stride)
    dx[i] = bf2f(y[i]) > 0.f ? dy[i] : uint16_t(0);
}

}  // namespace

hipError_t cast_rows_bf16(const float* in, int rows, int cols, uint16_t* out, int ldo, int ones, hipStream_t s) {
  const long n = static_cast<long>(rows) * (cols + 1);
  hipLaunchKernelGGL(k_cast_rows_bf16, dim3(stream_grid(n, 256)), dim3(256), 0, s, in, rows, cols, out, ldo, ones);
  return hipGetLastError();
}

hipError_t cast_f32_bf16(const float* in, uint16_t* out, long n, hipStream_t s) {
  hipLaunchKernelGGL(k_cast_f32_bf16, dim3(stream_grid(n, 256, 8)), dim3(256), 0, s, in, out, n);
  return hipGetLastError();
}
hipError_t cast_bf16_f32(const uint16_t* in, float* out, long n, hipStream_t s) {
  hipLaunchKernelGGL(k_cast_bf16_f32, dim3(stream_grid(n, 256, 8)), dim3(256), 0, s, in, out, n);
  return hipGetLastError();
}
hipError_t nchw_f32_to_nhwc_bf16(const float* in, uint16_t* out, int N, int C, int H, int W, int Cp,
                                 hipStream_t s) {
  const long total = static_cast<long>(N) * H * W * (Cp / 8);
  hipLaunchKernelGGL(k_nchw_to_nhwc, dim3(stream_grid(total, 256)), dim3(256), 0, s, in, out, N, C, H, W, Cp);
  return hipGetLastError();
}
hipError_t conv_weight_fwd_layout(const float* w, uint16_t* out, int Co, int Ci, int R, int S, int Cp, int Cop,
                                  hipStream_t s) {
  const long total = static_cast<long>(Cop) * R * S * Cp;
  hipLaunchKernelGGL(k_conv_w_fwd, dim3(stream_grid(total, 256)), dim3(256), 0, s, w, out, Co, Ci, R, S, Cp, Cop);
  return hipGetLastError();
}
hipError_t conv_weight_dgrad_layout(const float* w, uint16_t* out, int Co, int Ci, int R, int S, int Cip, int Cop,
                                    hipStream_t s) {
  const long total = static_cast<long>(Cop) * R * S * Cip;
  hipLaunchKernelGGL(k_conv_w_dgrad, dim3(stream_grid(total, 256)), dim3(256), 0, s, w, out, Co, Ci, R, S, Cip,
                     Cop);
  return hipGetLastError();
}
hipError_t conv_weight_layouts_multi(const ConvLayoutEntry* dev_table, int n, int blocks_x, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_conv_w_layouts_multi, dim3(blocks_x < 1 ? 1 : blocks_x, n), dim3(256), 0, s, dev_table);
  return hipGetLastError();
}
hipError_t conv_wgrad_to_oihw(const float* in, float* out, int Co, int Ci, int R, int S, int Cp, int accum,
                              hipStream_t s) {
  const long total = static_cast<long>(Co) * Ci * R * S;
  hipLaunchKernelGGL(k_wgrad_to_oihw, dim3(stream_grid(total, 256)), dim3(256), 0, s, in, out, Co, Ci, R, S,
                     Cp, accum);
  return hipGetLastError();
}
hipError_t colsum_bf16_ws(const uint16_t* x, float* out, int M, int N, int accum, float* ws, int ws_blocks,
                          hipStream_t s) {
  if (N % 8 == 0 && M <= 1024) {
    hipLaunchKernelGGL(k_colsum_cols, dim3(ceil_div(N / 8, 8)), dim3(256), 0, s, x, M, N, out, accum);
    return hipGetLastError();
  }
  if (N % 8 == 0 && ws != nullptr) {
    const int G = N / 8;
    const int rpi = 256 / (G < 256 ? G : 256);
    int nblk = ceil_div(M, rpi * 8);
    if (nblk > ws_blocks) nblk = ws_blocks;
    if (nblk < 1) nblk = 1;
    const int rpb = ceil_div(M, nblk);
    nblk = ceil_div(M, rpb);
    hipLaunchKernelGGL(k_colsum_vec, dim3(nblk), dim3(256), 0, s, x, M, N, rpb, ws);
    hipLaunchKernelGGL(k_colsum_final, dim3(ceil_div(N, 4)), dim3(256), 0, s, ws, nblk, N, out, accum);
    return hipGetLastError();
  }
  return colsum_bf16(x, out, M, N, accum, s);
}

hipError_t colsum_bf16(const uint16_t* x, float* out, int M, int N, int accum, hipStream_t s) {
  // accum is handled by the caller zeroing/keeping out; with a single row-block we overwrite.
  const int col_blocks = ceil_div(N, 64);
  int row_blocks = 1;
  while (row_blocks < 64 && col_blocks * row_blocks < 512 && M / (row_blocks * 2) >= 64) row_blocks *= 2;
  const int rpb = ceil_div(M, row_blocks);
  if (row_blocks > 1 && !accum) (void)hipMemsetAsync(out, 0, sizeof(float) * N, s);
  hipLaunchKernelGGL(k_colsum_bf16, dim3(col_blocks, row_blocks), dim3(256), 0, s, x, out, M, N, rpb, accum);
  return hipGetLastError();
}
hipError_t relu_bwd_bf16(const uint16_t* dy, const uint16_t* y, uint16_t* dx, long n, hipStream_t s) {
  hipLaunchKernelGGL(k_relu_bwd, dim3(stream_grid(n, 256, 8)), dim3(256), 0, s, dy, y, dx, n);
  return hipGetLastError();
}

// Batch gather driven by a DEVICE replay counter (elastic/rewire.py, utils/epoch_graph.py): rows [c x rows,
// (c + 1) x rows) of the epoch's index list idx (c = counter[0]) are gathered from the HBM-resident dataset into
// the captured step's static batch slots, and the launch's last workgroup advances the counter -- so a hipGraph
// replayed k times trains on k different slices of the epoch with no host work between replays (the host sets
// the counter once per epoch / resume).  Every workgroup reads the counter before it counts itself done, so
// the increment never races a read; counter[1] is the done count (re-zeroed by the last workgroup).
__global__ __launch_bounds__(256) void k_gather_rows_counter(const float4* __restrict__ src,
                                                             const int64_t* __restrict__ labels,
                                                             const int64_t* __restrict__ idx, int64_t n_idx,
                                                             uint32_t* counter, int rows, int row4,
                                                             float4* __restrict__ dst, int64_t* __restrict__ ydst) {
  __shared__ int64_t s_base;
  if (threadIdx.x == 0)
    s_base = static_cast<int64_t>(__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) * rows;
  __syncthreads();
  const int64_t base = s_base;
  const int64_t total = static_cast<int64_t>(rows) * row4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t row = t / row4, c = t - row * row4;
    int64_t k = base + row;
    k = k < n_idx ? k : n_idx - 1;  // (the host only replays whole slices; never read past the list)
    dst[t] = src[idx[k] * row4 + c];
  }
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; row < rows; row += stride) {
    int64_t k = base + row;
    k = k < n_idx ? k : n_idx - 1;
    ydst[row] = labels[idx[k]];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t n = __hip_atomic_fetch_add(counter + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (n == gridDim.x - 1) {
      __hip_atomic_store(counter + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

hipError_t gather_rows_counter(const float* src, const int64_t* labels, const int64_t* idx, int64_t n_idx,
                               uint32_t* counter, int rows, int row_elems, float* dst, int64_t* ydst, hipStream_t s) {
  if (rows <= 0 || row_elems % 4 != 0) return hipErrorInvalidValue;
  const int row4 = row_elems / 4;
  const int64_t total = static_cast<int64_t>(rows) * row4;
  const int grid = static_cast<int>(std::min<int64_t>(2048, (total + 255) / 256));
  hipLaunchKernelGGL(k_gather_rows_counter, dim3(grid), dim3(256), 0, s, reinterpret_cast<const float4*>(src), labels,
                     idx, n_idx, counter, rows, row4, reinterpret_cast<float4*>(dst), ydst);
  return hipGetLastError();
}

// One wall-clock timestamp (100 MHz constant clock) into stamps[slot]: a graph node at a phase boundary of a
// captured training step (bench phase attribution, utils/log.GraphPhaseTimer).
__global__ void k_time_stamp(unsigned long long* stamps, int slot) {
  if (threadIdx.x == 0) stamps[slot] = wall_clock64();
}

hipError_t time_stamp(unsigned long long* stamps, int slot, hipStream_t s) {
  hipLaunchKernelGGL(k_time_stamp, dim3(1), dim3(64), 0, s, stamps, slot);
  return hipGetLastError();
}

}  // namespace pde
