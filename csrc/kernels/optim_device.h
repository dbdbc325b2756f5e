// Multi-tensor optimiser update as a DEVICE function (SGD / Adam / AdamW over a range of chunks of a
// OptimEntry / OptimChunk table), shared by the standalone launch (optim.hip: k_optim) and the GEMM pair
// kernels (gemm.hip), which append optimiser blocks to a backward launch: the update of layer i+1 runs in the
// same grid as layer i's dgrad / wgrad GEMM tiles -- the HBM-bound update fills the CUs the latency-bound
// small GEMM leaves idle (OptimSeg, pde_kernels.h).  Same code path either way: bit-identical updates.
#pragma once
#include "common.cuh"
#include "pde_kernels.h"

namespace pde {
namespace optdev {

constexpr int kOptThreads = 256;
constexpr int kOptGroups = 4;                       // 16-byte groups per thread per chunk
constexpr int kOptChunk = kOptThreads * 4 * kOptGroups;   // elements per chunk (4096)

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

// 16-B state accesses.  NT 1: non-temporal (streaming) loads and stores -- every state byte is touched once
// per step, so keeping it in L2 / MALL only evicts the GEMMs' operands; NT 2: non-temporal loads, write-through
// (sc1) stores -- the updated state leaves L2 during the update instead of at the kernel boundary, ahead of the
// next step's first GEMM; NT 0: plain (A/B: PDE_OPTIM_NT)
template <int NT>
__device__ __forceinline__ f32x4 ld4(const float* p) {
  if constexpr (NT != 0) return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  else return *reinterpret_cast<const f32x4*>(p);
}
template <int NT>
__device__ __forceinline__ void st4(float* p, const f32x4& v) {
  if constexpr (NT == 2) st_vec(reinterpret_cast<f32x4*>(p), v, true);
  else if constexpr (NT == 1) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
  else *reinterpret_cast<f32x4*>(p) = v;
}

// One chunk's state for one thread: kOptGroups x 16 B of every state tensor, loaded before any math.
template <int MODE, int NT>
struct ChunkRegs {
  float p[kOptGroups][4], g[kOptGroups][4], m[kOptGroups][4], v[kOptGroups][4];
  int e0[kOptGroups], cnt[kOptGroups];
  int tensor;

  __device__ __forceinline__ void load(const OptimEntry* tab, const OptimChunk& ch, bool use_m) {
    tensor = ch.tensor;
    const OptimEntry& te = tab[ch.tensor];
    const int end = ch.start + ch.count;
#pragma unroll
    for (int u = 0; u < kOptGroups; ++u) {
      e0[u] = ch.start + (u * kOptThreads + threadIdx.x) * 4;
      cnt[u] = e0[u] < end ? min(4, end - e0[u]) : 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) p[u][k] = g[u][k] = m[u][k] = v[u][k] = 0.f;
      if (cnt[u] == 4 && te.vec) {
        const f32x4 pv = ld4<NT>(te.param + e0[u]);
        p[u][0] = pv[0]; p[u][1] = pv[1]; p[u][2] = pv[2]; p[u][3] = pv[3];
        if (te.grad) {
          const f32x4 gv = ld4<NT>(te.grad + e0[u]);
          g[u][0] = gv[0]; g[u][1] = gv[1]; g[u][2] = gv[2]; g[u][3] = gv[3];
        }
        if (use_m) {
          const f32x4 mv = ld4<NT>(te.exp_avg + e0[u]);
          m[u][0] = mv[0]; m[u][1] = mv[1]; m[u][2] = mv[2]; m[u][3] = mv[3];
        }
        if (MODE != 0) {
          const f32x4 vv = ld4<NT>(te.exp_avg_sq + e0[u]);
          v[u][0] = vv[0]; v[u][1] = vv[1]; v[u][2] = vv[2]; v[u][3] = vv[3];
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k < cnt[u]) {
            p[u][k] = te.param[e0[u] + k];
            if (te.grad) g[u][k] = te.grad[e0[u] + k];
            if (use_m) m[u][k] = te.exp_avg[e0[u] + k];
            if (MODE != 0) v[u][k] = te.exp_avg_sq[e0[u] + k];
          }
        }
      }
    }
  }

  __device__ __forceinline__ void finish(const Hyper& h, const OptimEntry* tab, bool use_m) {
    const OptimEntry& te = tab[tensor];
#pragma unroll
    for (int u = 0; u < kOptGroups; ++u) {
      if (cnt[u] == 0) continue;
#pragma unroll
      for (int k = 0; k < 4; ++k) update<MODE>(h, p[u][k], g[u][k], m[u][k], v[u][k]);
      const int i = e0[u];
      if (cnt[u] == 4 && te.vec) {
        st4<NT>(te.param + i, f32x4{p[u][0], p[u][1], p[u][2], p[u][3]});
        if (use_m) st4<NT>(te.exp_avg + i, f32x4{m[u][0], m[u][1], m[u][2], m[u][3]});
        if (MODE != 0) st4<NT>(te.exp_avg_sq + i, f32x4{v[u][0], v[u][1], v[u][2], v[u][3]});
        if (te.bf16_copy)
          st_vec(reinterpret_cast<u16x4*>(te.bf16_copy + i),
                 u16x4{f2bf(p[u][0]), f2bf(p[u][1]), f2bf(p[u][2]), f2bf(p[u][3])}, NT == 2);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k < cnt[u]) {
            te.param[i + k] = p[u][k];
            if (use_m) te.exp_avg[i + k] = m[u][k];
            if (MODE != 0) te.exp_avg_sq[i + k] = v[u][k];
            if (te.bf16_copy) te.bf16_copy[i + k] = f2bf(p[u][k]);
          }
        }
      }
    }
  }
};


// Chunks [c_begin, c_end) of the table, walked by `nblocks` blocks (this one is `block`), grid-stride and
// software-pipelined (the next chunk's loads are issued before the current chunk's math and stores).
// publish: the last of the `nblocks` blocks to finish stores the new step count (the final segment of a step).
// PIPE = false (the segments appended to GEMM launches: about one chunk per block, and the GEMM tiles' VGPR
// budget): one chunk's registers live at a time.
template <int MODE, int NT, bool PIPE = true>
__device__ __forceinline__ void run_chunks(const OptimEntry* __restrict__ tab, const OptimChunk* __restrict__ chunks,
                                           int c_begin, int c_end, const float* __restrict__ hp,
                                           int* __restrict__ step_ptr, int block, int nblocks, bool publish) {
  __shared__ int s_step;
  if (threadIdx.x == 0) s_step = step_ptr[0] + 1;  // step being taken (1-based)
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
  const bool use_m = MODE != 0 || h.mom != 0.f;
  if constexpr (PIPE) {
    ChunkRegs<MODE, NT> cur, nxt;
    int c = c_begin + block;
    if (c < c_end) cur.load(tab, chunks[c], use_m);
    for (; c < c_end; c += nblocks) {
      const int cn = c + nblocks;
      if (cn < c_end) nxt.load(tab, chunks[cn], use_m);
      cur.finish(h, tab, use_m);
      cur = nxt;
    }
  } else {
    for (int c = c_begin + block; c < c_end; c += nblocks) {
      ChunkRegs<MODE, NT> cur;
      cur.load(tab, chunks[c], use_m);
      cur.finish(h, tab, use_m);
    }
  }
  if (!publish) return;
  // The last block to finish publishes the new step count.  Every block read the old count before its
  // arrival (the value was consumed before the barrier above), and the next launch sees the store
  // across the kernel boundary: a relaxed device-scope ticket is enough (no fence).
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = atomicAdd(step_ptr + 1, 1);
    if (prev == nblocks - 1) {
      step_ptr[0] = s_step;
      step_ptr[1] = 0;
    }
  }
}

// Runtime mode dispatch (NT loads / stores: every state byte is touched once per step).
__device__ __forceinline__ void run_segment(const OptimSeg& s, int block) {
  if (s.mode == 0)
    run_chunks<0, 1, false>(s.tab, s.chunks, s.c0, s.c1, s.hp, s.step, block, s.blocks, s.publish != 0);
  else if (s.mode == 1)
    run_chunks<1, 1, false>(s.tab, s.chunks, s.c0, s.c1, s.hp, s.step, block, s.blocks, s.publish != 0);
  else
    run_chunks<2, 1, false>(s.tab, s.chunks, s.c0, s.c1, s.hp, s.step, block, s.blocks, s.publish != 0);
}

}  // namespace optdev
}  // namespace pde
