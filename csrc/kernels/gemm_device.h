// Device side of the bf16 MFMA GEMM (see gemm.hip for the design notes): operand loaders, the register-ring
// and LDS-DMA main loops, epilogues, kernels, and the host-side launch templates of the DMA core.  Included
// by gemm.hip and by the gemm_dma_*.hip translation units, which instantiate the DMA kernels in parallel
// builds (one 128x128 instantiation takes minutes of register allocation).  Everything is in an anonymous
// namespace: each translation unit gets its own copies.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "common.cuh"
#include "pde_kernels.h"
#include "optim_device.h"

namespace pde {

// dims of a paired launch's two problems (tiles along M / N, K per split, vector flags, splits)
struct PairDims {
  int tm[2], tn[2], kps[2], av[2], bv[2], nz[2];
};

namespace {


constexpr int kThreads = 256;
// Minimum waves per SIMD the 64x64 tiles are compiled for (-DPDE_GEMM_WPE=N to sweep): 4 caps them at 128 VGPRs
#ifndef PDE_GEMM_WPE
#define PDE_GEMM_WPE 4
#endif
// K-tiles in flight in the FAST loaders' register ring (-DPDE_FAST_STAGES=N to sweep)
#ifndef PDE_FAST_STAGES
#define PDE_FAST_STAGES 4
#endif

// LDS images are unpadded K-contiguous rows (BK = 32 -> 64 B, four 16-byte K-chunks) with an XOR swizzle
// of the chunk index: chunk c of row r lives at c ^ H[(r >> 2) & 3] ^ ((r >> 4) & 3), H = {0, 3, 2, 1}.
// gfx950 services ds_read_b128 in four NON-contiguous 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,
// 28-31}, ...): an MFMA fragment read (lane -> row lane & 15, chunk lane >> 4) puts every row of the
// fragment in each group, rows 0-3 / 12-15 at chunk c and rows 4-11 at chunk c+1.  With a 64-B pitch the
// 16-B slot of (r, c) is 4 (r & 3) + chunk', and H makes the four rows sharing r & 3 land on four
// different chunks in every group: conflict-free reads (an 80-B padded pitch, the previous layout, was
// 2-way conflicted on exactly this grouping: SQ_LDS_BANK_CONFLICT = 50 % of SQ_LDS_IDX_ACTIVE in
// profiles/r1h_resnet50_sq_counters.txt).  The (r >> 4) term is constant per 16-row fragment (reads stay
// conflict-free) and spreads the row-contiguous loader's transposing 2-byte scatter (8 rows 8 apart) over
// more banks; 16-B K-contiguous stores (8 contiguous lanes = 2 rows x 4 chunks) are conflict-free.
__device__ __forceinline__ int swz_chunk(int row, int chunk) {
  return chunk ^ ((-(row >> 2)) & 3) ^ ((row >> 4) & 3);
}

__device__ __forceinline__ u16x8 zero8() { return u16x8{0, 0, 0, 0, 0, 0, 0, 0}; }

// Row-contiguous LDS image: [BK = 32][BROWS] -- row k holds BROWS consecutive row (M/N) elements, its
// 16-B chunks XOR-swizzled by rc_swz(k).  A 16x16x32 fragment (lane l: row rb + (l & 15), k = 8 (l >> 4)
// + j) is two ds_read_b64_tr_b16: the 16-lane group g reads the 4 x 16 blocks k = 8g..8g+3 and 8g+4..8g+7
// (lane 4q + p addresses row k0 + q, columns rb + 4p..4p+3; lane i receives column i).  A 32-lane half
// then touches rows {k0..k0+3, k0+8..k0+11} x 2 chunks each; the swizzle gives those 16 (row, chunk) pairs
// distinct 4-bank slots (bank = (k * 2 BROWS + 16 chunk') / 4 mod 64), so the reads are conflict-free.
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

template <int BROWS>
__device__ __forceinline__ int rc_swz(int k) {
  constexpr int CH = BROWS / 8;  // 16-B chunks per row
  static_assert(CH == 4 || CH == 8 || CH == 16, "row-contiguous image widths 32 / 64 / 128");
  if constexpr (CH == 4) return 2 * ((k >> 3) & 1);
  else if constexpr (CH == 8) return 2 * ((k >> 1) & 1) + 4 * ((k >> 3) & 1);
  else return 2 * (k & 3) + 8 * ((k >> 3) & 1);
}

template <int BROWS>
__device__ __forceinline__ bf16x8 rc_frag(const uint16_t* lds, int rb, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int c = (rb >> 3) + (p >> 1);
  const int k1 = 8 * g + q, k2 = k1 + 4;
  const uint16_t* a1 = lds + k1 * BROWS + ((c ^ rc_swz<BROWS>(k1)) << 3) + 4 * (p & 1);
  const uint16_t* a2 = lds + k2 * BROWS + ((c ^ rc_swz<BROWS>(k2)) << 3) + 4 * (p & 1);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  const s16x4 r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a2));
  const s16x8 v = __builtin_shufflevector(r1, r2, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// Dense K-contiguous / row-contiguous element loads (operand kind 0).
__device__ __forceinline__ u16x8 load_dense_kc(const Operand& op, int rows, int K, int r, int k0, bool vec_ok) {
  u16x8 v = zero8();
  if (r >= rows || k0 >= K) return v;
  const uint16_t* p = static_cast<const uint16_t*>(op.ptr);
  const long base = static_cast<long>(r) * op.ld_r;
  if (vec_ok && k0 + 8 <= K) {
    v = *reinterpret_cast<const u16x8*>(p + base + k0);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (k0 + i < K) v[i] = p[base + static_cast<long>(k0 + i) * op.ld_k];
  }
  return v;
}

__device__ __forceinline__ u16x8 load_dense_rc(const Operand& op, int rows, int K, int r0, int k, bool vec_ok) {
  u16x8 v = zero8();
  if (r0 >= rows || k >= K) return v;
  const uint16_t* p = static_cast<const uint16_t*>(op.ptr);
  const long base = static_cast<long>(k) * op.ld_k;
  if (vec_ok && r0 + 8 <= rows) {
    v = *reinterpret_cast<const u16x8*>(p + base + r0);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (r0 + i < rows) v[i] = p[base + static_cast<long>(r0 + i) * op.ld_r];
  }
  return v;
}

// Branch-free 16-B operand load through a buffer descriptor: an invalid slot (out of the tile's rows, past
// K, or a conv tap in the padding) gets an out-of-range offset and the hardware returns zeros.  With no
// divergent branches around the loads the compiler can count them (s_waitcnt vmcnt(N)), which is what
// lets the register ring keep several K-tiles in flight (FAST loaders; operand extents < 2 GB).
constexpr uint32_t kOob = 0x80000000u;
__device__ __forceinline__ u16x8 bload16(__amdgpu_buffer_rsrc_t r, bool ok, long elem_off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, ok ? static_cast<uint32_t>(elem_off * 2) : kOob, 0, 0);
  return __builtin_bit_cast(u16x8, v);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t operand_rsrc(const Operand& op, int kind, int rows, int K,
                                                               bool kc) {
  long elems;
  if (kind == 0)  // row-contiguous: whole 8-row groups (rows past the end are padding, host-checked)
    elems = kc ? static_cast<long>(rows - 1) * op.ld_r + K : static_cast<long>(K - 1) * op.ld_k + (rows + 7) / 8 * 8;
  else
    elems = static_cast<long>(op.g.N) * op.g.H * op.g.W * op.g.C;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(op.ptr), 0, static_cast<int>(elems * 2), 0x00020000);
}

// K-contiguous operand (kinds 0, 1, 3): each slot loads 8 consecutive K elements of one row.
template <int BROWS, int BK, int KIND>  // KIND >= 0: compile-time operand kind, branch-free FAST loads
struct KcLoader {
  static constexpr bool FAST = KIND >= 0;
  __device__ static __forceinline__ int kind_of(const Operand& op) {
    if constexpr (KIND >= 0) return KIND;
    else return op.kind;
  }
  static constexpr int kVecs = BROWS * BK / 8;
  static constexpr int kPer = (kVecs + kThreads - 1) / kThreads;
  int k0[kPer];                 // the slot's current reduction index
  int c[kPer], kw[kPer], kh[kPer];
  int by[kPer], bx[kPer];       // kind 1: oy*s - pad, ox*s - pad;  kind 3: h + pad, w + pad
  long nb[kPer];                // image base offset in elements; -1: row out of range
  __amdgpu_buffer_rsrc_t rsrc;  // FAST: descriptor over the operand's valid extent

  __device__ __forceinline__ void init(const Operand& op, int rows, int row0, int kbeg, int K) {
    if constexpr (FAST) rsrc = operand_rsrc(op, KIND, rows, K, true);
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int v = threadIdx.x + i * kThreads;
      const int row = v / (BK / 8), kv = v - row * (BK / 8);
      k0[i] = kbeg + kv * 8;
      nb[i] = -1;
      c[i] = kw[i] = kh[i] = by[i] = bx[i] = 0;
      if (kind_of(op) == 0 || v >= kVecs) continue;
      const ConvGeom& g = op.g;
      c[i] = k0[i] % g.C;  // C % 8 == 0: the slot's 8 elements share (kh, kw)
      const int rs = k0[i] / g.C;
      kw[i] = rs % g.S;
      kh[i] = rs / g.S;
      const int r = row0 + row;
      if (r < rows) {
        const int HWo = g.Ho * g.Wo;
        const int n = r / HWo, rem = r - n * HWo, oy = rem / g.Wo, ox = rem - oy * g.Wo;
        nb[i] = static_cast<long>(n) * g.H * g.W * g.C;
        if (kind_of(op) == 1) {
          by[i] = oy * g.stride - g.pad;
          bx[i] = ox * g.stride - g.pad;
        } else {  // kind 3: (oy, ox) are dx coordinates; dy has dims H x W
          by[i] = oy + g.pad;
          bx[i] = ox + g.pad;
        }
      }
    }
  }

  __device__ __forceinline__ void advance(const Operand& op) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      k0[i] += BK;
      if (kind_of(op) != 0) {
        c[i] += BK;
        while (c[i] >= op.g.C) {
          c[i] -= op.g.C;
          if (++kw[i] == op.g.S) {
            kw[i] = 0;
            ++kh[i];
          }
        }
      }
    }
  }

  __device__ __forceinline__ void load(const Operand& op, int rows, int K, int row0, bool vec_ok,
                                       u16x8 (&regs)[kPer]) {
    if constexpr (FAST) {
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int v = threadIdx.x + i * kThreads;
        bool ok = v < kVecs && k0[i] < K;
        long off;
        if (kind_of(op) == 0) {
          const int r = row0 + v / (BK / 8);
          ok = ok && r < rows;
          off = static_cast<long>(r) * op.ld_r + k0[i];
        } else {
          const ConvGeom& g = op.g;
          int iy, ix;
          if (kind_of(op) == 1) {
            iy = by[i] + kh[i];
            ix = bx[i] + kw[i];
          } else {
            iy = by[i] - kh[i];
            ix = bx[i] - kw[i];
            ok = ok && iy >= 0 && ix >= 0;
            if (g.stride == 2) {
              ok = ok && ((iy | ix) & 1) == 0;
              iy >>= 1;
              ix >>= 1;
            } else if (g.stride > 2) {
              ok = ok && (iy % g.stride) == 0 && (ix % g.stride) == 0;
              iy /= g.stride;
              ix /= g.stride;
            }
          }
          ok = ok && nb[i] >= 0 && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
          off = nb[i] + (static_cast<long>(iy) * g.W + ix) * g.C + c[i];
        }
        regs[i] = bload16(rsrc, ok, off);
      }
      return;
    }
    const uint16_t* p = static_cast<const uint16_t*>(op.ptr);
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int v = threadIdx.x + i * kThreads;
      u16x8 val = zero8();
      if (v < kVecs && k0[i] < K) {
        if (kind_of(op) == 0) {
          val = load_dense_kc(op, rows, K, row0 + v / (BK / 8), k0[i], vec_ok);
        } else if (nb[i] >= 0) {
          const ConvGeom& g = op.g;
          int iy, ix;
          bool ok = true;
          if (kind_of(op) == 1) {
            iy = by[i] + kh[i];
            ix = bx[i] + kw[i];
          } else {
            iy = by[i] - kh[i];
            ix = bx[i] - kw[i];
            ok = iy >= 0 && ix >= 0;
            if (g.stride == 2) {
              ok = ok && ((iy | ix) & 1) == 0;
              iy >>= 1;
              ix >>= 1;
            } else if (g.stride > 2) {
              ok = ok && (iy % g.stride) == 0 && (ix % g.stride) == 0;
              iy /= g.stride;
              ix /= g.stride;
            }
          }
          if (ok && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W)
            val = *reinterpret_cast<const u16x8*>(p + nb[i] + (static_cast<long>(iy) * g.W + ix) * g.C + c[i]);
        }
      }
      regs[i] = val;
    }
  }

  __device__ __forceinline__ void store(uint16_t* lds, const u16x8 (&regs)[kPer]) {  // lds: [BROWS][BK]
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int v = threadIdx.x + i * kThreads;
      if (v < kVecs) {
        const int row = v / (BK / 8);
        const int kv = v - row * (BK / 8);
        *reinterpret_cast<u16x8*>(lds + row * BK + swz_chunk(row, kv) * 8) = regs[i];
      }
    }
  }

  // Folded BatchNorm (consumer side, FAST kinds 0 / 1): what load() just issued for each slot, for the
  // transforming store of the same ring stage -- mc = channel of the slot's 8 elements (-1: a zero slot:
  // out of range or a padding tap, which must stay zero), mr = activation row the slot's transformed values
  // belong to (-1: not written: a non-centre tap of a 3x3 gather).
  __device__ __forceinline__ void meta(const Operand& op, int rows, int K, int row0, int center, int (&mc)[kPer],
                                       int (&mr)[kPer]) const {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int v = threadIdx.x + i * kThreads;
      const int r = row0 + v / (BK / 8);
      bool ok = v < kVecs && k0[i] < K && r < rows;
      int ch = k0[i];
      bool wr = ok;
      if constexpr (KIND == 1) {
        const ConvGeom& g = op.g;
        const int iy = by[i] + kh[i], ix = bx[i] + kw[i];
        ok = ok && nb[i] >= 0 && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
        ch = c[i];
        wr = ok && center && kh[i] == 1 && kw[i] == 1;
      }
      mc[i] = ok ? ch : -1;
      mr[i] = wr ? r : -1;
    }
  }

  // store() with relu(x * scale[c] + shift[c]) applied to every live slot (ss: LDS [2][C] scale, shift);
  // `write`: also store the transformed 16 B to act[mr][mc] (the first N-tile's blocks)
  __device__ __forceinline__ void store_bn(uint16_t* lds, u16x8 (&regs)[kPer], const int (&mc)[kPer],
                                           const int (&mr)[kPer], const float* ss, int C, int relu, bool write,
                                           uint16_t* act) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int v = threadIdx.x + i * kThreads;
      if (v < kVecs && mc[i] >= 0) {
        const f32x4* sc = reinterpret_cast<const f32x4*>(ss + mc[i]);
        const f32x4* sh = reinterpret_cast<const f32x4*>(ss + C + mc[i]);
        const f32x4 s0 = sc[0], s1 = sc[1], h0 = sh[0], h1 = sh[1];
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = bf2f(regs[i][j]) * (j < 4 ? s0[j] : s1[j - 4]) + (j < 4 ? h0[j] : h1[j - 4]);
          if (relu) t = fmaxf(t, 0.f);
          o[j] = f2bf(t);
        }
        regs[i] = o;
        if (write && mr[i] >= 0) *reinterpret_cast<u16x8*>(act + static_cast<long>(mr[i]) * C + mc[i]) = o;
      }
    }
    store(lds, regs);
  }
};

// Row-contiguous operand (kinds 0 and 2): each slot loads 8 consecutive ROW elements at one k.
// Kind 2 (weight-gradient B operand): rows are (kh, kw, c) of the conv (fixed per slot), k is the output
// pixel (n, oy, ox), advanced incrementally.
template <int BROWS, int BK, int KIND>  // KIND >= 0: compile-time operand kind, branch-free FAST loads
struct RcLoader {
  static constexpr bool FAST = KIND >= 0;
  __device__ static __forceinline__ int kind_of(const Operand& op) {
    if constexpr (KIND >= 0) return KIND;
    else return op.kind;
  }
  static constexpr int kVecs = BROWS * BK / 8;
  static constexpr int kPer = (kVecs + kThreads - 1) / kThreads;
  int k[kPer];
  int c0[kPer], kw[kPer], kh[kPer];
  int n[kPer], oy[kPer], ox[kPer];
  bool rok[kPer];
  __amdgpu_buffer_rsrc_t rsrc;  // FAST: descriptor over the operand's valid extent

  __device__ __forceinline__ void init(const Operand& op, int rows, int row0, int kbeg, int K) {
    if constexpr (FAST) rsrc = operand_rsrc(op, KIND, rows, K, false);
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int v = threadIdx.x + i * kThreads;
      const int kk = v / (BROWS / 8), rv = v - kk * (BROWS / 8);
      const int r0 = row0 + rv * 8;
      k[i] = kbeg + kk;
      rok[i] = v < kVecs && r0 < rows;
      c0[i] = kw[i] = kh[i] = n[i] = oy[i] = ox[i] = 0;
      if (kind_of(op) != 2 || !rok[i]) continue;
      const ConvGeom& g = op.g;
      c0[i] = r0 % g.C;
      const int rs = r0 / g.C;
      kw[i] = rs % g.S;
      kh[i] = rs / g.S;
      const int HWo = g.Ho * g.Wo;
      n[i] = k[i] / HWo;
      const int rem = k[i] - n[i] * HWo;
      oy[i] = rem / g.Wo;
      ox[i] = rem - oy[i] * g.Wo;
    }
  }

  __device__ __forceinline__ void advance(const Operand& op) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      k[i] += BK;
      if (kind_of(op) == 2) {
        ox[i] += BK;
        while (ox[i] >= op.g.Wo) {
          ox[i] -= op.g.Wo;
          if (++oy[i] == op.g.Ho) {
            oy[i] = 0;
            ++n[i];
          }
        }
      }
    }
  }

  __device__ __forceinline__ void load(const Operand& op, int rows, int K, int row0, bool vec_ok,
                                       u16x8 (&regs)[kPer]) {
    if constexpr (FAST) {
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int v = threadIdx.x + i * kThreads;
        bool ok = v < kVecs && k[i] < K;
        long off;
        if (kind_of(op) == 0) {
          const int r0 = row0 + (v % (BROWS / 8)) * 8;  // FAST dense: the 8-row group is allocated
          ok = ok && r0 < rows;
          off = static_cast<long>(k[i]) * op.ld_k + r0;
        } else {
          const ConvGeom& g = op.g;
          const int iy = oy[i] * g.stride - g.pad + kh[i];
          const int ix = ox[i] * g.stride - g.pad + kw[i];
          ok = ok && rok[i] && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
          off = ((static_cast<long>(n[i]) * g.H + iy) * g.W + ix) * g.C + c0[i];
        }
        regs[i] = bload16(rsrc, ok, off);
      }
      return;
    }
    const uint16_t* p = static_cast<const uint16_t*>(op.ptr);
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int v = threadIdx.x + i * kThreads;
      u16x8 val = zero8();
      if (v < kVecs && k[i] < K) {
        if (kind_of(op) == 0) {
          val = load_dense_rc(op, rows, K, row0 + (v % (BROWS / 8)) * 8, k[i], vec_ok);
        } else if (rok[i]) {
          const ConvGeom& g = op.g;
          const int iy = oy[i] * g.stride - g.pad + kh[i];
          const int ix = ox[i] * g.stride - g.pad + kw[i];
          if (iy >= 0 && iy < g.H && ix >= 0 && ix < g.W)
            val = *reinterpret_cast<const u16x8*>(
                p + ((static_cast<long>(n[i]) * g.H + iy) * g.W + ix) * g.C + c0[i]);
        }
      }
      regs[i] = val;
    }
  }

  __device__ __forceinline__ void store(uint16_t* lds, const u16x8 (&regs)[kPer]) {  // [BK][BROWS] (rc_swz)
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int v = threadIdx.x + i * kThreads;
      if (v < kVecs) {
        const int kk = v / (BROWS / 8);
        const int rv = v - kk * (BROWS / 8);
        *reinterpret_cast<u16x8*>(lds + kk * BROWS + ((rv ^ rc_swz<BROWS>(kk)) << 3)) = regs[i];
      }
    }
  }
};

template <int BROWS, int BK, bool KC, int KIND>
using Loader = typename std::conditional<KC, KcLoader<BROWS, BK, KIND>, RcLoader<BROWS, BK, KIND>>::type;

__device__ __forceinline__ float apply_epi(float v, int epi, int m, int n, const GemmArgs& a) {
  if ((epi & EPI_BIAS) && n < a.nbias) v += a.bias[n];
  if (epi & EPI_DRELU) v = (bf2f(a.aux[static_cast<long>(m) * a.ldaux + n]) > 0.f) ? v : 0.f;
  if (epi & EPI_ADD_AUX) v += bf2f(a.aux[static_cast<long>(m) * a.ldaux + n]);
  if (epi & EPI_RELU) v = fmaxf(v, 0.f);
  return v;
}

__device__ __forceinline__ void store_out(float v, int epi, int m, int n, const GemmArgs& a) {
  if (a.bias_grad != nullptr && n >= a.bias_col) {  // ones-column bias gradient (fp32 outputs only)
    if (n == a.bias_col) a.bias_grad[m] = (epi & EPI_ACCUM) ? a.bias_grad[m] + v : v;
    return;
  }
  long off;
  if (epi & EPI_OIHW) {  // m = co, n = (r*S + s)*Cp + ci  ->  [co][ci][r][s]
    const int rs = n / a.oihw_cp, ci = n - rs * a.oihw_cp;
    if (ci >= a.oihw_ci) return;
    off = (static_cast<long>(m) * a.oihw_ci + ci) * a.oihw_rs + rs;
  } else {
    off = static_cast<long>(m) * a.ldo + n;
  }
  if (epi & EPI_OUT_F32) {
    float* o = static_cast<float*>(a.out);
    if (epi & EPI_ACCUM) v += o[off];
    o[off] = v;
  } else {
    static_cast<uint16_t*>(a.out)[off] = f2bf(v);
  }
}

// Split-K with the reduction inside the launch: every K-slice block stores its fp32 partial tile to the
// slab workspace, then the tile's LAST arriving block (per-tile ticket) reduces all slabs in z order and
// runs the epilogue.  Publish / consume is the write-through form of cdna_hip_programming.md §6
// Guideline 16 (counter row of MI355X_MICROARCH.md § visibility): slab bytes are stored sc1 (through to
// memory, so no L2 write-back fence -- an agent-scope release here costs every K-slice block a write-back
// of its XCD's dirty L2 and measured 2x slower end to end), every storing wave drains, the block meets,
// one lane takes a relaxed agent-scope ticket; the reducer reads every slab with sc1 loads (L1 bypassed,
// so no acquire).  The reducer resets the ticket (the array starts zeroed, so every launch finds 0).
constexpr int kMaxInKernelSplits = 8;  // more slabs per tile: the serial combine loses to a reduce launch
// K-tiles staged per LDS buffer and consumed per barrier (-DPDE_GEMM_SUB=N to sweep): the MFMAs of kSub
// consecutive 32-deep K-tiles run between two barriers, each K-tile keeping its own swizzled image.
#ifndef PDE_GEMM_SUB
#define PDE_GEMM_SUB 2
#endif
constexpr int kSub = PDE_GEMM_SUB;
template <int BM, int BN>
constexpr int SMEM_BYTES_OF() { return 2 * kSub * (BM + BN) * 32 * 2; }  // gemm_kernel's LDS (BK = 32, bf16)

// ---- BatchNorm folded into the convolutions (pde_kernels.h BnStatsOut / BnFoldIn) --------------------
constexpr double kBnS1 = 4294967296.0;  // fixed-point scale of sum x   (2^32)
constexpr double kBnS2 = 1048576.0;     // fixed-point scale of sum x^2 (2^20)

// Producer epilogue: per-column sums of the tile's stored bf16 outputs (st: [BM][BN] in LDS), combined in a
// fixed order inside the block and added to the group's fixed-point sums (exact int64 atomics).  red: LDS
// scratch of 2 * (kThreads / BN) * BN floats.  Block-collective.
template <int BM, int BN>
__device__ __forceinline__ void tile_bn_stats(const GemmArgs& a, const uint16_t* st, int m0, int n0, float* red) {
  constexpr int RG = kThreads / BN, RPG = BM / RG;
  static_assert(RG * BN == kThreads && RPG * RG == BM, "stats tiling");
  if (a.bn_out.debug & 2) return;
  const int nl = threadIdx.x % BN, rg = threadIdx.x / BN;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll 4
  for (int r = 0; r < RPG; ++r) {
    const int ml = rg * RPG + r;
    if (m0 + ml < a.M) {
      const float v = bf2f(st[ml * BN + nl]);
      s1 += v;
      s2 += v * v;
    }
  }
  red[rg * BN + nl] = s1;
  red[(RG + rg) * BN + nl] = s2;
  __syncthreads();
  const int n = n0 + threadIdx.x;
  if (threadIdx.x < BN && n < a.bn_out.C) {
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int q = 0; q < RG; ++q) {
      t1 += red[q * BN + threadIdx.x];
      t2 += red[(RG + q) * BN + threadIdx.x];
    }
    const int shard = (m0 / BM) % kBnShards;
    long long* sg = a.bn_out.sums +
                    (static_cast<long>(shard) * a.bn_out.G + m0 / a.bn_out.rows_per_group) * 2 * a.bn_out.C;
    atomicAdd(reinterpret_cast<unsigned long long*>(sg + n),
              static_cast<unsigned long long>(__double2ll_rn(static_cast<double>(t1) * kBnS1)));
    atomicAdd(reinterpret_cast<unsigned long long*>(sg + a.bn_out.C + n),
              static_cast<unsigned long long>(__double2ll_rn(static_cast<double>(t2) * kBnS2)));
  }
}

// Producer, after the block's tile is done (every block, whatever its split-K role): arrival on the launch's
// ticket behind its statistics atomics; the LAST block reads and zeroes the shards and finalizes the
// BatchNorm for every (group, channel), in group
// order for the running statistics, then resets the ticket.  Block-collective; `flag`: one LDS int.
__device__ __forceinline__ void bn_stats_finalize(const GemmArgs& a, int* flag) {
  const BnStatsOut& f = a.bn_out;
  if (f.debug & 1) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's statistics atomics are performed
  __syncthreads();
  if (threadIdx.x == 0)
    flag[0] = __hip_atomic_fetch_add(f.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == f.nblocks - 1;
  __syncthreads();
  if (!flag[0]) return;
  const double n = static_cast<double>(f.rows_per_group);
  for (int c = threadIdx.x; c < f.C; c += kThreads) {
    const float gm = f.gamma ? f.gamma[c] : 1.f, bt = f.beta ? f.beta[c] : 0.f;
    float rm = f.running_mean ? f.running_mean[c] : 0.f, rv = f.running_var ? f.running_var[c] : 1.f;
    for (int g = 0; g < f.G; ++g) {
      // exact integer sums (two's complement wraps consistently).  Agent-scope loads: the adds were performed
      // at the memory side and no block of this launch cached these lines, so every load reads them; all
      // 2 x kBnShards loads of a (group, channel) are in flight at once, then the shards are zeroed for the
      // next step (plain stores, written back at the kernel boundary before the next producer's adds)
      long long s1 = 0, s2 = 0;
#pragma unroll
      for (int sh = 0; sh < kBnShards; ++sh) {
        long long* sg = f.sums + (static_cast<long>(sh) * f.G + g) * 2 * f.C;
        s1 += __hip_atomic_load(sg + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s2 += __hip_atomic_load(sg + f.C + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int sh = 0; sh < kBnShards; ++sh) {
        long long* sg = f.sums + (static_cast<long>(sh) * f.G + g) * 2 * f.C;
        sg[c] = 0;
        sg[f.C + c] = 0;
      }
      const double mean_d = static_cast<double>(s1) / kBnS1 / n;
      double var = static_cast<double>(s2) / kBnS2 / n - mean_d * mean_d;
      if (var < 0.0) var = 0.0;
      const float mean = static_cast<float>(mean_d);
      const float invstd = rsqrtf(static_cast<float>(var) + f.eps);
      const float vu = f.rows_per_group > 1 ? static_cast<float>(var * n / (n - 1.0)) : static_cast<float>(var);
      f.save_mean[g * f.C + c] = mean;
      f.save_invstd[g * f.C + c] = invstd;
      f.ss[static_cast<long>(g) * 2 * f.C + c] = gm * invstd;
      f.ss[static_cast<long>(g) * 2 * f.C + f.C + c] = bt - mean * gm * invstd;
      rm = (1.f - f.momentum) * rm + f.momentum * mean;
      rv = (1.f - f.momentum) * rv + f.momentum * vu;
    }
    if (f.running_mean) {
      f.running_mean[c] = rm;
      f.running_var[c] = rv;
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(f.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Consumer: the block's group's scale / shift into LDS ss[0..C) / ss[C..2C).  Block-collective.
__device__ __forceinline__ void bn_fold_prologue(const GemmArgs& a, int m0, float* ss) {
  const BnFoldIn& f = a.bn_in;
  const float* src = f.ss + static_cast<long>(m0 / f.rows_per_group) * 2 * f.C;
  for (int i = threadIdx.x * 4; i < 2 * f.C; i += kThreads * 4)
    *reinterpret_cast<f32x4*>(ss + i) = *reinterpret_cast<const f32x4*>(src + i);
  __syncthreads();
}

template <int BM, int BN, int FM, int FN, int WTM, int WTN>
__device__ __forceinline__ void write_slab_and_reduce(const GemmArgs& args, const f32x4 (&acc)[FM][FN],
                                                      uint16_t* smem, int m0, int n0, int kz, int wm, int wn,
                                                      int lane, int splits, int slot) {
  float* ws = args.workspace;
  const long MN = static_cast<long>(args.M) * args.N;
  // one buffer descriptor over all slabs (host checks splits*M*N*4 < 2^31)
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(ws, 0, static_cast<int>(splits * MN * 4), 0x00020000);
  constexpr int SC1 = 16;  // aux bit: write-through store / L1-bypassing load
  const bool vec = args.N % 4 == 0 && (reinterpret_cast<uintptr_t>(ws) & 15) == 0;
  if (vec && BM * BN * 4 <= SMEM_BYTES_OF<BM, BN>()) {
    // stage the partial tile in the idle LDS, then 16-byte row stores
    float* st = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int nl = wn * WTN + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) st[(wm * WTM + i * 16 + (lane >> 4) * 4 + r) * BN + nl] = acc[i][j][r];
      }
    __syncthreads();
    for (int q = threadIdx.x; q < BM * BN / 4; q += kThreads) {
      const int ml = q / (BN / 4), nl = (q % (BN / 4)) * 4;
      const int m = m0 + ml, n = n0 + nl;
      if (m < args.M && n < args.N) {
        const int off = static_cast<int>((kz * MN + static_cast<long>(m) * args.N + n) * 4);
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(st + ml * BN + nl), rsrc, off, 0, SC1);
      }
    }
  } else {
    float* slab = ws + kz * MN;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * WTN + j * 16 + (lane & 15);
        if (n >= args.N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WTM + i * 16 + (lane >> 4) * 4 + r;
          if (m < args.M)
            __hip_atomic_store(slab + static_cast<long>(m) * args.N + n, acc[i][j][r], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
      }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its slab stores
  __syncthreads();
  int* last = reinterpret_cast<int*>(smem);  // staging reads are behind the barrier: LDS is free
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(args.tickets + slot, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last[0] = t == splits - 1;
  }
  __syncthreads();
  if (!last[0]) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
  const bool out_vec = vec && !(args.epi & (EPI_OIHW | EPI_OUT_F32)) && args.ldo % 4 == 0 &&
                       (reinterpret_cast<uintptr_t>(args.out) & 7) == 0;
  if (vec) {
    // the slab loads of QG outputs per thread in flight at once (splits <= kMaxInKernelSplits, host-checked);
    // groups of QG bound the registers of the big tiles (all 16 outputs of a 128x128 tile would need 512)
    constexpr int QI = BM * BN / 4 / kThreads;
    constexpr int QG = QI < 4 ? QI : 4;
    static_assert(QI % QG == 0, "output groups");
    const bool stats = out_vec && args.bn_out.sums != nullptr;
    uint16_t* st = smem;  // [BM][BN] bf16 staging for the BatchNorm statistics
    if (stats) __syncthreads();  // every thread has read `last` (aliases st) before anyone stages
#pragma unroll 1
    for (int i0 = 0; i0 < QI; i0 += QG) {
      f32x4 v[QG];
#pragma unroll
      for (int ii = 0; ii < QG; ++ii) {
        const int q = threadIdx.x + (i0 + ii) * kThreads;
        const int m = m0 + q / (BN / 4), n = n0 + (q % (BN / 4)) * 4;
        const bool ok = m < args.M && n < args.N;
        const int off = ok ? static_cast<int>((static_cast<long>(m) * args.N + n) * 4) : 0;
        u32x4 u[kMaxInKernelSplits];
#pragma unroll
        for (int z = 0; z < kMaxInKernelSplits; ++z)
          if (z < splits) u[z] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off + static_cast<int>(z * MN * 4), 0, SC1);
        v[ii] = *reinterpret_cast<const f32x4*>(&u[0]);
#pragma unroll
        for (int z = 1; z < kMaxInKernelSplits; ++z)
          if (z < splits) v[ii] += *reinterpret_cast<const f32x4*>(&u[z]);
      }
#pragma unroll
      for (int ii = 0; ii < QG; ++ii) {
        const int q = threadIdx.x + (i0 + ii) * kThreads;
        const int m = m0 + q / (BN / 4), n = n0 + (q % (BN / 4)) * 4;
        if (stats) {  // rows / columns past the tile's extent stage zeros (skipped by the statistics)
          u16x4 z = u16x4{0, 0, 0, 0};
          if (m < args.M && n < args.N) {
#pragma unroll
            for (int j = 0; j < 4; ++j) z[j] = f2bf(apply_epi(v[ii][j], args.epi, m, n + j, args));
          }
          *reinterpret_cast<u16x4*>(st + (q / (BN / 4)) * BN + (q % (BN / 4)) * 4) = z;
        }
        if (m >= args.M || n >= args.N) continue;
        if (out_vec) {
          u16x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = f2bf(apply_epi(v[ii][j], args.epi, m, n + j, args));
          st_vec(reinterpret_cast<u16x4*>(static_cast<uint16_t*>(args.out) + static_cast<long>(m) * args.ldo + n), o,
                 args.wt != 0);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            store_out(apply_epi(v[ii][j], args.epi, m, n + j, args), args.epi, m, n + j, args);
        }
      }
    }
  } else {
    for (int q = threadIdx.x; q < BM * BN; q += kThreads) {
      const int ml = q / BN, nl = q % BN;
      const int m = m0 + ml, n = n0 + nl;
      if (m >= args.M || n >= args.N) continue;
      const long off = static_cast<long>(m) * args.N + n;
      float v = 0.f;
      for (int z = 0; z < splits; ++z) v += __hip_atomic_load(ws + z * MN + off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      store_out(apply_epi(v, args.epi, m, n, args), args.epi, m, n, args);
    }
  }
  if (vec && out_vec && args.bn_out.sums != nullptr) {
    __syncthreads();
    tile_bn_stats<BM, BN>(args, smem, m0, n0, reinterpret_cast<float*>(smem + BM * BN));
  }
  if (threadIdx.x == 0) __hip_atomic_store(args.tickets + slot, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The epilogue of one output tile from its accumulators (shared by the register-ring and LDS-DMA main loops).
// C/D map of 16x16x32: col = lane & 15, row = (lane >> 4) * 4 + reg.  smem: the block's (idle) LDS, at least
// SMEM_BYTES bytes; the caller's K loop ended with a barrier.
template <int BM, int BN, int FM, int FN, int WTM, int WTN, int SMEM_BYTES>
__device__ __forceinline__ void tile_epilogue(const GemmArgs& args, const f32x4 (&acc)[FM][FN], uint16_t* smem,
                                              const int m0, const int n0, const int kz, const int nz, const int wm,
                                              const int wn, const int lane, const int orig) {
  // A lane's outputs are 4
  // rows of one column, so direct stores are 2-byte (bf16) / 4-byte (slab) scatters.  Where the tile fits
  // the (now idle) LDS, it is staged there and written back as 16-byte row vectors instead.
  const bool split = nz > 1;
  float* ws = args.workspace;
  if (split && args.tickets != nullptr) {
    write_slab_and_reduce<BM, BN, FM, FN, WTM, WTN>(args, acc, smem, m0, n0, kz, wm, wn, lane, nz, orig);
    return;
  }
  const bool vec_bf16 = !split && !(args.epi & (EPI_OIHW | EPI_OUT_F32)) && args.N % 8 == 0 && args.ldo % 8 == 0 &&
                        (reinterpret_cast<uintptr_t>(args.out) & 15) == 0;
  const bool vec_f32 = split && args.N % 4 == 0 && (reinterpret_cast<uintptr_t>(ws) & 15) == 0;
  if constexpr (BM * BN * 2 <= SMEM_BYTES) {
    if (vec_bf16) {
      uint16_t* st = smem;  // [BM][BN] bf16 (the K loop ended with a barrier: LDS is free)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int nl = wn * WTN + j * 16 + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int ml = wm * WTM + i * 16 + (lane >> 4) * 4 + r;
            const int m = m0 + ml, n = n0 + nl;
            float v = 0.f;
            if (m < args.M && n < args.N) v = apply_epi(acc[i][j][r], args.epi, m, n, args);
            st[ml * BN + nl] = f2bf(v);
          }
        }
      __syncthreads();
      uint16_t* out = static_cast<uint16_t*>(args.out);
      for (int q = threadIdx.x; q < BM * BN / 8; q += kThreads) {
        const int ml = q / (BN / 8), nl = (q % (BN / 8)) * 8;
        const int m = m0 + ml, n = n0 + nl;
        if (m < args.M && n < args.N)
          st_vec(reinterpret_cast<u16x8*>(out + static_cast<long>(m) * args.ldo + n),
                 *reinterpret_cast<const u16x8*>(st + ml * BN + nl), args.wt != 0);
      }
      if constexpr (BM * BN * 2 + 2 * BN * (kThreads / BN) * 4 <= SMEM_BYTES && kThreads % BN == 0) {
        if (args.bn_out.sums != nullptr)  // producer of a folded BatchNorm: its statistics from the staged tile
          tile_bn_stats<BM, BN>(args, st, m0, n0, reinterpret_cast<float*>(st + BM * BN));
      }
      return;
    }
  }
  // fp32 outputs (weight gradients) without split: staged in LDS, written as 16-B row vectors with the
  // epilogue (accumulate, ones-column bias routing) applied per element
  const bool vec_f32o = !split && (args.epi & EPI_OUT_F32) && !(args.epi & EPI_OIHW) && args.ldo % 4 == 0 &&
                        (reinterpret_cast<uintptr_t>(args.out) & 15) == 0;
  if constexpr (BM * BN * 4 <= SMEM_BYTES) {
    if (vec_f32o) {
      float* st = reinterpret_cast<float*>(smem);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int nl = wn * WTN + j * 16 + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r) st[(wm * WTM + i * 16 + (lane >> 4) * 4 + r) * BN + nl] = acc[i][j][r];
        }
      __syncthreads();
      const int nvec = args.bias_grad != nullptr ? args.bias_col : args.N;  // columns with a dense home
      float* out = static_cast<float*>(args.out);
      for (int q = threadIdx.x; q < BM * BN / 4; q += kThreads) {
        const int ml = q / (BN / 4), nl = (q % (BN / 4)) * 4;
        const int m = m0 + ml, n = n0 + nl;
        if (m >= args.M || n >= args.N) continue;
        const f32x4 v = *reinterpret_cast<const f32x4*>(st + ml * BN + nl);
        if (n + 4 <= nvec) {
          f32x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = apply_epi(v[j], args.epi, m, n + j, args);
          f32x4* dst = reinterpret_cast<f32x4*>(out + static_cast<long>(m) * args.ldo + n);
          if (args.epi & EPI_ACCUM) o += *dst;
          st_vec(dst, o, args.wt != 0);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (n + j < args.N) store_out(apply_epi(v[j], args.epi, m, n + j, args), args.epi, m, n + j, args);
        }
      }
      return;
    }
    if (vec_f32) {
      float* st = reinterpret_cast<float*>(smem);  // [BM][BN] fp32 partials
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int nl = wn * WTN + j * 16 + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r) st[(wm * WTM + i * 16 + (lane >> 4) * 4 + r) * BN + nl] = acc[i][j][r];
        }
      __syncthreads();
      for (int q = threadIdx.x; q < BM * BN / 4; q += kThreads) {
        const int ml = q / (BN / 4), nl = (q % (BN / 4)) * 4;
        const int m = m0 + ml, n = n0 + nl;
        if (m < args.M && n < args.N)
          st_vec(reinterpret_cast<f32x4*>(ws + (static_cast<long>(kz) * args.M + m) * args.N + n),
                 *reinterpret_cast<const f32x4*>(st + ml * BN + nl), args.wt != 0);
      }
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * WTN + j * 16 + (lane & 15);
      if (n >= args.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WTM + i * 16 + (lane >> 4) * 4 + r;
        if (m >= args.M) continue;
        float v = acc[i][j][r];
        if (split) {
          ws[(static_cast<long>(kz) * args.M + m) * args.N + n] = v;
        } else {
          v = apply_epi(v, args.epi, m, n, args);
          store_out(v, args.epi, m, n, args);
        }
      }
    }
  }
}

// One output tile (and K slice kz of nz) of a GEMM: the body of gemm_kernel, also run by gemm_pair_kernel for
// either of its two problems.  `orig` is the block's tile slot within its problem, `smem` the block's LDS
// (SMEM_BYTES_OF<BM, BN>() bytes).
template <int BM, int BN, int BK, int WM, int WN, bool AKC, bool BKC, int AKIND, int BKIND, int STAGES,
          bool BNF = false>
__device__ __forceinline__ void gemm_tile(const GemmArgs& args, int tiles_m, int tiles_n, int k_per_split, int a_vec,
                                          int b_vec, const int orig, const int kz, const int nz, uint16_t* smem,
                                          float* bn_ss = nullptr) {
  static_assert(!BNF || (AKC && (AKIND == 0 || AKIND == 1)), "folded BatchNorm: FAST K-contiguous dense / im2col A");
  static_assert(WM * WN == 4, "4 waves per block");
  static_assert(BK == 32, "swz_chunk assumes 4 16-byte K-chunks (64 B) per LDS row");
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int LDS_A = BM * BK, LDS_B = BN * BK;
  constexpr int SMEM_BYTES = SMEM_BYTES_OF<BM, BN>();
  constexpr int KSUB = (STAGES % kSub == 0) ? kSub : 1;  // the register ring holds whole K-tile groups
  constexpr int SUBT = LDS_A + LDS_B;                    // one K-tile image (A then B)
  constexpr int BUF = KSUB * SUBT;                       // one LDS buffer: KSUB K-tile images
  static_assert(2 * BUF * 2 <= SMEM_BYTES, "LDS budget");

  // XCD-aware tile id remap (bijective; see cdna_hip_programming.md §5 "XCD swizzle").
  const int ntiles = tiles_m * tiles_n;
  int tile = orig;
  if (ntiles > 8) {
    const int q = ntiles / 8, r = ntiles % 8, xcd = orig % 8;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  // group tiles along M in bands of 8 so co-resident tiles reuse B columns
  constexpr int GROUP = 8;
  const int group_sz = GROUP * tiles_n;
  const int gid = tile / group_sz;
  const int first_m = gid * GROUP;
  const int gm = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (tile % group_sz) % gm;
  const int tn = (tile % group_sz) / gm;

  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = kz * k_per_split;
  const int kend = min(args.K, kbeg + k_per_split);
  const int nk = (kend - kbeg + BK - 1) / BK;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const bool bn_write = BNF && tn == 0;  // the first N-tile's blocks materialise the activation

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  using LA = Loader<BM, BK, AKC, AKIND>;
  using LB = Loader<BN, BK, BKC, BKIND>;
  // FAST (both kinds compile-time): every load is issued unconditionally (past the end it is masked to
  // zeros with no memory traffic), so the waits before the LDS stores are counted, not vmcnt(0)
  constexpr bool FASTK = AKIND >= 0 && BKIND >= 0;
  LA la;
  LB lb;
  const bool avec = a_vec != 0, bvec = b_vec != 0;
  la.init(args.a, args.M, m0, kbeg, args.K);
  lb.init(args.b, args.N, n0, kbeg, args.K);
  // Register ring of S K-tiles: the loads of tile t + S are issued at iteration t (before its MFMAs), so
  // S tiles of global round trips are in flight; tile t + 1 is written to the other LDS buffer after the
  // MFMAs of tile t.  Reduction bound for the loaders is kend (zero fill past the split's end).
  constexpr int S = STAGES;
  u16x8 ra[S][LA::kPer], rb[S][LB::kPer];
  // folded BatchNorm: per ring stage, the channel / activation row of each A slot (KcLoader::meta)
  [[maybe_unused]] int mca[BNF ? S : 1][LA::kPer], mra[BNF ? S : 1][LA::kPer];
  const int bn_center = BNF ? args.bn_in.center : 0;
  auto a_meta = [&](int u) {
    if constexpr (BNF) la.meta(args.a, args.M, kend, m0, bn_center, mca[u], mra[u]);
  };
  auto a_store = [&](uint16_t* dst, int u) {
    if constexpr (BNF) {
      if (args.bn_in.debug & 4)
        la.store(dst, ra[u]);
      else
        la.store_bn(dst, ra[u], mca[u], mra[u], bn_ss, args.bn_in.C, args.bn_in.relu, bn_write, args.bn_in.act);
    } else {
      la.store(dst, ra[u]);
    }
  };
  if (nk > 0) {
    la.load(args.a, args.M, kend, m0, avec, ra[0]);
    a_meta(0);
    lb.load(args.b, args.N, kend, n0, bvec, rb[0]);
#pragma unroll
    for (int u = 1; u < S; ++u) {
      if (FASTK || u < nk) {
        la.advance(args.a);
        lb.advance(args.b);
        la.load(args.a, args.M, kend, m0, avec, ra[u]);
        a_meta(u);
        lb.load(args.b, args.N, kend, n0, bvec, rb[u]);
      }
    }
    // folded BatchNorm: the coefficients' L2 round trip overlaps the ring loads just issued
    if constexpr (BNF) bn_fold_prologue(args, m0, bn_ss);
#pragma unroll
    for (int q = 0; q < KSUB; ++q) {
      if (q < nk) {
        a_store(smem + q * SUBT, q);
        lb.store(smem + q * SUBT + LDS_A, rb[q]);
      }
    }
  } else if constexpr (BNF) {
    bn_fold_prologue(args, m0, bn_ss);  // (block-collective: every block takes part)
  }
  __syncthreads();

  // one K-tile's MFMAs from its LDS image
  auto mma_tile = [&](const uint16_t* As) {
    const uint16_t* Bs = As + LDS_A;
    bf16x8 af[FM], bfr[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if constexpr (AKC) {
        const int row = wm * WTM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(As + row * BK + swz_chunk(row, lane >> 4) * 8);
      } else {
        af[i] = rc_frag<BM>(As, wm * WTM + i * 16, lane);
      }
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if constexpr (BKC) {
        const int row = wn * WTN + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + swz_chunk(row, lane >> 4) * 8);
      } else {
        bfr[j] = rc_frag<BN>(Bs, wn * WTN + j * 16, lane);
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  };

  for (int kt = 0; kt < nk; kt += S) {
#pragma unroll
    for (int u = 0; u < S; u += KSUB) {
      const int t = kt + u;  // first K-tile of this group (its KSUB images are in LDS buffer (t / KSUB) & 1)
#pragma unroll
      for (int q = 0; q < KSUB; ++q) {
        if (FASTK || t + q + S < nk) {  // refill these slots (their tiles went to LDS one group ago)
          la.advance(args.a);
          lb.advance(args.b);
          la.load(args.a, args.M, kend, m0, avec, ra[u + q]);
          a_meta(u + q);
          lb.load(args.b, args.N, kend, n0, bvec, rb[u + q]);
        }
      }
      if (t < nk) {
        const uint16_t* buf = smem + ((t / KSUB) & 1) * BUF;
#pragma unroll
        for (int q = 0; q < KSUB; ++q)
          if (q == 0 || t + q < nk) mma_tile(buf + q * SUBT);
        uint16_t* nxt = smem + (((t / KSUB) + 1) & 1) * BUF;
#pragma unroll
        for (int q = 0; q < KSUB; ++q) {
          if (t + KSUB + q < nk) {
            a_store(nxt + q * SUBT, (u + KSUB + q) % S);
            lb.store(nxt + q * SUBT + LDS_A, rb[(u + KSUB + q) % S]);
          }
        }
        __syncthreads();
      }
    }
  }

  tile_epilogue<BM, BN, FM, FN, WTM, WTN, SMEM_BYTES>(args, acc, smem, m0, n0, kz, nz, wm, wn, lane, orig);
}

template <int BM, int BN, int BK, int WM, int WN, bool AKC, bool BKC, int AKIND, int BKIND, int STAGES,
          bool BNF = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu((BM * BN >= 128 * 128) ? 1 : PDE_GEMM_WPE))) void gemm_kernel(GemmArgs args, int tiles_m, int tiles_n,
                                                        int k_per_split, int a_vec, int b_vec) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM_BYTES_OF<BM, BN>() / 2];
  float* bn_ss = nullptr;
  if constexpr (BNF) {
    __shared__ __attribute__((aligned(16))) float ss[2 * kBnFoldMaxC + 4];
    bn_ss = ss;
  }
  gemm_tile<BM, BN, BK, WM, WN, AKC, BKC, AKIND, BKIND, STAGES, BNF>(args, tiles_m, tiles_n, k_per_split, a_vec,
                                                                     b_vec, blockIdx.x, blockIdx.z, gridDim.z, smem,
                                                                     bn_ss);
  if constexpr (BM == 64 && BN == 64 && AKC && BKC && (AKIND == 0 || AKIND == 1)) {
    if (args.bn_out.sums != nullptr) {  // producer of a folded BatchNorm: the last block finalizes it
      __syncthreads();                  // (LDS is free: every epilogue path ended its LDS use)
      bn_stats_finalize(args, reinterpret_cast<int*>(smem));
    }
  }
}

// Two independent GEMMs in ONE launch (a layer's data gradient and weight gradient): blocks [0, nb0) run
// problem 0's (tile, K-slice) grid, the rest problem 1's.  Both use the 64x64 FAST configuration; the
// operand kinds are per problem.  At the reference's small per-GPU batches each backward GEMM alone leaves
// CUs idle (ResNet-50 layer4: 512 output rows; the MLP: 128) and pays its own launch boundary; the pair
// fills the chip with both grids and costs one boundary.  (A second HIP stream does not help here: a
// branched hipGraph is launched node by node on ROCm, measured 12 % slower for ResNet-50 -- ops/streams.py.)
template <bool AKC0, bool BKC0, int AK0, int BK0, bool AKC1, bool BKC1, int AK1, int BK1>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(PDE_GEMM_WPE))) void gemm_pair_kernel(
    GemmArgs a0, GemmArgs a1, PairDims d, OptimSeg seg) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM_BYTES_OF<64, 64>() / 2];
  const int t0 = d.tm[0] * d.tn[0];
  const int nb0 = t0 * d.nz[0];
  int b = blockIdx.x;
  const int nbg = nb0 + d.tm[1] * d.tn[1] * d.nz[1];
  if (b >= nbg) {  // appended optimiser blocks (another layer's update; never a tensor these GEMMs touch)
    optdev::run_segment(seg, b - nbg);
    return;
  }
  if (b < nb0) {
    gemm_tile<64, 64, 32, 2, 2, AKC0, BKC0, AK0, BK0, PDE_FAST_STAGES>(a0, d.tm[0], d.tn[0], d.kps[0], d.av[0], d.bv[0], b % t0,
                                                         b / t0, d.nz[0], smem);
  } else {
    b -= nb0;
    const int t1 = d.tm[1] * d.tn[1];
    gemm_tile<64, 64, 32, 2, 2, AKC1, BKC1, AK1, BK1, PDE_FAST_STAGES>(a1, d.tm[1], d.tn[1], d.kps[1], d.av[1], d.bv[1], b % t1,
                                                         b / t1, d.nz[1], smem);
  }
}

// ---- LDS-DMA core --------------------------------------------------------------------------------------
// The main loop above stages operands global -> VGPR ring -> LDS: every K-tile in flight costs registers, so the
// ring is 4 tiles deep at most and the 64x64 instantiations spill at the 128-VGPR cap of 4 waves / SIMD.  This core
// moves operands with gfx950's buffer_load ... lds (LDS-DMA: a 16-B per-lane load whose data goes straight into
// LDS, no VGPR destination): the staging costs no registers at all, so
//   * K-tiles are 64 deep (one barrier per 64 K, half the barriers of the ring core) and S of them are in flight
//     in an S-slot LDS ring (S = 3..4: 48-128 KB of the CU's 160 KB);
//   * the waves' registers go to accumulators: 128x128 tiles (64x64 per wave, 64 accumulator VGPRs) fit without
//     spilling (profiles/r5_gemm_regs.md);
//   * out-of-range rows, K past the split's end and conv padding taps are an out-of-range buffer offset: the
//     hardware writes zeros to LDS, no branch around any load, so every wave issues the same count per K-tile
//     and the wait for tile t is a COUNTED `s_waitcnt vmcnt(N)` that leaves tiles t+1 .. t+S-2 in flight across
//     the raw s_barrier (cdna_hip_programming.md §5 "Pipelining across barriers").
// LDS images are the ring core's, written by DMA: the LDS side of a DMA is lane-linear (wave base + 16 lane),
// so the swizzles move to the SOURCE: the lane that fills a slot fetches the chunk the swizzled image keeps there.
//   K-contiguous [rows][64] (128-B rows, eight 16-B chunks): chunk c of row r sits at slot c ^ (r & 6).  A
//     16x16x32 fragment read (ds_read_b128, lane -> row lane & 15, chunk 4h + (lane >> 4)) puts rows r / r+8 of a
//     lane group on different 16-B slots of the 256-B bank row (r & 6 spreads the four row pairs, parity picks
//     the half), so fragment reads are conflict-free.  The filling lane's row is 8 w + 32 i + lane / 8, so its
//     chunk (lane & 7) ^ ((lane >> 3) & 6) is the same for all its slots and K-tiles.
//   row-contiguous [64 k][rows]: the ring core's rc_swz image, read with ds_read_b64_tr_b16 (rc_frag).
constexpr int kDmaBK = 64;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, uint16_t* lds_wave, bool ok, long elem_off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(lds_wave), 16,
                                           ok ? static_cast<uint32_t>(elem_off * 2) : kOob, 0, 0, 0);
}

// K-contiguous operand (kinds 0 dense, 1 im2col, 3 dgrad gather): slot v = tid + 256 i holds row v / 8.
template <int ROWS, int KIND>
struct DmaKc {
  static constexpr int kPer = ROWS * 8 / kThreads;
  static_assert(kPer >= 1 && kPer * kThreads == ROWS * 8, "K-contiguous DMA rows: a multiple of 32");
  int k0;                 // reduction index of this lane's chunk at the current K-tile
  int c, kw, kh;          // kinds 1 / 3: (channel, tap) of k0
  long nb[kPer];          // row base (kind 0: row * ld_r; kinds 1 / 3: image offset), -1: row out of range
  int by[kPer], bx[kPer];
  __amdgpu_buffer_rsrc_t rsrc;

  __device__ __forceinline__ void init(const Operand& op, int rows, int row0, int kbeg, int K) {
    rsrc = operand_rsrc(op, KIND, rows, K, true);
    const int lane = threadIdx.x & 63;
    k0 = kbeg + 8 * ((lane & 7) ^ ((lane >> 3) & 6));
    c = kw = kh = 0;
    if constexpr (KIND != 0) {
      const ConvGeom& g = op.g;
      c = k0 % g.C;
      const int rs = k0 / g.C;
      kw = rs % g.S;
      kh = rs / g.S;
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int r = row0 + ((threadIdx.x + i * kThreads) >> 3);
      nb[i] = -1;
      by[i] = bx[i] = 0;
      if (r >= rows) continue;
      if constexpr (KIND == 0) {
        nb[i] = static_cast<long>(r) * op.ld_r;
      } else {
        const ConvGeom& g = op.g;
        const int HWo = g.Ho * g.Wo;
        const int n = r / HWo, rem = r - n * HWo, oy = rem / g.Wo, ox = rem - oy * g.Wo;
        nb[i] = static_cast<long>(n) * g.H * g.W * g.C;
        if constexpr (KIND == 1) {
          by[i] = oy * g.stride - g.pad;
          bx[i] = ox * g.stride - g.pad;
        } else {  // (oy, ox) are dx coordinates; dy has dims H x W
          by[i] = oy + g.pad;
          bx[i] = ox + g.pad;
        }
      }
    }
  }

  __device__ __forceinline__ void advance(const Operand& op) {
    k0 += kDmaBK;
    if constexpr (KIND != 0) {
      c += kDmaBK;
      while (c >= op.g.C) {
        c -= op.g.C;
        if (++kw == op.g.S) {
          kw = 0;
          ++kh;
        }
      }
    }
  }

  // issue this K-tile's slots into the [ROWS][64] image at `img` (K = the split's end)
  __device__ __forceinline__ void issue(const Operand& op, int K, uint16_t* img, int wave) const {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      bool ok = k0 < K && nb[i] >= 0;
      long off;
      if constexpr (KIND == 0) {
        off = nb[i] + k0;
      } else {
        const ConvGeom& g = op.g;
        int iy, ix;
        if constexpr (KIND == 1) {
          iy = by[i] + kh;
          ix = bx[i] + kw;
        } else {
          iy = by[i] - kh;
          ix = bx[i] - kw;
          ok = ok && iy >= 0 && ix >= 0;
          if (g.stride == 2) {
            ok = ok && ((iy | ix) & 1) == 0;
            iy >>= 1;
            ix >>= 1;
          } else if (g.stride > 2) {
            ok = ok && (iy % g.stride) == 0 && (ix % g.stride) == 0;
            iy /= g.stride;
            ix /= g.stride;
          }
        }
        ok = ok && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
        off = nb[i] + (static_cast<long>(iy) * g.W + ix) * g.C + c;
      }
      dma16(rsrc, img + (i * kThreads + wave * 64) * 8, ok, off);
    }
  }
};

// Row-contiguous operand (kinds 0 dense, 2 im2col^T): slot v = tid + 256 i holds k-row v / (ROWS / 8) and, at
// position p = v % (ROWS / 8), the 8 consecutive rows of chunk p ^ rc_swz(k-row).
template <int ROWS, int KIND>
struct DmaRc {
  static constexpr int CH = ROWS / 8;
  static constexpr int kPer = kDmaBK * CH / kThreads;
  static_assert(kPer >= 1 && kPer * kThreads == kDmaBK * CH, "row-contiguous DMA widths 32 / 64 / 128");
  int k[kPer];             // reduction index (kind 2: output pixel) of each slot
  int c0[kPer], kw[kPer], kh[kPer];
  int n[kPer], oy[kPer], ox[kPer];
  int r0[kPer];            // first of the slot's 8 rows (kind 0), -1: out of range
  __amdgpu_buffer_rsrc_t rsrc;

  __device__ __forceinline__ void init(const Operand& op, int rows, int row0, int kbeg, int K) {
    rsrc = operand_rsrc(op, KIND, rows, K, false);
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int v = threadIdx.x + i * kThreads;
      const int kk = v / CH, p = v - kk * CH;
      const int rv = p ^ rc_swz<ROWS>(kk);
      const int rr = row0 + rv * 8;
      k[i] = kbeg + kk;
      r0[i] = rr < rows ? rr : -1;
      c0[i] = kw[i] = kh[i] = n[i] = oy[i] = ox[i] = 0;
      if constexpr (KIND == 2) {
        if (rr < rows) {
          const ConvGeom& g = op.g;
          c0[i] = rr % g.C;
          const int rs = rr / g.C;
          kw[i] = rs % g.S;
          kh[i] = rs / g.S;
        }
        const ConvGeom& g = op.g;
        const int HWo = g.Ho * g.Wo;
        n[i] = k[i] / HWo;
        const int rem = k[i] - n[i] * HWo;
        oy[i] = rem / g.Wo;
        ox[i] = rem - oy[i] * g.Wo;
      }
    }
  }

  __device__ __forceinline__ void advance(const Operand& op) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      k[i] += kDmaBK;
      if constexpr (KIND == 2) {
        ox[i] += kDmaBK;
        while (ox[i] >= op.g.Wo) {
          ox[i] -= op.g.Wo;
          if (++oy[i] == op.g.Ho) {
            oy[i] = 0;
            ++n[i];
          }
        }
      }
    }
  }

  __device__ __forceinline__ void issue(const Operand& op, int K, uint16_t* img, int wave) const {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      bool ok = k[i] < K && r0[i] >= 0;
      long off;
      if constexpr (KIND == 0) {
        off = static_cast<long>(k[i]) * op.ld_k + r0[i];
      } else {
        const ConvGeom& g = op.g;
        const int iy = oy[i] * g.stride - g.pad + kh[i];
        const int ix = ox[i] * g.stride - g.pad + kw[i];
        ok = ok && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
        off = ((static_cast<long>(n[i]) * g.H + iy) * g.W + ix) * g.C + c0[i];
      }
      dma16(rsrc, img + (i * kThreads + wave * 64) * 8, ok, off);
    }
  }
};

template <int ROWS, bool KC, int KIND>
using DmaLoader = typename std::conditional<KC, DmaKc<ROWS, KIND>, DmaRc<ROWS, KIND>>::type;

template <int BM, int BN, int S>
constexpr int dma_smem_bytes() { return S * (BM + BN) * kDmaBK * 2; }

// One output tile (K slice kz of nz) on the LDS-DMA core; smem: dma_smem_bytes<BM, BN, S>() bytes.
template <int BM, int BN, int WM, int WN, int S, bool AKC, bool BKC, int AKIND, int BKIND>
__device__ __forceinline__ void dma_tile(const GemmArgs& args, int tiles_m, int tiles_n, int k_per_split,
                                         const int orig, const int kz, const int nz, uint16_t* smem) {
  static_assert(WM * WN == 4, "4 waves per block");
  static_assert(S >= 2, "at least a double-buffered ring");
  constexpr int BK = kDmaBK;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int LDS_A = BM * BK, STAGE = (BM + BN) * BK;  // elements
  using LA = DmaLoader<BM, AKC, AKIND>;
  using LB = DmaLoader<BN, BKC, BKIND>;
  constexpr int PER_TILE = LA::kPer + LB::kPer;  // DMA instructions per thread per K-tile

  // XCD-aware tile id remap + bands of 8 row tiles (as gemm_tile)
  const int ntiles = tiles_m * tiles_n;
  int tile = orig;
  if (ntiles > 8) {
    const int q = ntiles / 8, r = ntiles % 8, xcd = orig % 8;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  constexpr int GROUP = 8;
  const int group_sz = GROUP * tiles_n;
  const int gid = tile / group_sz;
  const int first_m = gid * GROUP;
  const int gm = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (tile % group_sz) % gm;
  const int tn = (tile % group_sz) / gm;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = kz * k_per_split;
  const int kend = min(args.K, kbeg + k_per_split);
  const int nk = (kend - kbeg + BK - 1) / BK;

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  LA la;
  LB lb;
  la.init(args.a, args.M, m0, kbeg, kend);
  lb.init(args.b, args.N, n0, kbeg, kend);
  // prologue: K-tiles 0 .. S-2 in flight (tiles past the split's end are all-zero slots: uniform counts)
#pragma unroll
  for (int u = 0; u < S - 1; ++u) {
    la.issue(args.a, kend, smem + u * STAGE, wid);
    lb.issue(args.b, kend, smem + u * STAGE + LDS_A, wid);
    la.advance(args.a);
    lb.advance(args.b);
  }
  uint16_t* cur = smem;                    // stage of tile t
  uint16_t* nxt = smem + (S - 1) * STAGE;  // stage tile t + S - 1 goes to
  uint16_t* const last = smem + (S - 1) * STAGE;
  for (int t = 0; t < nk; ++t) {
    // tile t has landed (this wave's DMA: counted wait; every wave's: the barrier); tiles t+1 .. t+S-2 stay in flight
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_TILE * (S - 2)) : "memory");
    __builtin_amdgcn_s_barrier();
    // refill the slot every wave finished reading in iteration t - 1 (its MFMAs consumed those reads)
    la.issue(args.a, kend, nxt, wid);
    lb.issue(args.b, kend, nxt + LDS_A, wid);
    la.advance(args.a);
    lb.advance(args.b);
    const uint16_t* As = cur;
    const uint16_t* Bs = cur + LDS_A;
#pragma unroll
    for (int h = 0; h < BK / 32; ++h) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if constexpr (AKC) {
          const int row = wm * WTM + i * 16 + (lane & 15);
          af[i] = *reinterpret_cast<const bf16x8*>(As + row * BK + (((4 * h + (lane >> 4)) ^ (row & 6)) << 3));
        } else {
          af[i] = rc_frag<BM>(As + 32 * h * BM, wm * WTM + i * 16, lane);
        }
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if constexpr (BKC) {
          const int row = wn * WTN + j * 16 + (lane & 15);
          bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + (((4 * h + (lane >> 4)) ^ (row & 6)) << 3));
        } else {
          bfr[j] = rc_frag<BN>(Bs + 32 * h * BN, wn * WTN + j * 16, lane);
        }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    cur = cur == last ? smem : cur + STAGE;
    nxt = nxt == last ? smem : nxt + STAGE;
  }
  // drain the DMA still in flight (tail tiles past the end: zero slots) before the LDS is reused
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  tile_epilogue<BM, BN, FM, FN, WTM, WTN, dma_smem_bytes<BM, BN, S>()>(args, acc, smem, m0, n0, kz, nz, wm, wn, lane,
                                                                       orig);
}

// Blocks of a DMA kernel that fit a CU by LDS (160 KB), capped at 4: its waves / SIMD -- the register budget the
// kernel is compiled for (amdgpu_waves_per_eu), so VGPRs never cost occupancy the LDS ring leaves.
template <int BM, int BN, int S>
constexpr int dma_wpe() {
  constexpr int b = (160 * 1024) / dma_smem_bytes<BM, BN, S>();
  return b < 1 ? 1 : (b > 4 ? 4 : b);
}

template <int BM, int BN, int WM, int WN, int S, bool AKC, bool BKC, int AKIND, int BKIND>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(dma_wpe<BM, BN, S>()))) void gemm_dma_kernel(
    GemmArgs args, int tiles_m, int tiles_n, int k_per_split) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[dma_smem_bytes<BM, BN, S>() / 2];
  dma_tile<BM, BN, WM, WN, S, AKC, BKC, AKIND, BKIND>(args, tiles_m, tiles_n, k_per_split, blockIdx.x, blockIdx.z,
                                                      gridDim.z, smem);
  if constexpr (AKC && BKC && (AKIND == 0 || AKIND == 1)) {
    if (args.bn_out.sums != nullptr) {  // producer of a folded BatchNorm: the last block finalizes it
      __syncthreads();
      bn_stats_finalize(args, reinterpret_cast<int*>(smem));
    }
  }
}

// dgrad + wgrad pair on the DMA core (64x64 tiles, S-slot ring), optional optimiser blocks appended (as
// gemm_pair_kernel)
template <int S, bool AKC0, bool BKC0, int AK0, int BK0, bool AKC1, bool BKC1, int AK1, int BK1>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(dma_wpe<64, 64, S>()))) void
gemm_dma_pair_kernel(GemmArgs a0, GemmArgs a1, PairDims d, OptimSeg seg) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[dma_smem_bytes<64, 64, S>() / 2];
  const int t0 = d.tm[0] * d.tn[0];
  const int nb0 = t0 * d.nz[0];
  int b = blockIdx.x;
  const int nbg = nb0 + d.tm[1] * d.tn[1] * d.nz[1];
  if (b >= nbg) {
    optdev::run_segment(seg, b - nbg);
    return;
  }
  if (b < nb0) {
    dma_tile<64, 64, 2, 2, S, AKC0, BKC0, AK0, BK0>(a0, d.tm[0], d.tn[0], d.kps[0], b % t0, b / t0, d.nz[0], smem);
  } else {
    b -= nb0;
    const int t1 = d.tm[1] * d.tn[1];
    dma_tile<64, 64, 2, 2, S, AKC1, BKC1, AK1, BK1>(a1, d.tm[1], d.tn[1], d.kps[1], b % t1, b / t1, d.nz[1], smem);
  }
}

// ---- Skinny GEMMs: a handful of output tiles over a long K (the MLP's batch-128 linears) ---------------
// A 128 x 1024 output is 32 tiles of 64x64: too few blocks for 256 CUs, so the tile path splits K across
// blocks and pays an fp32 slab round trip plus a reduce launch per GEMM.  Here the split is ACROSS THE
// WAVES of one workgroup: a 16FM x 16FN tile per block (M=128, N=1024: 256 blocks), wave w takes K-steps
// w, w + NW, ... (32 deep), every lane loads its MFMA fragments straight from global memory (K-contiguous
// operands: one 16-B buffer load per lane per fragment, all U K-steps of a batch in flight at once;
// a row-contiguous B -- the dgrad's weight [K][N] -- goes through a wave-private LDS image read back with
// ds_read_b64_tr_b16), and the NW partial tiles meet in LDS, summed in wave order (deterministic) with the
// epilogue applied.  One launch, no slabs, no reduce kernel.  Requires dense operands, K-contiguous A, 16-B
// aligned rows, K % 8 == 0 (host-checked: skinny_ok).
constexpr int kSkinnyFM = 1, kSkinnyFN = 2, kSkinnyNW = kThreads / 64;
template <bool BKC>
constexpr int skinny_u() { return BKC ? 8 : 4; }  // K-steps per wave per batch
template <int FM, int FN, int NW, bool BKC>
constexpr int skinny_smem_bytes() {
  constexpr int img = BKC ? 0 : NW * skinny_u<BKC>() * 32 * 16 * FN * 2;
  constexpr int red = NW * FM * FN * 64 * 16;
  return img > red ? img : red;
}
template <int FM, int FN, int NW, bool BKC>
__device__ __forceinline__ void skinny_tile(const GemmArgs& args, int tiles_m, int tiles_n, int orig,
                                            uint16_t* smem) {
  constexpr int U = skinny_u<BKC>();
  constexpr int TM = 16 * FM, TN = 16 * FN;
  static_assert(BKC || TN == 32 || TN == 64 || TN == 128, "row-contiguous B image widths (rc_swz)");
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware: consecutive tile ids (the tiles_m row tiles of one B column block) on one XCD's L2
  const int ntiles = tiles_m * tiles_n;
  int tile = orig;
  if (ntiles > 8) {
    const int q = ntiles / 8, r = ntiles % 8, xcd = orig % 8;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  const int tn = tile / tiles_m, tm = tile - tn * tiles_m;
  const int m0 = tm * TM, n0 = tn * TN;
  const int K = args.K, nks = (K + 31) / 32;
  const auto ra = operand_rsrc(args.a, 0, args.M, K, true);
  const auto rb = operand_rsrc(args.b, 0, args.N, K, BKC);
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint16_t* img = smem + w * (U * 32 * TN);  // row-contiguous B only: [U][32 k][TN] per wave
  const int kq = 8 * (lane >> 4);
  for (int b0 = 0; b0 < nks; b0 += NW * U) {  // uniform trip count: the barriers below are legal
    u16x8 fa[U][FM], fb[U][FN];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ks = b0 + w + u * NW;
      const int k = ks * 32 + kq;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = m0 + 16 * i + (lane & 15);
        fa[u][i] = bload16(ra, ks < nks && m < args.M && k < K, static_cast<long>(m) * args.a.ld_r + k);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if constexpr (BKC) {
          const int n = n0 + 16 * j + (lane & 15);
          fb[u][j] = bload16(rb, ks < nks && n < args.N && k < K, static_cast<long>(n) * args.b.ld_r + k);
        } else {  // chunk c = lane + 64 j of the 32 x TN block: row c / (TN / 8), 8 columns at c % (TN / 8)
          const int c = lane + 64 * j, kr = c / (TN / 8), n = n0 + (c % (TN / 8)) * 8, kk = ks * 32 + kr;
          fb[u][j] = bload16(rb, ks < nks && kk < K && n < args.N, static_cast<long>(kk) * args.b.ld_k + n);
        }
      }
    }
    if constexpr (!BKC) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int c = lane + 64 * j, kr = c / (TN / 8), cc = c % (TN / 8);
          *reinterpret_cast<u16x8*>(img + u * 32 * TN + kr * TN + ((cc ^ rc_swz<TN>(kr)) << 3)) = fb[u][j];
        }
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (b0 + w + u * NW >= nks) continue;  // wave-uniform
      bf16x8 bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if constexpr (BKC) bfr[j] = __builtin_bit_cast(bf16x8, fb[u][j]);
        else bfr[j] = rc_frag<TN>(img + u * 32 * TN, 16 * j, lane);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[u][i]), bfr[j],
                                                              acc[i][j], 0, 0, 0);
    }
    if constexpr (!BKC) __syncthreads();  // images read before the next batch overwrites them
  }
  __syncthreads();  // the LDS is reused for the partial tiles
  f32x4* red = reinterpret_cast<f32x4*>(smem);  // [NW][FM][FN][64 lanes]
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) red[((w * FM + i) * FN + j) * 64 + lane] = acc[i][j];
  __syncthreads();
  // output o = ((i FN + j) 64 + lane') 4 + r: C/D map of 16x16x32 -- column lane' & 15, row 4 (lane' >> 4) + r
  for (int o = threadIdx.x; o < TM * TN; o += NW * 64) {
    const int r = o & 3, ln = (o >> 2) & 63, ij = o >> 8;
    const int i = ij / FN, j = ij - i * FN;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) v += red[((ww * FM + i) * FN + j) * 64 + ln][r];
    const int m = m0 + 16 * i + 4 * (ln >> 4) + r, n = n0 + 16 * j + (ln & 15);
    if (m < args.M && n < args.N) store_out(apply_epi(v, args.epi, m, n, args), args.epi, m, n, args);
  }
}

template <bool BKC>
__global__ __launch_bounds__(kThreads) void gemm_skinny_kernel(GemmArgs args, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[skinny_smem_bytes<kSkinnyFM, kSkinnyFN, kSkinnyNW, BKC>() / 2];
  skinny_tile<kSkinnyFM, kSkinnyFN, kSkinnyNW, BKC>(args, tiles_m, tiles_n, blockIdx.x, smem);
}

// A layer's skinny dgrad (problem 0) and its weight gradient on the 64x64 FAST tile (problem 1) in one launch.
template <bool BKC0, bool AKC1, bool BKC1, int AK1, int BK1>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void gemm_pair_skinny_kernel(
    GemmArgs a0, int tm0, int tn0, GemmArgs a1, PairDims d, OptimSeg seg) {
  constexpr int kS = skinny_smem_bytes<kSkinnyFM, kSkinnyFN, kSkinnyNW, BKC0>();
  constexpr int kT = SMEM_BYTES_OF<64, 64>();
  __shared__ __attribute__((aligned(16))) uint16_t smem[(kS > kT ? kS : kT) / 2];
  const int nb0 = tm0 * tn0;
  const int b = blockIdx.x;
  const int nbg = nb0 + d.tm[1] * d.tn[1] * d.nz[1];
  if (b >= nbg) {  // appended optimiser blocks
    optdev::run_segment(seg, b - nbg);
    return;
  }
  if (b < nb0) {
    skinny_tile<kSkinnyFM, kSkinnyFN, kSkinnyNW, BKC0>(a0, tm0, tn0, b, smem);
  } else {
    const int t1 = d.tm[1] * d.tn[1], b1 = b - nb0;
    gemm_tile<64, 64, 32, 2, 2, AKC1, BKC1, AK1, BK1, PDE_FAST_STAGES>(a1, d.tm[1], d.tn[1], d.kps[1], d.av[1],
                                                                       d.bv[1], b1 % t1, b1 / t1, d.nz[1], smem);
  }
}

// Split-K slab reduction, scalar form (N % 4 != 0).
__global__ void gemm_splitk_reduce(GemmArgs args, int splits) {
  const long total = static_cast<long>(args.M) * args.N;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    float v = 0.f;
    for (int z = 0; z < splits; ++z) v += args.workspace[z * total + i];
    const int m = static_cast<int>(i / args.N);
    const int n = static_cast<int>(i - static_cast<long>(m) * args.N);
    v = apply_epi(v, args.epi, m, n, args);
    store_out(v, args.epi, m, n, args);
  }
}

// Split-K slab reduction, vector form (N % 4 == 0): a block covers COLS float4 columns of the [M][N]
// output with LANES slab-lanes each (thread = column + COLS x lane); partials meet in LDS in a fixed
// order (deterministic), then the epilogue runs on the 4 outputs of each column.
template <int LANES>
__device__ __forceinline__ void splitk_reduce4_block(const GemmArgs& args, int splits, int block) {
  constexpr int COLS = 256 / LANES;
  __shared__ f32x4 part[LANES][COLS];
  const int total4 = args.M * (args.N / 4);
  const int col = threadIdx.x % COLS, sl = threadIdx.x / COLS;
  const int c4 = block * COLS + col;
  const f32x4* w4 = reinterpret_cast<const f32x4*>(args.workspace);
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
  if (c4 < total4) {
    int z = sl;
    for (; z + LANES < splits; z += 2 * LANES) {
      a0 += w4[static_cast<long>(z) * total4 + c4];
      a1 += w4[static_cast<long>(z + LANES) * total4 + c4];
    }
    for (; z < splits; z += LANES) a0 += w4[static_cast<long>(z) * total4 + c4];
  }
  f32x4 v = a0 + a1;
  if constexpr (LANES > 1) {
    part[sl][col] = v;
    __syncthreads();
    if (sl == 0) {
#pragma unroll
      for (int k = 1; k < LANES; ++k) v += part[k][col];
    }
  }
  if (sl == 0 && c4 < total4) {
    const int q = args.N / 4;
    const int m = c4 / q, n = (c4 - m * q) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) store_out(apply_epi(v[j], args.epi, m, n + j, args), args.epi, m, n + j, args);
  }
}
template <int LANES>
__global__ __launch_bounds__(256) void gemm_splitk_reduce4(GemmArgs args, int splits) {
  splitk_reduce4_block<LANES>(args, splits, blockIdx.x);
}
// the slab reductions of a GEMM pair in one launch (blocks [0, nb0): problem 0)
template <int L0, int L1>
__global__ __launch_bounds__(256) void gemm_splitk_reduce4_pair(GemmArgs a0, int s0, int nb0, GemmArgs a1, int s1) {
  if (static_cast<int>(blockIdx.x) < nb0)
    splitk_reduce4_block<L0>(a0, s0, blockIdx.x);
  else
    splitk_reduce4_block<L1>(a1, s1, blockIdx.x - nb0);
}

// Deferred weight-gradient slab reductions, batched: up to kMaxReduceJobs split-K GEMMs whose outputs are
// only read later (weight gradients accumulated into .grad) reduce in ONE launch at the end of backward
// instead of one launch per layer.  The job table travels by value in the kernel arguments (no host
// buffer the hipGraph would have to keep alive); block b reduces job j for b in [first[j], first[j+1]).
struct ReduceJobs {
  ReduceJob job[kMaxReduceJobs];
  int first[kMaxReduceJobs + 1];
  int n;
};
__global__ __launch_bounds__(256) void gemm_splitk_reduce_jobs(ReduceJobs t) {
  int j = 0;
  while (j + 1 < t.n && static_cast<int>(blockIdx.x) >= t.first[j + 1]) ++j;
  const ReduceJob& r = t.job[j];
  GemmArgs a{};
  a.M = r.M; a.N = r.N; a.out = r.out; a.ldo = r.ldo; a.epi = r.epi; a.workspace = r.workspace;
  a.oihw_ci = r.oihw_ci; a.oihw_rs = r.oihw_rs; a.oihw_cp = r.oihw_cp;
  a.bias_grad = r.bias_grad; a.bias_col = r.bias_col;
  // the same slab-lane count as the immediate reduction of this split count: identical summation order
  const int b = blockIdx.x - t.first[j];
  if (r.splits <= 2)
    splitk_reduce4_block<1>(a, r.splits, b);
  else if (r.splits <= 16)
    splitk_reduce4_block<4>(a, r.splits, b);
  else
    splitk_reduce4_block<16>(a, r.splits, b);
}


// ---- LDS-DMA kernel launchers (host templates; instantiated by gemm_dma_*.hip) ----------------------------
// a paired launch's operand orientation + kinds, one code per problem
constexpr int kind_code(bool akc, bool bkc, int ak, int bk) { return (akc ? 1 : 0) | (bkc ? 2 : 0) | (ak << 2) | (bk << 4); }
template <int BM, int BN, int S, bool AKC, bool BKC, int AK, int BKN>
void launch_dma1(dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps) {
  hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, 2, 2, S, AKC, BKC, AK, BKN>), grid, dim3(kThreads), 0, s, ka, tm, tn,
                     kps);
}
template <int BM, int BN, int S, bool AKC, bool BKC>
bool launch_dma_kinds(dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps) {
  const int ak = ka.a.kind, bk = ka.b.kind;
  if constexpr (AKC && BKC) {
    if (bk != 0) return false;
    if (ak == 0) return launch_dma1<BM, BN, S, true, true, 0, 0>(grid, s, ka, tm, tn, kps), true;
    if (ak == 1) return launch_dma1<BM, BN, S, true, true, 1, 0>(grid, s, ka, tm, tn, kps), true;
    if (ak == 3) return launch_dma1<BM, BN, S, true, true, 3, 0>(grid, s, ka, tm, tn, kps), true;
  } else if constexpr (AKC && !BKC) {
    if (bk != 0) return false;  // (an im2col^T B only occurs with a row-contiguous A: weight gradients)
    if (ak == 0) return launch_dma1<BM, BN, S, true, false, 0, 0>(grid, s, ka, tm, tn, kps), true;
    if (ak == 3) return launch_dma1<BM, BN, S, true, false, 3, 0>(grid, s, ka, tm, tn, kps), true;
  } else if constexpr (!AKC && BKC) {
    if (ak == 0 && bk == 0) return launch_dma1<BM, BN, S, false, true, 0, 0>(grid, s, ka, tm, tn, kps), true;
  } else {
    if (ak != 0) return false;
    if (bk == 0) return launch_dma1<BM, BN, S, false, false, 0, 0>(grid, s, ka, tm, tn, kps), true;
    if (bk == 2) return launch_dma1<BM, BN, S, false, false, 0, 2>(grid, s, ka, tm, tn, kps), true;
  }
  return false;
}
// the 64x64 tile's ring depths (a launch-time choice: deep rings for grids of <= 1 block per CU with long K,
// shallow ones -- more blocks per CU -- for big grids); the bigger tiles use 3 slots
constexpr int kDmaS64[5] = {2, 3, 4, 6, 8};
template <bool AKC, bool BKC>
bool launch_dma_cfg(int cfg, int s64, dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps) {
  switch (cfg) {
    case 3: return launch_dma_kinds<128, 128, 3, AKC, BKC>(grid, s, ka, tm, tn, kps);
    case 1: return launch_dma_kinds<128, 64, 3, AKC, BKC>(grid, s, ka, tm, tn, kps);
    case 2: return launch_dma_kinds<64, 128, 3, AKC, BKC>(grid, s, ka, tm, tn, kps);
    default:
      switch (s64) {
        case 2: return launch_dma_kinds<64, 64, 2, AKC, BKC>(grid, s, ka, tm, tn, kps);
        case 4: return launch_dma_kinds<64, 64, 4, AKC, BKC>(grid, s, ka, tm, tn, kps);
        case 6: return launch_dma_kinds<64, 64, 6, AKC, BKC>(grid, s, ka, tm, tn, kps);
        case 8: return launch_dma_kinds<64, 64, 8, AKC, BKC>(grid, s, ka, tm, tn, kps);
        default: return launch_dma_kinds<64, 64, 3, AKC, BKC>(grid, s, ka, tm, tn, kps);
      }
  }
}

}  // namespace

// implemented in gemm_dma_{tt,tf,ft,ff}.hip (operand orientations: K-contiguous A / B or not), gemm_dma_pair.hip
// cfg: 0 64x64, 1 128x64, 2 64x128, 3 128x128; s64: ring slots of the 64x64 tile (kDmaS64).  false: no
// instantiation for these operand kinds.
bool dma_launch_tt(int cfg, int s64, dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps);
bool dma_launch_tf(int cfg, int s64, dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps);
bool dma_launch_ft(int cfg, int s64, dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps);
bool dma_launch_ff(int cfg, int s64, dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps);
// pairs: s = 3 or 6 ring slots
bool dma_launch_pair(int s, int k0, int k1, dim3 grid, hipStream_t st, const GemmArgs& a0, const GemmArgs& a1,
                     const PairDims& d, const OptimSeg& seg);

}  // namespace pde
