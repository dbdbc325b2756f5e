// Device side of the bf16 MFMA GEMM shared by both main loops (see gemm.hip for the design notes): operand
// loaders and swizzles, epilogues (split-K slabs, in-launch reduction, BatchNorm statistics), constants.
// gemm_ring.h (register-ring core, skinny + reduce kernels; instantiated by gemm.hip) and gemm_dma.h (LDS-DMA
// core; instantiated by the gemm_dma_*.hip translation units, built in parallel) build on it.  Everything is
// in an anonymous namespace: each translation unit gets its own copies.
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
#include "gemm_dma_api.h"

namespace pde {

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
    // the slab loads of QG outputs per thread, ZC slabs at a time, in flight at once (splits <= kMaxInKernelSplits,
    // host-checked): QG x ZC x 16 B = 64 VGPRs.  (All kMaxInKernelSplits slabs of QG outputs at once -- 128 VGPRs of
    // loads -- was where every 4-wave tile instantiation spilled: 136-208 B of scratch per lane, r5_gemm_regs.md.)
    // Summation stays in slab order z = 0, 1, ... (bitwise the reduce launch's order).
    constexpr int QI = BM * BN / 4 / kThreads;
    constexpr int QG = QI < 4 ? QI : 4;
    constexpr int ZC = 4;
    static_assert(QI % QG == 0 && kMaxInKernelSplits % ZC == 0, "output groups / slab chunks");
    const bool stats = out_vec && args.bn_out.sums != nullptr;
    uint16_t* st = smem;  // [BM][BN] bf16 staging for the BatchNorm statistics
    if (stats) __syncthreads();  // every thread has read `last` (aliases st) before anyone stages
#pragma unroll 1
    for (int i0 = 0; i0 < QI; i0 += QG) {
      f32x4 v[QG];
      int off[QG];
#pragma unroll
      for (int ii = 0; ii < QG; ++ii) {
        const int q = threadIdx.x + (i0 + ii) * kThreads;
        const int m = m0 + q / (BN / 4), n = n0 + (q % (BN / 4)) * 4;
        const bool ok = m < args.M && n < args.N;
        off[ii] = ok ? static_cast<int>((static_cast<long>(m) * args.N + n) * 4) : 0;
      }
#pragma unroll
      for (int z0 = 0; z0 < kMaxInKernelSplits; z0 += ZC) {
        if (z0 >= splits) break;  // block-uniform
        u32x4 u[QG][ZC];
#pragma unroll
        for (int ii = 0; ii < QG; ++ii)
#pragma unroll
          for (int zz = 0; zz < ZC; ++zz)
            if (z0 + zz < splits)
              u[ii][zz] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off[ii] + static_cast<int>((z0 + zz) * MN * 4), 0,
                                                                SC1);
#pragma unroll
        for (int ii = 0; ii < QG; ++ii)
#pragma unroll
          for (int zz = 0; zz < ZC; ++zz) {
            if (z0 + zz >= splits) continue;
            const f32x4 x = *reinterpret_cast<const f32x4*>(&u[ii][zz]);
            if (z0 + zz == 0) v[ii] = x;
            else v[ii] += x;
          }
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

// a paired launch's operand orientation + kinds, one code per problem
constexpr int kind_code(bool akc, bool bkc, int ak, int bk) { return (akc ? 1 : 0) | (bkc ? 2 : 0) | (ak << 2) | (bk << 4); }

}  // namespace

}  // namespace pde
