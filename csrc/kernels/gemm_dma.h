// LDS-DMA GEMM core (buffer_load ... lds into an S-slot LDS ring, counted vmcnt waits, software-pipelined
// fragment reads) and its host-side launch templates.  Instantiated by the gemm_dma_*.hip translation units.
#pragma once

#include "gemm_common.h"
#include "gemm_dma_api.h"

namespace pde {

namespace {

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
  // one 32-deep half (h) of a K-tile's fragments from its LDS image
  auto read_frags = [&](const uint16_t* st, int h, bf16x8 (&af)[FM], bf16x8 (&bfr)[FN]) {
    const uint16_t* As = st;
    const uint16_t* Bs = st + LDS_A;
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
  };
  auto mma = [&](const bf16x8 (&af)[FM], const bf16x8 (&bfr)[FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  };
  // Software pipeline (all S ring slots in flight; tiles past the split's end are all-zero slots, so every wave
  // issues the same DMA count per K-tile and the waits are counted):
  //   prologue: DMA tiles 0 .. S-1; wait tile 0; barrier; read F0 = (tile 0, half 0)
  //   iteration t: read F1 = (t, half 1) | MFMA F0 | this wave's LDS reads drained, tile t+1 landed (counted
  //   vmcnt), barrier -> nobody reads tile t's slot any more: DMA tile t+S into it | read F0 = (t+1, half 0) |
  //   MFMA F1 -- every fragment read overlaps the MFMAs of the other half, one barrier per 64-deep K-tile.
#pragma unroll
  for (int u = 0; u < S; ++u) {
    la.issue(args.a, kend, smem + u * STAGE, wid);
    lb.issue(args.b, kend, smem + u * STAGE + LDS_A, wid);
    la.advance(args.a);
    lb.advance(args.b);
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_TILE * (S - 1)) : "memory");
  __builtin_amdgcn_s_barrier();
  bf16x8 fa0[FM], fb0[FN], fa1[FM], fb1[FN];
  read_frags(smem, 0, fa0, fb0);
  uint16_t* cur = smem;  // slot of tile t
  uint16_t* const last = smem + (S - 1) * STAGE;
  for (int t = 0; t < nk; ++t) {
    uint16_t* nxt = cur == last ? smem : cur + STAGE;  // slot of tile t + 1
    read_frags(cur, 1, fa1, fb1);
    __builtin_amdgcn_sched_barrier(0);
    mma(fa0, fb0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of tile t are done
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_TILE * (S - 2)) : "memory");  // tile t+1 landed (this wave)
    __builtin_amdgcn_s_barrier();                         // (every wave)
    la.issue(args.a, kend, cur, wid);                     // tile t+S -> tile t's slot
    lb.issue(args.b, kend, cur + LDS_A, wid);
    la.advance(args.a);
    lb.advance(args.b);
    read_frags(nxt, 0, fa0, fb0);
    __builtin_amdgcn_sched_barrier(0);
    mma(fa1, fb1);
    __builtin_amdgcn_sched_barrier(0);
    cur = nxt;
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


// ---- LDS-DMA kernel launchers (host templates; instantiated by gemm_dma_*.hip) ----------------------------
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

}  // namespace pde
