// Register-ring GEMM core (global -> VGPR ring -> LDS), its dgrad + wgrad pair kernel, the skinny (K split over
// waves) kernels and the split-K slab reductions.  Instantiated by gemm.hip.
#pragma once

#include "gemm_common.h"

namespace pde {

namespace {

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
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
  if (c4 < total4) {
    // four slabs per trip, all loads issued before the adds (a lane sums <= 4 slabs at every split count the
    // lane choice allows: one memory round trip instead of two or four dependent ones)
    int z = sl;
    for (; z + 3 * LANES < splits; z += 4 * LANES) {
      const f32x4 x0 = w4[static_cast<long>(z) * total4 + c4];
      const f32x4 x1 = w4[static_cast<long>(z + LANES) * total4 + c4];
      const f32x4 x2 = w4[static_cast<long>(z + 2 * LANES) * total4 + c4];
      const f32x4 x3 = w4[static_cast<long>(z + 3 * LANES) * total4 + c4];
      a0 += x0;
      a1 += x1;
      a2 += x2;
      a3 += x3;
    }
    for (; z < splits; z += LANES) a0 += w4[static_cast<long>(z) * total4 + c4];
  }
  f32x4 v = (a0 + a1) + (a2 + a3);
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



}  // namespace

}  // namespace pde
