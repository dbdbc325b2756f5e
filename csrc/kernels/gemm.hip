// bf16 MFMA GEMM / implicit-GEMM convolution for gfx950 (CDNA4).
//
//   C[m, n] = epilogue( sum_k A[m, k] * B[n, k] )
//
// One kernel template serves every matmul-shaped op of the suite: nn.Linear
// forward / dgrad / wgrad, and NHWC implicit-GEMM convolution forward / dgrad / wgrad (the
// operands are gathered from the activation on the fly -- no im2col buffer in HBM).
//
// Structure (cdna_hip_programming.md §5 "standard MFMA GEMM main loop"):
//   * 256 threads = 4 wave64s arranged WM x WN, each wave owns a (BM/WM) x (BN/WN) sub-tile made
//     of 16x16 fragments computed with v_mfma_f32_16x16x32_bf16 (fp32 accumulate).
//   * A and B tiles are staged global -> registers (a ring of STAGES K-tiles) -> LDS, double-buffered:
//     the global loads of K-tile t+STAGES are issued before the MFMAs of tile t and tile t+1 is written to
//     the other LDS buffer after
//     them (async-STAGE split, T14), one barrier per K-tile.
//   * K-contiguous operands: LDS images are unpadded K-contiguous 64-B rows with an XOR chunk swizzle, so
//     MFMA fragments are single conflict-free ds_read_b128 (see swz_chunk).
//     Operands contiguous along the row (M/N) dimension -- the transposed operands of dgrad / wgrad -- are
//     stored as loaded: [k][row] images written with 16-B stores, and the MFMA fragments are read with
//     gfx950's transposing LDS read (ds_read_b64_tr_b16, two per fragment; see rc_swz / rc_frag), so no
//     operand is ever scattered element-wise into LDS.
//   * Implicit-GEMM gathers keep per-slot state: a row's (image, output-pixel) decomposition is done
//     once per block, and the slot's (kh, kw, c) -- or, for the weight-gradient operand, its output
//     pixel -- is advanced incrementally by BK per K-tile, so the K loop has no integer division.
//   * Tiles are mapped XCD-aware (T1): consecutive tile ids go to the same XCD group so tiles
//     sharing A rows / B columns hit the same L2.
//   * Split-K writes fp32 partial slabs, summed in fixed z order (deterministic) by a vectorised
//     slab-reduction kernel that applies the fused epilogue.  Opt-in (PDE_GEMM_INKERNEL_SPLITK=1): the LAST
//     K-slice block of a tile to arrive reduces in the same launch (write-through slabs -> per-tile ticket,
//     cdna_hip_programming.md §5 "in-launch split-K reduction") -- measured slower here, see split_tickets.
//   * Epilogue options: bias, ReLU, ReLU-mask (backward), fp32 / bf16 output, accumulate, and an OIHW
//     remap that writes a conv weight gradient straight into the parameter's [Co][Ci][R][S] fp32 grad.
#include "gemm_ring.h"
#include "gemm_lowk.h"

namespace pde {

namespace {

// Per-tile arrival counters for the in-kernel split-K reduction: one zeroed device array per GPU, handed
// out in rolling windows (consecutive launches on one stream may share slots -- each launch leaves its
// tickets at 0 -- and the window keeps launches on different streams apart).  Allocated on first use
// outside a graph capture; until then (or if allocation fails) split GEMMs use the reduce kernel.
// OPT-IN (PDE_GEMM_INKERNEL_SPLITK=1): measured on MI355X (scripts/gpu_gemm_ab.sh, profiles/README.md r2c)
// the last-arriver combine is slower than the separate, chip-wide reduce launch on both the MLP
// (0.39 vs 0.33 ms/step) and ResNet-50 (5.89 vs 5.80 ms/step): the tile's reducer is one workgroup reading
// up to 8 slabs after the whole K range finished, a serial tail the 1.5-2 us launch boundary does not cost.
constexpr int kTicketSlots = 1 << 22;
// force: a producer of BatchNorm statistics needs the in-launch combine (its last arriver emits them)
int* split_tickets(int tiles, hipStream_t s, bool force = false) {
  static int* base[64] = {};
  static int next[64] = {};
  static bool enabled = std::getenv("PDE_GEMM_INKERNEL_SPLITK") != nullptr &&
                        std::getenv("PDE_GEMM_INKERNEL_SPLITK")[0] == '1';
  if ((!enabled && !force) || tiles > kTicketSlots) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (base[dev] == nullptr) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return nullptr;
    void* p = nullptr;
    if (hipMalloc(&p, sizeof(int) * kTicketSlots) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, sizeof(int) * kTicketSlots) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(p);
      return nullptr;
    }
    base[dev] = static_cast<int*>(p);
  }
  if (next[dev] + tiles > kTicketSlots) next[dev] = 0;
  int* t = base[dev] + next[dev];
  next[dev] += tiles;
  return t;
}

// FAST instantiations: (A kind, B kind) pairs that occur -- K-contiguous A: dense, im2col, dgrad gather;
// row-contiguous A: dense (dy^T); K-contiguous B: dense weights; row-contiguous B: dense, im2col^T.
constexpr int kFastStages = PDE_FAST_STAGES;
template <int BM, int BN, int BK, int WM, int WN, bool AKC, bool BKC, int AK, int BKN>
void launch_fast1(dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps, int av, int bv) {
  hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, AKC, BKC, AK, BKN, kFastStages>), grid, dim3(kThreads), 0, s,
                     ka, tm, tn, kps, av, bv);
}
template <int BM, int BN, int BK, int WM, int WN, bool AKC, bool BKC, int AK>
bool launch_fast_b(dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps, int av, int bv) {
  const int bk = ka.b.kind;
  if (bk == 0) {
    launch_fast1<BM, BN, BK, WM, WN, AKC, BKC, AK, 0>(grid, s, ka, tm, tn, kps, av, bv);
    return true;
  }
  if constexpr (!BKC) {
    if (bk == 2) {
      launch_fast1<BM, BN, BK, WM, WN, AKC, BKC, AK, 2>(grid, s, ka, tm, tn, kps, av, bv);
      return true;
    }
  }
  return false;
}
template <int BM, int BN, int BK, int WM, int WN, bool AKC, bool BKC>
bool launch_fast(dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps, int av, int bv) {
  const int ak = ka.a.kind;
  if (ak == 0) return launch_fast_b<BM, BN, BK, WM, WN, AKC, BKC, 0>(grid, s, ka, tm, tn, kps, av, bv);
  if constexpr (AKC) {
    if (ak == 1) return launch_fast_b<BM, BN, BK, WM, WN, AKC, BKC, 1>(grid, s, ka, tm, tn, kps, av, bv);
    if (ak == 3) return launch_fast_b<BM, BN, BK, WM, WN, AKC, BKC, 3>(grid, s, ka, tm, tn, kps, av, bv);
  }
  return false;
}

// Slab reduction of a split-K GEMM: the vector form's slab-lane count follows the split count.
bool reduce_vec_ok(const GemmArgs& a) {
  const long total = static_cast<long>(a.M) * a.N;
  return a.N % 4 == 0 && total / 4 < (1L << 30) && (reinterpret_cast<uintptr_t>(a.workspace) & 15) == 0;
}
int reduce_lanes(int splitk) { return splitk <= 2 ? 1 : (splitk <= 16 ? 4 : 16); }
void launch_reduce(const GemmArgs& a, int splitk, hipStream_t s) {
  const long total = static_cast<long>(a.M) * a.N;
  if (reduce_vec_ok(a)) {
    const long t4 = total / 4;
    const int lanes = reduce_lanes(splitk);
    if (lanes == 1)
      hipLaunchKernelGGL(gemm_splitk_reduce4<1>, dim3(ceil_div(t4, 256)), dim3(256), 0, s, a, splitk);
    else if (lanes == 4)
      hipLaunchKernelGGL(gemm_splitk_reduce4<4>, dim3(ceil_div(t4, 64)), dim3(256), 0, s, a, splitk);
    else
      hipLaunchKernelGGL(gemm_splitk_reduce4<16>, dim3(ceil_div(t4, 16)), dim3(256), 0, s, a, splitk);
  } else {
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3(stream_grid(total, 256)), dim3(256), 0, s, a, splitk);
  }
}

// Vector (16 B) loads are legal when the contiguous dimension and the other stride keep every 8-element
// group 16-byte aligned.
int vec_ok(const Operand& o, bool kc) {
  if (o.kind != 0) return 1;
  if (kc) return (o.ld_k == 1 && o.ld_r % 8 == 0 && (reinterpret_cast<uintptr_t>(o.ptr) & 15) == 0) ? 1 : 0;
  return (o.ld_r == 1 && o.ld_k % 8 == 0 && (reinterpret_cast<uintptr_t>(o.ptr) & 15) == 0) ? 1 : 0;
}
// FAST: the operand can be loaded branch-free through a buffer descriptor (gathers always; dense operands
// when every 16-B group is whole and aligned, extents < 2 GB).
bool fast_ok(const GemmArgs& a, const Operand& o, bool kc, int rows) {
  long elems;
  if (o.kind != 0) {
    elems = static_cast<long>(o.g.N) * o.g.H * o.g.W * o.g.C;
  } else {
    if (!vec_ok(o, kc)) return false;
    // K-contiguous: whole 8-element K groups; row-contiguous: whole 8-row groups, or a row pitch that
    // holds the padded group (the loads past `rows` only feed outputs beyond M / N, never stored)
    if (kc ? (a.K % 8 != 0) : (rows % 8 != 0 && o.ld_k < (rows + 7) / 8 * 8)) return false;
    elems = kc ? static_cast<long>(rows - 1) * o.ld_r + a.K
               : static_cast<long>(a.K - 1) * o.ld_k + (rows + 7) / 8 * 8;
  }
  return elems * 2 < (1L << 31) - 16;
}
bool generic_only() {
  static const bool g = std::getenv("PDE_GEMM_GENERIC") != nullptr;  // A/B switch
  return g;
}

// PDE_GEMM_LOG=1: one stderr line per GEMM launch decision (shape, operand kinds, tile, grid, split) -- the
// shape table behind the per-kernel traces (scripts/gemm_shape_table.py joins the two).
bool gemm_log_on() {
  static const bool on = std::getenv("PDE_GEMM_LOG") != nullptr && std::getenv("PDE_GEMM_LOG")[0] == '1';
  return on;
}
void gemm_log(const char* what, const GemmArgs& a, int bm, int bn, int tiles, int split) {
  if (!gemm_log_on()) return;
  std::fprintf(stderr, "[gemm] %s M=%d N=%d K=%d akind=%d bkind=%d tile=%dx%d tiles=%d split=%d gflop=%.4f\n", what,
               a.M, a.N, a.K, a.a.kind, a.b.kind, bm, bn, tiles, split, 2e-9 * a.M * a.N * static_cast<double>(a.K));
}

template <int BM, int BN, int BK, int WM, int WN, bool AKC, bool BKC>
hipError_t launch_cfg(const GemmArgs& a, hipStream_t s, int splitk) {
  const int tm = ceil_div(a.M, BM), tn = ceil_div(a.N, BN);
  int kps = ceil_div(a.K, splitk);
  kps = ceil_div(kps, BK) * BK;
  splitk = ceil_div(a.K, kps);
  const int av = vec_ok(a.a, AKC), bv = vec_ok(a.b, BKC);
  dim3 grid(tm * tn, 1, splitk);
  gemm_log("single", a, BM, BN, tm * tn, splitk);
  GemmArgs ka = a;
  const bool in_kernel = splitk > 1 && splitk <= kMaxInKernelSplits && a.splits_out == nullptr &&
                         static_cast<long>(splitk) * a.M * a.N * 4 < (1L << 31);  // buffer offsets
  const bool stats = a.bn_out.sums != nullptr;
  ka.tickets = in_kernel ? split_tickets(tm * tn, s, stats) : nullptr;
  if (stats && splitk > 1 && ka.tickets == nullptr) return hipErrorInvalidValue;  // gemm_bn_stats_ok said no
  if (stats) ka.bn_out.nblocks = tm * tn * splitk;
  if (a.splits_out != nullptr) *a.splits_out = splitk;  // the consumer reduces the slabs (no reduce launch)
  if constexpr (BM == 64 && BN == 64 && AKC && BKC) {
    if (a.bn_in.ss != nullptr) {  // folded BatchNorm in the A loader (gemm_bn_fold_ok checked the shape)
      if (a.a.kind == 0)
        hipLaunchKernelGGL((gemm_kernel<64, 64, 32, 2, 2, true, true, 0, 0, kFastStages, true>), grid, dim3(kThreads),
                           0, s, ka, tm, tn, kps, av, bv);
      else
        hipLaunchKernelGGL((gemm_kernel<64, 64, 32, 2, 2, true, true, 1, 0, kFastStages, true>), grid, dim3(kThreads),
                           0, s, ka, tm, tn, kps, av, bv);
      if (splitk > 1 && ka.tickets == nullptr && a.splits_out == nullptr) launch_reduce(a, splitk, s);
      return hipGetLastError();
    }
  }
  // FAST: both operands loaded branch-free through buffer descriptors (gathers always; dense operands when
  // every 16-B group is whole and aligned, extents < 2 GB) with compile-time operand kinds -- then the loads
  // are counted and a register ring of kFastStages K-tiles stays in flight.  The generic loaders' divergent scalar fallbacks make the
  // compiler wait for every load (vmcnt(0)) before each LDS store, so a deeper ring buys nothing there
  // (measured r2g), and they run at depth 1.
  constexpr bool kFastTile = BM * BN < 128 * 128;  // the 128x128 tile already spills: generic only
  const bool fast = kFastTile && !generic_only() && fast_ok(a, a.a, AKC, a.M) && fast_ok(a, a.b, BKC, a.N);
  bool launched = false;
  if constexpr (kFastTile) {
    if (fast) launched = launch_fast<BM, BN, BK, WM, WN, AKC, BKC>(grid, s, ka, tm, tn, kps, av, bv);
  }
  if (!launched)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, AKC, BKC, -1, -1, 1>), grid, dim3(kThreads), 0, s, ka, tm,
                       tn, kps, av, bv);
  if (splitk > 1 && ka.tickets == nullptr && a.splits_out == nullptr) launch_reduce(a, splitk, s);
  return hipGetLastError();
}

// Tile policy (measured on ResNet-50 128^2 b32 and the 5x1024 MLP, profiles/README.md r1h).  The K loop is
// bound by global round trips (SQ_WAIT_ANY ~60% of wave cycles at 1 block per CU), so prefer the 64x64
// tile (more blocks per CU) unless the 128x128 grid already has t128_min tiles.  Split-K until the grid
// reaches split_target blocks, each split keeping >= split_min_kt K-tiles; outputs of at most
// small_mn elements (cheap fp32 slabs: the MLP's linears) split further (small_* knobs).
// PDE_GEMM_* environment variables override the knobs for tuning sweeps (read once).
struct TilePolicy {
  // r2j sweep (FAST loaders): ResNet-50 4.66 -> 4.48 ms; r2m sweep after dgrad/wgrad pairing (a paired
  // launch already fills the chip with two grids, so each member needs less split-K): split targets
  // 512 -> 256 blocks, small outputs >= 8 K-tiles per split -- ResNet-50 3.97 -> 3.84 ms, MLP 0.235 -> 0.228 ms
  // r5x re-sweep after the first-write gradient change: K-tiles per split 16 -> 8 -- ResNet-50 level (3.134 ms),
  // pipeline stage 2 at m = 8 1.398 -> 1.353 ms (profiles/r5x_split_policy_sweep.txt)
  long t128_min = 2048, split_target = 256, small_mn = 262144, small_split_target = 256;
  int split_min_kt = 8, small_split_min_kt = 8;
  // 128x64 tile (64x32 per wave: 25 % less LDS traffic per MFMA than the 64x64 tile's 32x32 wave tiles) for
  // unpaired GEMMs with at least wide_min 64x64 tiles (0: off)
  long wide_min = 0;
  TilePolicy() {
    auto env_l = [](const char* n, long& v) { if (const char* e = std::getenv(n)) v = std::atol(e); };
    auto env_i = [](const char* n, int& v) { if (const char* e = std::getenv(n)) v = std::atoi(e); };
    env_l("PDE_GEMM_T128_MIN", t128_min);
    env_l("PDE_GEMM_SPLIT_TARGET", split_target);
    env_i("PDE_GEMM_SPLIT_MIN_KT", split_min_kt);
    env_l("PDE_GEMM_SMALL_MN", small_mn);
    env_l("PDE_GEMM_SMALL_SPLIT_TARGET", small_split_target);
    env_i("PDE_GEMM_SMALL_SPLIT_MIN_KT", small_split_min_kt);
    env_l("PDE_GEMM_WIDE_MIN", wide_min);
  }
};
const TilePolicy& tile_policy() {
  static const TilePolicy p;
  return p;
}

enum TileCfg { kTile128x32, kTile32x128, kTile128, kTile64, kTile128x64 };
// The tile configuration and split-K count of a GEMM (split-K only where a workspace was provided:
// a.splitk slabs, never exceeded).  `wide`: the 128x64 tile may be chosen (single launches; pairs keep 64x64).
TileCfg choose_tiles(const GemmArgs& a, int& split, bool wide = false) {
  const TilePolicy& tp = tile_policy();
  const long t128 = static_cast<long>(ceil_div(a.M, 128)) * ceil_div(a.N, 128);
  const long t64 = static_cast<long>(ceil_div(a.M, 64)) * ceil_div(a.N, 64);
  const bool small = static_cast<long>(a.M) * a.N <= tp.small_mn;
  const long target = small ? tp.small_split_target : tp.split_target;
  const int min_kt = small ? tp.small_split_min_kt : tp.split_min_kt;
  auto pick_split = [&](long tiles, int bk) {
    if (a.workspace == nullptr || a.splitk <= 1) return 1;
    int sk = 1;
    while (sk * 2 <= a.splitk && tiles * sk < target && a.K / (sk * 2) >= min_kt * bk) sk *= 2;
    return sk;
  };
  if (a.N <= 32) {
    split = pick_split(static_cast<long>(ceil_div(a.M, 128)) * ceil_div(a.N, 32), 32);
    return kTile128x32;
  }
  if (a.M <= 32) {
    split = pick_split(static_cast<long>(ceil_div(a.M, 32)) * ceil_div(a.N, 128), 32);
    return kTile32x128;
  }
  if (t128 >= tp.t128_min) {
    split = pick_split(t128, 32);
    return kTile128;
  }
  if (wide && tp.wide_min > 0 && t64 >= tp.wide_min) {
    split = pick_split(static_cast<long>(ceil_div(a.M, 128)) * ceil_div(a.N, 64), 32);
    return kTile128x64;
  }
  split = pick_split(t64, 32);
  return kTile64;
}

// ---- LDS-DMA core dispatch --------------------------------------------------------------------------------
// PDE_GEMM_CORE=dma|ring selects the main loop (A/B switch); PDE_GEMM_DMA_TILE=64x64|128x64|64x128|128x128 forces
// the DMA tile (shape sweeps, scripts/gemm_bench.py).
#ifndef PDE_GEMM_CORE_DEFAULT
#define PDE_GEMM_CORE_DEFAULT 0
#endif
// 0 ring, 1 dma, 2 hybrid: the DMA core for the shapes where it measured faster (profiles/r5d: 3x3 forward
// convolutions up to M = 8192, and long-K problems with M <= 2048), the ring core elsewhere
int gemm_core_mode() {
  static const int mode = [] {
    const char* e = std::getenv("PDE_GEMM_CORE");
    if (e == nullptr) return static_cast<int>(PDE_GEMM_CORE_DEFAULT);
    if (std::strcmp(e, "dma") == 0) return 1;
    if (std::strcmp(e, "hybrid") == 0) return 2;
    return 0;
  }();
  return mode;
}
bool dma_core_on() { return gemm_core_mode() != 0; }
bool dma_shape_ok(const GemmArgs& a) {
  if (gemm_core_mode() != 2) return true;
  return (a.a.kind == 1 && a.M <= 8192) || (a.K >= 512 && a.M <= 2048);
}
enum DmaCfg { kD64 = 0, kD128x64 = 1, kD64x128 = 2, kD128 = 3 };
int dma_forced_tile() {
  static const int f = [] {
    const char* e = std::getenv("PDE_GEMM_DMA_TILE");
    if (e == nullptr) return -1;
    if (std::strcmp(e, "64x64") == 0) return static_cast<int>(kD64);
    if (std::strcmp(e, "128x64") == 0) return static_cast<int>(kD128x64);
    if (std::strcmp(e, "64x128") == 0) return static_cast<int>(kD64x128);
    if (std::strcmp(e, "128x128") == 0) return static_cast<int>(kD128);
    return -1;
  }();
  return f;
}
struct DmaPolicy {
  long min_blocks = 256;  // prefer the largest tile whose grid (with split-K) reaches this many blocks
  int min_k_split = 512;  // every K slice keeps at least this much K (8 DMA K-tiles)
  DmaPolicy() {
    if (const char* e = std::getenv("PDE_DMA_MIN_BLOCKS")) min_blocks = std::atol(e);
    if (const char* e = std::getenv("PDE_DMA_MIN_KSPLIT")) min_k_split = std::atoi(e);
  }
};
const DmaPolicy& dma_policy() {
  static const DmaPolicy p;
  return p;
}
int dma_split(const GemmArgs& a, long tiles) {
  const DmaPolicy& p = dma_policy();
  if (a.workspace == nullptr || a.splitk <= 1) return 1;
  int sk = 1;
  while (sk * 2 <= a.splitk && tiles * sk < p.min_blocks && a.K / (sk * 2) >= p.min_k_split) sk *= 2;
  return sk;
}
DmaCfg choose_dma(const GemmArgs& a, int& split) {
  static const int bm[4] = {64, 128, 64, 128}, bn[4] = {64, 64, 128, 128};
  const int forced = dma_forced_tile();
  if (forced >= 0) {
    split = dma_split(a, static_cast<long>(ceil_div(a.M, bm[forced])) * ceil_div(a.N, bn[forced]));
    return static_cast<DmaCfg>(forced);
  }
  const DmaPolicy& p = dma_policy();
  // largest tile first (area, then the wider side along the bigger problem dimension)
  const int order[4] = {kD128, a.M >= a.N ? kD128x64 : kD64x128, a.M >= a.N ? kD64x128 : kD128x64, kD64};
  for (int o : order) {
    if (o != kD64 && ((bm[o] == 128 && a.M < 128) || (bn[o] == 128 && a.N < 128))) continue;
    const long tiles = static_cast<long>(ceil_div(a.M, bm[o])) * ceil_div(a.N, bn[o]);
    const int sk = dma_split(a, tiles);
    if (o == kD64 || tiles * sk >= p.min_blocks) {
      split = sk;
      return static_cast<DmaCfg>(o);
    }
  }
  split = 1;
  return kD64;
}

// Ring slots of a 64x64 DMA launch of `blocks` workgroups with K slices of `kps`: PDE_DMA_S64=2|3|4|6|8 forces;
// by default the LDS ring trades blocks per CU for K-tiles in flight -- a grid of at most one block per CU
// gets the deepest ring its K slice can use (the latency-bound small layers), bigger grids more blocks per CU.
int dma_s64(long blocks, int kps) {
  static const int forced = std::getenv("PDE_DMA_S64") ? std::atoi(std::getenv("PDE_DMA_S64")) : 0;
  if (forced == 2 || forced == 3 || forced == 4 || forced == 6 || forced == 8) return forced;
  const int kt = (kps + kDmaBK - 1) / kDmaBK;
  if (blocks <= 256 && kt >= 8) return 8;
  if (blocks <= 512 && kt >= 4) return 4;
  return kt <= 2 ? 2 : 3;
}
int dma_spair(long blocks) {
  static const int forced = std::getenv("PDE_DMA_SPAIR") ? std::atoi(std::getenv("PDE_DMA_SPAIR")) : 0;
  if (forced == 3 || forced == 6) return forced;
  return blocks <= 384 ? 6 : 3;
}

// false: not launched (the caller falls back to the ring core)
bool launch_dma(int cfg, bool akc, bool bkc, const GemmArgs& a, hipStream_t s, int splitk, hipError_t& err) {
  static const int bm[4] = {64, 128, 64, 128}, bn[4] = {64, 64, 128, 128};
  const int BM = bm[cfg], BN = bn[cfg];
  const int tm = ceil_div(a.M, BM), tn = ceil_div(a.N, BN);
  int kps = ceil_div(ceil_div(a.K, splitk), kDmaBK) * kDmaBK;
  splitk = ceil_div(a.K, kps);
  const dim3 grid(tm * tn, 1, splitk);
  GemmArgs ka = a;
  const bool in_kernel = splitk > 1 && splitk <= kMaxInKernelSplits && a.splits_out == nullptr &&
                         static_cast<long>(splitk) * a.M * a.N * 4 < (1L << 31);
  const bool stats = a.bn_out.sums != nullptr;
  ka.tickets = in_kernel ? split_tickets(tm * tn, s, stats) : nullptr;
  if (stats && splitk > 1 && ka.tickets == nullptr) return false;
  if (stats) ka.bn_out.nblocks = tm * tn * splitk;
  const int s64 = cfg == kD64 ? dma_s64(static_cast<long>(tm) * tn * splitk, kps) : 3;
  bool ok;
  if (akc && bkc) ok = dma_launch_tt(cfg, s64, grid, s, ka, tm, tn, kps);
  else if (akc) ok = dma_launch_tf(cfg, s64, grid, s, ka, tm, tn, kps);
  else if (bkc) ok = dma_launch_ft(cfg, s64, grid, s, ka, tm, tn, kps);
  else ok = dma_launch_ff(cfg, s64, grid, s, ka, tm, tn, kps);
  if (!ok) return false;
  if (gemm_log_on()) {
    char what[16];
    std::snprintf(what, sizeof(what), "dma.s%d", cfg == kD64 ? s64 : 3);
    gemm_log(what, a, BM, BN, tm * tn, splitk);
  }
  if (a.splits_out != nullptr) *a.splits_out = splitk;
  if (splitk > 1 && ka.tickets == nullptr && a.splits_out == nullptr) launch_reduce(a, splitk, s);
  err = hipGetLastError();
  return true;
}
template <bool AKC, bool BKC>
bool dispatch_dma(const GemmArgs& a, hipStream_t s, hipError_t& err) {
  if (!dma_core_on() || generic_only() || a.bn_in.ss != nullptr) return false;  // (BN fold: ring core only)
  if (!dma_shape_ok(a)) return false;
  if (!fast_ok(a, a.a, AKC, a.M) || !fast_ok(a, a.b, BKC, a.N)) return false;
  int split = 1;
  const int cfg = choose_dma(a, split);
  return launch_dma(cfg, AKC, BKC, a, s, split, err);
}

template <bool AKC, bool BKC>
hipError_t dispatch_tiles(const GemmArgs& a, hipStream_t s) {
  hipError_t derr = hipSuccess;
  if (dispatch_dma<AKC, BKC>(a, s, derr)) return derr;
  int split = 1;
  switch (choose_tiles(a, split, true)) {
    case kTile128x64: return launch_cfg<128, 64, 32, 2, 2, AKC, BKC>(a, s, split);
    case kTile128x32: return launch_cfg<128, 32, 32, 4, 1, AKC, BKC>(a, s, split);
    case kTile32x128: return launch_cfg<32, 128, 32, 1, 4, AKC, BKC>(a, s, split);
    case kTile128: return launch_cfg<128, 128, 32, 2, 2, AKC, BKC>(a, s, split);
    default: return launch_cfg<64, 64, 32, 2, 2, AKC, BKC>(a, s, split);
  }
}

bool is_kc(const Operand& o) {
  if (o.kind == 1 || o.kind == 3) return true;
  if (o.kind == 2) return false;
  return o.ld_k == 1;
}

// Host mirrors of the dispatch decisions the folded BatchNorm depends on (see pde_kernels.h).
bool skinny_ok(const GemmArgs& a);
bool bn_stats_ok_impl(const GemmArgs& a, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0 || generic_only() || a.bn_out.C <= 0 || a.bn_out.rows_per_group <= 0) return false;
  if (a.epi != 0 || a.splits_out != nullptr || a.N % 8 != 0 || a.ldo % 8 != 0 || a.bn_out.C > a.N ||
      (reinterpret_cast<uintptr_t>(a.out) & 15) != 0)
    return false;
  if (a.bn_out.rows_per_group % 64 != 0 || a.M % a.bn_out.rows_per_group != 0) return false;
  if (skinny_ok(a) || !is_kc(a.a) || !is_kc(a.b)) return false;
  int split = 1;
  if (!fast_ok(a, a.a, true, a.M) || !fast_ok(a, a.b, true, a.N)) return false;
  if (dma_core_on() && dma_shape_ok(a)) {  // the DMA core emits statistics on every tile: no tile across groups
    static const int bm[4] = {64, 128, 64, 128};
    if (a.bn_out.rows_per_group % bm[choose_dma(a, split)] != 0) return false;
  } else if (choose_tiles(a, split, true) != kTile64) {
    return false;
  }
  if (split > 1) {  // the in-launch combine: its last arriver emits the statistics
    if (split > kMaxInKernelSplits || static_cast<long>(split) * a.M * a.N * 4 >= (1L << 31)) return false;
    if (split_tickets(1, s, true) == nullptr) return false;  // allocated (outside a capture) or not
  }
  return true;
}

bool bn_fold_ok_impl(const GemmArgs& a) {
  const BnFoldIn& f = a.bn_in;
  if (a.M <= 0 || a.N <= 0 || generic_only() || f.C <= 0 || f.C > kBnFoldMaxC || f.C % 8 != 0) return false;
  if (f.rows_per_group <= 0 || f.rows_per_group % 64 != 0 || f.G * f.rows_per_group != a.M) return false;
  if (skinny_ok(a) || !is_kc(a.a) || !is_kc(a.b) || a.b.kind != 0) return false;
  if (a.a.kind == 0) {
    if (a.K != f.C) return false;  // A = x [rows][C]: K index == channel
  } else if (a.a.kind == 1) {
    const ConvGeom& g = a.a.g;
    if (g.C != f.C) return false;
    if (f.center && !(g.R == 3 && g.S == 3 && g.stride == 1 && g.pad == 1 && g.Ho == g.H && g.Wo == g.W))
      return false;
  } else {
    return false;
  }
  int split = 1;
  if (choose_tiles(a, split, true) != kTile64) return false;
  return fast_ok(a, a.a, true, a.M) && fast_ok(a, a.b, true, a.N);
}

// ---- GEMM pairs ------------------------------------------------------------------------------------
int kind_code_of(const GemmArgs& a) { return kind_code(is_kc(a.a), is_kc(a.b), a.a.kind, a.b.kind); }

// Launch plan of one pair member: false unless the single-GEMM dispatch would run it on the 64x64 FAST tile
// (so the pair computes exactly what two separate launches would).
bool pair_member_plan(const GemmArgs& a, int& tm, int& tn, int& kps, int& split, int& av, int& bv,
                      bool dma = false) {
  if (a.M <= 0 || a.N <= 0 || generic_only()) return false;
  const long t64 = static_cast<long>(ceil_div(a.M, 64)) * ceil_div(a.N, 64);
  if (dma) {
    split = dma_split(a, t64);
  } else if (choose_tiles(a, split) != kTile64) {
    // a narrow (<= 32 rows or columns), short-K problem the lone launch would give a 32-wide tile: in a pair
    // it takes 64x64 tiles without split -- half-empty tiles, but one launch fewer (the MLP's 10-wide last
    // layer: its weight gradient joins the dgrad launch)
    if (!((a.M <= 32 || a.N <= 32) && t64 <= 64 && a.K <= 1024)) return false;
    split = 1;
  }
  const bool akc = is_kc(a.a), bkc = is_kc(a.b);
  if (!fast_ok(a, a.a, akc, a.M) || !fast_ok(a, a.b, bkc, a.N)) return false;
  tm = ceil_div(a.M, 64);
  tn = ceil_div(a.N, 64);
  const int bk = dma ? kDmaBK : 32;
  kps = ceil_div(ceil_div(a.K, split), bk) * bk;
  split = ceil_div(a.K, kps);
  av = vec_ok(a.a, akc);
  bv = vec_ok(a.b, bkc);
  return true;
}

template <bool AKC1, bool BKC1, int AK1, int BK1>
bool launch_pair_k0(int k0, dim3 grid, hipStream_t s, const GemmArgs& a0, const GemmArgs& a1, const PairDims& d,
                    const OptimSeg& seg) {
  switch (k0) {  // data-gradient kinds: dgrad gather / dense dy x {dgrad layout, forward copy read transposed}
#define PDE_PAIR(AKC0, BKC0, AK0, BK0)                                                                          \
  case kind_code(AKC0, BKC0, AK0, BK0):                                                                         \
    hipLaunchKernelGGL((gemm_pair_kernel<AKC0, BKC0, AK0, BK0, AKC1, BKC1, AK1, BK1>), grid, dim3(kThreads), 0, s, \
                       a0, a1, d, seg);                                                                         \
    return true;
    PDE_PAIR(true, true, 3, 0)
    PDE_PAIR(true, true, 0, 0)
    PDE_PAIR(true, false, 0, 0)
    PDE_PAIR(true, false, 3, 0)
#undef PDE_PAIR
    default: return false;
  }
}

// Skinny path (skinny_tile): dense operands, K-contiguous A, 16-B aligned rows, whole 8-element K groups, a
// plain epilogue, and an output the 64x64 tile path would cover with too few blocks for the chip (it would
// split K across blocks) while K is long enough for the in-block wave split to pay.
bool skinny_enabled() {
  static const bool on = !(std::getenv("PDE_GEMM_SKINNY") && std::getenv("PDE_GEMM_SKINNY")[0] == '0');
  return on;
}
bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
bool skinny_ok(const GemmArgs& a) {
  if (!skinny_enabled() || generic_only() || a.a.kind != 0 || a.b.kind != 0) return false;
  if (a.epi & EPI_OIHW || a.bias_grad != nullptr || a.splits_out != nullptr) return false;
  if (a.a.ld_k != 1 || a.a.ld_r % 8 != 0 || !aligned16(a.a.ptr) || a.K % 8 != 0) return false;
  const bool bkc = is_kc(a.b);
  if (bkc ? (a.b.ld_r % 8 != 0) : (a.b.ld_r != 1 || a.b.ld_k % 8 != 0 || a.N % 8 != 0)) return false;
  if (!aligned16(a.b.ptr)) return false;
  if (static_cast<long>(a.M) * a.a.ld_r * 2 >= (1L << 31) || static_cast<long>(a.K) * a.N * 2 >= (1L << 31))
    return false;
  const long t64 = static_cast<long>(ceil_div(a.M, 64)) * ceil_div(a.N, 64);
  return t64 < 128 && a.K >= 256 && a.M <= 1024;
}
void skinny_grid(const GemmArgs& a, int& tm, int& tn) {
  tm = ceil_div(a.M, 16 * kSkinnyFM);
  tn = ceil_div(a.N, 16 * kSkinnyFN);
}
hipError_t launch_skinny(const GemmArgs& a, hipStream_t s) {
  int tm, tn;
  skinny_grid(a, tm, tn);
  gemm_log("skinny", a, 16 * kSkinnyFM, 16 * kSkinnyFN, tm * tn, 1);
  if (is_kc(a.b))
    hipLaunchKernelGGL(gemm_skinny_kernel<true>, dim3(tm * tn), dim3(kThreads), 0, s, a, tm, tn);
  else
    hipLaunchKernelGGL(gemm_skinny_kernel<false>, dim3(tm * tn), dim3(kThreads), 0, s, a, tm, tn);
  return hipGetLastError();
}
// Low-K path (gemm_lowk.h): dense K-contiguous operands, K <= 64 (<= 128 with PDE_GEMM_LOWK_MAX_K), a bf16 output with at most bias / ReLU in the
// epilogue, and enough rows for the streamed column strips to pay.  PDE_GEMM_LOWK=0: off; PDE_GEMM_LOWK_MIN_M:
// fewest rows (default 4096); PDE_GEMM_LOWK_BLOCKS: grid cap (default 256; row tiles beyond it are walked by the
// same blocks, the next tile's loads overlapping the current one's stores).
struct LowkPolicy {
  bool on = true;
  long min_m = 4096, max_blocks = 256;  // r6q sweep: 256 / 512 / 1024 / 2048 -> 256 (one block per CU)
  // K <= 64 only by default (r6r, in ResNet-50 b32's eager trace): 32768x256x64 11.75 us vs the tile core's 12.84,
  // 32768x64x64 6.4 vs 8.2, but 8192x512x128 11.2 vs 8.9 (level in isolation, 7.5 vs 7.4): PDE_GEMM_LOWK_MAX_K
  int max_k = 64;
  LowkPolicy() {
    if (const char* e = std::getenv("PDE_GEMM_LOWK")) on = e[0] != '0';
    if (const char* e = std::getenv("PDE_GEMM_LOWK_MIN_M")) min_m = std::atol(e);
    if (const char* e = std::getenv("PDE_GEMM_LOWK_BLOCKS")) max_blocks = std::max(1L, std::atol(e));
    if (const char* e = std::getenv("PDE_GEMM_LOWK_MAX_K")) max_k = std::min(128, std::atoi(e));
  }
};
const LowkPolicy& lowk_policy() {
  static const LowkPolicy p;
  return p;
}
bool lowk_ok(const GemmArgs& a) {
  const LowkPolicy& p = lowk_policy();
  if (!p.on || generic_only() || a.a.kind != 0 || a.b.kind != 0) return false;
  if (a.M < p.min_m || a.K > p.max_k || a.K % 8 != 0 || a.N < 64 || a.N % 4 != 0) return false;
  if ((a.epi & ~(EPI_BIAS | EPI_RELU)) != 0 || a.bias_grad != nullptr || a.bn_out.sums != nullptr ||
      a.bn_in.ss != nullptr)
    return false;
  if (a.a.ld_k != 1 || a.b.ld_k != 1 || a.a.ld_r % 8 != 0 || a.b.ld_r % 8 != 0 || !aligned16(a.a.ptr) ||
      !aligned16(a.b.ptr))
    return false;
  if (a.ldo % 8 != 0 || !aligned16(a.out)) return false;
  return fast_ok(a, a.a, true, a.M) && fast_ok(a, a.b, true, a.N);
}
hipError_t launch_lowk(const GemmArgs& a, hipStream_t s) {
  const int fn = a.N % 128 == 0 ? 8 : 4;  // column strips of 128 (64 when N is not a multiple of 128)
  const int tm = ceil_div(a.M, kLowkBM), tn = ceil_div(a.N, 16 * fn);
  long blocks = static_cast<long>(tm) * tn;
  const long cap = std::max<long>(tn, lowk_policy().max_blocks / tn * tn);  // a multiple of tn
  if (blocks > cap) blocks = cap;
  if (a.splits_out != nullptr) *a.splits_out = 1;
  gemm_log("lowk", a, kLowkBM, 16 * fn, tm * tn, 1);
  const dim3 grid(static_cast<unsigned>(blocks));
  if (a.K <= 64) {
    if (fn == 8) hipLaunchKernelGGL((gemm_lowk_kernel<2, 8>), grid, dim3(kThreads), 0, s, a, tm, tn);
    else hipLaunchKernelGGL((gemm_lowk_kernel<2, 4>), grid, dim3(kThreads), 0, s, a, tm, tn);
  } else {
    if (fn == 8) hipLaunchKernelGGL((gemm_lowk_kernel<4, 8>), grid, dim3(kThreads), 0, s, a, tm, tn);
    else hipLaunchKernelGGL((gemm_lowk_kernel<4, 4>), grid, dim3(kThreads), 0, s, a, tm, tn);
  }
  return hipGetLastError();
}
// skinny problem 0 + 64x64 FAST-tile problem 1 (a weight gradient: dy^T x dense activation)
bool launch_pair_skinny(const GemmArgs& a0, const GemmArgs& a1, const PairDims& d, hipStream_t s,
                        const OptimSeg& seg) {
  if (kind_code_of(a1) != kind_code(false, false, 0, 0)) return false;
  int tm0, tn0;
  skinny_grid(a0, tm0, tn0);
  const dim3 grid(static_cast<unsigned>(tm0 * tn0 + d.tm[1] * d.tn[1] * d.nz[1] + seg.blocks));
  gemm_log("pair-skinny.0", a0, 16 * kSkinnyFM, 16 * kSkinnyFN, tm0 * tn0, 1);
  gemm_log("pair-skinny.1", a1, 64, 64, d.tm[1] * d.tn[1], d.nz[1]);
  if (is_kc(a0.b))
    hipLaunchKernelGGL((gemm_pair_skinny_kernel<true, false, false, 0, 0>), grid, dim3(kThreads), 0, s, a0, tm0, tn0,
                       a1, d, seg);
  else
    hipLaunchKernelGGL((gemm_pair_skinny_kernel<false, false, false, 0, 0>), grid, dim3(kThreads), 0, s, a0, tm0,
                       tn0, a1, d, seg);
  return true;
}

}  // namespace

bool gemm_bn_stats_ok(const GemmArgs& a, hipStream_t s) { return bn_stats_ok_impl(a, s); }
bool gemm_bn_fold_ok(const GemmArgs& a) { return bn_fold_ok_impl(a); }

// Vector epilogue / slab stores write-through (GemmArgs::wt); PDE_GEMM_WT=0 plain.  r4l: ResNet-50 3.317 -> 3.248
// ms/step, MLP level
int gemm_wt() {
  static const int on = std::getenv("PDE_GEMM_WT") ? std::atoi(std::getenv("PDE_GEMM_WT")) : 1;
  return on;
}

hipError_t gemm_bf16(const GemmArgs& a_in, hipStream_t s) {
  if (a_in.M <= 0 || a_in.N <= 0) return hipSuccess;
  GemmArgs a = a_in;
  a.wt = gemm_wt();
  if (skinny_ok(a)) return launch_skinny(a, s);
  if (lowk_ok(a)) return launch_lowk(a, s);
  const bool akc = is_kc(a.a), bkc = is_kc(a.b);
  if (akc && bkc) return dispatch_tiles<true, true>(a, s);
  if (akc && !bkc) return dispatch_tiles<true, false>(a, s);
  if (!akc && bkc) return dispatch_tiles<false, true>(a, s);
  return dispatch_tiles<false, false>(a, s);
}

hipError_t gemm_reduce_slabs_bf16(float* ws, int splits, int M, int N, uint16_t* out, hipStream_t s) {
  GemmArgs a{};
  a.M = M;
  a.N = N;
  a.workspace = ws;
  a.out = out;
  a.ldo = N;
  a.epi = 0;
  launch_reduce(a, splits, s);
  return hipGetLastError();
}

hipError_t gemm_reduce_jobs(const ReduceJob* jobs, int n, hipStream_t s) {
  for (int base = 0; base < n; base += kMaxReduceJobs) {
    ReduceJobs t{};
    t.n = std::min(kMaxReduceJobs, n - base);
    int blocks = 0;
    for (int j = 0; j < t.n; ++j) {
      t.job[j] = jobs[base + j];
      t.first[j] = blocks;
      blocks += ceil_div(static_cast<long>(t.job[j].M) * t.job[j].N / 4, 256 / reduce_lanes(t.job[j].splits));
    }
    t.first[t.n] = blocks;
    hipLaunchKernelGGL(gemm_splitk_reduce_jobs, dim3(blocks), dim3(256), 0, s, t);
  }
  return hipGetLastError();
}

bool pair_balance_on() {  // opt-in (PDE_GEMM_PAIR_BALANCE=1): measured slower, r3s (more slab traffic)
  static const bool on = std::getenv("PDE_GEMM_PAIR_BALANCE") && std::getenv("PDE_GEMM_PAIR_BALANCE")[0] == '1';
  return on;
}

bool gemm_pair_enabled() {
  static const bool on = !(std::getenv("PDE_GEMM_PAIR") && std::getenv("PDE_GEMM_PAIR")[0] == '0');
  return on;
}

hipError_t gemm_bf16_pair(const GemmArgs& a0_in, const GemmArgs& a1_in, hipStream_t s, int* defer_split1,
                          const OptimSeg* seg_in, int* defer_split0) {
  GemmArgs a0 = a0_in, a1 = a1_in;
  a0.wt = a1.wt = gemm_wt();
  if (defer_split1 != nullptr) *defer_split1 = 0;
  if (defer_split0 != nullptr) *defer_split0 = 0;
  OptimSeg seg{};  // blocks = 0: no optimiser segment
  if (seg_in != nullptr && seg_in->c1 > seg_in->c0 && seg_in->blocks > 0) seg = *seg_in;
  PairDims d{};
  int sp0 = 1, sp1 = 1;
  if (gemm_pair_enabled() && skinny_ok(a0) &&
      pair_member_plan(a1, d.tm[1], d.tn[1], d.kps[1], sp1, d.av[1], d.bv[1]) && (sp1 == 1 || reduce_vec_ok(a1))) {
    // skinny dgrad + tile wgrad: problem 0 needs no reduction at all
    GemmArgs g1 = a1;
    g1.tickets = nullptr;
    d.nz[1] = sp1;
    if (static_cast<long>(d.tm[1]) * d.tn[1] * sp1 < (1L << 30) && launch_pair_skinny(a0, g1, d, s, seg)) {
      if (defer_split1 != nullptr && sp1 > 1) {
        *defer_split1 = sp1;
      } else if (sp1 > 1) {
        launch_reduce(a1, sp1, s);
      }
      return hipGetLastError();
    }
  }
  d = PairDims{};
  sp1 = 1;
  const bool dma = gemm_core_mode() == 1;  // (hybrid: paired launches stay on the ring core)
  const bool ok = gemm_pair_enabled() &&
                  pair_member_plan(a0, d.tm[0], d.tn[0], d.kps[0], sp0, d.av[0], d.bv[0], dma) &&
                  pair_member_plan(a1, d.tm[1], d.tn[1], d.kps[1], sp1, d.av[1], d.bv[1], dma) &&
                  (sp0 == 1 || reduce_vec_ok(a0)) && (sp1 == 1 || reduce_vec_ok(a1));
  if (ok && !dma && pair_balance_on()) {
    // a paired launch lasts as long as its longest K slice: while one member's slices are >= 2x the other's,
    // split it further (within its workspace, <= 64 MB of slabs): e.g. layer4's 3x3 dgrad (36 K-tiles per
    // slice at split 4) next to its weight gradient (16)
    for (int it = 0; it < 4; ++it) {
      const int kt0 = d.kps[0] / 32, kt1 = d.kps[1] / 32;
      const int w = kt0 >= 2 * kt1 ? 0 : (kt1 >= 2 * kt0 ? 1 : -1);
      if (w < 0) break;
      const GemmArgs& a = w ? a1 : a0;
      int& sp = w ? sp1 : sp0;
      int nsp = sp * 2;
      if (a.workspace == nullptr || nsp > a.splitk || static_cast<long>(nsp) * a.M * a.N * 4 > (64L << 20) ||
          !reduce_vec_ok(a))
        break;
      const int kps = ceil_div(ceil_div(a.K, nsp), 32) * 32;
      nsp = ceil_div(a.K, kps);
      if (nsp <= sp) break;
      sp = nsp;
      d.kps[w] = kps;
    }
  }
  const int k0 = ok ? kind_code_of(a0) : -1, k1 = ok ? kind_code_of(a1) : -1;
  d.nz[0] = sp0;
  d.nz[1] = sp1;
  const long blocks = static_cast<long>(d.tm[0]) * d.tn[0] * sp0 + static_cast<long>(d.tm[1]) * d.tn[1] * sp1 +
                      seg.blocks;
  bool launched = false;
  if (ok && blocks < (1L << 31)) {
    const int spair = dma ? dma_spair(blocks) : 0;
    gemm_log(dma ? (spair == 6 ? "dpair6.0" : "dpair3.0") : "pair.0", a0, 64, 64, d.tm[0] * d.tn[0], sp0);
    gemm_log(dma ? (spair == 6 ? "dpair6.1" : "dpair3.1") : "pair.1", a1, 64, 64, d.tm[1] * d.tn[1], sp1);
    GemmArgs g0 = a0, g1 = a1;
    g0.tickets = g1.tickets = nullptr;  // pair: split-K partials always go through the reduce launch
    const dim3 grid(static_cast<unsigned>(blocks));
    if (dma) {
      launched = dma_launch_pair(spair, k0, k1, grid, s, g0, g1, d, seg);
    } else switch (k1) {  // weight-gradient kinds: dy^T x {im2col^T gather, dense activation}
      case kind_code(false, false, 0, 2):
        launched = launch_pair_k0<false, false, 0, 2>(k0, grid, s, g0, g1, d, seg);
        break;
      case kind_code(false, false, 0, 0):
        launched = launch_pair_k0<false, false, 0, 0>(k0, grid, s, g0, g1, d, seg);
        break;
      default: break;
    }
  }
  if (!launched) {  // not a pairable configuration: two ordinary launches, problem 0 first (+ the optimiser)
    hipError_t e = gemm_bf16(a0, s);
    if (e == hipSuccess) e = gemm_bf16(a1, s);
    if (e == hipSuccess && seg.blocks > 0)
      e = multi_tensor_optim_range(seg.mode, seg.tab, seg.chunks, seg.c0, seg.c1, seg.hp, seg.step, seg.publish, s);
    return e;
  }
  if (defer_split1 != nullptr && sp1 > 1) {  // problem 1's slabs are reduced later by gemm_reduce_jobs
    *defer_split1 = sp1;
    sp1 = 1;
  }
  if (defer_split0 != nullptr && sp0 > 1) {  // problem 0's slabs are summed by their consumer (bn_bwd's dys)
    *defer_split0 = sp0;
    sp0 = 1;
  }
  if (sp0 > 1 && sp1 > 1) {
    const int l0 = reduce_lanes(sp0), l1 = reduce_lanes(sp1);
    const int nb0 = static_cast<int>(ceil_div(static_cast<long>(a0.M) * a0.N / 4, 256 / l0));
    const int nb1 = static_cast<int>(ceil_div(static_cast<long>(a1.M) * a1.N / 4, 256 / l1));
    const dim3 g(nb0 + nb1);
#define PDE_RED(L0, L1) \
  if (l0 == L0 && l1 == L1) hipLaunchKernelGGL((gemm_splitk_reduce4_pair<L0, L1>), g, dim3(256), 0, s, a0, sp0, nb0, a1, sp1);
    PDE_RED(1, 1) PDE_RED(1, 4) PDE_RED(1, 16) PDE_RED(4, 1) PDE_RED(4, 4) PDE_RED(4, 16) PDE_RED(16, 1) PDE_RED(16, 4)
    PDE_RED(16, 16)
#undef PDE_RED
  } else if (sp0 > 1) {
    launch_reduce(a0, sp0, s);
  } else if (sp1 > 1) {
    launch_reduce(a1, sp1, s);
  }
  return hipGetLastError();
}

}  // namespace pde
