// Whole training step of the elastic-DDP MLP (pytorch_elastic/mnist_ddp_elastic.py:133-173: Linear+ReLU stacks,
// cross-entropy, Adam) as ONE persistent launch on gfx950: forward, loss, backward and the optimiser update of
// every layer, phase after phase, with a grid barrier between phases.
//
// Why: at the reference batch (128) every GEMM of the 5x1024 MLP is 0.27 GFLOP -- a few hundred nanoseconds of
// matrix-core time -- yet a launch costs 5-8 us (launch, first-load latency, drain), so the layer-by-layer step
// (FusedMLP: 17 launches) is launch- and latency-bound.  Here one workgroup per CU stays resident for the whole
// step and each phase is ONE global round trip: a workgroup issues every load of the phase -- the MFMA fragments
// of its data-gradient tile, of its weight-gradient tile and the optimiser state of the weight tile it updates --
// before its first MFMA (fragments straight from memory into VGPRs, 16 bytes per lane, K split over the 4 waves).
//
// Layouts (B = batch, rows of 8 bf16 per lane read as one 16-byte load):
//   forward   C[B][out] = A[B][in] . W[out][in]^T      A: activations row-major, W: the optimiser-maintained bf16
//                                                      copy (row-major) -- both K-contiguous
//   dgrad     D[B][in] = G[B][out] . W^T[in][out]^T    G: the gradient row-major, W^T: a bf16 transposed copy the
//                                                      update keeps current (functional.maintain_transposed_copy)
//   wgrad     dW[out][in] = G^T[out][B] . A^T[in][B]^T G^T and A^T: transposed copies written by the producing
//                                                      epilogues
// Every epilogue writes its 32x16 tile twice, row-major and transposed, staged through LDS so that each lane
// stores 16 bytes.  The ReLU mask of the backward comes from the saved activation (a > 0).
//
// Phases for L layers (L = 7 for the reference model: 15 phases, 14 grid barriers):
//   F0..F(L-2)  hidden forwards (F0 also writes x^T, the first layer's wgrad operand; x fp32 -> bf16 on load)
//   CE          last layer's logits + softmax cross-entropy (mean) + d logits, per 32-row tile (DPP row reductions)
//   Bj (j = L-1..0): dgrad of layer j (j >= 1), then the weight + bias gradient of layer j and its UPDATE straight
//               from the accumulators (the W^T tile parked in LDS until the next window: W^T is still being read
//               by other workgroups' dgrads until this phase's barrier) -- every layer's 64x64 gradient tiles fit
//               the grid; otherwise (PDE_MLP_FUSE=0 too) the update of layer j + 1, read back from gw, one window
//               later.  After B0: the step's mean loss, the device step counter
//
// Inter-workgroup visibility (MI355X_MICROARCH.md, "Valid forms"; cdna_hip_programming.md Guideline 16): every byte
// handed from one workgroup to another inside the launch (activations, gradients, d logits, x^T, loss partials) is
// stored write-through (sc1, 16 / 8-byte buffer stores) and EVERY load of it is an sc1 buffer load; each storing
// wave drains (vmcnt(0)) before the workgroup barrier behind which lane 0 arrives -- so the grid barrier needs no
// release or acquire fence.  Weight gradients and optimiser state never cross workgroups: the workgroup that
// computes a 64x64 weight-gradient tile updates that tile one phase later (same tile decomposition).  The barrier is
// one monotonic arrival counter zeroed by a memset node before every launch; barrier k waits for (k + 1) x grid
// arrivals (sc1 poll, bounded: a timeout sets the error word instead of hanging).  Requires every workgroup
// resident at once (one per CU, checked on the host).  Within a workgroup only LDS-scoped barriers (no vmcnt wait:
// stores drain under the next phase's loads).
#include "common.cuh"
#include "mlp_train.h"
#include "optim_device.h"
#include "pde_kernels.h"
#include "xgmi_device.h"

namespace pde {

namespace {

constexpr int MT = 256;  // 4 waves
constexpr int KW = 8;    // k-steps (of 32) per wave in a row-GEMM tile: K <= 4 * 8 * 32 = 1024
constexpr int OOB = static_cast<int>(0x80000000u);  // a buffer offset past every range: the load returns zeros

using rsrc_t = __amdgpu_buffer_rsrc_t;

__device__ __forceinline__ rsrc_t mkbuf(const void* p, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, static_cast<int>(bytes), 0x00020000);
}
template <int AUX>
__device__ __forceinline__ u16x8 bld16(rsrc_t r, int off) {
  return __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
}
__device__ __forceinline__ u16x4 bld8_sc1(rsrc_t r, int off) {
  return __builtin_bit_cast(u16x4, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 16));
}
__device__ __forceinline__ void bst16_sc1(rsrc_t r, int off, const u16x8& v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 16);
}

__device__ __forceinline__ f32x4 mfma16(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// LDS-only workgroup barrier: LDS accesses complete, then s_barrier -- global loads and stores stay in flight
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// DPP row (16-lane) reductions: after the four steps every lane holds the op over its row.  Whole wave active.
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <class Op>
__device__ __forceinline__ float row16(float v, Op op) {
  v = op(v, dppf<0xB1>(v));   // quad_perm xor 1
  v = op(v, dppf<0x4E>(v));   // quad_perm xor 2
  v = op(v, dppf<0x141>(v));  // row_half_mirror
  v = op(v, dppf<0x140>(v));  // row_mirror
  return v;
}

// Grid barrier k, split and XCD-hierarchical: grid_arrive -- every wave drains its stores (the hand-off bytes, all
// sc1), then lane 0 adds one arrival to its group's counter (group = workgroup index mod 8, the XCD round-robin of
// the dispatcher; only the contention depends on that, not correctness), and the group's last arrival adds one to
// the top counter; grid_wait -- lane 0 polls the top counter (sc1) until this barrier's count has arrived.  Counters
// are monotonic ACROSS launches (each on its own 128-byte line): barrier k of launch n waits for (n x nbar + k + 1)
// arrivals per member, n = the launch word every workgroup reads at its start and workgroup 0 advances at its end
// (after its last barrier, so every workgroup of the launch has read it) -- no memset node per launch.  Work that
// neither produces nor consumes a hand-off (the optimiser update, prefetching the next phase's weight fragments)
// runs between arrive and wait and hides the barrier's latency.
constexpr int kBarGroups = 8, kBarStride = 32;  // top at [0], group g at [32 (g + 1)], the launch word at [32 x 9]
constexpr int kBarWords = kBarStride * (kBarGroups + 2);
struct Bar {
  unsigned* w;
  unsigned base;  // n x nbar
};
__device__ __forceinline__ void grid_arrive(const Bar& b, int k) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (threadIdx.x == 0) {
    const unsigned g = blockIdx.x % kBarGroups, grid = gridDim.x;
    const unsigned members = (grid - g + kBarGroups - 1) / kBarGroups;
    const unsigned old = __hip_atomic_fetch_add(b.w + kBarStride * (g + 1), 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == (b.base + static_cast<unsigned>(k) + 1) * members)
      __hip_atomic_fetch_add(b.w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ void grid_wait(const Bar& b, int* err, int k) {
  if (threadIdx.x == 0) {
    const unsigned groups = gridDim.x < kBarGroups ? gridDim.x : kBarGroups;
    const unsigned target = (b.base + static_cast<unsigned>(k) + 1) * groups;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    // wrap-safe: the counters run on across launches and wrap after ~2^32 / (groups x nbar) steps
    while (static_cast<int>(__hip_atomic_load(b.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s at 100 MHz
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the poll
}

struct Smem {
  f32x4 red[3][2][64];      // row-GEMM: waves 1..3's K-quarter partials
  uint16_t ep[32][24];      // row-GEMM epilogue: the 32x16 bf16 tile (wave 0)
  uint16_t tr[64][72];      // update: the W^T tile (fused form: parked here until the next window)
  float gt[64][68];         // fused form: the weight-gradient tile, accumulator layout -> update layout
  float gb[64];             //             and its bias gradients
};

// ---- row-GEMM tile: C[m0, m0+32) x [n0, n0+16) of A[M][K] . W[N][K]^T, K split over the 4 waves ----------------
struct RowLoads {
  u16x8 a0[KW], a1[KW], b[KW];
  u16x4 mask[2];  // dgrad: act^T[n][m .. m+3] of the two 16-row halves (wave 0)
  float bias;     // forward / CE: the bias of the lane's column (wave 0)
  int tg[2][4];   // CE: the labels of the lane's rows (wave 0)
};

// The weight fragments of a tile (plain loads: written by an earlier launch) -- issued ahead of the barrier that
// precedes the tile's phase.
__device__ __forceinline__ void row_load_w(RowLoads& L, const uint16_t* W, int ldb, int N, int K, int n0) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nks = (K + 31) >> 5, kr = 8 * (lane >> 4), rl = lane & 15;
  const rsrc_t rw = mkbuf(W, static_cast<long>(N) * ldb * 2);
#pragma unroll
  for (int u = 0; u < KW; ++u) {
    const int ks = w + 4 * u, k = ks * 32 + kr, rn = n0 + rl;
    L.b[u] = bld16<0>(rw, ks < nks && k < K && rn < N ? (rn * ldb + k) * 2 : OOB);
  }
}

// The activation fragments: bf16 hand-off payload (sc1 loads) or, AF32, the fp32 images (plain, rounded to bf16)
template <bool AF32>
__device__ __forceinline__ void row_load_a(RowLoads& L, const void* A, int lda, int M, int K, int m0) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nks = (K + 31) >> 5, kr = 8 * (lane >> 4), rl = lane & 15;
  const rsrc_t ra = mkbuf(A, static_cast<long>(M) * lda * 2);
#pragma unroll
  for (int u = 0; u < KW; ++u) {
    const int ks = w + 4 * u, k = ks * 32 + kr;
    const bool kok = ks < nks && k < K;
    if constexpr (AF32) {
      const float* X = static_cast<const float*>(A);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = m0 + 16 * h + rl;
        u16x8 o{0, 0, 0, 0, 0, 0, 0, 0};
        if (kok && r < M) {
          const f32x4* q = reinterpret_cast<const f32x4*>(X + static_cast<long>(r) * lda + k);
          const f32x4 x0 = q[0], x1 = q[1];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            o[j] = f2bf(x0[j]);
            o[4 + j] = f2bf(x1[j]);
          }
        }
        (h ? L.a1[u] : L.a0[u]) = o;
      }
    } else {
      const int r0 = m0 + rl, r1 = m0 + 16 + rl;
      L.a0[u] = bld16<16>(ra, kok && r0 < M ? (r0 * lda + k) * 2 : OOB);
      L.a1[u] = bld16<16>(ra, kok && r1 < M ? (r1 * lda + k) * 2 : OOB);
    }
  }
}

// MFMAs + the K-quarter reduction: wave 0 returns the sums (c0 rows m0..+15, c1 rows m0+16..+31)
__device__ __forceinline__ void row_mma(const RowLoads& L, f32x4& c0, f32x4& c1, Smem& sm) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  c0 = f32x4{0.f, 0.f, 0.f, 0.f};
  c1 = c0;
#pragma unroll
  for (int u = 0; u < KW; ++u) {
    c0 = mfma16(L.a0[u], L.b[u], c0);
    c1 = mfma16(L.a1[u], L.b[u], c1);
  }
  if (w > 0) {
    sm.red[w - 1][0][lane] = c0;
    sm.red[w - 1][1][lane] = c1;
  }
  lds_sync();
  if (w == 0) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      c0 += sm.red[q][0][lane];
      c1 += sm.red[q][1][lane];
    }
  }
}

// Wave 0: the tile (v[s][r] = row m0 + 16 s + 4 (lane >> 4) + r, column n0 + (lane & 15)) as bf16, stored row-major
// into out (pitch ldo) and transposed into outT (pitch B), 16 bytes per lane each, write-through.  N % 8 == 0.
__device__ __forceinline__ void ep_store(Smem& sm, const float (&v)[2][4], rsrc_t out, int ldo, rsrc_t outT, int B,
                                         int m0, int n0, int N) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) sm.ep[16 * s + 4 * (lane >> 4) + r][lane & 15] = f2bf(v[s][r]);
  {  // row-major: lane -> (row, 8-column half)
    const int row = lane >> 1, h = lane & 1, n = n0 + 8 * h;
    const u16x8 x = *reinterpret_cast<const u16x8*>(&sm.ep[row][8 * h]);
    if (n < N) bst16_sc1(out, ((m0 + row) * ldo + n) * 2, x);
  }
  {  // transposed: lane -> (column, 8-row quarter)
    const int c = lane >> 2, q = lane & 3, n = n0 + c;
    u16x8 x;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = sm.ep[8 * q + j][c];
    if (n < N) bst16_sc1(outT, (n * B + m0 + 8 * q) * 2, x);
  }
}

// ---- weight-gradient tile: gw[o0, o0+64) x [i0, i0+64) = G^T[o][b] . A^T[i][b], 128 batch columns per pass -----
struct WgLoads {
  u16x8 a[4][2], b[4][2];
  u16x8 g[4];  // bias gradient: this thread's quarter of one G^T row (column-block-0 tiles)
};

__device__ __forceinline__ void wg_load(WgLoads& L, rsrc_t rg, rsrc_t ra, int B, int out, int in, int o0, int i0,
                                        int kb, bool bias) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wo = w >> 1, wi = w & 1;
  const int kr = 8 * (lane >> 4), rl = lane & 15;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = kb + 32 * u + kr;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int o = o0 + 32 * wo + 16 * e + rl, i = i0 + 32 * wi + 16 * e + rl;
      L.a[u][e] = bld16<16>(rg, k < B && o < out ? (o * B + k) * 2 : OOB);
      L.b[u][e] = bld16<16>(ra, k < B && i < in ? (i * B + k) * 2 : OOB);
    }
  }
  const int o = o0 + (threadIdx.x >> 2), q = threadIdx.x & 3, span = B / 4;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int b = q * span + 8 * c;
    L.g[c] = bld16<16>(rg, bias && kb == 0 && 8 * c < span && o < out ? (o * B + b) * 2 : OOB);
  }
}

__device__ __forceinline__ void wg_mma(const WgLoads& L, f32x4 (&acc)[2][2]) {
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int f = 0; f < 2; ++f) acc[e][f] = mfma16(L.a[u][e], L.b[u][f], acc[e][f]);
}

// ---- optimiser update of a 64x64 weight tile (+ the tile's 64 biases on column-block-0 tiles) -------------------
struct UpLoads {
  f32x4 p[4], g[4], m[4], v[4];
  float bp, bg, bm, bv;
};

__device__ __forceinline__ void up_load(UpLoads& U, const MlpLayerArgs& L, int o0, int i0, bool use_m, bool use_v,
                                        bool load_g = true) {
  const int tc = threadIdx.x & 15, tr0 = threadIdx.x >> 4, i = i0 + 4 * tc;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int o = o0 + tr0 + 16 * q;
    const long e = (o < L.out && i < L.in) ? static_cast<long>(o) * L.in + i : 0;  // clamped: loaded, not stored
    U.p[q] = optdev::ld4<1>(L.w + e);
    if (load_g) U.g[q] = optdev::ld4<1>(L.gw + e);
    U.m[q] = use_m ? optdev::ld4<1>(L.mw + e) : f32x4{0.f, 0.f, 0.f, 0.f};
    U.v[q] = use_v ? optdev::ld4<1>(L.vw + e) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int ob = o0 + threadIdx.x;
  U.bp = U.bg = U.bm = U.bv = 0.f;
  if (i0 == 0 && threadIdx.x < 64 && ob < L.out) {
    U.bp = L.b[ob];
    if (load_g) U.bg = L.gb[ob];
    if (use_m) U.bm = L.mb[ob];
    if (use_v) U.bv = L.vb[ob];
  }
}

__device__ __forceinline__ void wt_flush(const MlpLayerArgs& L, int o0, int i0, Smem& sm);

template <int MODE>
__device__ __forceinline__ void up_finish(UpLoads& U, const MlpLayerArgs& L, const optdev::Hyper& h, int o0, int i0,
                                          bool use_m, Smem& sm, bool park = false) {
  const int tc = threadIdx.x & 15, tr0 = threadIdx.x >> 4, i = i0 + 4 * tc;
  float pv[4][4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float p[4], g[4], m[4], v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      p[c] = U.p[q][c]; g[c] = U.g[q][c]; m[c] = U.m[q][c]; v[c] = U.v[q][c];
      optdev::update<MODE>(h, p[c], g[c], m[c], v[c]);
      pv[q][c] = p[c];
    }
    const int o = o0 + tr0 + 16 * q;
    if (o < L.out && i < L.in) {
      const long e = static_cast<long>(o) * L.in + i;
      optdev::st4<1>(L.w + e, f32x4{p[0], p[1], p[2], p[3]});
      if (use_m) optdev::st4<1>(L.mw + e, f32x4{m[0], m[1], m[2], m[3]});
      if (MODE != 0) optdev::st4<1>(L.vw + e, f32x4{v[0], v[1], v[2], v[3]});
      *reinterpret_cast<u16x4*>(L.wbf + e) = u16x4{f2bf(p[0]), f2bf(p[1]), f2bf(p[2]), f2bf(p[3])};
    }
  }
  const int ob = o0 + threadIdx.x;
  if (i0 == 0 && threadIdx.x < 64 && ob < L.out) {
    optdev::update<MODE>(h, U.bp, U.bg, U.bm, U.bv);
    L.b[ob] = U.bp;
    if (use_m) L.mb[ob] = U.bm;
    if (MODE != 0) L.vb[ob] = U.bv;
  }
  if (L.wtbf == nullptr) return;
  // the transposed copy: the tile through LDS, each thread then writes 16 consecutive output rows of one input row
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int c = 0; c < 4; ++c) sm.tr[4 * tc + c][tr0 + 16 * q] = f2bf(pv[q][c]);
  if (!park) wt_flush(L, o0, i0, sm);
}

// The W^T tile in sm.tr (64 input rows x 64 outputs) to L.wtbf: each thread 16 consecutive outputs of one input row
__device__ __forceinline__ void wt_flush(const MlpLayerArgs& L, int o0, int i0, Smem& sm) {
  if (L.wtbf == nullptr) return;
  lds_sync();
  const int il = threadIdx.x >> 2, part = threadIdx.x & 3;
  const int ii = i0 + il, ob16 = o0 + 16 * part;
  if (ii < L.in) {
    uint16_t* dst = L.wtbf + static_cast<long>(ii) * L.ldt + ob16;
    if (ob16 + 16 <= L.out) {
      u16x8 x0, x1;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        x0[c] = sm.tr[il][16 * part + c];
        x1[c] = sm.tr[il][16 * part + 8 + c];
      }
      reinterpret_cast<u16x8*>(dst)[0] = x0;
      reinterpret_cast<u16x8*>(dst)[1] = x1;
    } else {
      for (int c = 0; c < 16 && ob16 + c < L.out; ++c) dst[c] = sm.tr[il][16 * part + c];
    }
  }
  lds_sync();
}

// ---- phases -----------------------------------------------------------------------------------------------------
// Each phase function runs this workgroup's tiles; the FIRST tile's weight fragments were prefetched into `R` by
// the caller (ahead of the barrier), later tiles (more tiles than workgroups) load their own.
template <bool AF32>
__device__ __forceinline__ void fwd_phase(const MlpTrainArgs& a, int l, RowLoads& R, Smem& sm) {
  const MlpLayerArgs& L = a.L[l];
  const int B = a.B, mt = B / 32, nt = (L.out + 15) / 16, lane = threadIdx.x & 63;
  const void* A = AF32 ? static_cast<const void*>(a.x) : static_cast<const void*>(a.act[l]);
  const rsrc_t ro = mkbuf(a.act[l + 1], static_cast<long>(B) * L.out * 2);
  const rsrc_t rot = mkbuf(a.actT[l + 1], static_cast<long>(B) * L.out * 2);
  for (int t = blockIdx.x; t < mt * nt; t += gridDim.x) {
    const int m0 = (t % mt) * 32, n0 = (t / mt) * 16;
    if (t != blockIdx.x) {
      row_load_w(R, L.wbf, L.in, L.out, L.in, n0);
      R.bias = n0 + (lane & 15) < L.out ? L.b[n0 + (lane & 15)] : 0.f;
    }
    row_load_a<AF32>(R, A, L.in, B, L.in, m0);
    f32x4 c0, c1;
    row_mma(R, c0, c1, sm);
    if (threadIdx.x < 64) {
      const float bias = R.bias;
      float v[2][4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[0][r] = fmaxf(c0[r] + bias, 0.f);
        v[1][r] = fmaxf(c1[r] + bias, 0.f);
      }
      ep_store(sm, v, ro, L.out, rot, B, m0, n0, L.out);
    }
    lds_sync();  // red / ep reuse by the next tile
  }
}
__device__ __forceinline__ void fwd_prefetch(const MlpTrainArgs& a, int l, RowLoads& R) {
  const MlpLayerArgs& L = a.L[l];
  const int mt = a.B / 32, nt = (L.out + 15) / 16, t = blockIdx.x;
  if (t < mt * nt) {
    const int n = (t / mt) * 16 + (threadIdx.x & 15);
    row_load_w(R, L.wbf, L.in, L.out, L.in, (t / mt) * 16);
    R.bias = n < L.out ? L.b[n] : 0.f;
  }
}

// The last layer's weight fragments, its bias and the labels of CE tile t (none of them a hand-off)
__device__ __forceinline__ void ce_loads_w(const MlpTrainArgs& a, RowLoads& R, int t) {
  const MlpLayerArgs& L = a.L[a.nl - 1];
  const int lane = threadIdx.x & 63, n = lane & 15;
  row_load_w(R, L.wbf, L.in, L.out, L.in, 0);
  R.bias = n < L.out ? L.b[n] : 0.f;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) R.tg[s][r] = static_cast<int>(a.y[t * 32 + 16 * s + 4 * (lane >> 4) + r]);
}

// Last layer (out <= 16) + mean softmax cross-entropy: d logits (both layouts, 16 columns) and one loss partial
// per 32-row tile.
template <bool AF32>
__device__ __forceinline__ void ce_phase(const MlpTrainArgs& a, RowLoads& R, Smem& sm) {
  const int l = a.nl - 1;
  const MlpLayerArgs& L = a.L[l];
  const int B = a.B, mt = B / 32, lane = threadIdx.x & 63;
  const void* A = AF32 ? static_cast<const void*>(a.x) : static_cast<const void*>(a.act[l]);
  const float inv_b = 1.f / static_cast<float>(B);
  const rsrc_t rd = mkbuf(a.dlog, static_cast<long>(B) * 32 * 2);
  const rsrc_t rdt = mkbuf(a.dlogT, static_cast<long>(B) * 32 * 2);
  for (int t = blockIdx.x; t < mt; t += gridDim.x) {
    const int m0 = t * 32;
    if (t != blockIdx.x) ce_loads_w(a, R, t);
    row_load_a<AF32>(R, A, L.in, B, L.in, m0);
    f32x4 c0, c1;
    row_mma(R, c0, c1, sm);
    if (threadIdx.x < 64) {
      const int n = lane & 15;
      const bool valid = n < L.out;
      const float bias = R.bias;
      float lsum = 0.f, dv[2][4];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const f32x4& c = s ? c1 : c0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float z = valid ? c[r] + bias : -INFINITY;
          const float mx = row16(z, [](float x, float y) { return fmaxf(x, y); });
          const float se = row16(valid ? __expf(z - mx) : 0.f, [](float x, float y) { return x + y; });
          const float lse = mx + __logf(se);
          const int tg = R.tg[s][r];
          const float zt = row16(n == tg ? z : 0.f, [](float x, float y) { return x + y; });
          lsum += n == 0 ? lse - zt : 0.f;
          dv[s][r] = valid ? (__expf(z - lse) - (n == tg ? 1.f : 0.f)) * inv_b : 0.f;
        }
      }
      ep_store(sm, dv, rd, 32, rdt, B, m0, 0, 16);
      const float tot = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lsum), 0)) +
                        __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lsum), 16)) +
                        __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lsum), 32)) +
                        __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lsum), 48));
      if (lane == 0) __hip_atomic_store(a.loss_part + t, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    lds_sync();
  }
}
__device__ __forceinline__ void ce_prefetch(const MlpTrainArgs& a, RowLoads& R) {
  if (static_cast<int>(blockIdx.x) < a.B / 32) ce_loads_w(a, R, blockIdx.x);
}

// dgrad of layer j (j >= 1): d_j = (G . W_j^T^T) * (act_j > 0); G = d logits (K padded to 32) or d_{j+1}
struct DgradGeom {
  const uint16_t* G;
  int ldg, K, n;
};
__device__ __forceinline__ DgradGeom dgrad_geom(const MlpTrainArgs& a, int j) {
  const bool last = j == a.nl - 1;
  const MlpLayerArgs& L = a.L[j];
  return {last ? a.dlog : a.d[j + 1], last ? 32 : L.out, last ? 32 : L.out,
          j >= 1 ? (a.B / 32) * ((L.in + 15) / 16) : 0};
}
__device__ __forceinline__ void dgrad_prefetch(const MlpTrainArgs& a, int j, RowLoads& R) {
  const MlpLayerArgs& L = a.L[j];
  const DgradGeom g = dgrad_geom(a, j);
  const int mt = a.B / 32, t = blockIdx.x;
  if (t < g.n) row_load_w(R, L.wtbf, L.ldt, L.in, g.K, (t / mt) * 16);
}

// The weight + bias gradient of one 64x64 tile from its loaded operands: stored to gw / gb and, `sm` given, also
// left in sm->gt / sm->gb for the fused update (accumulator layout; read back in the update layout after a sync)
__device__ __forceinline__ void wgrad_tile(const MlpLayerArgs& L, WgLoads& WW, rsrc_t rg, rsrc_t ra, int B, int o0, int i0, Smem* sm) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wo = w >> 1, wi = w & 1;
  f32x4 acc[2][2];
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int f = 0; f < 2; ++f) acc[e][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  wg_mma(WW, acc);
  float bsum = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) bsum += bf2f(WW.g[c][jj]);
  for (int kb = 128; kb < B; kb += 128) {  // batches beyond 128: further passes (loads not overlapped)
    wg_load(WW, rg, ra, B, L.out, L.in, o0, i0, kb, false);
    wg_mma(WW, acc);
  }
  if (i0 == 0) {  // bias gradient: 4 threads per row
    const int o = o0 + (threadIdx.x >> 2), q = threadIdx.x & 3, span = B / 4;
    for (int b = q * span + 32; b < (q + 1) * span; b += 8) {  // spans beyond the 4 preloaded vectors
      const u16x8 x = bld16<16>(rg, o < L.out ? (o * B + b) * 2 : OOB);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) bsum += bf2f(x[jj]);
    }
    bsum += __shfl_xor(bsum, 1, 64);
    bsum += __shfl_xor(bsum, 2, 64);
    if (q == 0 && o < L.out) L.gb[o] = bsum;
    if (sm != nullptr && q == 0) sm->gb[threadIdx.x >> 2] = bsum;
  }
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int il = 32 * wi + 16 * f + (lane & 15), i = i0 + il;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int ol = 32 * wo + 16 * e + 4 * (lane >> 4), o = o0 + ol;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (i < L.in && o + r < L.out) L.gw[static_cast<long>(o + r) * L.in + i] = acc[e][f][r];
        if (sm != nullptr) sm->gt[ol + r][il] = acc[e][f][r];
      }
    }
  }
}

// Backward phase of layer j: this workgroup's dgrad tile(s) (weights prefetched) and weight-gradient tile(s).
// `U`: the optimiser state of this workgroup's first update tile of layer j + 1 (`UL`), loaded right behind the
// GEMM operands so that its HBM traffic overlaps the GEMMs' latency; the update itself runs after the arrive.
// part 0: the dgrad tiles (the phase's hand-off, before the barrier's arrive); part 1: the weight-gradient tiles,
// with the update state of layer j + 1 loaded behind their operands (between arrive and wait).
__device__ __forceinline__ void bwd_phase(const MlpTrainArgs& a, int j, int part, RowLoads& R, Smem& sm, UpLoads& U,
                                          bool pre, const MlpLayerArgs& UL, bool use_m, bool use_v) {
  const MlpLayerArgs& L = a.L[j];
  const bool last = j == a.nl - 1;
  const int B = a.B, mt = B / 32, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const DgradGeom g = dgrad_geom(a, j);
  const uint16_t* GT = last ? a.dlogT : a.dT[j + 1];
  const int ot = (L.out + 63) / 64, nwg = ot * ((L.in + 63) / 64);
  const rsrc_t rg = mkbuf(GT, static_cast<long>(last ? 32 : L.out) * B * 2);
  const rsrc_t ra = mkbuf(a.actT[j], static_cast<long>(L.in) * B * 2);
  const rsrc_t rm = mkbuf(a.actT[j], static_cast<long>(L.in) * B * 2);

  auto dgrad_load = [&](int tt) {
    const int m0 = (tt % mt) * 32, n0 = (tt / mt) * 16;
    if (tt != static_cast<int>(blockIdx.x)) row_load_w(R, L.wtbf, L.ldt, L.in, g.K, n0);
    row_load_a<false>(R, g.G, g.ldg, B, g.K, m0);
    if (w == 0) {
      const int n = n0 + (lane & 15);
#pragma unroll
      for (int s = 0; s < 2; ++s)
        R.mask[s] = bld8_sc1(rm, n < L.in ? (n * B + m0 + 16 * s + 4 * (lane >> 4)) * 2 : OOB);
    }
  };
  auto dgrad_finish = [&](int tt) {
    const int m0 = (tt % mt) * 32, n0 = (tt / mt) * 16;
    f32x4 c0, c1;
    row_mma(R, c0, c1, sm);
    if (threadIdx.x < 64) {
      float v[2][4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[0][r] = bf2f(R.mask[0][r]) > 0.f ? c0[r] : 0.f;
        v[1][r] = bf2f(R.mask[1][r]) > 0.f ? c1[r] : 0.f;
      }
      ep_store(sm, v, mkbuf(a.d[j], static_cast<long>(B) * L.in * 2), L.in,
               mkbuf(a.dT[j], static_cast<long>(B) * L.in * 2), B, m0, n0, L.in);
    }
    lds_sync();
  };
  auto wgrad_finish = [&](WgLoads& WW, int o0, int i0) { wgrad_tile(L, WW, rg, ra, B, o0, i0, nullptr); };

  const int t = blockIdx.x;
  if (part == 0) {
    for (int tt = t; tt < g.n; tt += gridDim.x) {  // (more tiles than workgroups: one after another)
      dgrad_load(tt);
      dgrad_finish(tt);
    }
    return;
  }
  WgLoads Wg;
  const bool do_wg = t < nwg;
  const int wo0 = (t % ot) * 64, wi0 = (t / ot) * 64;
  if (do_wg) wg_load(Wg, rg, ra, B, L.out, L.in, wo0, wi0, 0, wi0 == 0);
  if (pre) {
    const int uot = (UL.out + 63) / 64, nup = uot * ((UL.in + 63) / 64);
    if (t < nup) up_load(U, UL, (t % uot) * 64, (t / uot) * 64, use_m, use_v);
  }
  if (do_wg) wgrad_finish(Wg, wo0, wi0);
  for (int tt = t + gridDim.x; tt < nwg; tt += gridDim.x) {
    const int o0 = (tt % ot) * 64, i0 = (tt / ot) * 64;
    wg_load(Wg, rg, ra, B, L.out, L.in, o0, i0, 0, i0 == 0);
    wgrad_finish(Wg, o0, i0);
  }
}

// Fused backward window of layer j (every layer's weight-gradient tiles fit the grid: at most one per workgroup):
// the weight + bias gradient of this workgroup's 64x64 tile of layer j and, straight from the accumulators (through
// LDS: no gradient read-back from memory, no extra window), the optimiser update of the same tile -- its state
// loaded right behind the GEMM operands.  The updated W^T tile cannot be stored yet (other workgroups' dgrads of
// layer j read W^T until this phase's barrier completes): with `park` it stays in LDS and is stored at the start
// of this workgroup's next window (`pk`), after that barrier.  j = 0 (no dgrad reads W_0^T): stored at once.
struct Park {
  int l, o0, i0;
};

// In-launch gradient exchange of this workgroup's tile of layer j (world > 1, fused form), on the tile the
// weight-gradient GEMM left in LDS (sm.gt / sm.gb, read back below in the update layout by the SAME threads, so no
// extra barrier): stage it (write-through) into my slot at the tile's offset, raise flag value (epoch x nl + exchange
// index + 1) in every rank's flag array, wait for every rank's, then sum the N ranks' tiles in rank order
// (bit-identical on every rank), scale by xscale and write the average back to LDS and to gw / gb (DDP's averaged
// .grad).  Few values are live here (the tile stays in LDS), so the exchange adds no spills to the update's state.
// A timed-out wait leaves the local gradient (the error words are set; the host raises at its check).
// Block-collective.
__device__ __forceinline__ void xchg_tile(const MlpTrainArgs& a, const XgmiView& xv, int j, int t, uint32_t epoch,
                                          int* s_fail, Smem& sm, int o0, int i0) {
  const long off = a.xoff[j] + static_cast<long>(t) * kMlpXchgTile;
  const int tc = threadIdx.x & 15, tr0 = threadIdx.x >> 4;
  const bool bias = i0 == 0 && threadIdx.x < 64;
  float* mine = xgmi_slot(xv, xv.rank, epoch) + off;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    st_vec(reinterpret_cast<f32x4*>(mine + (tr0 + 16 * q) * 64 + 4 * tc),
           *reinterpret_cast<const f32x4*>(&sm.gt[tr0 + 16 * q][4 * tc]), true);
  if (bias) mine[4096 + threadIdx.x] = sm.gb[threadIdx.x];
  const uint32_t k = static_cast<uint32_t>(a.nl - 1 - j);
  // every kernel argument the code below needs is read BEFORE the flag wait: behind its asm memory clobbers a read of
  // the argument block would make the compiler keep a private copy of the whole block (1.7 KB of scratch per lane)
  const float xscale = a.xscale;
  float* const gw = a.L[j].gw;
  float* const gbp = a.L[j].gb;
  const int lin = a.L[j].in, lout = a.L[j].out;
  const uint32_t flag = epoch * static_cast<uint32_t>(a.nl) + k + 1u;
  if (!xgmi_publish_and_wait(xv, blockIdx.x, flag, s_fail)) return;
  const int i = i0 + 4 * tc;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = (tr0 + 16 * q) * 64 + 4 * tc;
    f32x4 acc = *reinterpret_cast<const f32x4*>(xgmi_slot(xv, 0, epoch) + off + row);
    for (int r = 1; r < xv.size; ++r) acc += *reinterpret_cast<const f32x4*>(xgmi_slot(xv, r, epoch) + off + row);
    acc *= xscale;
    *reinterpret_cast<f32x4*>(&sm.gt[tr0 + 16 * q][4 * tc]) = acc;
    const int o = o0 + tr0 + 16 * q;
    if (o < lout && i < lin) *reinterpret_cast<f32x4*>(gw + static_cast<long>(o) * lin + i) = acc;
  }
  if (bias) {
    float b = xgmi_slot(xv, 0, epoch)[off + 4096 + threadIdx.x];
    for (int r = 1; r < xv.size; ++r) b += xgmi_slot(xv, r, epoch)[off + 4096 + threadIdx.x];
    b *= xscale;
    sm.gb[threadIdx.x] = b;
    if (o0 + static_cast<int>(threadIdx.x) < lout) gbp[o0 + threadIdx.x] = b;
  }
}

template <int MODE, bool XCHG>
__device__ __forceinline__ void bwd_fused(const MlpTrainArgs& a, int j, const optdev::Hyper& h, bool use_m, Smem& sm, Park& pk,
                          bool park, uint32_t xepoch, int* s_fail, const XgmiView* xv) {
  const MlpLayerArgs& L = a.L[j];
  const bool last = j == a.nl - 1;
  const int B = a.B, t = blockIdx.x;
  const uint16_t* GT = last ? a.dlogT : a.dT[j + 1];
  const int ot = (L.out + 63) / 64, nwg = ot * ((L.in + 63) / 64);
  const rsrc_t rg = mkbuf(GT, static_cast<long>(last ? 32 : L.out) * B * 2);
  const rsrc_t ra = mkbuf(a.actT[j], static_cast<long>(L.in) * B * 2);
  const bool mine = t < nwg;
  const int o0 = (t % ot) * 64, i0 = (t / ot) * 64;
  WgLoads Wg;
  UpLoads U;
  if (mine) {
    wg_load(Wg, rg, ra, B, L.out, L.in, o0, i0, 0, i0 == 0);
    up_load(U, L, o0, i0, use_m, MODE != 0, false);
  }
  if (pk.l >= 0) {  // layer j + 1's parked W^T tile (its dgrads all finished before the last barrier)
    wt_flush(a.L[j + 1], pk.o0, pk.i0, sm);
    pk.l = -1;
  }
  if (!mine) return;
  wgrad_tile(L, Wg, rg, ra, B, o0, i0, &sm);
  lds_sync();
  const int tc = threadIdx.x & 15, tr0 = threadIdx.x >> 4;
  if constexpr (XCHG) xchg_tile(a, *xv, j, t, xepoch, s_fail, sm, o0, i0);
#pragma unroll
  for (int q = 0; q < 4; ++q) U.g[q] = *reinterpret_cast<const f32x4*>(&sm.gt[tr0 + 16 * q][4 * tc]);
  if (i0 == 0 && threadIdx.x < 64) U.bg = sm.gb[threadIdx.x];
  up_finish<MODE>(U, L, h, o0, i0, use_m, sm, park);
  if (park) pk = Park{j, o0, i0};
  else lds_sync();  // gt / gb reuse
}

// The update of layer l (tiles of this workgroup: the ones whose weight gradient it computed)
template <int MODE>
__device__ __forceinline__ void update_layer(const MlpTrainArgs& a, int l, const optdev::Hyper& h, bool use_m, Smem& sm,
                                             UpLoads& P, bool pre) {
  const MlpLayerArgs& L = a.L[l];
  const int uot = (L.out + 63) / 64, nup = uot * ((L.in + 63) / 64);
  for (int t = blockIdx.x; t < nup; t += gridDim.x) {
    UpLoads U;
    const int o0 = (t % uot) * 64, i0 = (t / uot) * 64;
    if (pre && t == static_cast<int>(blockIdx.x)) {
      up_finish<MODE>(P, L, h, o0, i0, use_m, sm);  // the first tile's state was loaded during the GEMMs
      continue;
    }
    up_load(U, L, o0, i0, use_m, MODE != 0);
    up_finish<MODE>(U, L, h, o0, i0, use_m, sm);
  }
}

// Phase stamps (optional, int64[128]): [k] workgroup 0's 100 MHz wall clock at boundary k, [64 + k] the latest
// workgroup's (atomic max).
__device__ __forceinline__ void stamp(const MlpTrainArgs& a, int& k) {
  if (a.stamps != nullptr && threadIdx.x == 0) {
    const long long t = static_cast<long long>(__builtin_amdgcn_s_memrealtime());
    if (blockIdx.x == 0) a.stamps[k] = t;
    atomicMax(reinterpret_cast<unsigned long long*>(a.stamps + 64 + k), static_cast<unsigned long long>(t));
  }
  ++k;
}

// x^T (bf16, the first layer's weight-gradient operand, read in B0): 8 batch rows of one input column per thread
__device__ __forceinline__ void write_xT(const MlpTrainArgs& a) {
  const int in0 = a.L[0].in, nb = a.B / 8;
  const rsrc_t rx = mkbuf(a.actT[0], static_cast<long>(in0) * a.B * 2);
  for (int e = blockIdx.x * MT + threadIdx.x; e < in0 * nb; e += gridDim.x * MT) {
    const int i = e / nb, m = (e % nb) * 8;
    u16x8 o;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) o[jj] = f2bf(a.x[static_cast<long>(m + jj) * in0 + i]);
    bst16_sc1(rx, (i * a.B + m) * 2, o);
  }
}

template <int MODE, bool XCHG>
__global__ __launch_bounds__(MT) void k_mlp_train(MlpTrainArgs a) {
  __shared__ Smem sm;
  __shared__ int s_step;
  __shared__ unsigned s_launch;
  __shared__ uint32_t s_xepoch;
  __shared__ int s_xfail;
  // the peer view in LDS: its per-lane indexed arrays (base[rank]) must not be indexed in the kernel-argument block
  // (a divergent index there makes the compiler copy the whole argument block to scratch)
  __shared__ XgmiView s_xv;
  int ks = 0, kb = 0;
  stamp(a, ks);
  // world > 1: this launch's exchange epoch (block-collective; the last workgroup to finish advances it)
  uint32_t xepoch = 0u;
  if constexpr (XCHG) {
    if (threadIdx.x == 0) {  // field by field (a struct copy out of the argument block is a memcpy that keeps a
                             // private copy of the whole block alive)
#pragma unroll
      for (int r = 0; r < kXgmiMaxRanks; ++r) s_xv.base[r] = a.xv.base[r];
      s_xv.state = a.xv.state;
      s_xv.host = a.xv.host;
      s_xv.timeout_ticks = a.xv.timeout_ticks;
      s_xv.read_delay_ticks = a.xv.read_delay_ticks;
      s_xv.flag_bytes = a.xv.flag_bytes;
      s_xv.slot_bytes = a.xv.slot_bytes;
      s_xv.rank = a.xv.rank;
      s_xv.size = a.xv.size;
      s_xv.blocks = a.xv.blocks;
    }
    __syncthreads();
    xepoch = xgmi_epoch(s_xv, blockIdx.x, &s_xepoch);
  }
  if (threadIdx.x == 0) {
    s_step = __hip_atomic_load(a.step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    s_launch = __hip_atomic_load(a.bar + kBarStride * (kBarGroups + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const int nbar = 2 * a.nl - 1;  // F0..F(L-2), CE, B(L-1)..B1
  const Bar bar{a.bar, s_launch * static_cast<unsigned>(nbar)};
  optdev::Hyper h;
  h.lr = a.hp[HP_LR]; h.b1 = a.hp[HP_BETA1]; h.b2 = a.hp[HP_BETA2]; h.eps = a.hp[HP_EPS];
  h.wd = a.hp[HP_WD]; h.mom = a.hp[HP_MOMENTUM]; h.gscale = a.hp[HP_GRAD_SCALE];
  h.step = s_step;
  h.step_size = 0.f;
  h.inv_sqrt_bc2 = 1.f;
  if (MODE != 0) {
    const float bc1 = 1.f - __powf(h.b1, static_cast<float>(h.step));
    const float bc2 = 1.f - __powf(h.b2, static_cast<float>(h.step));
    h.step_size = h.lr / bc1;
    h.inv_sqrt_bc2 = rsqrtf(bc2);
  }
  const bool use_m = MODE != 0 || h.mom != 0.f;
  const int nl = a.nl, B = a.B;
  RowLoads R;
  if (nl > 1) fwd_prefetch(a, 0, R); else ce_prefetch(a, R);
  if (nl > 1) {
    fwd_phase<true>(a, 0, R, sm);
    stamp(a, ks);
    grid_arrive(bar, kb);
    write_xT(a);  // drained by the next arrive, read only in B0
    if (nl > 2) fwd_prefetch(a, 1, R); else ce_prefetch(a, R);
    grid_wait(bar, a.err, kb++);
    stamp(a, ks);
    for (int l = 1; l < nl - 1; ++l) {
      fwd_phase<false>(a, l, R, sm);
      stamp(a, ks);
      grid_arrive(bar, kb);
      if (l + 1 < nl - 1) fwd_prefetch(a, l + 1, R); else ce_prefetch(a, R);
      grid_wait(bar, a.err, kb++);
      stamp(a, ks);
    }
    ce_phase<false>(a, R, sm);
  } else {
    write_xT(a);
    ce_phase<true>(a, R, sm);
  }
  stamp(a, ks);
  grid_arrive(bar, kb);
  dgrad_prefetch(a, nl - 1, R);
  grid_wait(bar, a.err, kb++);
  stamp(a, ks);
  UpLoads U;
  // (SGD keeps the unfused form: with both forms in its body the compiler spills 1.6 KB per lane)
  bool fuse = MODE != 0 && (a.flags & 2) == 0;
  for (int l = 0; l < nl; ++l)
    fuse = fuse && ((a.L[l].out + 63) / 64) * ((a.L[l].in + 63) / 64) <= static_cast<int>(gridDim.x);
  if (fuse) {
    // Bj: the dgrad tiles (the hand-off), then -- between arrive and wait -- this workgroup's weight-gradient tile
    // of layer j updated straight from its accumulators (W^T parked until the next window) and the next dgrad's
    // weight fragments.  B0: layer 1's parked W^T, layer 0's gradient and update (no barrier left).
    Park pk{-1, 0, 0};
    for (int j = nl - 1; j >= 1; --j) {
      bwd_phase(a, j, 0, R, sm, U, false, a.L[j], use_m, MODE != 0);
      stamp(a, ks);
      grid_arrive(bar, kb);
      bwd_fused<MODE, XCHG>(a, j, h, use_m, sm, pk, true, xepoch, &s_xfail, &s_xv);
      dgrad_prefetch(a, j - 1, R);
      stamp(a, ks);
      grid_wait(bar, a.err, kb++);
      stamp(a, ks);
    }
    bwd_fused<MODE, XCHG>(a, 0, h, use_m, sm, pk, false, xepoch, &s_xfail, &s_xv);
    stamp(a, ks);  // (an empty phase: the boundary count of the unfused form)
  } else {
    // B(nl-1) .. B1: the dgrad tiles (the hand-off), then -- between arrive and wait -- the weight-gradient tiles of
    // layer j, the update of layer j + 1 (its weight-gradient tiles are this workgroup's from B(j+1)'s window; every
    // dgrad that read its W^T finished before that barrier) and the next dgrad's weight fragments
    for (int j = nl - 1; j >= 1; --j) {
      const bool up = j + 1 < nl;
      const bool pre = up && (a.flags & 1) == 0;
      bwd_phase(a, j, 0, R, sm, U, false, a.L[j], use_m, MODE != 0);
      stamp(a, ks);
      grid_arrive(bar, kb);
      bwd_phase(a, j, 1, R, sm, U, pre, a.L[up ? j + 1 : j], use_m, MODE != 0);
      if (up) update_layer<MODE>(a, j + 1, h, use_m, sm, U, pre);
      dgrad_prefetch(a, j - 1, R);
      stamp(a, ks);
      grid_wait(bar, a.err, kb++);
      stamp(a, ks);
    }
    // B0: layer 0's weight gradient and the updates of layers 1 and 0 (no hand-off left: no barrier).  Gradient tiles
    // stored by OTHER threads of this workgroup earlier (layer 1 in B1's window, layer 0 just below) are drained and
    // met before the updates read them (the other layers have a grid barrier's arrive in between)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const bool pre0 = nl > 1 && (a.flags & 1) == 0;
    bwd_phase(a, 0, 1, R, sm, U, pre0, a.L[nl > 1 ? 1 : 0], use_m, MODE != 0);
    stamp(a, ks);
    if (nl > 1) update_layer<MODE>(a, 1, h, use_m, sm, U, pre0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    update_layer<MODE>(a, 0, h, use_m, sm, U, false);
  }
  stamp(a, ks);
  if constexpr (XCHG) xgmi_finish(s_xv, blockIdx.x, xepoch);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    float s = 0.f;
    for (int t = 0; t < B / 32; ++t) s += __hip_atomic_load(a.loss_part + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.loss[0] = s / static_cast<float>(B);
    // every workgroup read the old count (and the launch word) at its start, before the first barrier
    __hip_atomic_store(a.step, s_step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.bar + kBarStride * (kBarGroups + 1), s_launch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

int mlp_train_grid(int device) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) return 0;
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&k_mlp_train<1, false>), MT, 0) !=
          hipSuccess ||
      per < 1)
    return 0;
  return cus;  // one workgroup per CU: every one resident (the grid barrier needs it)
}

hipError_t mlp_train_step(const MlpTrainArgs& a, int grid, hipStream_t s) {
  if (grid <= 0 || a.nl < 1 || a.nl > kMlpMaxLayers || a.B % 32 != 0) return hipErrorInvalidValue;
  if (a.xchg) {  // the exchange rides on the fused form only, with one flag word per workgroup of the view
    if (a.mode == 0 || (a.flags & 2) != 0 || a.xv.blocks < grid) return hipErrorInvalidValue;
    for (int l = 0; l < a.nl; ++l)
      if (((a.L[l].out + 63) / 64) * ((a.L[l].in + 63) / 64) > grid) return hipErrorInvalidValue;
    int in[kMlpMaxLayers], out[kMlpMaxLayers];
    for (int l = 0; l < a.nl; ++l) { in[l] = a.L[l].in; out[l] = a.L[l].out; }
    if (mlp_xchg_floats(in, out, a.nl) * 4 > a.xv.slot_bytes) return hipErrorInvalidValue;
  }
  if (a.xchg) {
    switch (a.mode) {
      case 1: hipLaunchKernelGGL((k_mlp_train<1, true>), dim3(grid), dim3(MT), 0, s, a); break;
      case 2: hipLaunchKernelGGL((k_mlp_train<2, true>), dim3(grid), dim3(MT), 0, s, a); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  switch (a.mode) {
    case 0: hipLaunchKernelGGL((k_mlp_train<0, false>), dim3(grid), dim3(MT), 0, s, a); break;
    case 1: hipLaunchKernelGGL((k_mlp_train<1, false>), dim3(grid), dim3(MT), 0, s, a); break;
    case 2: hipLaunchKernelGGL((k_mlp_train<2, false>), dim3(grid), dim3(MT), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace pde
