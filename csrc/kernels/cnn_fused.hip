// Fused MNIST-CNN training step for gfx950: the whole of horovod/mnist_horovod.py:9-25's `Net`
// (conv5x5 1->10, maxpool2, ReLU, conv5x5 10->20, Dropout2d, maxpool2, ReLU, fc 320->50, ReLU,
// dropout, fc 50->10, log_softmax) + NLL loss + the complete backward pass, with every activation
// resident in LDS.
//
// Why: the network is 21,840 parameters and ~1 MFLOP/image forward; at the reference batch (1024 per
// worker) the layer-by-layer path is ~40 kernels of a few microseconds each, every one far below the
// chip's roofline.  Here ONE workgroup (16 wave64s, one per CU: the LDS image is
// ~122 KB) trains NI=4 images end to end.  Every phase is a short dependent chain (LDS gathers feeding a
// few MFMAs, L2 weight loads feeding a dot product), so the kernel is latency-bound: 16 waves (4 per
// SIMD, <= 128 VGPRs) hide twice the latency of 8 and cut each phase's per-wave trip count in half:
//   * the five convolution GEMMs -- conv1 fwd, conv2 fwd, conv2 dgrad, conv2 wgrad, conv1 wgrad -- run
//     on the matrix cores (v_mfma_f32_16x16x32_bf16, fp32 accumulate) as implicit GEMMs whose operand
//     fragments are gathered straight from the LDS-resident bf16 activations (im2col never exists);
//   * the conv weights are re-laid out ONCE per workgroup into LDS in MFMA B-fragment order (one 16-byte
//     ds_read per lane per fragment); fc1's 64 KB weight matrix is read from L2 (shared by all WGs);
//   * the forward M dimension is ordered (pooled cell, 2x2 tap), so an MFMA lane's 4 accumulator rows
//     are exactly the 4 taps of one pooling window: max-pool, argmax, bias, dropout2d and ReLU are done
//     on the accumulators, and no pre-pool activation is ever stored;
//   * backward scatters the pooled gradients to their argmax taps once (a dense bf16 plane per channel)
//     and feeds it to the dgrad / wgrad GEMMs; small fc layers, softmax/NLL and masks stay in fp32 VALU;
//   * every weight gradient of the 4 images is complete after its phase and is written straight to the
//     workgroup's fp32 slab; k_cnn_reduce sums the slabs in a fixed order (deterministic) straight into
//     the flat gradient buffer (e.g. the DDP bucket).
// Dropout masks come from a counter-based hash keyed by a device-resident counter that k_cnn_reduce
// advances, so hipGraph replays draw fresh masks.  Precision: bf16 MFMA operands (images, conv weights,
// conv activations and their gradients), fp32 accumulation, fp32 fc layers / loss / gradients.
#include <cstddef>
#include <type_traits>

#include "common.cuh"
#include "optim_device.h"
#include "pde_kernels.h"
#include "xgmi_device.h"

namespace pde {

namespace {

constexpr int T = 1024;           // 16 waves
constexpr int NW = T / 64;
constexpr int NI = 4;             // images per workgroup
constexpr int C1 = 10, C2 = 20, KS = 5, H0 = 28, O1 = 24, P1 = 12, O2 = 8, P2 = 4, F1 = 50, F2 = 10;
constexpr int NX = H0 * H0, NC1 = P1 * P1, NR1 = C1 * NC1, NC2 = P2 * P2, NIN = C2 * NC2;  // 784 144 1440 16 320
// LDS channel pitches of the [ci][cell] planes (r1 in u16, a1 in bytes, e1 in u32): 144 cells padded so that the
// channels a wave touches at once fall in different banks (ds_*_b32 banks are (a / 4) mod 32; at a 288-byte
// pitch channels 0, 4, 8 share one: P1's stores and P9's reads ran 3-6 LDS cycles per instruction, r4s)
constexpr int RP16 = 146, RP8 = 148;
static_assert(RP16 >= NC1 && RP8 >= NC1, "channel planes hold the 144 cells");
static_assert(RP16 % 2 == 0 && RP8 % 4 == 0, "P9 reads 4 cells' argmax bytes as one aligned 4-byte word");
// e1: the conv1-output gradient of every pooled cell, written by P7b's epilogue as a bf16 pair positioned at its
// argmax tap's column (tap dx = 0 -> low half, 1 -> high half; 0 for a relu-dead cell) and read by P9 as 4 cells
// per 16-byte load.  592-byte channel rows: 16-byte aligned, and the 10 channels of a 16-lane b128 phase start
// 20 banks apart (disjoint 4-bank spans)
constexpr int EP = 148;
constexpr unsigned char AM_DEAD = 0xFF;  // a1 of a relu-dead cell (r1 == 0): no tap carries a gradient
// LDS row pitch of the images x / x1 (28 pixels + 8 zero columns): with x1 9 banks after x, P1's pixel-pair
// gathers take 2.75 LDS cycles per instruction instead of 4 (r4t model; columns 28.. are read by the zero-weight
// kx = 5 taps only)
constexpr int XP = 36, NXP = H0 * XP;
constexpr int DHP = 52;  // LDS row pitch (floats) of dh: 16-byte rows, P6 reads them as float4
constexpr int W1N = C1 * KS * KS, W2N = C2 * C1 * KS * KS, FC1N = F1 * NIN, FC2N = F2 * F1;
constexpr int K2 = C1 * KS * KS;       // 250: conv2 reduction (ci,ky,kx) in the weight's own order
// conv2 fwd: K ordered (tap, ci) with ci padded to 16 over a channel-last copy of r1, so a lane's 8
// k-values are ONE 16-byte LDS read: k = 32 ks + 8 lg + j -> tap 2 ks + lg/2, ci 8 (lg & 1) + j
constexpr int C1P = 16;
constexpr int KS2 = (KS * KS * C1P + 31) / 32;  // 13 k-steps (the last one half padding)
constexpr int KSW2 = NI * 8 * 8 / 32;           // 8 conv2-wgrad k-steps: K = (image, y, x)
// conv2 dgrad: K = (tap, co) with co padded to 24 = 3 groups of 8, packed: k-step ks, lane group lg holds
// group g = 4 ks + lg = (tap g / 3, channels 8 (g % 3) .. +7).  The gradient is kept with each co group of 8
// contiguous (co 20..23 zero), so a lane's 8 k-values are ONE 16-byte LDS read of its own position.
constexpr int CG = 3;                                // co groups of 8 per tap
constexpr int NGD = KS * KS * CG;                    // 75 (tap, co-group) pairs
constexpr int KSD = (NGD + 3) / 4;                   // 19 k-steps (25 with one k-step per tap)
// d2n layout (u16 units): element (im, Y, X, co) at im D2N_IM + Y D2N_RP + X D2N_P + (co / 8) D2N_Q + co % 8 --
// 48-byte positions, 528-byte rows, co groups 256 bytes apart (interleaved with other positions' slots).  A P7b
// A read (a 16-lane b128 group mixes two k-groups and two rows of the tile) models 5.6 LDS cycles per
// wave-instruction against 6.75 for plain [pos][40] rows (scripts/p7b_lds_model.py; 4 is conflict-free)
constexpr int D2N_P = 24, D2N_RP = 264, D2N_Q = 128;
constexpr int D2N_IM = 7 * D2N_RP + 7 * D2N_P + 2 * D2N_Q + 8;  // 2280: one past the last slot of an image
static_assert(D2N_IM % 8 == 0 && D2N_P % 8 == 0 && D2N_RP % 8 == 0 && D2N_Q % 8 == 0, "d2n: 16-byte slots");
__host__ __device__ constexpr int d2n_ofs(int im, int y, int x, int co) {
  return im * D2N_IM + y * D2N_RP + x * D2N_P + (co >> 3) * D2N_Q + (co & 7);
}
constexpr int D2R = O2 * O2 + 8;       // d2 plane row stride (u16): 144 B
constexpr int MT1 = O1 * O1 / 16;      // 36 conv1 M-tiles per image (4 cells x 4 taps each)
constexpr int MTD = NC1 * 1 / 16;      // 9 conv2-dgrad M-tiles per image (144 r1 positions)
constexpr int KSW1 = O1 * O1 / 32;     // 18 conv1-wgrad k-steps per image
// parameter offsets in the flat gradient (torch parameter order of Net)
constexpr int O_W1 = 0, O_B1 = O_W1 + W1N, O_W2 = O_B1 + C1, O_B2 = O_W2 + W2N, O_FC1W = O_B2 + C2,
              O_FC1B = O_FC1W + FC1N, O_FC2W = O_FC1B + F1, O_FC2B = O_FC2W + FC2N, NPARAM = O_FC2B + F2;
// Per-workgroup fp32 slabs hold every gradient EXCEPT fc1's weight (16,000 of the 21,840 parameters):
// that one is a rank-B product dW = dH^T . R2 over the whole batch, so each workgroup writes its 4 images'
// fc1 output gradients dH and inputs R2 (370 floats per image, K-contiguous) and k_cnn_reduce computes
// it as one f32-MFMA GEMM -- 1.5 MB of activations instead of 16 MB of slabs written and read back.
constexpr int NSLAB = NPARAM - FC1N;                     // 5,840 slab floats per workgroup
// (the slab's conv2-weight block [O_W2, O_W2 + W2N) holds dW2 as [co group of 4][kidx][4]: P7a's 16-byte
// stores of 16 consecutive kidx are 256 contiguous bytes; SLAB_OFS puts that block on a 128-byte line boundary
// and NSLABP pads each workgroup's slab to whole lines, so those stores are full-line writes)
static_assert(O_W2 % 4 == 0 && C2 % 4 == 0 && W2N % 4 == 0, "W2T: float4 columns of 4 co");
constexpr int SLAB_OFS = (32 - O_W2 % 32) % 32;                       // floats
constexpr int NSLABP = (SLAB_OFS + NSLAB + 31) / 32 * 32;             // slab pitch per workgroup (floats)
constexpr int S_FC1B = O_FC1B - FC1N, S_FC2W = O_FC2W - FC1N, S_FC2B = O_FC2B - FC1N;
constexpr int NACT = F1 + NIN;                           // activation rows: dH^T (50) then R2^T (320)
// row pitch (bf16 elements) of the activation image: the batch columns rounded up to 8 (16-byte operand loads)
__host__ __device__ constexpr int act_pitch(int nwg) { return (nwg * NI + 7) & ~7; }
static_assert(O_FC1W % 4 == 0 && FC1N % 4 == 0 && NSLAB % 4 == 0, "float4 slab columns");

__device__ __forceinline__ float hash_u01(unsigned long long seed, unsigned long long id) {
  unsigned long long z = seed + 0x9E3779B97F4A7C15ULL * (id + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return static_cast<float>(z >> 40) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ f32x4 mfma(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// Cross-lane helpers on DPP row operations and lane reads: no LDS round trip (a __shfl_xor butterfly is a chain
// of dependent ds_bpermutes, ~0.1 us each: P4's softmax ran 15 of them back to back).  Whole wave active.
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float lanef(float v, int l) {  // l wave-uniform
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;
// every lane: op over the wave (quads, 8-lane halves, 16-lane rows by DPP, then the 4 rows' values by lane reads)
template <class Op>
__device__ __forceinline__ float wave_all(float v, Op op) {
  v = op(v, dppf<DPP_XOR1>(v));
  v = op(v, dppf<DPP_XOR2>(v));
  v = op(v, dppf<DPP_HALF_MIRROR>(v));
  v = op(v, dppf<DPP_MIRROR>(v));
  return op(op(lanef(v, 0), lanef(v, 16)), op(lanef(v, 32), lanef(v, 48)));
}
__device__ __forceinline__ float wave_sum_dpp(float v) { return wave_all(v, [](float a, float b) { return a + b; }); }
__device__ __forceinline__ float wave_max_dpp(float v) { return wave_all(v, [](float a, float b) { return fmaxf(a, b); }); }

struct CnnSmem {
  // bf16 MFMA operands
  alignas(16) uint16_t r1n[NI][NC1][C1P];  // relu(maxpool(conv1)) channel-last, ci padded with zeros; e1 (P7b-P9)
                                           // later, spanning r1n and the front of w2f (both dead after P2)
  alignas(16) u16x8 w2f[KS2][2][64];   // conv2 fwd B fragments [kstep][ntile][lane]
  alignas(16) u16x8 w2d[KSD][64];      // conv2 dgrad B fragments [kstep][lane]: B[k=(tap,co)][n=ci]
  alignas(16) u16x8 w1f[64];           // conv1 B fragment
  // conv2-output gradient (non-zero only at the argmax taps), twice: channel-last for the dgrad A
  // fragments (co padded to 32 with zeros) and as 8x8 planes for the wgrad A fragments
  alignas(16) uint16_t d2n[NI * D2N_IM];     // (d2n_ofs layout)
  alignas(16) uint16_t d2[NI][C2][D2R];    // rows padded to 144 B: the 16 co rows of a wgrad A fragment hit
                                           // 16 distinct 16-B bank groups (128-B rows: 4-8-way conflicts)
  alignas(16) uint16_t zero16[8];      // 16 zero bytes: the target of every out-of-range operand read
  alignas(8) uint32_t p7tab[KSD * 4][2];  // P7b k-group g: {(ky << 16) | kx, d2n offset of the tap + co group}
  uint16_t x[NI][NXP];                 // images, rows of XP (columns 28.. zero)
  uint16_t xpad[18];                   // x1 starts 9 banks after x: P1 / P9 pixel-pair reads of x and x1 by
                                       // the same instruction no longer collide (8064-byte arrays)
  uint16_t x1[NI][NXP];                 // images shifted by one element (x1[i] = x[i + 1]): every pair of
                                       // consecutive pixels is ONE aligned 4-byte LDS read from x or x1
  uint16_t xonepad[48];                // xone starts 4 banks after x (36 words): P9's bias-column reads no longer
                                       // share a bank with the tap-(4,4) column (scripts/p9_lds_model.py)
  alignas(16) uint16_t xone[NI][NXP];  // bf16 1.0 everywhere: P9's B column 25 reads it (conv1's bias gradient)
  alignas(16) uint16_t r1[NI][C1 * RP16];   // relu(maxpool(conv1)), [ci][cell] (pitch RP16)
  // fp32 head
  alignas(16) float b1[C1];
  alignas(16) float b2[C2];
  alignas(16) float fc1b[F1];
  alignas(16) float fc2w[FC2N];
  alignas(16) float fc2b[F2];
  alignas(16) float r2[NI][NIN];       // fc1 input (NCHW flatten order); read as float4 in P3
  alignas(16) float dp2[NI][NIN];      // grad at the pooled conv2 output (dropout2d applied)
  float h1[NI][F1], m1[NI][F1], h1d[NI][F1];
  alignas(16) float dh[NI][DHP];       // rows padded to 16-byte multiples: P6 reads them as float4
  float mc2[NI][C2];
  float logit[NI][F2], dlog[NI][F2];
  float lossim[NI];                    // per-image loss terms (P4), summed at the end
  float valid[NI];
  int label[NI];
  alignas(16) unsigned char a1[NI][C1 * RP8];
  unsigned char a2[NI][NIN];
};
static_assert(sizeof(CnnSmem) <= 160 * 1024, "LDS budget");
static_assert((offsetof(CnnSmem, x1) - offsetof(CnnSmem, x)) / 4 % 32 == 9 &&
                  (offsetof(CnnSmem, xone) - offsetof(CnnSmem, x)) / 4 % 32 == 4,
              "x1 / xone bank offsets from x (P1 gathers, P9 B reads: scripts/p9_lds_model.py)");
static_assert(offsetof(CnnSmem, w2f) == offsetof(CnnSmem, r1n) + sizeof(uint16_t) * NI * NC1 * C1P &&
                  sizeof(uint32_t) * NI * C1 * EP <= sizeof(uint16_t) * NI * NC1 * C1P + sizeof(u16x8) * KS2 * 2 * 64,
              "e1 aliases r1n + w2f");
static_assert(offsetof(CnnSmem, d2n) == offsetof(CnnSmem, w1f) + sizeof(u16x8) * 64 &&
                  NW * 2 * 64 * sizeof(f32x4) <= sizeof(u16x8) * (KSD * 64 + 64) + sizeof(uint16_t) * NI * D2N_IM,
              "P9 partials alias w2d + w1f + d2n (not e1)");
static_assert(offsetof(CnnSmem, w2d) == offsetof(CnnSmem, w2f) + sizeof(u16x8) * KS2 * 2 * 64, "w2f, w2d adjacent");
constexpr int NT2 = 16 / NW;  // conv2-wgrad N-tiles (250 -> 16 x 16) per wave
constexpr int NFRAG = KS2 * 2 * 64 + KSD * 64 + 64;  // bf16 MFMA weight fragments (w2f, w2d, w1f)
static_assert(offsetof(CnnSmem, w1f) == offsetof(CnnSmem, w2d) + sizeof(u16x8) * KSD * 64, "w2d, w1f adjacent");
// fc1 forward: thread = (output j, 32-wide input chunk) over all images; fc1 backward dp2: thread = (input i,
// chunk of fc1 outputs).  Their partial sums live in the w2f region (dead after P2), combined in a fixed
// order (deterministic).
constexpr int FC1_KC = NIN / 32;        // 10 input chunks
constexpr int DP2_JC = 3;               // fc1-output chunks for dp2 (16, 16, 18 rows: float4-aligned starts)
constexpr int DP2_J = 16;               // rows per chunk (the last one takes the rest)
static_assert(F1 - DP2_J * (DP2_JC - 1) <= 20 && DP2_J % 4 == 0 && DHP >= DP2_J * (DP2_JC - 1) + 20, "dp2 chunks");
static_assert(F1 * FC1_KC <= T && NIN * DP2_JC <= T, "fc1 work split");
static_assert(sizeof(float) * NI * F1 * FC1_KC <= sizeof(u16x8) * KS2 * 2 * 64, "fc1 partials alias w2f");
static_assert(sizeof(float) * NI * NIN * DP2_JC <= sizeof(u16x8) * KS2 * 2 * 64, "dp2 partials alias w2f");
static_assert(NT2 * NW == 16, "conv2 wgrad tiling");

// Workgroup barrier for LDS hand-offs only: every wave's LDS accesses complete (lgkmcnt), then s_barrier --
// outstanding GLOBAL loads and stores stay in flight (an LDS-scoped fence; __syncthreads would also wait
// vmcnt(0)).  Waves of k_cnn_train only exchange data through LDS: the slab / activation stores drain under
// the following phases and prefetched weights (w3, w6) arrive across barriers.
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Single-process fused tail (cnn_train_fused with PDE_CNN_FUSED_TAIL): after P9 every workgroup of k_cnn_train
// meets at a grid barrier and the first RED_BLOCKS of them run k_cnn_reduce's roles (slab columns, fc1
// weight-gradient tiles, loss, SGD + fragment refresh) -- one launch per step instead of two, and no kernel
// boundary between the slabs' producers and their reducers.  Requires every workgroup resident at once (one
// 157 KB-LDS workgroup per CU: nwg <= CUs, checked on the host) and nothing else on the device: the barrier's
// bounded spin (2 s) sets `err` instead of hanging if that is ever violated.
struct CnnTail {
  const float* gscale;
  float* grads;
  float* loss;
  unsigned long long* rng;
  float* params;
  const float* hp;
  uint16_t* frag;
  int* step;
  unsigned* bar;  // [0] arrival counter, [1] generation
  int* err;
  int accumulate, B, on, pad;
};
__device__ void cnn_fused_tail(const CnnTail& tl, int rb, f32x4* part, uint32_t* s_epoch, int* s_fail,
                               const float* slabs, int nwg, const uint16_t* acts, const float* loss_part);

// Grid barrier over co-resident workgroups: every wave's global stores complete, one agent-scope release +
// arrival per workgroup; the last arrival resets the counter and bumps the generation; the others poll it
// (bounded), then acquire.
__device__ __forceinline__ void cnn_grid_barrier(unsigned* bar, unsigned n, int* err, unsigned* s_gen) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g0 = __hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned old = __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == n - 1) {
      __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
      __hip_atomic_fetch_add(bar + 1, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s at 100 MHz
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    *s_gen = g0;
  }
  __syncthreads();
}

// Stores of the per-workgroup outputs the reduction launch reads (slabs, activation columns, loss partials):
// SM 0 plain, 1 non-temporal, 2 write-through (sc1: the bytes leave the XCD's L2 under the remaining phases
// instead of at the kernel boundary), 3 write-through for the 8- / 16-byte stores only, the dword ones plain
// (narrow write-through stores cost several times their bytes' time).  Vector stores only.
template <int SM>
__device__ __forceinline__ void out_st(float* p, float v) {
  if constexpr (SM == 1) __builtin_nontemporal_store(v, p);
  else if constexpr (SM == 2) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else *p = v;
}
template <int SM>
__device__ __forceinline__ void out_st_u16x4(uint16_t* p, u16x4 v) {
  if constexpr (SM == 1) __builtin_nontemporal_store(v, reinterpret_cast<u16x4*>(p));
  else st_vec(reinterpret_cast<u16x4*>(p), v, SM >= 2);
}
template <int SM>
__device__ __forceinline__ void out_st4(float* p, f32x4 v) {
  if constexpr (SM == 1) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
  else if constexpr (SM >= 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else *reinterpret_cast<f32x4*>(p) = v;
}

// BREG: P7b's B operand (the conv2 data-gradient fragments, identical for every wave) is loaded from the
// fragment image into registers at the start of P7a instead of being staged in LDS -- a quarter of P7b's LDS
// traffic moves to the vector-memory path (L1 / L2 hits), which runs beside the LDS.
template <int SM, bool BREG>
__global__ __launch_bounds__(T) void k_cnn_train(const float* __restrict__ images, const int64_t* __restrict__ tgt,
                                                 int B, const float* __restrict__ params,
                                                 const u16x8* __restrict__ frag,
                                                 const unsigned long long* __restrict__ rng, float p_drop2,
                                                 float p_drop1, int training, float* __restrict__ slabs,
                                                 float* __restrict__ loss_part, uint16_t* __restrict__ acts,
                                                 unsigned long long* __restrict__ stamps, int stop_after,
                                                 CnnTail tail, int xmap) {
  // optional phase timestamps (diagnostic only: stamps == nullptr in production launches); stop_after = k
  // ends the kernel after phase stamp k (diagnostic: hardware counters of a kernel prefix)
#define PDE_STAMP(k)                                                                      \
  if (stamps != nullptr && threadIdx.x == 0) stamps[blockIdx.x * 16 + (k)] = wall_clock64(); \
  if (stop_after == (k)) return
  PDE_STAMP(0);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  CnnSmem& S = *reinterpret_cast<CnnSmem*>(smem_raw);
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);  // wave-uniform: scalar loop control / branches
  const int lr = lane & 15, lg = lane >> 4;  // fragment row/col (lane & 15) and k-group (lane >> 4)
  const float* gW1 = params + O_W1;
  const float* gW2 = params + O_W2;
  const float* gFC1W = params + O_FC1W;
  const float* gFC1B = params + O_FC1B;
  // xmap: workgroups that share an XCD (blockIdx % 8 under the observed round-robin placement) take
  // consecutive images, so the 8 workgroups writing one 128-B line of an activation row sit behind one L2
  const int lwg = (xmap & 1) ? (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int n0 = lwg * NI;

  // ---- P0: images -> bf16, weights -> bf16 MFMA fragments, fp32 head weights, dropout masks ------
  // every global load of the phase is issued first (unconditional, clamped addresses): conv1's fragment (w1f),
  // then the image quad.  Only w1f is stored to LDS now; conv2's forward fragments (w2f) are requested at the
  // end of P0 and stored at the end of P1, its data-gradient fragments (w2d) are requested in P4 and stored at
  // the end of P6 -- their latency is on no phase's critical path, and the burst of fragment reads every
  // workgroup makes at the start is 28 KB instead of 47 KB.
  // (vmcnt retires loads in issue order: the loads P0 itself consumes -- w1f, images, the head parameters --
  // are issued before the deferred fragment loads)
  static_assert(NI * NX / 4 <= T, "one image quad per thread");
  const int qi = min(t, NI * NX / 4 - 1);
  const int qim = (qi * 4) / NX, qoff = qi * 4 - qim * NX;
  constexpr int NF2F = KS2 * 2 * 64, NF2D = KSD * 64;  // fragment image: [w2f | w2d | w1f]
  static_assert(NF2F <= 2 * T && NF2D <= 2 * T && NF2F + NF2D + 64 == NFRAG, "fragment slots");
  u16x8 fr[2];
  const u16x8 fw1 = frag[NF2F + NF2D + (t & 63)];
  f32x4 img = *reinterpret_cast<const f32x4*>(images + static_cast<long>(min(n0 + qim, B - 1)) * NX + qoff);
  if (t < NI * NX / 4) {
    const int im = qim, off = qoff, n = n0 + im;
    const f32x4 v = n < B ? img : f32x4{0.f, 0.f, 0.f, 0.f};
    const int row = off / H0, col = off - row * H0;  // a quad never crosses a row (H0 % 4 == 0)
    uint16_t* dst = &S.x[im][row * XP + col];
    const uint16_t b0 = f2bf(v[0]), b1 = f2bf(v[1]), b2 = f2bf(v[2]), b3 = f2bf(v[3]);
    dst[0] = b0; dst[1] = b1; dst[2] = b2; dst[3] = b3;
    uint16_t* d1 = &S.x1[im][row * XP + col];
    if (col > 0) d1[-1] = b0;
    d1[0] = b1; d1[1] = b2; d1[2] = b3;
  }
  static_assert(H0 % 4 == 0 && XP >= H0 + 6, "image quads within a row; kx = 5 reads stay in the row");
  for (int i = t; i < NI * H0 * (XP - H0 + 1); i += T) {  // zero columns: x 28.., x1 27..
    const int r = i / (XP - H0 + 1), c = i - r * (XP - H0 + 1);
    if (c > 0) (&S.x[0][0])[r * XP + H0 - 1 + c] = 0;
    (&S.x1[0][0])[r * XP + H0 - 1 + c] = 0;
  }
  if (t < 64) S.w1f[t] = fw1;
  for (int i = t; i < NI * O2 * O2; i += T) {  // co group 2 zeroed (co 20..23 stay zero; 16..19 rewritten per step)
    const int im = i / (O2 * O2), pos = i - im * (O2 * O2);
    *reinterpret_cast<u16x8*>(&S.d2n[d2n_ofs(im, pos / O2, pos % O2, 16)]) = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  if (t < 8) S.zero16[t] = 0;
  static_assert((NI * NXP) % 8 == 0 && NI * NXP / 8 <= T, "xone: one 16-byte store per thread");
  if (t < NI * NXP / 8)
    reinterpret_cast<u16x8*>(&S.xone[0][0])[t] = u16x8{0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};
  if (t < KSD * 4) {  // P7b's per-k-group tap table (groups past NGD never match: ky = kx = 0x8000)
    const int g = t, tap = g / CG, cg = g - tap * CG, ky = tap / KS, kx = tap - ky * KS;
    S.p7tab[g][0] = g < NGD ? (static_cast<uint32_t>(ky) << 16) | static_cast<uint32_t>(kx) : 0x80008000u;
    S.p7tab[g][1] = static_cast<uint32_t>(g < NGD ? (-(ky * D2N_RP + kx * D2N_P) + cg * D2N_Q) * 2 : 0);  // bytes
  }
  for (int i = t; i < C1; i += T) S.b1[i] = params[O_B1 + i];
  for (int i = t; i < C2; i += T) S.b2[i] = params[O_B2 + i];
  for (int i = t; i < F1; i += T) S.fc1b[i] = gFC1B[i];
  for (int i = t; i < FC2N + F2; i += T) (&S.fc2w[0])[i] = params[O_FC2W + i];
  const unsigned long long seed = rng[0] * 0xD1B54A32D192ED03ULL;
  const float keep2 = training ? 1.f / (1.f - p_drop2) : 1.f;
  const float keep1 = training ? 1.f / (1.f - p_drop1) : 1.f;
  if (t < NI * C2) {
    const int im = t / C2, c = t - im * C2;
    const unsigned long long id = static_cast<unsigned long long>(n0 + im) * C2 + c;
    S.mc2[im][c] = (!training || hash_u01(seed ^ 0x5bd1e995ULL, id) >= p_drop2) ? keep2 : 0.f;
  } else if (t >= 128 && t < 128 + NI * F1) {
    const int u = t - 128, im = u / F1, j = u - im * F1;
    const unsigned long long id = static_cast<unsigned long long>(n0 + im) * F1 + j;
    S.m1[im][j] = (!training || hash_u01(seed ^ 0x27d4eb2fULL, id) >= p_drop1) ? keep1 : 0.f;
  } else if (t >= 384 && t < 384 + NI) {
    const int im = t - 384;
    const bool ok = n0 + im < B;
    S.valid[im] = ok ? 1.f : 0.f;
    S.label[im] = ok ? static_cast<int>(tgt[n0 + im]) : 0;
  }
  float* slab = slabs + static_cast<long>(blockIdx.x) * NSLABP + SLAB_OFS;
  fr[0] = frag[t];  // conv2 forward fragments: stored to LDS at the end of P1
  fr[1] = frag[min(t + T, NF2F - 1)];
  lds_sync();
  PDE_STAMP(1);

  // ---- P1: conv1 (MFMA, M = (cell, tap), K = (ky, kx6) 30 -> 32, N = co) + maxpool2 + relu ----------
  // K runs over 6-wide kernel rows (kx = 5 has zero weight): every k pair (kx even) is two consecutive
  // pixels, read as ONE aligned 4-byte LDS load -- from x when the window starts on an even column (dx = 0),
  // from the shifted copy x1 otherwise: 4 gathers per fragment instead of 8.
  {
    int koff[4];  // pair p: k = 8 lg + 2p = (ky, kx) offset into the image; pairs past k = 30 read offset 0
                  // (finite pixels times w1f's zero rows: no mask)
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int k = lg * 8 + 2 * p;
      koff[p] = k < KS * 6 ? (k / 6) * XP + (k % 6) : 0;
    }
    const u16x8 bw = S.w1f[lane];
    const int tap = lr & 3, dy = tap >> 1, dx = tap & 1;
    const uint16_t* xsrc = dx ? &S.x1[0][0] - 1 : &S.x[0][0];  // x1[i - 1] = x[i]: odd starts become even
    // a tile is 4 consecutive pooling cells of one cell row (12 % 4 == 0): image, cell row and first column
    // are wave-uniform (scalar), the lane adds its cell (lr >> 2) and tap -- no per-lane division
    static_assert(P1 % 4 == 0 && MT1 * 4 == NC1, "conv1 tiles: 4 cells of one row");
    const uint16_t* xlane = xsrc + dy * XP + 2 * (lr >> 2) + dx;
    auto gather = [&](int tile, u16x8& a) {
      const int im = tile / MT1, t4 = tile - im * MT1, py = t4 / (P1 / 4), px0 = (t4 - py * (P1 / 4)) * 4;
      const uint16_t* xb = xlane + im * NXP + 2 * py * XP + 2 * px0;
      u32x4 v;
#pragma unroll
      for (int p = 0; p < 4; ++p) v[p] = *reinterpret_cast<const uint32_t*>(xb + koff[p]);
      a = __builtin_bit_cast(u16x8, v);
    };
    static_assert((NI * MT1) % NW == 0, "every wave runs the same number of conv1 tiles");
    constexpr int NT1 = NI * MT1 / NW;  // 9 tiles per wave
    // all of the wave's gathers first, then its MFMAs, then the epilogues: no tile waits on another's LDS
    // round trip (a one-tile-ahead pipeline measured 3.0 us for this loop, r4p)
    u16x8 ag[NT1];
#pragma unroll
    for (int u = 0; u < NT1; ++u) gather(wid + u * NW, ag[u]);
    f32x4 accs[NT1];
#pragma unroll
    for (int u = 0; u < NT1; ++u) accs[u] = mfma(ag[u], bw, f32x4{0.f, 0.f, 0.f, 0.f});
    const float bias1 = lr < C1 ? S.b1[lr] : 0.f;
#pragma unroll
    for (int u = 0; u < NT1; ++u) {
      const int tile = wid + u * NW;
      const int im = tile / MT1, c0 = (tile - im * MT1) * 4;
      const f32x4 acc = accs[u];
      const int co = lr;  // rows (lg*4 + r) = taps r of cell c0 + lg
      // lanes co >= C1: w1f's columns and bias1 are zero there, so r == 0 -- r1n's ci padding gets its zeros;
      // their r1 / a1 stores are masked off (exec, no per-lane address selects)
      const bool live = co < C1;
      int am = 0;
      float m = acc[0];
      if (acc[1] > m) { m = acc[1]; am = 1; }
      if (acc[2] > m) { m = acc[2]; am = 2; }
      if (acc[3] > m) { m = acc[3]; am = 3; }
      const uint16_t r = f2bf(fmaxf(m + bias1, 0.f));
      if (r == 0) am = AM_DEAD;  // relu-dead: P7b's epilogue and P9 read the mask from a1
      S.r1n[im][c0 + lg][co] = r;
      if (live) {
        S.r1[im][co * RP16 + c0 + lg] = r;
        S.a1[im][co * RP8 + c0 + lg] = static_cast<unsigned char>(am);
      }
    }
  }
  if (stamps != nullptr) {  // diagnostic: conv1 done (waves 0 / 7 / 15), before the fragment stores
    if (t == 0) stamps[blockIdx.x * 16 + 13] = wall_clock64();
    if (t == 15 * 64) stamps[blockIdx.x * 16 + 15] = wall_clock64();
  }
  if (!(xmap & 2)) {  // conv2 forward fragments (loaded in P0): bf16 MFMA order, straight 16-byte stores
    // (xmap & 2: timing diagnostic, the stores and their wait skipped -- results invalid)
    u16x8* dst = &S.w2f[0][0][0];
    dst[t] = fr[0];
    if (t + T < NF2F) dst[t + T] = fr[1];
  }
  lds_sync();
  PDE_STAMP(2);

  // fc1's weights for P3 (32 per thread, 8 x 16-B L2 loads) are requested now: their latency hides under
  // conv2 (registers: 78 -> ~110 VGPRs, no spill at 4 waves per SIMD)
  f32x4 w3[8];
  if (t < F1 * FC1_KC) {
    const int j = t / FC1_KC, kc = t - j * FC1_KC;
    const f32x4* w4 = reinterpret_cast<const f32x4*>(gFC1W + j * NIN + kc * 4);
#pragma unroll
    for (int q = 0; q < 8; ++q) w3[q] = w4[q * (FC1_KC)];
  }

  // ---- P2: conv2 (MFMA, M = (cell, tap) 64/image = 4 M-tiles, K = (ci,ky,kx) 250 -> 256, N = co 20 -> 32)
  //          + dropout2d + maxpool2 + relu.  One (image, M-tile) per wave iteration, both N-tiles.
  for (int mtile = wid; mtile < NI * 4; mtile += NW) {
    const int im = mtile >> 2, mt = mtile & 3;
    const int tap = lr & 3, dy = tap >> 1, dx = tap & 1;
    const int cell = mt * 4 + (lr >> 2), py = cell >> 2, px = cell & 3;
    const int rb = (2 * py + dy) * P1 + 2 * px + dx;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    const uint16_t* r1n = &S.r1n[im][0][(lg & 1) * 8];
#pragma unroll
    for (int ks = 0; ks < KS2; ++ks) {
      const int tp = 2 * ks + (lg >> 1), ky = tp / KS, kx = tp - ky * KS;
      const u16x8 a = tp < KS * KS ? *reinterpret_cast<const u16x8*>(r1n + (rb + ky * P1 + kx) * C1P)
                                   : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      acc0 = mfma(a, S.w2f[ks][0][lane], acc0);
      acc1 = mfma(a, S.w2f[ks][1][lane], acc1);
    }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int co = nt * 16 + lr;
      if (co < C2) {
        const f32x4 v = nt == 0 ? acc0 : acc1;
        int am = 0;
        float m = v[0];
        if (v[1] > m) { m = v[1]; am = 1; }
        if (v[2] > m) { m = v[2]; am = 2; }
        if (v[3] > m) { m = v[3]; am = 3; }
        const int q = co * NC2 + mt * 4 + lg;
        S.r2[im][q] = fmaxf((m + S.b2[co]) * S.mc2[im][co], 0.f);
        S.a2[im][q] = static_cast<unsigned char>(am);
      }
    }
  }
  lds_sync();
  PDE_STAMP(3);

  // ---- P3: fc1 + relu + dropout.  Thread (j, kc): 32 weights of row j (8 x 16-B L2 loads, all in flight
  // together) against the 4 images' inputs; partials [kc][im][j] summed in kc order. -------------------
  {
    float* part = reinterpret_cast<float*>(&S.w2f[0][0][0]);
    if (t < F1 * FC1_KC) {
      const int j = t / FC1_KC, kc = t - j * FC1_KC;
      // chunk kc = inputs {40 q + 4 kc .. +3 : q = 0..7}: the 10 chunks of a wave read 10 consecutive
      // float4s of r2 (conflict-free), and adjacent lanes load adjacent 16 B of the weight row (w3, loaded
      // before P2)
      const f32x4* w = w3;
      float s4[NI] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int im = 0; im < NI; ++im) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(&S.r2[im][q * 4 * FC1_KC + kc * 4]);
          s4[im] += w[q][0] * x[0] + w[q][1] * x[1] + w[q][2] * x[2] + w[q][3] * x[3];
        }
#pragma unroll
      for (int im = 0; im < NI; ++im) part[(kc * NI + im) * F1 + j] = s4[im];
    }
    lds_sync();
    if (t < NI * F1) {
      const int im = t / F1, j = t - im * F1;
      float s1 = S.fc1b[j];
#pragma unroll
      for (int kc = 0; kc < FC1_KC; ++kc) s1 += part[(kc * NI + im) * F1 + j];
      const float h = fmaxf(s1, 0.f);
      S.h1[im][j] = h;
      S.h1d[im][j] = h * S.m1[im][j];
    }
  }
  lds_sync();
  PDE_STAMP(4);

  // fc1 weight columns for P6's dp2 (thread (i, jc): up to 17 rows of column i), requested now so their L2
  // latency hides under P4 / P5
  // (unconditional loads from clamped addresses -- no divergent branch around them, so the compiler tracks
  // them precisely; rows past the chunk / threads past NIN x DP2_JC load a valid element P6 never uses)
  constexpr int JPER = F1 - DP2_J * (DP2_JC - 1);  // 18: the longest chunk
  float w6[JPER];
  {
    const int tc = min(t, NIN * DP2_JC - 1);
    const int jc = tc / NIN, i = tc - jc * NIN;
#pragma unroll
    for (int u = 0; u < JPER; ++u) w6[u] = gFC1W[min(jc * DP2_J + u, F1 - 1) * NIN + i];
  }
  // conv2 data-gradient fragments for P7b: stored to LDS at the end of P6 (the w2d region is idle until then)
  u16x8 fd[2];
  if constexpr (!BREG) {
    fd[0] = frag[NF2F + t];
    fd[1] = frag[NF2F + min(t + T, NF2D - 1)];
  }

  // ---- P4: fc2 logits, then log_softmax + NLL + dlogits: ONE WAVE PER IMAGE, no block barrier in between.
  // Lane l < 4 F2 computes a quarter of logit v = l / 4 (rows j = l % 4 + 4 k), the quad sums it; the softmax
  // reductions run across the wave's lanes (one thread per image summing serially took ~1.5 us).
  static_assert(NI <= NW && 4 * F2 <= 64, "P4: a wave per image, a lane quad per logit");
  if (wid < NI) {
    const int im = wid, v = lane >> 2, p = lane & 3;
    const bool lv = v < F2;
    const int vr = lv ? v : 0;
    float s = 0.f;
    // (fully unrolled, like every loop between the w6 prefetch and P6: a loop header makes the compiler wait
    // for ALL outstanding global loads, w6 included)
#pragma unroll
    for (int k = 0; k < (F1 + 3) / 4; ++k) {
      const int j = p + 4 * k;
      if (j < F1) s += S.fc2w[vr * F1 + j] * S.h1d[im][j];
    }
    s += dppf<DPP_XOR1>(s);
    s += dppf<DPP_XOR2>(s);
    const float logit = s + S.fc2b[vr];
    const float m = wave_max_dpp(lv ? logit : -INFINITY);
    const float ex = __expf(logit - m);
    const float se = wave_sum_dpp(lv && p == 0 ? ex : 0.f);
    const float lse = m + __logf(se);
    const float val = S.valid[im];
    const int y = S.label[im];  // (loaded in P0: a global load here would wait behind the w6 prefetch)
    const float ly = lanef(logit, __builtin_amdgcn_readfirstlane(4 * y));  // y: the wave's image label
    const float inv_b = val / static_cast<float>(B);
    const float dl = (__expf(logit - lse) - (v == y ? 1.f : 0.f)) * inv_b;  // d logit v (lanes of quad v)
    if (lv && p == 0) S.dlog[im][v] = dl;
    if (lane == 0) S.lossim[im] = val * (lse - ly);
    // P5's dh = relu'(h1) * mask * (W2^T dlog) of THIS image, in the same wave: lane j < F1 gathers the 10
    // d logits from the quads by shuffles (the fc2 weight / bias gradients, which sum over the images, are
    // taken in P6 after the barrier)
    static_assert(F1 <= 64, "P4: a lane per fc1 output");
    const int j = lane < F1 ? lane : 0;
    float sh = 0.f;
#pragma unroll
    for (int vv = 0; vv < F2; ++vv) sh += S.fc2w[vv * F1 + j] * lanef(dl, 4 * vv);
    if (lane < F1) S.dh[im][lane] = (S.h1[im][lane] > 0.f) ? sh * S.m1[im][lane] : 0.f;
  }
  lds_sync();
  PDE_STAMP(5);
  PDE_STAMP(6);
  PDE_STAMP(7);

  // ---- P5 (fc2 backward) now lives in P4 (dh, per image) and P6 (the fc2 weight / bias gradients) -------

  // ---- P6: fc1 backward: dH / R2 columns for the batch-wide dW GEMM (k_cnn_reduce), db to the slab, and
  // dp2 = grad at the pooled conv2 output.  Columns n0..n0+3 of the K-contiguous bf16 [row][Bkp] image (the
  // reduction's bf16 MFMA operands): one 8-byte store per row (rows 0..49 dH^T, 50..369 R2^T); the workgroup
  // owning the last columns also zeroes the row padding up to Bkp (a multiple of 8).
  static_assert(FC2N + F2 <= T, "fc2 weight / bias gradients: one element per thread");
  if (t < FC2N) {  // fc2 weight gradient (all images' dlog / h1d, complete since P4's barrier)
    const int v = t / F1, j = t - v * F1;
    float s = 0.f;
#pragma unroll
    for (int im = 0; im < NI; ++im) s += S.dlog[im][v] * S.h1d[im][j];
    out_st<SM>(&slab[S_FC2W + t], s);
  } else if (t < FC2N + F2) {
    const int v = t - FC2N;
    float s = 0.f;
#pragma unroll
    for (int im = 0; im < NI; ++im) s += S.dlog[im][v];
    out_st<SM>(&slab[S_FC2B + v], s);
  }
  {
    const int Bk = gridDim.x * NI, Bkp = act_pitch(gridDim.x);
    const bool pad = Bkp != Bk && n0 + NI == Bk;
    for (int row = t; row < NACT; row += T) {
      u16x4 v;
#pragma unroll
      for (int im = 0; im < NI; ++im) v[im] = f2bf(row < F1 ? S.dh[im][row] : S.r2[im][row - F1]);
      out_st_u16x4<SM>(acts + static_cast<long>(row) * Bkp + n0, v);
      if (pad) out_st_u16x4<SM>(acts + static_cast<long>(row) * Bkp + n0 + NI, u16x4{0, 0, 0, 0});
    }
  }
  if (t < F1) {
    float s = 0.f;
#pragma unroll
    for (int im = 0; im < NI; ++im) s += S.dh[im][t];
    out_st<SM>(&slab[S_FC1B + t], s);
  }
  float* dpart = reinterpret_cast<float*>(&S.w2f[0][0][0]);  // [jc][im][i]
  if (t < NIN * DP2_JC) {  // thread (i, jc): sum over fc1 outputs j in chunk jc (column loads coalesced)
    const int jc = t / NIN, i = t - jc * NIN;
    const int j0 = jc * DP2_J, nj = jc == DP2_JC - 1 ? F1 - j0 : DP2_J;
    const float* w = w6;  // loaded before P4
    float s4[NI] = {0.f, 0.f, 0.f, 0.f};
    // dh read as float4 (5 per image instead of 18 scalars); products past the chunk are selected away
    // (the padding columns are never written: select, not multiply by zero)
#pragma unroll
    for (int im = 0; im < NI; ++im)
#pragma unroll
      for (int q = 0; q < (JPER + 3) / 4; ++q) {
        const f32x4 d = *reinterpret_cast<const f32x4*>(&S.dh[im][j0 + 4 * q]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int u = 4 * q + e;
          if (u < JPER) s4[im] += u < nj ? w[u] * d[e] : 0.f;
        }
      }
#pragma unroll
    for (int im = 0; im < NI; ++im) dpart[(jc * NI + im) * NIN + i] = s4[im];
  }
  lds_sync();
  // dp2 = grad at the pooled conv2 output, scattered to the argmax taps by the thread that combines it (both
  // layouts; every tap of every window is written) -- no barrier between the two; the conv2 bias gradient,
  // which needs every dp2 of a channel, runs after the phase's closing barrier
  for (int it = t; it < NI * NIN; it += T) {
    const int im = it / NIN, q = it - im * NIN, co = q / NC2, cell = q - co * NC2;
    float s1 = 0.f;
#pragma unroll
    for (int jc = 0; jc < DP2_JC; ++jc) s1 += dpart[(jc * NI + im) * NIN + q];
    const float v = (S.r2[im][q] > 0.f) ? s1 * S.mc2[im][co] : 0.f;
    S.dp2[im][q] = v;
    const int py = cell >> 2, px = cell & 3, a = S.a2[im][q];
    const uint16_t g = f2bf(v);
    const int p00 = (2 * py) * O2 + 2 * px;
    const uint32_t gv = g;
    *reinterpret_cast<uint32_t*>(&S.d2[im][co][p00]) = a == 0 ? gv : (a == 1 ? gv << 16 : 0u);
    *reinterpret_cast<uint32_t*>(&S.d2[im][co][p00 + O2]) = a == 2 ? gv : (a == 3 ? gv << 16 : 0u);
    uint16_t* dn = &S.d2n[d2n_ofs(im, 2 * py, 2 * px, co)];
    dn[0] = a == 0 ? g : 0;
    dn[D2N_P] = a == 1 ? g : 0;
    dn[D2N_RP] = a == 2 ? g : 0;
    dn[D2N_RP + D2N_P] = a == 3 ? g : 0;
  }
  if constexpr (!BREG) {
    u16x8* dst = &S.w2d[0][0];
    dst[t] = fd[0];
    if (t + T < NF2D) dst[t + T] = fd[1];
  }
  lds_sync();
  PDE_STAMP(8);
  if (t >= 448 && t < 448 + C2) {  // conv2 bias gradient (dp2 is not overwritten before P9)
    const int co = t - 448;
    f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int im = 0; im < NI; ++im)
#pragma unroll
      for (int c = 0; c < NC2; c += 4) s4 += *reinterpret_cast<const f32x4*>(&S.dp2[im][co * NC2 + c]);
    out_st<SM>(&slab[O_B2 + co], (s4[0] + s4[1]) + (s4[2] + s4[3]));
  }
  // BREG: the first KSB k-steps' B fragments of P7b requested now, ahead of P7a's slab stores (vmcnt retires
  // in issue order, so waiting for them never waits for those stores); P7b's k-step ks requests k-step
  // ks + KSB (all 19 held at once: 76 VGPRs, spills)
  constexpr int KSB = 8;
  u16x8 bd[BREG ? KSD : 1];
  if constexpr (BREG) {
#pragma unroll
    for (int ks = 0; ks < KSB; ++ks) bd[ks] = frag[NF2F + ks * 64 + lane];
  }

  // ---- P7a: conv2 wgrad (MFMA): dW2[co][(ci,ky,kx)] = sum_(im,y,x) d2[co][y][x] * r1[ci][y+ky][x+kx].
  // M = co (2 tiles), N = 250 -> 16 tiles (NT2 per wave), K = (im, y, x) 256 = 8 k-steps.  An A fragment
  // is one 16-byte row of the d2 plane.
  {
    // B gathers: the 8 consecutive u16 of a fragment start at a 2-byte-aligned address, so they are read as the
    // 5 aligned words covering them and funnel-shifted (v_alignbyte) when the start is odd -- one 16-byte read
    // there would be an unaligned LDS access (64 cycles), 8 masked u16 reads cost an exec round trip each
    // (columns kidx >= K2 and rows co >= C2 of the outputs are never stored: their lanes read real, finite
    // operands -- offset 0 / channel C2 - 1 -- instead of selecting zeros every k-step)
    int nb[NT2];
#pragma unroll
    for (int u = 0; u < NT2; ++u) {
      const int kidx = (wid * NT2 + u) * 16 + lr, ci = kidx / 25, r = kidx - ci * 25, ky = r / 5, kx = r - ky * 5;
      nb[u] = kidx < K2 ? ci * RP16 + ky * P1 + kx : 0;
    }
    const uint16_t* arow[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) arow[mt] = &S.d2[0][min(mt * 16 + lr, C2 - 1)][0];
    f32x4 acc[2][NT2];
#pragma unroll
    for (int u = 0; u < NT2; ++u) acc[0][u] = acc[1][u] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < KSW2; ++ks) {
      const int im = ks >> 1, y = (ks & 1) * 4 + lg;  // this lane's 8 positions: row y, x = 0..7
      u16x8 a[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) a[mt] = *reinterpret_cast<const u16x8*>(arow[mt] + im * C2 * D2R + y * O2);
#pragma unroll
      for (int u = 0; u < NT2; ++u) {
        const int e0 = nb[u] + y * P1;  // first element
        // (index arithmetic, not pointer casts: the loads must stay LDS loads, not generic flat ones)
        const uint32_t* wp = reinterpret_cast<const uint32_t*>(&S.r1[im][0]) + (e0 >> 1);
        const uint32_t sh = static_cast<uint32_t>(e0 & 1) * 2;  // 0 or 2 bytes
        uint32_t w[5];
#pragma unroll
        for (int q = 0; q < 5; ++q) w[q] = wp[q];
        u32x4 v;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = __builtin_amdgcn_alignbyte(w[q + 1], w[q], sh);
        const u16x8 b = __builtin_bit_cast(u16x8, v);
        acc[0][u] = mfma(a[0], b, acc[0][u]);
        acc[1][u] = mfma(a[1], b, acc[1][u]);
      }
    }
    // the slab's conv2-weight block is kept as [co group][kidx][4] (see SLAB_OFS): a lane's 4 accumulator rows
    // are 4 consecutive co of one kidx, so they leave as one 16-byte store, and the 16 lanes of a co group write
    // 256 contiguous bytes (5000 dword stores per workgroup before; narrow write-through stores cost several
    // times the bytes' time, MI355X_MICROARCH.md store rows)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int u = 0; u < NT2; ++u) {
        const int kidx = (wid * NT2 + u) * 16 + lr, cg = mt * 4 + lg;
        if (cg * 4 < C2 && kidx < K2) out_st4<SM>(&slab[O_W2 + (cg * K2 + kidx) * 4], acc[mt][u]);
      }
  }
  PDE_STAMP(9);

  // ---- P7b: conv2 dgrad (MFMA): dr1[ci][Y][X] = sum_(ky,kx) sum_co d2[Y-ky][X-kx][co] * w2[co][ci][ky][kx],
  // then relu'(r1).  M = r1 positions (9 tiles per image, 36 total, round-robin over waves), N = ci,
  // K = (tap, co24) packed into 19 k-steps: a lane's A fragment is the 16-byte co-group of ITS tap's source
  // position (Y-ky, X-kx), or the zero block when that position lies outside the 8x8 conv2 output -- every
  // read is unconditional, so the k-loop pipelines its LDS reads ahead of the MFMAs.
  {
    constexpr int MAXT = (NI * MTD + NW - 1) / NW;  // 3
    f32x4 acc[MAXT];
    int ty[MAXT], tx[MAXT], tb[MAXT];
    u16x2 tyx[MAXT];  // (ty, tx) packed: one packed subtract checks both tap offsets
#pragma unroll
    for (int u = 0; u < MAXT; ++u) {
      acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int tile = min(wid + u * NW, NI * MTD - 1);  // a 2-tile wave's third slot mirrors a real tile
      // (4x4-block tiles model fewer bank conflicts, 6.8 -> 6.0 LDS cycles per A read, but measured slower:
      // P7b 5.76 -> 5.96 us, r4t)
      const int im = tile / MTD, pos = (tile % MTD) * 16 + lr;
      ty[u] = pos / P1;
      tx[u] = pos - ty[u] * P1;
      tb[u] = d2n_ofs(im, ty[u], tx[u], 0) * 2;  // byte offset at tap (0,0), channel 0
      tyx[u] = u16x2{static_cast<uint16_t>(tx[u]), static_cast<uint16_t>(ty[u])};
    }
    const char* base = reinterpret_cast<const char*>(&S.d2n[0]);
    const char* zp = reinterpret_cast<const char*>(&S.zero16[0]);
    const char* tp[MAXT];  // each tile's tap-(0,0) address: a k-step adds the tap offset and selects
#pragma unroll
    for (int u = 0; u < MAXT; ++u) tp[u] = base + tb[u];
    const int ntile = wid < NI * MTD - 2 * NW ? 3 : 2;  // wave-uniform (36 tiles over 16 waves)

    // k-step ks, lane group lg: tap / co group of k-group g = 4 ks + lg from the LDS table (one 8-byte read
    // instead of the divisions), validity of (Y - ky, X - kx) for all tiles by one packed 16-bit subtract each
    // (r4af: P7b was the phase with the most VALU instructions)
    // (table entries are read one k-step before the loads that use them: the read's latency hides under the
    // previous k-step's MFMAs)
    auto tab = [&](int ks) { return *reinterpret_cast<const u32x2*>(&S.p7tab[min(ks, KSD - 1) * 4 + lg][0]); };
    auto load = [&](auto ntc, int ks, const u32x2& e, u16x8 (&a)[MAXT], u16x8& b) {
      const u16x2 kyx = __builtin_bit_cast(u16x2, e[0]);
      const int tofs = static_cast<int>(e[1]);
      if constexpr (BREG) b = bd[ks];
      else b = S.w2d[ks][lane];
#pragma unroll
      for (int u = 0; u < decltype(ntc)::value; ++u) {
        const bool ok = (__builtin_bit_cast(uint32_t, static_cast<u16x2>(tyx[u] - kyx)) & 0xFFF8FFF8u) == 0u;
        a[u] = *reinterpret_cast<const u16x8*>(ok ? tp[u] + tofs : zp);
      }
    };
    // the k-loop per tile count: a 2-tile wave neither reads nor multiplies a third tile (the phase is bound by
    // LDS bandwidth, and the mirrored third tile's A reads were ~20% of its bytes)
    auto kloop = [&](auto ntc) {
      constexpr int NT = decltype(ntc)::value;
      u16x8 an[MAXT], bn;
      load(ntc, 0, tab(0), an, bn);
      u32x2 en = tab(1);
#pragma unroll
      for (int ks = 0; ks < KSD; ++ks) {  // reads of k-step ks+1 are issued before the MFMAs of ks
        u16x8 ac[MAXT], bc = bn;
#pragma unroll
        for (int u = 0; u < NT; ++u) ac[u] = an[u];
        if constexpr (BREG) {
          if (ks + KSB < KSD) bd[ks + KSB] = frag[NF2F + (ks + KSB) * 64 + lane];
        }
        if (ks + 1 < KSD) {
          const u32x2 e = en;
          en = tab(ks + 2);
          load(ntc, ks + 1, e, an, bn);
        }
#pragma unroll
        for (int u = 0; u < NT; ++u) acc[u] = mfma(ac[u], bc, acc[u]);
      }
    };
    if (ntile == 3) kloop(std::integral_constant<int, 3>{});
    else kloop(std::integral_constant<int, 2>{});
    // epilogue: the lane's 4 consecutive cells as e1 words (relu'(r1) from a1's dead mark), one 16-byte store.
    // e1 aliases r1n / w2f, which no P7a / P7b wave reads (r1 itself is still P7a's B operand: no barrier here)
    uint32_t* e1 = reinterpret_cast<uint32_t*>(&S.r1n[0][0][0]);
#pragma unroll
    for (int u = 0; u < MAXT; ++u) {
      const int tile = wid + u * NW;
      const int ci = lr;
      if (tile < NI * MTD && ci < C1) {
        const int im = tile / MTD, cell = (tile % MTD) * 16 + lg * 4;
        const uint32_t am4 = *reinterpret_cast<const uint32_t*>(&S.a1[im][ci * RP8 + cell]);
        u32x4 e;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t am = (am4 >> (8 * r)) & 0xFFu;
          e[r] = am == AM_DEAD ? 0u : static_cast<uint32_t>(f2bf(acc[u][r])) << (16 * (am & 1u));
        }
        *reinterpret_cast<u32x4*>(&e1[(im * C1 + ci) * EP + cell]) = e;
      }
    }
  }
  lds_sync();
  PDE_STAMP(10);

  // ---- P9: conv1 wgrad (MFMA): dW1[co][(ky,kx)] = sum_(im,y,x) dconv1[co][y][x] * x[y+ky][x+kx], with
  // dconv1 = the pooled cell's gradient (e1) at its argmax tap.  M = co, N = 25 taps + the bias column (B = 1)
  // -> 2 tiles, K = (im, y, x) 2304 = 72 k-steps split over the waves; partials combined in LDS in a fixed order.
  // K order: a lane's 8 k-elements are 2 horizontally adjacent pooled cells x their 2x2 pooling windows, so its A
  // fragment is the 2 cells' e1 words placed by the argmax row (no per-position selects) and its B fragment 4
  // aligned pixel pairs (2 rows x 2 column pairs) of x or x1.
  {
    const uint16_t* xw[2];  // per N-tile column kidx: x (kx even) or x1 - 1 (kx odd) at the tap offset; the ones
                            // plane for the bias column 25; the discarded columns 26..31 read column 17's pixels
                            // (same addresses: a broadcast, no extra bank traffic)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k0 = u * 16 + lr, kidx = k0 > 25 ? 17 : k0;
      const int nb = (kidx / 5) * XP + kidx % 5;
      xw[u] = kidx == 25 ? &S.xone[0][0] : ((kidx % 5) & 1 ? &S.x1[0][0] - 1 : &S.x[0][0]) + nb;
    }
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const int co = lr;
    const int cr = co < C1 ? co : 0;  // rows co >= C1 are discarded: they read channel 0's (finite) data
    const uint32_t* e1 = reinterpret_cast<const uint32_t*>(&S.r1n[0][0][0]);
    // a fixed trip count (72 k-steps over 16 waves: 5 slots, the last one live on 8 waves -- a wave-uniform
    // skip): every slot's LDS reads are issued before the first select / MFMA
    constexpr int NK9 = (NI * KSW1 + NW - 1) / NW;
    static_assert(KSW1 * 4 * 2 == NC1 && P1 % 2 == 0, "P9: 4 lane groups x 2 cells per k-step");
    uint32_t m9[NK9];
    u32x2 e9[NK9];
    u16x8 b9[NK9][2];
#pragma unroll
    for (int u9 = 0; u9 < NK9; ++u9) {
      const int ks = wid + u9 * NW;
      if (ks >= NI * KSW1) break;  // wave-uniform
      const int im = ks / KSW1;
      const uint32_t gi = static_cast<uint32_t>((ks - im * KSW1) * 4 + lg);  // cell pair 0..71 of the image
      const uint32_t py = (gi * 43u) >> 8, pc = gi - py * 6u;               // gi / 6, gi % 6 (gi < 72)
      const int cell = static_cast<int>(py * P1 + pc * 2);
      m9[u9] = *reinterpret_cast<const uint16_t*>(&S.a1[im][cr * RP8 + cell]);
      e9[u9] = *reinterpret_cast<const u32x2*>(&e1[(im * C1 + cr) * EP + cell]);
      const int off = im * NXP + static_cast<int>(py * 2 * XP + pc * 4);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        // k order (dy, cell c, dx): pixel pairs (row 2py + dy, columns 4pc + 2c + {0, 1}), one ds_read2 per row
        // filling adjacent operand registers; never a 16-byte read at a 2-byte-aligned address, which the LDS
        // would replay as an unaligned access
        const uint16_t* src = xw[u] + off;
        u32x4 v;
        v[0] = *reinterpret_cast<const uint32_t*>(src);
        v[1] = *reinterpret_cast<const uint32_t*>(src + 2);
        v[2] = *reinterpret_cast<const uint32_t*>(src + XP);
        v[3] = *reinterpret_cast<const uint32_t*>(src + XP + 2);
        b9[u9][u] = __builtin_bit_cast(u16x8, v);
      }
    }
#pragma unroll
    for (int u9 = 0; u9 < NK9; ++u9) {
      if (wid + u9 * NW >= NI * KSW1) break;
      u32x4 a;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const bool lower = (m9[u9] >> (8 * c + 1)) & 1u;  // argmax in the window's second row (dead: e1 == 0)
        a[c] = lower ? 0u : e9[u9][c];
        a[2 + c] = lower ? e9[u9][c] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) acc[u] = mfma(__builtin_bit_cast(u16x8, a), b9[u9][u], acc[u]);
    }
    // w2d / w1f / d2n are dead after P7b (its last reads precede the barrier before P9): the per-wave partials go
    // there without another barrier (e1, still read by slower waves, lies before them)
    f32x4* part = reinterpret_cast<f32x4*>(&S.w2d[0][0]);
    part[(wid * 2 + 0) * 64 + lane] = acc[0];
    part[(wid * 2 + 1) * 64 + lane] = acc[1];
    lds_sync();
    if (stamps != nullptr && t == 0) stamps[blockIdx.x * 16 + 14] = wall_clock64();  // diagnostic: partials in LDS
    // conv1's weight and bias gradients (slab [O_W1, O_B1 + C1), contiguous): thread t sums gradient t over the
    // waves in a fixed order (bias c = B column 25 of channel c), each quad gathers its 4 sums with DPP and its
    // first lane writes them as one 16-byte store (r4ac: dword stores cost the step ~0.8 us; a staging pass
    // through LDS cost a barrier, and separate bias waves summing dr1 another ~0.3 us)
    static_assert(O_W1 == 0 && O_B1 == W1N && (W1N + C1) % 4 == 0, "conv1 gradients: one float4 run");
    if (wid * 64 < W1N + C1) {  // wave-uniform: waves 0-4
      const bool live = t < W1N + C1;
      const int c = t < W1N ? t / 25 : (live ? t - W1N : 0);
      const int kidx = t < W1N ? t - c * 25 : 25;
      const int u = kidx >> 4;
      const int l = (c >> 2) * 16 + (kidx & 15), r = c & 3;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += part[(w * 2 + u) * 64 + l][r];
      const int si = __builtin_bit_cast(int, s);
      const f32x4 q{s, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, si, 0x55, 0xF, 0xF, false)),
                    __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, si, 0xAA, 0xF, 0xF, false)),
                    __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, si, 0xFF, 0xF, 0xF, false))};
      if (live && (t & 3) == 0 && !(xmap & 4))  // (xmap & 4: timing diagnostic, stores skipped)
        out_st4<SM>(&slab[O_W1 + t], q);
    }
  }
  PDE_STAMP(11);

  // loss partial: the images' terms from P4
  if (wid == 0) {
    const float l = wave_sum_dpp(lane < NI ? S.lossim[lane] : 0.f);
    if (lane == 0) out_st<SM>(&loss_part[blockIdx.x], l);
  }
  if (stamps != nullptr) {  // diagnostic: every wave's stores drained, then the workgroup's last stamp
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    PDE_STAMP(12);
  }
  if (tail.on) {  // single process: the reduction roles in this launch (see CnnTail)
    __shared__ uint32_t s_epoch;
    __shared__ int s_fail;
    __shared__ unsigned s_gen;
    cnn_grid_barrier(tail.bar, gridDim.x, tail.err, &s_gen);
    // (w2f / w2d are dead after P9: the roles' 8 KB of partials live there)
    cnn_fused_tail(tail, blockIdx.x, reinterpret_cast<f32x4*>(&S.w2f[0][0][0]), &s_epoch, &s_fail, slabs,
                   gridDim.x, acts, loss_part);
  }
}

// The conv weights in bf16 MFMA B-fragment order (conv2 fwd [ks][ntile][lane], conv2 dgrad [tap][lane],
// conv1 [lane]), written once per step so every training workgroup loads them with 16-byte copies.
__global__ __launch_bounds__(256) void k_cnn_prep(const float* __restrict__ params, u16x8* __restrict__ frag) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= NFRAG) return;
  const float* gW1 = params + O_W1;
  const float* gW2 = params + O_W2;
  u16x8 f;
  if (e < KS2 * 2 * 64) {  // conv2 fwd: B[k=(tap, ci16)][n=co] = w2[co][ci][tap]
    const int ks = e >> 7, nt = (e >> 6) & 1, l = e & 63;
    const int co = nt * 16 + (l & 15), g = l >> 4, tap = 2 * ks + (g >> 1), c8 = (g & 1) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      f[j] = (co < C2 && tap < KS * KS && c8 + j < C1) ? f2bf(gW2[co * K2 + (c8 + j) * KS * KS + tap]) : 0;
  } else if (e < KS2 * 2 * 64 + KSD * 64) {  // conv2 dgrad: B[k=(tap, co24)][n=ci] = w2[co][ci][tap]
    const int e2 = e - KS2 * 2 * 64, ks = e2 >> 6, l = e2 & 63;
    const int ci = l & 15, g = ks * 4 + (l >> 4), tap = g / CG, c0 = (g - tap * CG) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      f[j] = (g < NGD && ci < C1 && c0 + j < C2) ? f2bf(gW2[(c0 + j) * K2 + ci * 25 + tap]) : 0;
  } else {  // conv1: B[k = (ky, kx6)][n = co] = w1[co][ky][kx] (kx = 5 and k >= 30: zero)
    const int l = e - KS2 * 2 * 64 - KSD * 64;
    const int co = l & 15, k0 = (l >> 4) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + j, ky = k / 6, kx = k - ky * 6;
      f[j] = (co < C1 && k < KS * 6 && kx < KS) ? f2bf(gW1[co * 25 + ky * KS + kx]) : 0;
    }
  }
  frag[e] = f;
}

// Single-element inverse of k_cnn_prep: parameter p (flat index) with new value w -> its bf16 slot(s) in
// the fragment image (conv2 weights appear twice: forward and dgrad layouts; conv1 once; everything else
// is not staged).  Padding slots are never touched, so the image stays valid once k_cnn_prep wrote it.
__device__ __forceinline__ void write_frag(uint16_t* __restrict__ f, int p, float w) {
  const uint16_t b = f2bf(w);
  if (p >= O_W2 && p < O_W2 + W2N) {
    const int q = p - O_W2, co = q / K2, r = q - co * K2, ci = r / (KS * KS), tap = r - ci * (KS * KS);
    const int g = ((tap & 1) << 1) | (ci >> 3);
    const int e = ((tap >> 1) << 7) | ((co >> 4) << 6) | (g << 4) | (co & 15);  // conv2 fwd [ks][ntile][lane]
    f[e * 8 + (ci & 7)] = b;
    const int gd = tap * CG + (co >> 3);                                         // conv2 dgrad [kstep][lane]
    const int e2 = KS2 * 2 * 64 + (gd >> 2) * 64 + (((gd & 3) << 4) | ci);
    f[e2 * 8 + (co & 7)] = b;
  } else if (p >= O_W1 && p < O_W1 + W1N) {
    const int co = p / (KS * KS), k25 = p - co * (KS * KS);
    const int k = (k25 / KS) * 6 + k25 % KS;                                     // (ky, kx6) order
    const int e = KS2 * 2 * 64 + KSD * 64 + (((k >> 3) << 4) | co);             // conv1 [lane]
    f[e * 8 + (k & 7)] = b;
  }
}

// Plain SGD (torch.optim.SGD, momentum 0, no weight decay: mnist_horovod.py:50) on the flat parameters
// with the fragment image refreshed in the same pass, so the next step needs no k_cnn_prep.
// hp: the fused optimiser's device hyper-parameters (HP_LR, HP_GRAD_SCALE).
__global__ __launch_bounds__(256) void k_cnn_sgd(float* __restrict__ params, const float* __restrict__ grads,
                                                 const float* __restrict__ hp, uint16_t* __restrict__ frag,
                                                 int* __restrict__ step) {
  if (step != nullptr && blockIdx.x == 0 && threadIdx.x == 0) step[0] += 1;  // the optimiser's device step
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= NPARAM) return;
  const float w = params[p] - hp[HP_LR] * (grads[p] * hp[HP_GRAD_SCALE]);
  params[p] = w;
  write_frag(frag, p, w);
}

// grads (+)= gscale * (sum_wg slabs[wg] | dH^T . R2) in a fixed order (deterministic).
//  * slab blocks (blockIdx < RED_SLAB_BLOCKS): 8 waves over 16 float4 slab columns; lane = column + 16 x
//    slab-lane, so one load instruction of a wave reads 4 slabs x 256 B and each thread keeps nwg/32
//    independent float4 loads in flight;
//  * fc1 blocks: one 16 x 16 tile of dW_fc1[j][i] = sum_n dH[n][j] R2[n][i] on the bf16 matrix cores
//    (16x16x32, fp32 accumulation; the operands are the bf16 activation columns, like every other weight
//    gradient here -- fp32 columns with f32 MFMAs moved twice the bytes, r4u), the batch K split over the 8
//    waves, partials summed in wave order.  Lane (lr, lg) loads 16 B (8 columns) of row j (A) / row i (B) at
//    k = kb + 8 lg;
//  * block 0 also reduces the per-workgroup loss partials and advances the dropout RNG counter.
// With hp (single process, no all-reduce in between) every block also applies the SGD update to the
// parameters it reduced and refreshes their bf16 fragment slots.
#ifndef PDE_CNN_RED_COLS
#define PDE_CNN_RED_COLS 16  // slab columns per reduce block (8: 183 blocks, measured slower, r4ag)
#endif
constexpr int RED_T = 512, RED_COLS = PDE_CNN_RED_COLS, RED_LANES = RED_T / RED_COLS;  // slab lanes per column
constexpr int NSLAB4 = NSLAB / 4;
constexpr int RED_SLAB_BLOCKS = (NSLAB4 + RED_COLS - 1) / RED_COLS;
constexpr int FC1_JT = (F1 + 15) / 16, FC1_IT = NIN / 16;   // 4 x 20 output tiles
constexpr int RED_BLOCKS = RED_SLAB_BLOCKS + FC1_JT * FC1_IT;
static_assert(NIN % 16 == 0, "fc1 input tiles");
static_assert(NI == 4, "activation columns are written as one 8-byte bf16 quad per row");

// w0 = params[p] and the hyper-parameters loaded at the start of the role (off the reduction's dependent chain)
__device__ __forceinline__ void sgd_update(float* params, float lr, float gsc, uint16_t* frag, int p, float w0,
                                           float g) {
  const float w = w0 - lr * (g * gsc);
  params[p] = w;
  write_frag(frag, p, w);
}

// One reduction role (rb = role block: slab columns for rb < RED_SLAB_BLOCKS, else an fc1 weight-gradient
// tile; role 0 also reduces the loss partials and advances the dropout RNG / SGD step counters), run by the
// first RED_T threads of a block whose every thread calls it (block barriers inside).  Called by k_cnn_reduce
// (one role per block) and, single process, by k_cnn_train's workgroups after a grid barrier.
__device__ __forceinline__ void cnn_reduce_role(int rb, f32x4* part, uint32_t* s_epoch, int* s_fail,
                                                const float* __restrict__ slabs, int nwg,
                                                const uint16_t* __restrict__ acts, const float* __restrict__ gscale,
                                                float* __restrict__ grads, int accumulate,
                                                const float* __restrict__ loss_part, int B, float* __restrict__ loss,
                                                unsigned long long* __restrict__ rng, float* __restrict__ params,
                                                const float* __restrict__ hp, uint16_t* __restrict__ frag,
                                                int* __restrict__ step, const XgmiView& xv, float xscale) {
  const int tid = threadIdx.x;
  const bool act = tid < RED_T;  // (k_cnn_train's threads past RED_T only join the barriers)
  const float gs = gscale ? gscale[0] : 1.f;
  // world > 1 with a peer view: this block's gradients go through the one-shot xGMI exchange (stage to my
  // slot, flags, read all ranks' values in rank order, x xscale) before the store + SGD update
  const bool xchg = xv.size > 1;
  // SGD operands requested up front: they do not depend on the reduction
  const float lrate = hp ? hp[HP_LR] : 0.f, gsc = hp ? hp[HP_GRAD_SCALE] : 0.f;
  const uint32_t epoch = xchg ? xgmi_epoch(xv, rb, s_epoch) : 0u;
  float* xmine = xchg ? xgmi_slot(xv, xv.rank, epoch) : nullptr;
  if (rb < RED_SLAB_BLOCKS) {
    const int col = tid % RED_COLS, sl = tid / RED_COLS;
    const int c4 = rb * RED_COLS + col;
    const f32x4* s4 = reinterpret_cast<const f32x4*>(slabs);
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
    const bool owner = act && sl == 0 && c4 < NSLAB4;
    // slab column -> parameter float4 (the xGMI staging index too); the conv2-weight block is [co group][kidx]
    // [4] in the slab (SLAB_OFS): its columns hold 4 co of one kidx, parameters K2 apart
    const int p4 = c4 < O_FC1W / 4 ? c4 : c4 + FC1N / 4;
    const bool w2t = c4 >= O_W2 / 4 && c4 < (O_W2 + W2N) / 4;
    int pj[4];
    {
      const int q = c4 - O_W2 / 4, cg = q / K2, kidx = q - cg * K2;
#pragma unroll
      for (int j = 0; j < 4; ++j) pj[j] = w2t ? O_W2 + (cg * 4 + j) * K2 + kidx : p4 * 4 + j;
    }
    f32x4 w0 = a0, g0 = a0;
    if (owner && w2t) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (hp) w0[j] = params[pj[j]];
        if (accumulate) g0[j] = grads[pj[j]];
      }
    } else {
      if (owner && hp) w0 = reinterpret_cast<const f32x4*>(params)[p4];
      if (owner && accumulate) g0 = reinterpret_cast<const f32x4*>(grads)[p4];
    }
    if (act && c4 < NSLAB4) {
      int b = sl;
      for (; b + 7 * RED_LANES < nwg; b += 8 * RED_LANES) {  // 8 independent loads in flight
        f32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = s4[static_cast<long>(b + u * RED_LANES) * (NSLABP / 4) + SLAB_OFS / 4 + c4];
        a0 += v[0] + v[4];
        a1 += v[1] + v[5];
        a2 += v[2] + v[6];
        a3 += v[3] + v[7];
      }
      for (; b + 3 * RED_LANES < nwg; b += 4 * RED_LANES) {  // 4 in flight (nwg / RED_LANES < 8)
        f32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = s4[static_cast<long>(b + u * RED_LANES) * (NSLABP / 4) + SLAB_OFS / 4 + c4];
        a0 += v[0];
        a1 += v[1];
        a2 += v[2];
        a3 += v[3];
      }
      for (; b < nwg; b += RED_LANES) a0 += s4[static_cast<long>(b) * (NSLABP / 4) + SLAB_OFS / 4 + c4];
    }
    if (act) part[sl * RED_COLS + col] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (owner) {
      v = part[col];
#pragma unroll 8
      for (int k = 1; k < RED_LANES; ++k) v += part[k * RED_COLS + col];
      v *= gs;
      if (xchg) reinterpret_cast<f32x4*>(xmine)[p4] = v;
    }
    bool ok = true;
    if (xchg) {
      ok = xgmi_publish_and_wait(xv, rb, epoch, s_fail);
      if (owner && ok) {
        f32x4 r4[kXgmiMaxRanks];
#pragma unroll
        for (int r = 0; r < kXgmiMaxRanks; ++r)
          if (r < xv.size) r4[r] = reinterpret_cast<const f32x4*>(xgmi_slot(xv, r, epoch))[p4];
        v = r4[0];
#pragma unroll
        for (int r = 1; r < kXgmiMaxRanks; ++r)
          if (r < xv.size) v += r4[r];
        v *= xscale;
      }
      xgmi_finish(xv, rb, epoch);
    }
    if (owner && ok) {
      if (accumulate) v += g0;
      if (w2t) {
#pragma unroll
        for (int j = 0; j < 4; ++j) grads[pj[j]] = v[j];
      } else {
        reinterpret_cast<f32x4*>(grads)[p4] = v;
      }
      if (hp) {
#pragma unroll
        for (int j = 0; j < 4; ++j) sgd_update(params, lrate, gsc, frag, pj[j], w0[j], v[j]);
      }
    }
  } else {
    const int fb = rb - RED_SLAB_BLOCKS;
    const int j0 = (fb / FC1_IT) * 16, i0 = (fb % FC1_IT) * 16;
    const int lane = tid & 63, wid = tid >> 6, lr = lane & 15, lg = lane >> 4;
    const int Bkp = act_pitch(nwg);  // columns Bk.. are zero
    const int kper = ((Bkp + 8 * 32 - 1) / (8 * 32)) * 32;  // this wave's K slice, a multiple of 32
    const int k0 = wid * kper, k1 = act ? min(Bkp, k0 + kper) : k0;
    const bool jv = j0 + lr < F1;
    float w0[4] = {0.f, 0.f, 0.f, 0.f}, g0[4] = {0.f, 0.f, 0.f, 0.f};  // wave 0's outputs (j0 + 4 lg + r, i0 + lr)
    if (wid == 0 && act) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = j0 + lg * 4 + r;
        if (j < F1) {
          const int p = O_FC1W + j * NIN + i0 + lr;
          if (hp) w0[r] = params[p];
          if (accumulate) g0[r] = grads[p];
        }
      }
    }
    const uint16_t* arow = acts + static_cast<long>(jv ? j0 + lr : 0) * Bkp;
    const uint16_t* brow = acts + static_cast<long>(F1 + i0 + lr) * Bkp;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    constexpr int CH = 4;  // 32-deep chunks per pass: all 2 x CH loads in flight before the first MFMA
    const u16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int kb = k0; kb < k1; kb += 32 * CH) {
      u16x8 a[CH], b[CH];
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int k = kb + 32 * c + 8 * lg;  // 8 whole columns: k and Bkp are multiples of 8
        const bool ok = k < k1;
        a[c] = (ok && jv) ? *reinterpret_cast<const u16x8*>(arow + k) : z8;
        b[c] = ok ? *reinterpret_cast<const u16x8*>(brow + k) : z8;
      }
#pragma unroll
      for (int c = 0; c < CH; c += 2) {
        acc0 = mfma(a[c], b[c], acc0);
        acc1 = mfma(a[c + 1], b[c + 1], acc1);
      }
    }
    f32x4* wpart = part;
    if (act) wpart[wid * 64 + lane] = acc0 + acc1;
    __syncthreads();
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    const int i = i0 + lr;
    if (wid == 0) {
      v = wpart[lane];
#pragma unroll
      for (int w = 1; w < RED_T / 64; ++w) v += wpart[w * 64 + lane];
      v *= gs;
      if (xchg) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = j0 + lg * 4 + r;
          if (j < F1) xmine[O_FC1W + j * NIN + i] = v[r];
        }
      }
    }
    bool ok = true;
    if (xchg) {
      ok = xgmi_publish_and_wait(xv, rb, epoch, s_fail);
      if (wid == 0 && ok) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = j0 + lg * 4 + r;
          const int p = O_FC1W + (j < F1 ? j : 0) * NIN + i;
          float a[kXgmiMaxRanks];
#pragma unroll
          for (int q = 0; q < kXgmiMaxRanks; ++q)
            if (q < xv.size) a[q] = xgmi_slot(xv, q, epoch)[p];
          float g = a[0];
#pragma unroll
          for (int q = 1; q < kXgmiMaxRanks; ++q)
            if (q < xv.size) g += a[q];
          v[r] = g * xscale;
        }
      }
      xgmi_finish(xv, rb, epoch);
    }
    if (wid == 0 && ok) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = j0 + lg * 4 + r;
        if (j < F1) {
          const int p = O_FC1W + j * NIN + i;
          float g = v[r];
          if (accumulate) g += g0[r];
          grads[p] = g;
          if (hp) sgd_update(params, lrate, gsc, frag, p, w0[r], g);
        }
      }
    }
  }
  if (rb == 0 && tid >= RED_T - 64 && tid < RED_T) {  // role 0's last active wave: loss
    const int lane = tid - (RED_T - 64);
    float s = 0.f;
    for (int b = lane; b < nwg; b += 64) s += loss_part[b];
    s = wave_sum(s);
    if (lane == 0) {
      loss[0] = s / static_cast<float>(B);
      rng[0] += 1;  // advance the dropout stream for the next step
      if (hp != nullptr && step != nullptr) step[0] += 1;  // the fused SGD's device step counter
    }
  }
}

__global__ __launch_bounds__(RED_T) void k_cnn_reduce(const float* __restrict__ slabs, int nwg,
                                                      const uint16_t* __restrict__ acts,
                                                      const float* __restrict__ gscale, float* __restrict__ grads,
                                                      int accumulate, const float* __restrict__ loss_part, int B,
                                                      float* __restrict__ loss, unsigned long long* __restrict__ rng,
                                                      float* __restrict__ params, const float* __restrict__ hp,
                                                      uint16_t* __restrict__ frag, int* __restrict__ step,
                                                      XgmiView xv, float xscale, int rb0) {
  __shared__ f32x4 part[RED_LANES * RED_COLS];  // slab: [lane][column]; fc1: [wave][lane] (same 8 KB)
  __shared__ uint32_t s_epoch;
  __shared__ int s_fail;
  cnn_reduce_role(rb0 + blockIdx.x, part, &s_epoch, &s_fail, slabs, nwg, acts, gscale, grads, accumulate, loss_part, B,
                  loss, rng, params, hp, frag, step, xv, xscale);
}

__device__ void cnn_fused_tail(const CnnTail& tl, int rb, f32x4* part, uint32_t* s_epoch, int* s_fail,
                               const float* slabs, int nwg, const uint16_t* acts, const float* loss_part) {
  if (rb >= RED_BLOCKS) return;  // block-uniform: workgroups past the roles are done
  XgmiView one{};
  one.size = 1;
  cnn_reduce_role(rb, part, s_epoch, s_fail, slabs, nwg, acts, tl.gscale, tl.grads, tl.accumulate, loss_part, tl.B,
                  tl.loss, tl.rng, tl.params, tl.hp, tl.frag, tl.step, one, 1.f);
}

}  // namespace

int cnn_num_params() { return NPARAM; }
// PDE_CNN_FUSED_TAIL=1: the single-process reduction inside k_cnn_train (CnnTail).  Off: measured SLOWER
// (r3v: 0.054 vs 0.041 ms/step) -- the grid barrier's agent-scope release / acquire in every workgroup writes
// back and invalidates the L2 of all 8 XCDs 256 times, where the kernel boundary does it once.
bool cnn_fused_tail_enabled() {
  const char* e = std::getenv("PDE_CNN_FUSED_TAIL");
  return e != nullptr && e[0] == '1';
}
int cnn_device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    hipDeviceProp_t prop{};
    cus = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
              ? prop.multiProcessorCount : -1;
  }
  return cus;
}
// The barrier's counter / generation words and error flag: one zeroed allocation per device, made outside any
// graph capture (until then the two-launch form runs).
bool cnn_barrier_words(hipStream_t s, unsigned** bar, int** err) {
  static unsigned* base[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  if (base[dev] == nullptr) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return false;
    void* p = nullptr;
    if (hipMalloc(&p, 64) != hipSuccess) return false;
    if (hipMemset(p, 0, 64) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(p);
      return false;
    }
    base[dev] = static_cast<unsigned*>(p);
  }
  *bar = base[dev];
  *err = reinterpret_cast<int*>(base[dev] + 4);
  return true;
}
int cnn_tail_error(int reset) {
  unsigned* bar = nullptr;
  int* err = nullptr;
  if (!cnn_barrier_words(nullptr, &bar, &err)) return 0;
  int v = 0;
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&v, err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  if (reset && v != 0) (void)hipMemset(err, 0, sizeof(int));
  return v;
}

size_t cnn_frag_bytes() { return sizeof(u16x8) * NFRAG; }
size_t cnn_smem_bytes() { return sizeof(CnnSmem); }
int cnn_images_per_workgroup() { return NI; }

int cnn_slab_floats() { return NSLABP; }  // per workgroup, padded (SLAB_OFS)
int cnn_act_rows() { return NACT; }
int cnn_act_pitch(int nwg) { return act_pitch(nwg); }

hipError_t cnn_train_fused(const float* images, const int64_t* tgt, int B, float* params, void* frag,
                           unsigned long long* rng, float p_drop2, float p_drop1, int training, float* slabs,
                           float* loss_part, uint16_t* acts, int nwg, float* loss, float* grads, const float* gscale,
                           int accumulate, hipStream_t s, unsigned long long* stamps, int prep,
                           const float* sgd_hp, int stop_after, int* sgd_step, const XgmiView* xv,
                           float xscale) {
  if (reinterpret_cast<uintptr_t>(grads) & 15) return hipErrorInvalidValue;  // float4 gradient stores
  XgmiView view{};
  view.size = 1;
  if (xv != nullptr && xv->size > 1) {
    // the exchange replaces the all-reduce of the gradients: no local accumulation in between, one flag
    // row and one staging float per parameter for each of this kernel's workgroups
    if (accumulate || xv->blocks < RED_BLOCKS || xv->slot_bytes < static_cast<int64_t>(NPARAM) * 4)
      return hipErrorInvalidValue;
    view = *xv;
  }
  const size_t sm = sizeof(CnnSmem);
  // PDE_CNN_STORE: store flavour of the slabs / activations (out_st).  Write-through (2) is the default: the
  // 7.5 MB the reduction launch reads no longer sit dirty in the XCD L2s at the kernel boundary (r4k: 0.0408 ->
  // 0.0381 ms/step; non-temporal 0.0390).  PDE_CNN_XMAP=1: XCD-grouped images (r4k: level, off)
  static const int smode = std::getenv("PDE_CNN_STORE") ? std::atoi(std::getenv("PDE_CNN_STORE")) : 2;
  static const int xmap_env = std::getenv("PDE_CNN_XMAP") ? std::atoi(std::getenv("PDE_CNN_XMAP")) : 0;
  static const int diag_frag = (std::getenv("PDE_CNN_DIAG_FRAG") ? 2 : 0) |  // timing only: see k_cnn_train
                               (std::getenv("PDE_CNN_DIAG_P9ST") ? 4 : 0);
  const int xmap = (xmap_env != 0 && nwg % 8 == 0 ? 1 : 0) | diag_frag;
  static const bool breg = std::getenv("PDE_CNN_BREG") != nullptr && std::getenv("PDE_CNN_BREG")[0] == '1';
  using TrainFn = decltype(&k_cnn_train<0, false>);
  static const TrainFn kTrain[2][4] = {
      {&k_cnn_train<0, false>, &k_cnn_train<1, false>, &k_cnn_train<2, false>, &k_cnn_train<3, false>},
      {&k_cnn_train<0, true>, &k_cnn_train<1, true>, &k_cnn_train<2, true>, &k_cnn_train<3, true>}};
  const int si = smode >= 0 && smode <= 3 ? smode : 0;
  const TrainFn train = kTrain[breg ? 1 : 0][si];
  static bool attr[2][4] = {};
  if (!attr[breg ? 1 : 0][si]) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(train), hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(sm));
    attr[breg ? 1 : 0][si] = true;
  }
  if (reinterpret_cast<uintptr_t>(frag) & 15) return hipErrorInvalidValue;
  if (prep)
    hipLaunchKernelGGL(k_cnn_prep, dim3(ceil_div(NFRAG, 256)), dim3(256), 0, s, params, static_cast<u16x8*>(frag));
  if (reinterpret_cast<uintptr_t>(acts) & 15) return hipErrorInvalidValue;
  CnnTail tail{};
  unsigned* bar = nullptr;
  int* berr = nullptr;
  if (view.size == 1 && stamps == nullptr && stop_after < 0 && cnn_fused_tail_enabled() && nwg >= RED_BLOCKS &&
      nwg <= cnn_device_cus() && cnn_barrier_words(s, &bar, &berr)) {
    tail.gscale = gscale; tail.grads = grads; tail.loss = loss; tail.rng = rng; tail.params = params;
    tail.hp = sgd_hp; tail.frag = static_cast<uint16_t*>(frag); tail.step = sgd_step; tail.bar = bar;
    tail.err = berr; tail.accumulate = accumulate; tail.B = B; tail.on = 1;
  }
  // PDE_CNN_DIAG (timing diagnostics only, results invalid): 1 no reduce launch, 2 no train launch, 4 reduce
  // slab-column roles only, 8 reduce fc1-tile roles only, 16 no SGD update / fragment refresh in the reduce
  static const int diag = std::getenv("PDE_CNN_DIAG") ? std::atoi(std::getenv("PDE_CNN_DIAG")) : 0;
  if (!(diag & 2))
    hipLaunchKernelGGL(train, dim3(nwg), dim3(T), sm, s, images, tgt, B, params,
                       static_cast<const u16x8*>(frag), rng, p_drop2, p_drop1, training, slabs, loss_part, acts,
                       stamps, stop_after, tail, xmap);
  if (!tail.on && !(diag & 1)) {
    const int rb0 = (diag & 8) ? RED_SLAB_BLOCKS : 0;
    const int nrb = (diag & 4) ? RED_SLAB_BLOCKS : (diag & 8) ? RED_BLOCKS - RED_SLAB_BLOCKS : RED_BLOCKS;
    hipLaunchKernelGGL(k_cnn_reduce, dim3(nrb), dim3(RED_T), 0, s, slabs, nwg, acts, gscale, grads,
                       accumulate, loss_part, B, loss, rng, params, (diag & 16) ? nullptr : sgd_hp,
                       static_cast<uint16_t*>(frag), sgd_step, view, xscale, rb0);
  }
  return hipGetLastError();
}

hipError_t cnn_sgd_fused(float* params, const float* grads, const float* hp, void* frag, hipStream_t s, int* step) {
  if (reinterpret_cast<uintptr_t>(frag) & 15) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_cnn_sgd, dim3(ceil_div(NPARAM, 256)), dim3(256), 0, s, params, grads, hp,
                     static_cast<uint16_t*>(frag), step);
  return hipGetLastError();
}

// AdamW (torch.optim.AdamW: the Horovod-elastic script's optimiser, horovod_mnist_elastic.py:41) on the flat
// parameters, its exp_avg / exp_avg_sq as flat buffers, with the fragment image refreshed in the same pass -- the
// multi-tensor update launch and the next step's fragment prep launch become ONE launch.  hp / step: the fused
// optimiser's device hyper-parameters and {steps taken, arrival counter}, read and advanced exactly as its own
// update kernel does (optim_device.h run_chunks), so its state_dict and later steps stay consistent.
__global__ __launch_bounds__(256) void k_cnn_adamw(float* __restrict__ params, const float* __restrict__ grads,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   const float* __restrict__ hp, int* __restrict__ step,
                                                   uint16_t* __restrict__ frag) {
  __shared__ int s_step;
  if (threadIdx.x == 0) s_step = step[0] + 1;
  __syncthreads();
  optdev::Hyper h;
  h.lr = hp[HP_LR]; h.b1 = hp[HP_BETA1]; h.b2 = hp[HP_BETA2]; h.eps = hp[HP_EPS];
  h.wd = hp[HP_WD]; h.mom = hp[HP_MOMENTUM]; h.gscale = hp[HP_GRAD_SCALE];
  h.step = s_step;
  const float bc1 = 1.f - __powf(h.b1, static_cast<float>(h.step));
  const float bc2 = 1.f - __powf(h.b2, static_cast<float>(h.step));
  h.step_size = h.lr / bc1;
  h.inv_sqrt_bc2 = rsqrtf(bc2);
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p < NPARAM) {
    float w = params[p], mm = m[p], vv = v[p];
    optdev::update<2>(h, w, grads[p], mm, vv);
    params[p] = w;
    m[p] = mm;
    v[p] = vv;
    write_frag(frag, p, w);
  }
  __syncthreads();  // (every block read the old count before its arrival: the last one publishes)
  if (threadIdx.x == 0) {
    const int prev = atomicAdd(step + 1, 1);
    if (prev == static_cast<int>(gridDim.x) - 1) {
      step[0] = s_step;
      step[1] = 0;
    }
  }
}

hipError_t cnn_adamw_fused(float* params, const float* grads, float* m, float* v, const float* hp, void* frag,
                           int* step, hipStream_t s) {
  hipLaunchKernelGGL(k_cnn_adamw, dim3(ceil_div(NPARAM, 256)), dim3(256), 0, s, params, grads, m, v, hp, step,
                     static_cast<uint16_t*>(frag));
  return hipGetLastError();
}

}  // namespace pde
