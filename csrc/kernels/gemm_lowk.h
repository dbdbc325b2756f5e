// Low-K GEMM: C[M, N] = epi(A[M, K] . B[N, K]^T) for K <= 128 with dense K-contiguous operands -- the 1x1
// convolutions at the ResNet stage entries (b32: 32768x256x64, 8192x512x128, 32768x64x64), where the tile core's
// 64x64 blocks do 2-4 K-steps each and the launch is a chain of load -> 2 MFMAs -> epilogue round trips
// (12.8 us for 20 MB: 1.6 TB/s, r6_resnet50_gemm_shapes.md).  Here the problem is streamed instead:
//   * a block owns one BN-wide column strip of C: its B strip (BN x K bf16, <= 32 KB) is read from global memory
//     ONCE into LDS and every wave keeps its MFMA B fragments of it in registers for every row tile;
//   * the block walks row tiles of BM = 128 (4 waves x 32 rows) grid-strided; a wave loads its A fragments
//     straight from global memory (16 B per lane, no LDS), and the NEXT tile's fragments are requested before the
//     current tile's MFMAs and stores, so a tile's A read and the previous tile's C write are in flight together;
//   * the MFMAs run transposed (D^T = B . A^T): a lane then holds 4 consecutive columns of one output row, which
//     are staged (8-byte LDS writes, epilogue applied) in the wave's own LDS rows and leave as 16-byte row chunks;
//     waves never wait for each other (no block barrier).
// The kernel is bandwidth-shaped: per 128-row tile it reads 128 K bf16 and writes 128 BN bf16, with ~1 us of MFMA
// work per CU against several us of HBM traffic.
#pragma once

#include "gemm_common.h"

namespace pde {

namespace {

constexpr int kLowkBM = 128;   // rows per tile: 4 waves x 32
constexpr int kLowkFM = 2;     // 16-row fragments per wave
template <int BN>
constexpr int kLowkPitch() { return BN + 8; }  // staging row pitch (elements): 16 B of padding per row

template <int KT, int FN>
__global__ __launch_bounds__(kThreads) void gemm_lowk_kernel(GemmArgs args, int tm, int tn) {
  constexpr int BN = 16 * FN;
  __shared__ __attribute__((aligned(16))) uint16_t stage[4][32 * kLowkPitch<BN>()];  // per-wave output staging
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int K = args.K, M = args.M, N = args.N;
  const int nt = blockIdx.x % tn;  // host: gridDim.x % tn == 0, so a block keeps its column strip
  const int n0 = nt * BN;
  const auto ra = operand_rsrc(args.a, 0, M, K, true);
  const auto rb = operand_rsrc(args.b, 0, N, K, true);
  const int kq = 8 * (lane >> 4), lr = lane & 15;
  // B strip -> LDS once per block (16-byte chunks, rows padded by 16 B), then every wave takes its B fragments
  // from there into registers, kept for every row tile: lane (lr, kq) holds B[n0 + 16 j + lr][32 ks + kq .. +7].
  // (Each wave loading its fragments from global memory made B -- 4 copies per block -- the bulk of the
  // launch's L2 traffic: 32 MB against 20 MB of A and C for 32768x256x64.)
  constexpr int KP = 32 * KT + 8;  // LDS row pitch (elements)
  __shared__ __attribute__((aligned(16))) uint16_t bimg[BN * KP];
  for (int q = threadIdx.x; q < BN * KT * 4; q += kThreads) {
    const int row = q / (KT * 4), c = q % (KT * 4), n = n0 + row, k = 8 * c;
    *reinterpret_cast<u16x8*>(bimg + row * KP + k) = bload16(rb, n < N && k < K, static_cast<long>(n) * args.b.ld_r + k);
  }
  __syncthreads();
  bf16x8 bfr[KT][FN];
#pragma unroll
  for (int ks = 0; ks < KT; ++ks)
#pragma unroll
    for (int j = 0; j < FN; ++j)
      bfr[ks][j] = *reinterpret_cast<const bf16x8*>(bimg + (16 * j + lr) * KP + 32 * ks + kq);
  const int mstep = gridDim.x / tn;
  int mt = blockIdx.x / tn;
  u16x8 an[KT][kLowkFM];
  auto load_a = [&](int t, u16x8 (&dst)[KT][kLowkFM]) {
#pragma unroll
    for (int ks = 0; ks < KT; ++ks)
#pragma unroll
      for (int i = 0; i < kLowkFM; ++i) {
        const int m = t * kLowkBM + 32 * w + 16 * i + lr, k = 32 * ks + kq;
        dst[ks][i] = bload16(ra, m < M && k < K, static_cast<long>(m) * args.a.ld_r + k);
      }
  };
  if (mt < tm) load_a(mt, an);
  const int epi = args.epi;
  uint16_t* out = static_cast<uint16_t*>(args.out);
  for (; mt < tm; mt += mstep) {  // trip count uniform per block
    u16x8 ac[KT][kLowkFM];
#pragma unroll
    for (int ks = 0; ks < KT; ++ks)
#pragma unroll
      for (int i = 0; i < kLowkFM; ++i) ac[ks][i] = an[ks][i];
    if (mt + mstep < tm) load_a(mt + mstep, an);  // next tile in flight under this one's MFMAs and stores
    f32x4 acc[kLowkFM][FN];
#pragma unroll
    for (int i = 0; i < kLowkFM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KT; ++ks)
#pragma unroll
      for (int i = 0; i < kLowkFM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)  // D^T tile: lane holds column m = lr, rows n = 4 (lane >> 4) + r
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[ks][j], __builtin_bit_cast(bf16x8, ac[ks][i]),
                                                              acc[i][j], 0, 0, 0);
    // epilogue: the wave's 32 x BN bf16 tile staged in its own LDS rows (8-byte writes: a lane's 4 consecutive
    // columns), then written back as 16-byte row chunks -- 8 lanes cover one 128-byte line
    uint16_t* st = &stage[w][0];
#pragma unroll
    for (int i = 0; i < kLowkFM; ++i) {
      const int ml = 16 * i + lr, m = mt * kLowkBM + 32 * w + ml;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int nl = 16 * j + 4 * (lane >> 4);
        u16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          o[r] = f2bf(epi ? apply_epi(acc[i][j][r], epi, m, n0 + nl + r, args) : acc[i][j][r]);
        *reinterpret_cast<u16x4*>(st + ml * kLowkPitch<BN>() + nl) = o;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    constexpr int CPR = BN / 8;  // 16-byte chunks per row
#pragma unroll
    for (int q = lane; q < 32 * CPR; q += 64) {
      const int ml = q / CPR, c = q % CPR;
      const int m = mt * kLowkBM + 32 * w + ml, n = n0 + 8 * c;
      const u16x8 v = *reinterpret_cast<const u16x8*>(st + ml * kLowkPitch<BN>() + 8 * c);
      if (m < M && n < N) {
        if (n + 8 <= N) {
          *reinterpret_cast<u16x8*>(out + static_cast<long>(m) * args.ldo + n) = v;
        } else {  // N % 4 == 0: a last half chunk
          *reinterpret_cast<u16x4*>(out + static_cast<long>(m) * args.ldo + n) = u16x4{v[0], v[1], v[2], v[3]};
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  }
}

}  // namespace

}  // namespace pde
