// Fused MNIST-CNN training step for gfx950: the whole of horovod/mnist_horovod.py:9-25's `Net`
// (conv5x5 1->10, maxpool2, ReLU, conv5x5 10->20, Dropout2d, maxpool2, ReLU, fc 320->50, ReLU,
// dropout, fc 50->10, log_softmax) + NLL loss + the complete backward pass, with every activation
// resident in LDS.
//
// Why: the network is 21,840 parameters and ~1 MFLOP/image forward; at the reference batch (1024 per
// worker) the layer-by-layer path is ~40 kernels of a few microseconds each, every one far below the
// chip's roofline.  Here ONE workgroup (8 wave64s) trains NI=4 images end to end,
// the 4 images side by side in every phase so each phase has 4x the independent work (ILP/TLP for a
// latency-bound, LDS-resident pipeline):
//   * conv1/conv2/fc2 weights are staged in LDS once per workgroup; fc1's 64 KB weight matrix is read
//     from L2 (shared by all workgroups), each load feeding all 4 images;
//   * pooling is computed from the conv outputs in registers (4 conv taps per pooled cell, the argmax
//     tap kept as a byte), so no pre-pool activation is ever stored;
//   * backward exploits the pooling sparsity: only the argmax tap of each pooled cell carries gradient,
//     so conv2-wgrad, conv2-dgrad and conv1-wgrad do 1/4 of the dense work;
//   * since the 4 images are processed together, every weight gradient is complete after its phase and
//     is written straight to the workgroup's fp32 slab (no accumulators to carry); k_cnn_reduce sums the slabs in a fixed order (deterministic) straight into the flat gradient
//     buffer (e.g. the DDP bucket).
// Dropout masks come from a counter-based hash keyed by a device-resident counter that k_cnn_loss
// advances, so hipGraph replays draw fresh masks.  All math is fp32.
#include "common.cuh"
#include "pde_kernels.h"

namespace pde {

namespace {

constexpr int T = 512;   // 8 waves
constexpr int NI = 4;    // images per workgroup, processed side by side
constexpr int C1 = 10, C2 = 20, KS = 5, H0 = 28, P1 = 12, P2 = 4, F1 = 50, F2 = 10;
constexpr int NX = H0 * H0, NR1 = C1 * P1 * P1, NIN = C2 * P2 * P2;  // 784, 1440, 320
constexpr int W1N = C1 * KS * KS, W2N = C2 * C1 * KS * KS, FC1N = F1 * NIN, FC2N = F2 * F1;
// parameter offsets in the flat gradient (torch parameter order of Net)
constexpr int O_W1 = 0, O_B1 = O_W1 + W1N, O_W2 = O_B1 + C1, O_B2 = O_W2 + W2N, O_FC1W = O_B2 + C2,
              O_FC1B = O_FC1W + FC1N, O_FC2W = O_FC1B + F1, O_FC2B = O_FC2W + FC2N, NPARAM = O_FC2B + F2;

__device__ __forceinline__ float hash_u01(unsigned long long seed, unsigned long long id) {
  unsigned long long z = seed + 0x9E3779B97F4A7C15ULL * (id + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return static_cast<float>(z >> 40) * (1.0f / 16777216.0f);
}

struct CnnSmem {
  float x[NI][NX];
  float w1[W1N], b1[C1], w2[W2N], b2[C2];   // contiguous: staged with one loop
  float fc2w[FC2N], fc2b[F2];
  float r1[NI][NR1];     // relu(maxpool(conv1))
  float dr1[NI][NR1];    // grad wrt r1 -> grad at the argmax tap of conv1
  float r2[NI][NIN];     // relu(maxpool(dropout2d(conv2))) == fc1 input (NCHW flatten order)
  alignas(16) float dp2[NI][NIN];    // grad at the argmax tap of conv2 (16-B rows: f32x4 loads)
  float h1[NI][F1], m1[NI][F1], h1d[NI][F1], dh[NI][F1];
  float mc2[NI][C2];
  float logit[NI][F2], dlog[NI][F2];
  float valid[NI];
  float gw1[W1N], gb1[C1];   // conv1 gradients (LDS atomics across the 4 images)
  unsigned char a1[NI][NR1];
  alignas(16) unsigned char a2[NI][NIN];
};

__global__ __launch_bounds__(T) void k_cnn_train(const float* __restrict__ images, const int64_t* __restrict__ tgt,
                                                 int B, const float* __restrict__ params,
                                                 const unsigned long long* __restrict__ rng, float p_drop2,
                                                 float p_drop1, int training, float* __restrict__ slabs,
                                                 float* __restrict__ loss_part,
                                                 unsigned long long* __restrict__ stamps) {
  // optional phase timestamps (diagnostic only: stamps == nullptr in production launches)
#define PDE_STAMP(k) \
  if (stamps != nullptr && threadIdx.x == 0) stamps[blockIdx.x * 16 + (k)] = wall_clock64()
  PDE_STAMP(0);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  CnnSmem& S = *reinterpret_cast<CnnSmem*>(smem_raw);
  const int t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  const float* gFC1W = params + O_FC1W;
  const float* gFC1B = params + O_FC1B;
  const int n0 = blockIdx.x * NI;

  // ---- P0: stage weights, zero accumulators, load the images and dropout masks --------------------
  for (int i = t; i < W1N + C1 + W2N + C2; i += T) (&S.w1[0])[i] = params[O_W1 + i];
  for (int i = t; i < FC2N + F2; i += T) (&S.fc2w[0])[i] = params[O_FC2W + i];
  for (int i = t; i < W1N + C1; i += T) (&S.gw1[0])[i] = 0.f;
  float* slab = slabs + static_cast<long>(blockIdx.x) * NPARAM;
  const unsigned long long seed = rng[0] * 0xD1B54A32D192ED03ULL;
  const float keep2 = training ? 1.f / (1.f - p_drop2) : 1.f;
  const float keep1 = training ? 1.f / (1.f - p_drop1) : 1.f;
  for (int i = t; i < NI * NX; i += T) {
    const int im = i / NX, n = n0 + im;
    S.x[im][i - im * NX] = n < B ? images[static_cast<long>(n) * NX + (i - im * NX)] : 0.f;
  }
  if (t < NI * C2) {
    const int im = t / C2, c = t - im * C2;
    const unsigned long long id = static_cast<unsigned long long>(n0 + im) * C2 + c;
    S.mc2[im][c] = (!training || hash_u01(seed ^ 0x5bd1e995ULL, id) >= p_drop2) ? keep2 : 0.f;
  } else if (t >= 128 && t < 128 + NI * F1) {
    const int u = t - 128, im = u / F1, j = u - im * F1;
    const unsigned long long id = static_cast<unsigned long long>(n0 + im) * F1 + j;
    S.m1[im][j] = (!training || hash_u01(seed ^ 0x27d4eb2fULL, id) >= p_drop1) ? keep1 : 0.f;
  } else if (t >= 384 && t < 384 + NI) {
    S.valid[t - 384] = (n0 + t - 384) < B ? 1.f : 0.f;
  }
  __syncthreads();
  PDE_STAMP(1);

  // ---- P1: conv1 + maxpool2 + relu: one pooled cell (4 conv taps) per item ----------------------
  for (int it = t; it < NI * NR1; it += T) {
    const int im = it / NR1, p = it - im * NR1;
    const int co = p / (P1 * P1), rem = p - co * P1 * P1, py = rem / P1, px = rem - py * P1;
    const float* xi = S.x[im] + (2 * py) * H0 + 2 * px;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
#pragma unroll
    for (int ky = 0; ky < KS; ++ky) {
      float row0[6], row1[6];
#pragma unroll
      for (int xx = 0; xx < 6; ++xx) { row0[xx] = xi[ky * H0 + xx]; row1[xx] = xi[(ky + 1) * H0 + xx]; }
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        const float w = S.w1[co * 25 + ky * 5 + kx];
        acc0 += w * row0[kx];
        acc1 += w * row0[kx + 1];
        acc2 += w * row1[kx];
        acc3 += w * row1[kx + 1];
      }
    }
    int am = 0;
    float m = acc0;
    if (acc1 > m) { m = acc1; am = 1; }
    if (acc2 > m) { m = acc2; am = 2; }
    if (acc3 > m) { m = acc3; am = 3; }
    S.r1[im][p] = fmaxf(m + S.b1[co], 0.f);
    S.a1[im][p] = static_cast<unsigned char>(am);
  }
  __syncthreads();
  PDE_STAMP(2);

  // ---- P2: conv2 + dropout2d + maxpool2 + relu -------------------------------------------------
  for (int it = t; it < NI * NIN; it += T) {
    const int im = it / NIN, q = it - im * NIN;
    const int co = q / (P2 * P2), rem = q - co * P2 * P2, py = rem / P2, px = rem - py * P2;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
    for (int ci = 0; ci < C1; ++ci) {
      const float* r = S.r1[im] + ci * P1 * P1 + (2 * py) * P1 + 2 * px;
      const float* w = S.w2 + (co * C1 + ci) * 25;
#pragma unroll
      for (int ky = 0; ky < KS; ++ky) {
        float row0[6], row1[6];
#pragma unroll
        for (int xx = 0; xx < 6; ++xx) { row0[xx] = r[ky * P1 + xx]; row1[xx] = r[(ky + 1) * P1 + xx]; }
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) {
          const float wv = w[ky * 5 + kx];
          acc0 += wv * row0[kx];
          acc1 += wv * row0[kx + 1];
          acc2 += wv * row1[kx];
          acc3 += wv * row1[kx + 1];
        }
      }
    }
    int am = 0;
    float m = acc0;
    if (acc1 > m) { m = acc1; am = 1; }
    if (acc2 > m) { m = acc2; am = 2; }
    if (acc3 > m) { m = acc3; am = 3; }
    S.r2[im][q] = fmaxf((m + S.b2[co]) * S.mc2[im][co], 0.f);
    S.a2[im][q] = static_cast<unsigned char>(am);
  }
  __syncthreads();
  PDE_STAMP(3);

  // ---- P3: fc1 + relu + dropout: wave per output row, lanes over inputs, 4 images per load ------
  for (int j = wid; j < F1; j += T / 64) {
    const float* wr = gFC1W + j * NIN;
    float s[NI] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NIN / 64; ++k) {
      const int i = lane + k * 64;
      const float w = wr[i];
#pragma unroll
      for (int im = 0; im < NI; ++im) s[im] += w * S.r2[im][i];
    }
#pragma unroll
    for (int im = 0; im < NI; ++im) s[im] = wave_sum(s[im]);
    if (lane < NI) {
      const float h = fmaxf(s[lane] + gFC1B[j], 0.f);
      S.h1[lane][j] = h;
      S.h1d[lane][j] = h * S.m1[lane][j];
    }
  }
  __syncthreads();
  PDE_STAMP(4);

  // ---- P4: fc2 logits, then log_softmax + NLL + dlogits per image ---------------------------------
  if (t < NI * F2) {
    const int im = t / F2, v = t - im * F2;
    float s = S.fc2b[v];
#pragma unroll 10
    for (int j = 0; j < F1; ++j) s += S.fc2w[v * F1 + j] * S.h1d[im][j];
    S.logit[im][v] = s;
  }
  __syncthreads();
  PDE_STAMP(5);
  float loss_acc = 0.f;
  if (t < NI) {
    const int im = t;
    float m = S.logit[im][0];
    for (int v = 1; v < F2; ++v) m = fmaxf(m, S.logit[im][v]);
    float se = 0.f;
    for (int v = 0; v < F2; ++v) se += __expf(S.logit[im][v] - m);
    const float lse = m + __logf(se);
    const float val = S.valid[im];
    const int y = val > 0.f ? static_cast<int>(tgt[n0 + im]) : 0;
    loss_acc = val * (lse - S.logit[im][y]);
    const float inv_b = val / static_cast<float>(B);
    for (int v = 0; v < F2; ++v) S.dlog[im][v] = (__expf(S.logit[im][v] - lse) - (v == y ? 1.f : 0.f)) * inv_b;
  }
  __syncthreads();
  PDE_STAMP(6);

  // ---- P5: fc2 backward; dh = relu'(h1) * mask * (W2^T dlog) ------------------------------------
  for (int i = t; i < FC2N; i += T) {
    const int v = i / F1, j = i - v * F1;
    float s = 0.f;
#pragma unroll
    for (int im = 0; im < NI; ++im) s += S.dlog[im][v] * S.h1d[im][j];
    slab[O_FC2W + i] = s;
  }
  if (t < F2) {
    float s = 0.f;
#pragma unroll
    for (int im = 0; im < NI; ++im) s += S.dlog[im][t];
    slab[O_FC2B + t] = s;
  }
  if (t >= 256 && t < 256 + NI * F1) {
    const int u = t - 256, im = u / F1, j = u - im * F1;
    float s = 0.f;
#pragma unroll
    for (int v = 0; v < F2; ++v) s += S.fc2w[v * F1 + j] * S.dlog[im][v];
    S.dh[im][j] = (S.h1[im][j] > 0.f) ? s * S.m1[im][j] : 0.f;
  }
  __syncthreads();
  PDE_STAMP(7);

  // ---- P6: fc1 backward: dW, db (straight to the slab), dr2 -> grad at conv2's argmax tap ---------
  for (int idx = t; idx < FC1N; idx += T) {
    const int j = idx / NIN, i = idx - j * NIN;
    float s = 0.f;
#pragma unroll
    for (int im = 0; im < NI; ++im) s += S.dh[im][j] * S.r2[im][i];
    slab[O_FC1W + idx] = s;
  }
  if (t < F1) {
    float s = 0.f;
#pragma unroll
    for (int im = 0; im < NI; ++im) s += S.dh[im][t];
    slab[O_FC1B + t] = s;
  }
  if (t < NIN) {
    const int i = t, co = i / (P2 * P2);
    float s[NI] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 10
    for (int j = 0; j < F1; ++j) {
      const float w = gFC1W[j * NIN + i];
#pragma unroll
      for (int im = 0; im < NI; ++im) s[im] += w * S.dh[im][j];
    }
#pragma unroll
    for (int im = 0; im < NI; ++im) S.dp2[im][i] = (S.r2[im][i] > 0.f) ? s[im] * S.mc2[im][co] : 0.f;
  }
  __syncthreads();
  PDE_STAMP(8);

  // ---- P7a: conv2 wgrad (sparse: one tap per pooled cell).  Item = (co, ci, ky) computing the 5 kx
  // taps together: each (cell, image) costs 2 index loads + one 5-wide r1 row segment.
  for (int it = t; it < C2 * C1 * KS; it += T) {
    const int co = it / (C1 * KS), rem = it - co * C1 * KS, ci = rem / KS, ky = rem - ci * KS;
    float s[KS] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int im = 0; im < NI; ++im) {
      const float* r = S.r1[im] + ci * P1 * P1 + ky * P1;
#pragma unroll 4
      for (int c = 0; c < P2 * P2; ++c) {
        const int q = co * 16 + c, py = c >> 2, px = c & 3;
        const float g = S.dp2[im][q];
        const int a = S.a2[im][q];
        const float* rr = r + (2 * py + (a >> 1)) * P1 + 2 * px + (a & 1);
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) s[kx] += g * rr[kx];
      }
    }
    float* dst = slab + O_W2 + (co * C1 + ci) * 25 + ky * 5;
#pragma unroll
    for (int kx = 0; kx < KS; ++kx) dst[kx] = s[kx];
  }
  if (t >= 448 && t < 448 + C2) {
    const int co = t - 448;
    float s = 0.f;
    for (int im = 0; im < NI; ++im)
      for (int c = 0; c < 16; ++c) s += S.dp2[im][co * 16 + c];
    slab[O_B2 + co] = s;
  }
  PDE_STAMP(9);
  // ---- P7b: conv2 dgrad as a row gather (no atomics, deterministic) + relu'(r1).  Item = one row y of
  // one (image, ci) plane; the 12 outputs stay in registers.  Only cells whose argmax tap row lies in
  // [y-4, y] can reach row y: py in [(y-4)/2, y/2].  (A 4-lanes-per-row split with shuffle reduction
  // measured slower: 46 vs 37 us per workgroup -- LDS weight-read conflicts across co.)
  for (int it = t; it < NI * C1 * P1; it += T) {
    const int im = it / (C1 * P1), rem = it - im * C1 * P1, ci = rem / P1, y = rem - ci * P1;
    float s[P1];
#pragma unroll
    for (int xx = 0; xx < P1; ++xx) s[xx] = 0.f;
    const int py_lo = max(0, (y - 4) >> 1), py_hi = min(P2 - 1, y >> 1);
    for (int co = 0; co < C2; ++co) {
      const float* w = S.w2 + (co * C1 + ci) * 25;
      for (int py = py_lo; py <= py_hi; ++py) {
#pragma unroll
        for (int px = 0; px < P2; ++px) {
          const int q = co * 16 + py * 4 + px;
          const float g = S.dp2[im][q];
          const int a = S.a2[im][q];
          const int ky = y - (2 * py + (a >> 1));
          if (ky >= 0 && ky < KS && g != 0.f) {
            const float* wr = w + ky * 5;
            if (a & 1) {
#pragma unroll
              for (int kx = 0; kx < KS; ++kx) s[2 * px + 1 + kx] += g * wr[kx];
            } else {
#pragma unroll
              for (int kx = 0; kx < KS; ++kx) s[2 * px + kx] += g * wr[kx];
            }
          }
        }
      }
    }
    const float* r1 = S.r1[im] + ci * P1 * P1 + y * P1;
    float* d = S.dr1[im] + ci * P1 * P1 + y * P1;
#pragma unroll
    for (int xx = 0; xx < P1; ++xx) d[xx] = r1[xx] > 0.f ? s[xx] : 0.f;
  }
  __syncthreads();
  PDE_STAMP(10);

  // ---- P9: conv1 wgrad at the argmax taps.  Item = (co, ky, image, half of the cells) computing the 5
  // kx taps together; combined with LDS atomics (400 items x 5 adds).  Bias grad alongside.
  for (int it = t; it < C1 * KS * NI * 2; it += T) {
    const int co = it / (KS * NI * 2), rem = it - co * KS * NI * 2, ky = rem / (NI * 2), r2_ = rem - ky * NI * 2;
    const int im = r2_ >> 1, half = r2_ & 1;
    const float* g = S.dr1[im] + co * 144;
    const unsigned char* am = S.a1[im] + co * 144;
    const float* xi = S.x[im] + ky * H0;
    float s[KS] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int c = half * 72; c < half * 72 + 72; ++c) {
      const float gv = g[c];
      const int py = c / P1, px = c - py * P1, a = am[c];
      const float* xr = xi + (2 * py + (a >> 1)) * H0 + 2 * px + (a & 1);
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) s[kx] += gv * xr[kx];
    }
#pragma unroll
    for (int kx = 0; kx < KS; ++kx) atomicAdd(&S.gw1[co * 25 + ky * 5 + kx], s[kx]);
  }
  if (t >= 448 && t < 448 + NI * C1) {
    const int u = t - 448, im = u / C1, co = u - im * C1;
    float s = 0.f;
    for (int c = 0; c < 144; ++c) s += S.dr1[im][co * 144 + c];
    atomicAdd(&S.gb1[co], s);
  }
  __syncthreads();
  PDE_STAMP(11);

  // ---- conv1 gradients to the slab; loss partial -----------------------------------------------------
  for (int i = t; i < W1N + C1; i += T) slab[O_W1 + i] = (&S.gw1[0])[i];
  // loss: threads 0..NI-1 of wave 0 hold it
  if (wid == 0) {
    const float l = wave_sum(loss_acc);
    if (lane == 0) loss_part[blockIdx.x] = l;
  }
}

// grads[i] (+)= gscale * sum_wg slabs[wg][i].  4 waves split the slabs, fixed order, LDS combine.
__global__ __launch_bounds__(256) void k_cnn_reduce(const float* __restrict__ slabs, int nwg, const float* __restrict__ gscale,
                                                    float* __restrict__ grads, int accumulate) {
  __shared__ float part[4][64];
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  float s0 = 0.f, s1 = 0.f;
  if (i < NPARAM) {
    int b = w;
    for (; b + 4 < nwg; b += 8) {
      s0 += slabs[static_cast<long>(b) * NPARAM + i];
      s1 += slabs[static_cast<long>(b + 4) * NPARAM + i];
    }
    if (b < nwg) s0 += slabs[static_cast<long>(b) * NPARAM + i];
  }
  part[w][threadIdx.x & 63] = s0 + s1;
  __syncthreads();
  if (w == 0 && i < NPARAM) {
    const float v = (part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x]) *
                    (gscale ? gscale[0] : 1.f);
    grads[i] = accumulate ? grads[i] + v : v;
  }
}

__global__ void k_cnn_loss(const float* __restrict__ part, int nwg, int B, float* __restrict__ loss,
                           unsigned long long* __restrict__ rng) {
  float s = 0.f;
  for (int b = threadIdx.x; b < nwg; b += 64) s += part[b];
  s = wave_sum(s);
  if (threadIdx.x == 0) {
    loss[0] = s / static_cast<float>(B);
    rng[0] += 1;  // advance the dropout stream for the next step
  }
}

}  // namespace

int cnn_num_params() { return NPARAM; }
size_t cnn_smem_bytes() { return sizeof(CnnSmem); }
int cnn_images_per_workgroup() { return NI; }

hipError_t cnn_train_fused(const float* images, const int64_t* tgt, int B, const float* params,
                           unsigned long long* rng, float p_drop2, float p_drop1, int training, float* slabs,
                           float* loss_part, int nwg, float* loss, hipStream_t s,
                           unsigned long long* stamps) {
  const size_t sm = sizeof(CnnSmem);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_cnn_train), hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(sm));
    attr = true;
  }
  hipLaunchKernelGGL(k_cnn_train, dim3(nwg), dim3(T), sm, s, images, tgt, B, params, rng, p_drop2, p_drop1, training,
                     slabs, loss_part, stamps);
  hipLaunchKernelGGL(k_cnn_loss, dim3(1), dim3(64), 0, s, loss_part, nwg, B, loss, rng);
  return hipGetLastError();
}

hipError_t cnn_reduce_grads(const float* slabs, int nwg, const float* gscale, float* grads, int accumulate,
                            hipStream_t s) {
  hipLaunchKernelGGL(k_cnn_reduce, dim3(ceil_div(NPARAM, 64)), dim3(256), 0, s, slabs, nwg, gscale, grads,
                     accumulate);
  return hipGetLastError();
}

}  // namespace pde
