// dgrad + wgrad pairs on the LDS-DMA core (gemm_dma_pair_kernel, gemm_dma.h): the combinations that occur --
// data gradients: dgrad gather / dense dy x {dgrad-layout weights, forward copy read transposed}; weight gradients:
// dy^T x {im2col^T gather, dense activation}.
#include "gemm_dma.h"

namespace pde {

namespace {

template <int S, bool AKC1, bool BKC1, int AK1, int BK1>
bool pair_k0(int k0, dim3 grid, hipStream_t s, const GemmArgs& a0, const GemmArgs& a1, const PairDims& d,
             const OptimSeg& seg) {
  switch (k0) {
#define PDE_DPAIR(AKC0, BKC0, AK0, BK0)                                                                          \
  case kind_code(AKC0, BKC0, AK0, BK0):                                                                          \
    hipLaunchKernelGGL((gemm_dma_pair_kernel<S, AKC0, BKC0, AK0, BK0, AKC1, BKC1, AK1, BK1>), grid, dim3(kThreads), 0, \
                       s, a0, a1, d, seg);                                                                       \
    return true;
    PDE_DPAIR(true, true, 3, 0)
    PDE_DPAIR(true, true, 0, 0)
    PDE_DPAIR(true, false, 0, 0)
    PDE_DPAIR(true, false, 3, 0)
#undef PDE_DPAIR
    default: return false;
  }
}

}  // namespace

template <int S>
bool pair_k1(int k0, int k1, dim3 grid, hipStream_t s, const GemmArgs& a0, const GemmArgs& a1, const PairDims& d,
             const OptimSeg& seg) {
  switch (k1) {
    case kind_code(false, false, 0, 2): return pair_k0<S, false, false, 0, 2>(k0, grid, s, a0, a1, d, seg);
    case kind_code(false, false, 0, 0): return pair_k0<S, false, false, 0, 0>(k0, grid, s, a0, a1, d, seg);
    default: return false;
  }
}

bool dma_launch_pair(int s, int k0, int k1, dim3 grid, hipStream_t st, const GemmArgs& a0, const GemmArgs& a1,
                     const PairDims& d, const OptimSeg& seg) {
  return s >= 6 ? pair_k1<6>(k0, k1, grid, st, a0, a1, d, seg) : pair_k1<3>(k0, k1, grid, st, a0, a1, d, seg);
}

}  // namespace pde
