// LDS-DMA GEMM kernels with K-contiguous A and row-contiguous B operands (gemm_dma.h); a translation unit of its own so the
// instantiations compile in parallel with gemm.hip.
#include "gemm_dma.h"

namespace pde {

bool dma_launch_tf(int cfg, int s64, dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps) {
  return launch_dma_cfg<true, false>(cfg, s64, grid, s, ka, tm, tn, kps);
}

}  // namespace pde
