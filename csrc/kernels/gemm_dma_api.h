// Host-side entry points of the LDS-DMA GEMM core (gemm_dma.h), for gemm.hip's dispatch.
#pragma once

#include <hip/hip_runtime.h>

#include "pde_kernels.h"
#include "optim_device.h"

namespace pde {

constexpr int kDmaBK = 64;  // K depth of one DMA K-tile

// dims of a paired launch's two problems (tiles along M / N, K per split, vector flags, splits)
struct PairDims {
  int tm[2], tn[2], kps[2], av[2], bv[2], nz[2];
};

// implemented in gemm_dma_{tt,tf,ft,ff}.hip (operand orientations: K-contiguous A / B or not), gemm_dma_pair.hip
// cfg: 0 64x64, 1 128x64, 2 64x128, 3 128x128; s64: ring slots of the 64x64 tile (kDmaS64).  false: no
// instantiation for these operand kinds.
bool dma_launch_tt(int cfg, int s64, dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps);
bool dma_launch_tf(int cfg, int s64, dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps);
bool dma_launch_ft(int cfg, int s64, dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps);
bool dma_launch_ff(int cfg, int s64, dim3 grid, hipStream_t s, const GemmArgs& ka, int tm, int tn, int kps);
// pairs: s = 3 or 6 ring slots
bool dma_launch_pair(int s, int k0, int k1, dim3 grid, hipStream_t st, const GemmArgs& a0, const GemmArgs& a1,
                     const PairDims& d, const OptimSeg& seg);


}  // namespace pde
