// Fused multi-tensor optimisers (gfx950): SGD (+momentum), Adam, AdamW over ALL parameter tensors
// of a model in ONE launch ("one fused multi-tensor Adam kernel").
//
// Work decomposition: the host cuts every tensor into chunks of at most kChunk elements (a chunk never
// straddles two tensors) and uploads a chunk list once.  A block walks chunks grid-stride; the chunk's
// tensor entry is block-uniform (scalar loads), and each thread moves kGroups x 16 B of every state
// tensor per chunk with all loads issued before the math (memory-level parallelism; no per-element
// search over tensor offsets).
//
// Hyper-parameters and the step counter live in device memory so the update can be replayed inside a
// hipGraph while the LR changes between replays (elastic LR rescale, horovod_mnist_elastic.py:80-82).
// fp32 master weights.  Besides the update the kernel refreshes the MFMA kernels' bf16 compute copy of
// the weight it just wrote (linear weights, and 1x1 conv weights whose OIHW layout IS the implicit-GEMM
// layout), with contiguous 8-byte stores -- so those layers run no per-step cast / layout kernel.  The
// step counter is int32[2] = {steps taken, arrival counter}: the last block to finish advances it.
#include <cstdlib>

#include "optim_device.h"

namespace pde {

namespace {

using optdev::kOptChunk;
using optdev::kOptThreads;

template <int MODE, int NT>
__global__ __launch_bounds__(kOptThreads) void k_optim(const OptimEntry* __restrict__ tab,
                                                       const OptimChunk* __restrict__ chunks, int c_begin, int c_end,
                                                       const float* __restrict__ hp, int* __restrict__ step_ptr,
                                                       int publish) {
  optdev::run_chunks<MODE, NT>(tab, chunks, c_begin, c_end, hp, step_ptr, blockIdx.x, gridDim.x, publish != 0);
}

}  // namespace

int optim_chunk_elems() { return kOptChunk; }

int optim_segment_blocks(int nchunks) {
  // ~3 blocks per CU, each walking several chunks with the next one's loads in flight (pipelined loop)
  static const int kMaxBlocks = std::getenv("PDE_OPTIM_BLOCKS") ? std::atoi(std::getenv("PDE_OPTIM_BLOCKS")) : 768;
  return nchunks < kMaxBlocks ? nchunks : kMaxBlocks;
}

hipError_t multi_tensor_optim_range(int mode, const OptimEntry* dev_table, const OptimChunk* dev_chunks, int c_begin,
                                    int c_end, const float* dev_hparams, int* dev_step, int publish, hipStream_t s) {
  if (c_end <= c_begin) return hipSuccess;
  // PDE_OPTIM_NT: 0 plain, 1 non-temporal loads + stores, 2 non-temporal loads + write-through stores (ld4/st4).
  // Default by size: non-temporal from 8M elements per launch up (the state streams through once and would only
  // evict the next step's operands from L2 / MALL), plain below.  r4x, MLP Adam (6M): plain 31.2 us, write-through
  // 35.1, non-temporal 37.9; r6ah, ResNet stage 2 SGD (24M): non-temporal 1.2439 vs plain 1.2626 ms per step,
  // ResNet-50 b32 (25.5M, write-through) level
  static const int nt_env = std::getenv("PDE_OPTIM_NT") ? std::atoi(std::getenv("PDE_OPTIM_NT")) : -1;
  const int nt = nt_env >= 0 ? nt_env : (static_cast<long>(c_end - c_begin) * kOptChunk >= (8L << 20) ? 1 : 0);
  dim3 grid(static_cast<unsigned>(optim_segment_blocks(c_end - c_begin)));
#define PDE_OPT(M)                                                                                            \
  if (nt == 2)                                                                                                \
    hipLaunchKernelGGL((k_optim<M, 2>), grid, dim3(kOptThreads), 0, s, dev_table, dev_chunks, c_begin, c_end, \
                       dev_hparams, dev_step, publish);                                                      \
  else if (nt == 1)                                                                                           \
    hipLaunchKernelGGL((k_optim<M, 1>), grid, dim3(kOptThreads), 0, s, dev_table, dev_chunks, c_begin, c_end, \
                       dev_hparams, dev_step, publish);                                                      \
  else                                                                                                        \
    hipLaunchKernelGGL((k_optim<M, 0>), grid, dim3(kOptThreads), 0, s, dev_table, dev_chunks, c_begin, c_end, \
                       dev_hparams, dev_step, publish);
  if (mode == 0) {
    PDE_OPT(0)
  } else if (mode == 1) {
    PDE_OPT(1)
  } else {
    PDE_OPT(2)
  }
#undef PDE_OPT
  return hipGetLastError();
}

hipError_t multi_tensor_optim(int mode, const OptimEntry* dev_table, const OptimChunk* dev_chunks, int nchunks,
                              const float* dev_hparams, int* dev_step, hipStream_t s) {
  return multi_tensor_optim_range(mode, dev_table, dev_chunks, 0, nchunks, dev_hparams, dev_step, 1, s);
}

}  // namespace pde
