// One-launch MLP training step (csrc/kernels/mlp_fused.hip): argument block and entry points.  Kept out of
// pde_kernels.h so that the kernel's iteration does not rebuild every translation unit.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "xgmi_view.h"

namespace pde {

// Whole MLP training step in ONE persistent launch (mlp_fused.hip): forward, mean softmax cross-entropy, backward
// and the optimiser update (mode 0 SGD, 1 Adam, 2 AdamW; hyper-parameters / step count as optim_step) of every
// Linear(+ReLU) layer, grid barriers between phases.  Layer l: fp32 master weight w [out][in] / bias, gradients,
// optimiser state (mw / vw, mb / vb: nullptr when the mode has none), the bf16 copy wbf [out][in] (refreshed) and,
// for l >= 1, the transposed bf16 copy wtbf [in][ldt] (ldt = out, or 32 for the last layer: zero-padded columns).
// act[l] (l >= 1): [B][in_l] bf16 input of layer l; actT[l]: [in_l][B] (actT[0] = x^T, written by the kernel);
// d / dT[l] (l >= 1): the gradient at act[l] (ReLU applied); dlog [B][32] / dlogT [32][B] zero-initialised.
// B % 32 == 0, every in / out % 8 == 0 except the last out (<= 16), in <= 1024 (one row-GEMM tile's K).
constexpr int kMlpMaxLayers = 8;
struct MlpLayerArgs {
  float *w, *b, *gw, *gb, *mw, *vw, *mb, *vb;
  uint16_t *wbf, *wtbf;
  int in, out, ldt;
};
struct MlpTrainArgs {
  MlpLayerArgs L[kMlpMaxLayers];
  int nl, B, mode;
  const float* x;
  const int64_t* y;
  uint16_t* act[kMlpMaxLayers];
  uint16_t* actT[kMlpMaxLayers];
  uint16_t* d[kMlpMaxLayers];
  uint16_t* dT[kMlpMaxLayers];
  uint16_t *dlog, *dlogT;
  float *loss_part, *loss;
  const float* hp;
  int* step;
  unsigned* bar;  // [320], zeroed ONCE: the grid barrier's counters and launch word (monotonic across launches)
  int* err;
  long long* stamps;  // optional [128]: workgroup 0's / the latest workgroup's wall clock at each phase boundary
  int flags;          // bit 0: load the update state after the weight-gradient tiles, not with them (PDE_MLP_PRELOAD=0)
                      // bit 1: no fused wgrad + update (PDE_MLP_FUSE=0)
  // world > 1 (one node): every 64x64 weight-gradient tile (+ its bias slice) is exchanged over xGMI INSIDE the
  // launch, between its weight-gradient GEMM and its update -- staged into this rank's slot of `xv` at the tile's
  // offset (kMlpXchgTile floats per tile, layers in order), one flag per (workgroup, exchange), summed over all
  // ranks in rank order and scaled by xscale (1 / world: DDP's average).  xchg == 0: no exchange.
  XgmiView xv;
  float xscale;
  int xchg;
  long xoff[kMlpMaxLayers];  // first float of layer l's tiles in the exchange slot (host-computed)
};
constexpr int kMlpXchgTile = 64 * 64 + 64;
// floats of the exchange slot the layers' tiles need (the XgmiAllreduce instance's max_bytes must cover 4x this)
inline long mlp_xchg_floats(const int* in, const int* out, int nl) {
  long n = 0;
  for (int l = 0; l < nl; ++l) n += static_cast<long>((out[l] + 63) / 64) * ((in[l] + 63) / 64) * kMlpXchgTile;
  return n;
}
int mlp_train_grid(int device);  // workgroups of the persistent launch (one per CU), 0 if it cannot be resident
hipError_t mlp_train_step(const MlpTrainArgs& a, int grid, hipStream_t s);

}  // namespace pde
