#pragma once
#include <hip/hip_runtime.h>

namespace pde {

constexpr int kMaxPackSegs = 96;  // per launch (kernel-argument table); larger batches are chunked

struct PackSeg {
  void* ptr;     // tensor data
  long n;        // elements
  long offset;   // element offset in the fused buffer
  int dtype;     // 0 f32, 1 bf16
};

struct PackTable {
  int count;
  PackSeg seg[kMaxPackSegs];
};

// tensors -> fused buffer (x scale), fused -> tensors (x scale); fused_dt: 0 f32, 1 bf16
hipError_t fusion_pack(const PackTable& t, void* fused, int fused_dt, float scale, hipStream_t s);
hipError_t fusion_unpack(const PackTable& t, const void* fused, int fused_dt, float scale, hipStream_t s);

}  // namespace pde
