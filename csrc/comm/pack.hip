// Fusion-buffer pack / unpack for the Horovod-style engine (gfx950): many tensors <-> one contiguous
// buffer in ONE launch per direction (Horovod does a memcpy per tensor).  Unpack fuses the
// post-scale (1/size for Average, gradient_predivide_factor) into the copy.  Optional dtype change on
// the fly implements fp32 <-> bf16 compression on the wire.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pack.h"

namespace pde {

namespace {

__device__ __forceinline__ float load_as_f32(const void* p, long i, int dt) {
  if (dt == 0) return static_cast<const float*>(p)[i];
  const uint16_t b = static_cast<const uint16_t*>(p)[i];
  return __uint_as_float(static_cast<uint32_t>(b) << 16);
}
__device__ __forceinline__ void store_from_f32(void* p, long i, int dt, float v) {
  if (dt == 0) {
    static_cast<float*>(p)[i] = v;
  } else {
    __bf16 h = static_cast<__bf16>(v);
    static_cast<uint16_t*>(p)[i] = __builtin_bit_cast(uint16_t, h);
  }
}

// blockIdx.y = segment; grid-stride over the segment's elements.
__global__ void k_pack(PackTable tab, void* fused, int fused_dt, float scale) {
  const PackSeg& sg = tab.seg[blockIdx.y];
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < sg.n;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const float v = load_as_f32(sg.ptr, i, sg.dtype) * scale;
    store_from_f32(fused, sg.offset + i, fused_dt, v);
  }
}

__global__ void k_unpack(PackTable tab, const void* fused, int fused_dt, float scale) {
  const PackSeg& sg = tab.seg[blockIdx.y];
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < sg.n;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const float v = load_as_f32(fused, sg.offset + i, fused_dt) * scale;
    store_from_f32(sg.ptr, i, sg.dtype, v);
  }
}

int grid_x(const PackTable& t) {
  long mx = 1;
  for (int i = 0; i < t.count; ++i) mx = t.seg[i].n > mx ? t.seg[i].n : mx;
  long b = (mx + 255) / 256;
  if (b > 256) b = 256;
  return static_cast<int>(b);
}

}  // namespace

hipError_t fusion_pack(const PackTable& t, void* fused, int fused_dt, float scale, hipStream_t s) {
  if (t.count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pack, dim3(grid_x(t), t.count), dim3(256), 0, s, t, fused, fused_dt, scale);
  return hipGetLastError();
}

hipError_t fusion_unpack(const PackTable& t, const void* fused, int fused_dt, float scale, hipStream_t s) {
  if (t.count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_unpack, dim3(grid_x(t), t.count), dim3(256), 0, s, t, fused, fused_dt, scale);
  return hipGetLastError();
}

}  // namespace pde
