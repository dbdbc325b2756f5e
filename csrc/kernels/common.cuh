// Shared device helpers for the gfx950 kernels: bf16 conversion, vector types, wave reductions.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace pde {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

// 16- / 8-byte global store, write-through (sc1) when `wt`: the bytes leave the XCD's L2 while the kernel
// runs, so the next launch (its blocks on any XCD) does not first wait for an end-of-kernel write-back of
// them -- that boundary cost grows with the bytes a kernel leaves dirty (MI355X_MICROARCH.md, boundary row).
// Narrower write-through stores are one fabric write each (slow): callers keep the plain path for those.
template <typename V>
__device__ __forceinline__ void st_vec(V* p, const V& v, bool wt) {
  static_assert(sizeof(V) == 16 || sizeof(V) == 8, "16- or 8-byte stores");
  if (wt) {
    if constexpr (sizeof(V) == 16)
      asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(__builtin_bit_cast(u32x4, v)) : "memory");
    else
      asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(__builtin_bit_cast(u32x2, v)) : "memory");
  } else {
    *p = v;
  }
}

__device__ __forceinline__ float bf2f(uint16_t b) {
  return __uint_as_float(static_cast<uint32_t>(b) << 16);
}
// Round-to-nearest-even via the native cast (hipcc emits v_cvt_pk_bf16_f32; NaN stays NaN).
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 h = static_cast<__bf16>(f);
  return __builtin_bit_cast(uint16_t, h);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

inline int ceil_div(long a, long b) { return static_cast<int>((a + b - 1) / b); }

// Grid size for a grid-stride memory-bound kernel: enough blocks to fill 256 CUs, capped.
inline int stream_grid(long n, int block, int per_thread = 1, long cap = 2048) {
  long blocks = (n + static_cast<long>(block) * per_thread - 1) / (static_cast<long>(block) * per_thread);
  if (blocks < 1) blocks = 1;
  if (blocks > cap) blocks = cap;
  return static_cast<int>(blocks);
}

}  // namespace pde
