// Shared device helpers for the dstack_amd CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dsa {

typedef unsigned short bf16_t;  // raw bf16 storage
typedef unsigned short us8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// round-to-nearest-even float -> bf16 (hipcc lowers the pattern to v_cvt_pk_bf16_f32 on gfx950)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ void unpack8(const us8& v, float (&o)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = bf2f(v[i]);
}

__device__ __forceinline__ us8 pack8(const float (&o)[8]) {
  us8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = f2bf(o[i]);
  return v;
}

// 64-lane wave reductions (wave64: __shfl_xor spans all 64 lanes)
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

}  // namespace dsa

#define DSA_CHECK(expr)                                                              \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess) return _e;                                                 \
  } while (0)
