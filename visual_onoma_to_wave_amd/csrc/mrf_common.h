// Helpers shared by the fused MRF kernels (resblock.hip, resblock3.hip): 16-byte staging
// vectors, the conflict-free LDS row swizzle and packed-bf16 leaky ReLU.
#pragma once

#include "vo_common.h"

namespace vo {

// staging registers use a clang vector type: HIP's uint4 struct is copied with memcpy, which
// kept the streamed-weight registers in scratch memory
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// LDS rows of 64 B (32 bf16 of one 32-channel plane); 16-byte chunk q of row r sits at chunk
// q ^ ((r >> (sh - 1)) & 2): the fragment reads of 16 consecutive rows hit distinct banks
__device__ __forceinline__ int rb_off(int r, int q, int sh) { return r * 32 + 8 * (q ^ ((r >> (sh - 1)) & 2)); }

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return pk_bf16(lo, hi);
}

// leaky ReLU of 8 packed bf16 (0 <= slope <= 1: lrelu(v) = max(v, slope * v))
__device__ __forceinline__ u32x4 lrelu8(u32x4 u, float s) {
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = __uint_as_float(w[i] << 16), hi = __uint_as_float(w[i] & 0xffff0000u);
    w[i] = pk_bf16(lrelu_max(lo, s), lrelu_max(hi, s));
  }
  return u32x4{w[0], w[1], w[2], w[3]};
}

// packed-fp32 forms (v_pk_mul_f32 / v_pk_add_f32: two values per VALU instruction) for the
// epilogues, whose VALU work -- not the MFMAs -- bound the narrow MRF kernels (round-3 counters:
// 6-9 VALU instructions per MFMA in the k = 3 blocks)
typedef float f32x2v __attribute__((ext_vector_type(2)));

// bf16 pair of leaky-ReLU(a), leaky-ReLU(b): one packed multiply, two maxima, one packed convert
__device__ __forceinline__ uint32_t lrelu_pk(float a, float b, float s) {
  const f32x2v m = f32x2v{a, b} * s;
  return pk_bf16(__builtin_elementwise_maximum(a, m.x), __builtin_elementwise_maximum(b, m.y));
}

// lrelu8 with the packed multiply: 8 packed bf16 -> 8 packed bf16
__device__ __forceinline__ u32x4 lrelu8_pk(u32x4 u, float s) {
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = lrelu_pk(__uint_as_float(w[i] << 16), __uint_as_float(w[i] & 0xffff0000u), s);
  return u32x4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ void unpack8(u32x4 u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

}  // namespace vo
