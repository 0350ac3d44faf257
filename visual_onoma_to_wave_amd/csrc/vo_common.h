// Shared device helpers for the gfx950 (CDNA4) kernels of the synthesis path.
// Wave = 64 lanes; MFMA 16x16x32 bf16 (or 8 x 16x16x4 f32 in the fp32 parity mode).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "../../include/vonoma.h"

typedef unsigned short bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace vo {

// ---------------------------------------------------------------- scalar conversion
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16_t x) { return __uint_as_float(((uint32_t)x) << 16); }

template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16_t from_f32<bf16_t>(float x) {
  __hip_bfloat16 b = __float2bfloat16(x);  // round-to-nearest-even, NaN stays NaN
  return *reinterpret_cast<bf16_t*>(&b);
}

// Two floats -> one packed bf16 pair in ONE v_cvt_pk_bf16_f32 (round to nearest even, NaN stays
// NaN).  The pair of scalar conversions compiled to two v_cvt_pk_bf16_f32 and a v_or_b32_sdwa.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
}
// leaky ReLU max(v, s v) for 0 <= s <= 1.  IEEE maximum: unlike fmaxf it needs no operand
// canonicalisation (fmaxf of a value bit-cast from bf16 compiled to two v_max_f32); the results
// are identical (a NaN input gives a NaN either way).
__device__ __forceinline__ float lrelu_max(float v, float s) { return __builtin_elementwise_maximum(v, v * s); }

// Index of the table entry owning item x: the last i < n with start[i] <= x (start ascending,
// start[0] = 0) -- a binary search over a table in the kernel arguments, so a workgroup near the
// end of a 32-entry table pays 5 dependent scalar loads instead of 32.
__device__ __forceinline__ int table_find(const int* start, int n, int x) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (start[mid] <= x) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Workgroups are dispatched round-robin over the 8 XCDs by linear id (w -> XCD w % 8), and each
// XCD has its own L2.  xcd_grouped_id(w, n) maps linear id w of an n-workgroup grid to a logical id
// in [0, n) such that consecutive logical ids run on one XCD: workgroups that read the same bytes
// (the query tiles of one attention head, ...) take logical ids next to each other and share that
// XCD's L2 instead of every XCD fetching them.
__device__ __forceinline__ int xcd_grouped_id(int w, int n) {
  const int x = w & 7, k = w >> 3, q = n >> 3, r = n & 7;
  return x * q + (x < r ? x : r) + k;
}

// Workgroup barrier for LDS hand-offs: this wave's LDS operations drained, then s_barrier.
// __syncthreads() adds a workgroup-scope release fence, and on gfx950 that fence waits vmcnt(0):
// every outstanding global load or store of the wave (an epilogue's y stores, a prefetch meant to
// stay in flight across the barrier) is drained at each barrier.  LDS-DMA destinations still
// need their own vmcnt wait before this barrier; no global memory is handed between waves.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---------------------------------------------------------------- counter-based dropout mask
// Element i of a dropout site is kept iff drop_hash(s0, s1, i) >= p 2^32 (vo_dropout, and the LayerNorm kernels
// that apply a sublayer's dropout in-pass): (s0, s1) from the step's device seed and the site's salt.
__device__ __forceinline__ uint32_t drop_mix(uint32_t h) {  // murmur3 finaliser
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t drop_hash(uint32_t s0, uint32_t s1, uint32_t i) {
  return drop_mix(drop_mix(i * 0x9E3779B9u ^ s0) + s1);
}
__device__ __forceinline__ void drop_keys(const int64_t* seed, uint32_t salt, uint32_t& s0, uint32_t& s1) {
  const uint64_t sd = (uint64_t)seed[0];
  s0 = (uint32_t)sd ^ drop_mix(salt + 0x3C6EF372u);
  s1 = (uint32_t)(sd >> 32);
}

// ---------------------------------------------------------------- 8-element vectors
// Load 8 consecutive elements (16 B for bf16, 32 B for f32) as floats.
__device__ __forceinline__ void load8(const bf16_t* p, float (&v)[8]) {
  uint4 u = *reinterpret_cast<const uint4*>(p);
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void store8(bf16_t* p, const float (&v)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    w[i] = pk_bf16(v[2 * i], v[2 * i + 1]);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ void store8(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void store4(bf16_t* p, const float (&v)[4]) {
  uint32_t a = pk_bf16(v[0], v[1]);
  uint32_t b = pk_bf16(v[2], v[3]);
  *reinterpret_cast<uint2*>(p) = make_uint2(a, b);
}
__device__ __forceinline__ void store4(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void load4(const bf16_t* p, float (&v)[4]) {
  uint2 u = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
}
__device__ __forceinline__ void load4(const float* p, float (&v)[4]) {
  float4 a = *reinterpret_cast<const float4*>(p);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}

// ---------------------------------------------------------------- MFMA fragments
// A fragment holds A[row = lane&15][k = 8*(lane>>4) + j], B holds B[k = 8*(lane>>4)+j][col = lane&15]
// (j = 0..7).  For bf16 that is exactly one v_mfma_f32_16x16x32_bf16.  For f32 the same
// 32-deep k-slice is split into 8 v_mfma_f32_16x16x4_f32 whose k index (lane>>4) maps to
// k = 8*(lane>>4) + j -- any consistent k permutation of A and B gives the same sum.
template <typename TC> struct Frag;
template <> struct Frag<bf16_t> {
  bf16x8 v;
  __device__ __forceinline__ void load(const bf16_t* p) { v = *reinterpret_cast<const bf16x8*>(p); }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (__bf16)0.0f;
  }
};
template <> struct Frag<float> {
  float v[8];
  __device__ __forceinline__ void load(const float* p) {
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.f;
  }
};

__device__ __forceinline__ f32x4 mfma(const Frag<bf16_t>& a, const Frag<bf16_t>& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma(const Frag<float>& a, const Frag<float>& b, f32x4 c) {
#pragma unroll
  for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[j], b.v[j], c, 0, 0, 0);
  return c;
}

// ---------------------------------------------------------------- split-bf16 fp32 contractions (VO_F32X3)
// An fp32 operand v is held as hi = bf16(v), lo = bf16(v - hi) (v - hi is exact in fp32), and a product
// as hi a * hi b + hi a * lo b + lo a * hi b: three 16x16x32 bf16 MFMAs with fp32 accumulation in place
// of eight 16x16x4 f32 ones (5.3x fewer MFMA cycles).  Per product the dropped lo a * lo b and the
// rounding of the lo parts leave <= 3 * 2^-18 of |a b| (~1e-5) -- fp32-class accuracy, not bit-exact
// fp32.  bx3_t is the LDS element of such a tile: 8 channels = 32 bytes = [hi x 8 | lo x 8], so an
// 8-element vector sits where an fp32 tile would put it (same offsets, same 4-byte element).
struct bx3_t { uint32_t u; };
__device__ __forceinline__ void split8(const float (&v)[8], uint4& hi, uint4& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    h[i] = pk_bf16(v[2 * i], v[2 * i + 1]);
    const float r0 = v[2 * i] - __uint_as_float(h[i] << 16);
    const float r1 = v[2 * i + 1] - __uint_as_float(h[i] & 0xffff0000u);
    l[i] = pk_bf16(r0, r1);
  }
  hi = make_uint4(h[0], h[1], h[2], h[3]);
  lo = make_uint4(l[0], l[1], l[2], l[3]);
}
__device__ __forceinline__ void store8(bx3_t* p, const float (&v)[8]) {
  uint4 hi, lo;
  split8(v, hi, lo);
  reinterpret_cast<uint4*>(p)[0] = hi;
  reinterpret_cast<uint4*>(p)[1] = lo;
}
template <> struct Frag<bx3_t> {
  bf16x8 hi, lo;
  __device__ __forceinline__ void load(const bx3_t* p) {
    hi = reinterpret_cast<const bf16x8*>(p)[0];
    lo = reinterpret_cast<const bf16x8*>(p)[1];
  }
};
__device__ __forceinline__ f32x4 mfma(const Frag<bx3_t>& a, const Frag<bx3_t>& b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo, b.hi, c, 0, 0, 0);  // small terms first
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.lo, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, c, 0, 0, 0);
}

// ---------------------------------------------------------------- activations
__device__ __forceinline__ float act(int kind, float x, float slope) {
  switch (kind) {
    case VO_ACT_RELU: return x > 0.f ? x : 0.f;
    case VO_ACT_LRELU: return x > 0.f ? x : x * slope;
    case VO_ACT_TANH: return tanhf(x);
    default: return x;
  }
}

// ---------------------------------------------------------------- wave reductions (64 lanes)
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

}  // namespace vo

// error plumbing shared by the launchers (vo_runtime.cpp)
extern "C" void vo_set_error(const char* fmt, ...);
extern "C" int vo_tune_get(const char* key);

#define VO_CHECK_ARG(cond, ...)                \
  do {                                         \
    if (!(cond)) {                             \
      vo_set_error(__VA_ARGS__);               \
      return VO_ERR_INVALID;                   \
    }                                          \
  } while (0)

#define VO_RETURN_LAUNCH()                                       \
  do {                                                           \
    hipError_t e_ = hipGetLastError();                           \
    if (e_ != hipSuccess) {                                      \
      vo_set_error("launch failed: %s", hipGetErrorString(e_));  \
      return (int)e_;                                            \
    }                                                            \
    return VO_OK;                                                \
  } while (0)
