// HiFi-GAN tail and layout/weight preparation kernels.
//
// conv_post_kernel: lrelu(0.01) -> Conv1d(C -> 1, k7, pad 3) -> tanh over channels-last
//   activations (scripts/hifigan/models.py:161-163).  HBM-bound: C*2 bytes in, 4 out per
//   sample; a workgroup stages 256 + K - 1 rows in LDS and every lane reduces K*C products.
// transpose_bct_kernel: (B, C, T) fp32 mel -> channels-last (B, T, ldy), zero channel pad.
// pack_weight_kernel: weight-norm fold (models.py:105-109,167-174), BatchNorm fold and the
//   [K][Co][Ci] / polyphase ConvTranspose1d layouts the conv1d kernel reads.

#include <algorithm>

#include "vo_common.h"

namespace vo {

constexpr int CP_ROWS = 256;

// CC > 0: compile-time channel count (HiFi-GAN V1: 32) -- the staging loads are then issued
// as one batch (a runtime-trip loop serialises one HBM round trip per iteration); CC = 0:
// any C (multiple of 8).
template <typename TX, int CC>
__global__ void __launch_bounds__(256) conv_post_kernel(const TX* __restrict__ x, const float* __restrict__ w,
                                                        float bias, int T, int C_, int K, float slope,
                                                        float* __restrict__ y) {
  const int C = CC > 0 ? CC : C_;
  extern __shared__ __attribute__((aligned(16))) float cp_lds[];
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * CP_ROWS;
  const int pad = (K - 1) / 2;
  const int rows = CP_ROWS + K - 1;
  // pitch C + 4 floats: 16-byte aligned rows, and the 16 lanes of a ds_read_b128 group
  // (consecutive rows, same channels) land on distinct 4-bank groups
  const int P = C + 4;
  const TX* xb = x + (int64_t)b * T * C;
  const int vpr = C / 4;
  // staging: unconditional (clamped) loads, zeroed out of range -- a load under a divergent
  // branch is waited for immediately
  auto stage = [&](int v, const float (&q0)[4]) {
    const int r = v / vpr, c = (v - r * vpr) * 4;
    const int t = t0 - pad + r;
    const bool in = t >= 0 && t < T;
    float q[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) q[e] = in ? fmaxf(q0[e], q0[e] * slope) : 0.f;  // 0 <= slope <= 1
    *reinterpret_cast<float4*>(cp_lds + r * P + c) = make_float4(q[0], q[1], q[2], q[3]);
  };
  auto src = [&](int v) {
    const int r = v / vpr, c = (v - r * vpr) * 4;
    return xb + (int64_t)min(max(t0 - pad + r, 0), T - 1) * C + c;
  };
  if constexpr (CC > 0) {
    constexpr int NV = ((CP_ROWS + 30) * (CC / 4) + 255) / 256;  // K <= 31
    float q[NV][4];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = min(threadIdx.x + i * 256, rows * vpr - 1);
      load4(src(v), q[i]);
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = threadIdx.x + i * 256;
      if (v < rows * vpr) stage(v, q[i]);
    }
  } else {
    for (int v = threadIdx.x; v < rows * vpr; v += 256) {
      float q[4];
      load4(src(v), q);
      stage(v, q);
    }
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= T) return;
  float acc0 = bias, acc1 = 0.f;
  for (int k = 0; k < K; ++k) {
    const float* row = cp_lds + (threadIdx.x + k) * P;
    const float* wk = w + k * C;  // wave-uniform: scalar loads
    for (int c = 0; c < C; c += 8) {
      const float4 a = *reinterpret_cast<const float4*>(row + c);
      const float4 d = *reinterpret_cast<const float4*>(row + c + 4);
      acc0 += wk[c] * a.x + wk[c + 1] * a.y + wk[c + 2] * a.z + wk[c + 3] * a.w;
      acc1 += wk[c + 4] * d.x + wk[c + 5] * d.y + wk[c + 6] * d.z + wk[c + 7] * d.w;
    }
  }
  y[(int64_t)b * T + t] = tanhf(acc0 + acc1);
}

// conv_post_rows_kernel (bf16, compile-time C and K; HiFi-GAN V1: 32, 7): each thread reads
// ONE input row straight from HBM (C bf16, lrelu'd in registers) and reduces it against all K
// taps, z[k][r] = sum_c w[k][c] x[r][c]; after one barrier output t0 + r is tanh(bias +
// sum_k z[k][r + k]).  A row is read once (LDS traffic 2K floats per sample) instead of K
// times from an LDS tile by every output (the stencil kernel above: K*C floats per sample).
// 256 rows per workgroup give 256 - (K - 1) outputs.
template <int C, int K>
__global__ void __launch_bounds__(256) conv_post_rows_kernel(const bf16_t* __restrict__ x, const float* __restrict__ w,
                                                             float bias, int T, float slope, float* __restrict__ y) {
  constexpr int OUT = 256 - (K - 1);
  constexpr int PAD = (K - 1) / 2;
  __shared__ float z[K][256];
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * OUT;
  const int r = threadIdx.x;
  const int t = t0 - PAD + r;
  const bool in = t >= 0 && t < T;
  const bf16_t* src = x + ((int64_t)b * T + min(max(t, 0), T - 1)) * C;
  float f[C];
#pragma unroll
  for (int c = 0; c < C; c += 8) load8(src + c, *reinterpret_cast<float(*)[8]>(f + c));
#pragma unroll
  for (int c = 0; c < C; ++c) f[c] = in ? fmaxf(f[c], f[c] * slope) : 0.f;  // 0 <= slope <= 1
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float p0 = 0.f, p1 = 0.f;
#pragma unroll
    for (int c = 0; c < C; c += 2) {
      p0 = fmaf(w[k * C + c], f[c], p0);  // wave-uniform weights: scalar loads
      p1 = fmaf(w[k * C + c + 1], f[c + 1], p1);
    }
    z[k][r] = p0 + p1;
  }
  __syncthreads();
  if (r >= OUT || t0 + r >= T) return;
  float acc = bias;
#pragma unroll
  for (int k = 0; k < K; ++k) acc += z[k][r + k];
  y[(int64_t)b * T + t0 + r] = tanhf(acc);
}

template <typename TY>
__global__ void transpose_bct_kernel(const float* __restrict__ x, int C, int T, TY* __restrict__ y, int ldy) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z;
  const int t0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, t = t0 + tx;
    tile[k][tx] = (c < C && t < T) ? x[((int64_t)b * C + c) * T + t] : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int t = t0 + k, c = c0 + tx;
    if (t < T && c < ldy) y[((int64_t)b * T + t) * ldy + c] = from_f32<TY>(tile[tx][k]);
  }
}

// one workgroup per dim-0 slice of src (Co for conv, Ci for transposed conv)
template <typename TD>
__global__ void __launch_bounds__(256) pack_weight_kernel(const float* __restrict__ src, const float* __restrict__ g,
                                                          const float* __restrict__ row_scale, int mode, int Co,
                                                          int Ci, int K, int stride, TD* __restrict__ dst) {
  __shared__ float red[4];
  const int s0 = blockIdx.x;
  const int n = (mode == VO_PACK_CONVT) ? Co * K : Ci * K;  // elements per slice
  const float* sp = src + (int64_t)s0 * n;
  float mul = 1.f;
  if (g) {
    float ss = 0.f;
    for (int e = threadIdx.x; e < n; e += 256) ss += sp[e] * sp[e];
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    const float norm = sqrtf(red[0] + red[1] + red[2] + red[3]);
    mul = g[s0] / norm;
  }
  for (int e = threadIdx.x; e < n; e += 256) {
    if (mode == VO_PACK_CONV) {
      // src (Co, Ci, K): s0 = co, e = ci*K + k  -> dst[k][co][ci]
      const int ci = e / K, k = e - ci * K;
      const float rs = row_scale ? row_scale[s0] : 1.f;
      dst[((int64_t)k * Co + s0) * Ci + ci] = from_f32<TD>(sp[e] * mul * rs);
    } else if (mode == VO_PACK_DGRAD) {
      // src (Co, Ci, K): the input-gradient conv uses taps reversed and C_in/C_out swapped:
      // dst[K-1-k][ci][co] = src[co][ci][k]
      const int ci = e / K, k = e - ci * K;
      const float rs = row_scale ? row_scale[s0] : 1.f;
      dst[((int64_t)(K - 1 - k) * Ci + ci) * Co + s0] = from_f32<TD>(sp[e] * mul * rs);
    } else {
      // src (Ci, Co, 2s): s0 = ci, e = co*K + kt; tap kt = r + s*(1-kk) -> dst[kk][r*Co + co][ci]
      const int co = e / K, kt = e - co * K;
      const int r = kt % stride, kk = 1 - kt / stride;
      const float rs = row_scale ? row_scale[co] : 1.f;
      dst[((int64_t)kk * stride * Co + (int64_t)r * Co + co) * Ci + s0] = from_f32<TD>(sp[e] * mul * rs);
    }
  }
}

// without the weight-norm fold: one thread per DESTINATION element (grid-stride), the source
// gathered -- the whole weight is L2-resident while it is walked, and the stores, which the
// per-row kernel above scattered 2 bytes at a time across the taps (8 us for a 256 x 256 x 9
// training weight), go out as contiguous 128-byte wave rows
template <typename TD>
__global__ void __launch_bounds__(256) pack_weight_lin_kernel(const float* __restrict__ src,
                                                              const float* __restrict__ row_scale, int mode, int Co,
                                                              int Ci, int K, int stride, TD* __restrict__ dst) {
  const int64_t n = (int64_t)Co * Ci * K;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    int64_t si;
    int co;
    if (mode == VO_PACK_CONV) {  // dst[k][co][ci] <- src[co][ci][k]
      const int ci = (int)(i % Ci);
      const int64_t r = i / Ci;
      co = (int)(r % Co);
      const int k = (int)(r / Co);
      si = ((int64_t)co * Ci + ci) * K + k;
    } else if (mode == VO_PACK_DGRAD) {  // dst[K-1-k][ci][co] <- src[co][ci][k]
      co = (int)(i % Co);
      const int64_t r = i / Co;
      const int ci = (int)(r % Ci);
      const int k = K - 1 - (int)(r / Ci);
      si = ((int64_t)co * Ci + ci) * K + k;
    } else {  // ConvTranspose1d: dst[kk][r*Co + co][ci] <- src[ci][co][r + s*(1-kk)]
      const int ci = (int)(i % Ci);
      const int64_t q = i / Ci;
      const int col = (int)(q % ((int64_t)stride * Co)), kk = (int)(q / ((int64_t)stride * Co));
      const int rr = col / Co;
      co = col - rr * Co;
      si = ((int64_t)ci * Co + co) * K + rr + stride * (1 - kk);
    }
    dst[i] = from_f32<TD>(src[si] * (row_scale ? row_scale[co] : 1.f));
  }
}

}  // namespace vo

using namespace vo;

extern "C" int vo_conv_post(const void* x, int x_dtype, const float* w, float bias, int B, int T, int C, int K,
                            float slope, float* y, void* stream) {
  VO_CHECK_ARG(x && w && y, "conv_post: null pointer");
  VO_CHECK_ARG(C % 8 == 0 && K % 2 == 1 && C <= 512 && K <= 31, "conv_post: C=%d K=%d unsupported", C, K);
  VO_CHECK_ARG(slope >= 0.f && slope <= 1.f, "conv_post: slope %g outside [0, 1]", slope);
  VO_CHECK_ARG(B > 0 && T > 0, "conv_post: empty");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (x_dtype == VO_BF16 && C == 32 && K == 7 && vo_tune_get("post_cfg") != 1) {  // post_cfg 1: stencil kernel
    constexpr int OUT = 256 - 6;
    dim3 g2((unsigned)((T + OUT - 1) / OUT), (unsigned)B);
    hipLaunchKernelGGL((conv_post_rows_kernel<32, 7>), g2, dim3(256), 0, st, (const bf16_t*)x, w, bias, T, slope, y);
    VO_RETURN_LAUNCH();
  }
  dim3 grid((unsigned)((T + CP_ROWS - 1) / CP_ROWS), (unsigned)B);
  const size_t lds = (size_t)(CP_ROWS + K - 1) * (C + 4) * sizeof(float);
  if (x_dtype == VO_BF16 && C == 32)
    hipLaunchKernelGGL((conv_post_kernel<bf16_t, 32>), grid, dim3(256), lds, st, (const bf16_t*)x, w, bias, T, C, K, slope, y);
  else if (x_dtype == VO_BF16)
    hipLaunchKernelGGL((conv_post_kernel<bf16_t, 0>), grid, dim3(256), lds, st, (const bf16_t*)x, w, bias, T, C, K, slope, y);
  else
    hipLaunchKernelGGL((conv_post_kernel<float, 0>), grid, dim3(256), lds, st, (const float*)x, w, bias, T, C, K, slope, y);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_transpose_bct(const float* x, int B, int C, int T, void* y, int y_dtype, int ldy, void* stream) {
  VO_CHECK_ARG(x && y && ldy >= C, "transpose_bct: bad arguments");
  if (B == 0 || T == 0) return VO_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((unsigned)((T + 31) / 32), (unsigned)((ldy + 31) / 32), (unsigned)B);
  if (y_dtype == VO_BF16)
    hipLaunchKernelGGL(transpose_bct_kernel<bf16_t>, grid, dim3(256), 0, st, x, C, T, (bf16_t*)y, ldy);
  else
    hipLaunchKernelGGL(transpose_bct_kernel<float>, grid, dim3(256), 0, st, x, C, T, (float*)y, ldy);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_pack_weight(const float* src, const float* g, const float* row_scale, int mode, int Co, int Ci,
                              int K, int stride, void* dst, int dst_dtype, void* stream) {
  VO_CHECK_ARG(src && dst, "pack_weight: null pointer");
  VO_CHECK_ARG(mode == VO_PACK_CONV || mode == VO_PACK_DGRAD || (mode == VO_PACK_CONVT && stride >= 1 && K == 2 * stride),
               "pack_weight: bad mode/stride (K must be 2*stride for ConvTranspose1d)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (!g) {
    const int64_t n = (int64_t)Co * Ci * K;
    const dim3 lg((unsigned)std::min<int64_t>((n + 255) / 256, 8192));
    if (dst_dtype == VO_BF16)
      hipLaunchKernelGGL(pack_weight_lin_kernel<bf16_t>, lg, dim3(256), 0, st, src, row_scale, mode, Co, Ci, K, stride,
                         (bf16_t*)dst);
    else
      hipLaunchKernelGGL(pack_weight_lin_kernel<float>, lg, dim3(256), 0, st, src, row_scale, mode, Co, Ci, K, stride,
                         (float*)dst);
    VO_RETURN_LAUNCH();
  }
  dim3 grid((unsigned)(mode == VO_PACK_CONVT ? Ci : Co));
  if (dst_dtype == VO_BF16)
    hipLaunchKernelGGL(pack_weight_kernel<bf16_t>, grid, dim3(256), 0, st, src, g, row_scale, mode, Co, Ci, K, stride,
                       (bf16_t*)dst);
  else
    hipLaunchKernelGGL(pack_weight_kernel<float>, grid, dim3(256), 0, st, src, g, row_scale, mode, Co, Ci, K, stride,
                       (float*)dst);
  VO_RETURN_LAUNCH();
}
