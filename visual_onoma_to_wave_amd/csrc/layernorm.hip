// Residual + LayerNorm + pad-mask over channels-last rows, one wave per row.
// Replaces: LayerNorm(out + residual) of MultiHeadAttention / PositionwiseFeedForward
// (scripts/transformer/SubLayers.py:55,91) fused with FFTBlock.masked_fill(mask, 0)
// (scripts/transformer/Layers.py:25,28), and the VariancePredictor LayerNorms
// (scripts/model/modules.py:197-206).  HBM-bound: reads x (+res), writes y.

#include "vo_common.h"

namespace vo {

template <typename TX, typename TR, typename TY, int NPL>
__global__ void __launch_bounds__(256) layernorm_kernel(const TX* __restrict__ x, const TR* __restrict__ res,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta,
                                                        const int32_t* __restrict__ lens, int B, int T,
                                                        float eps, TY* __restrict__ y) {
  constexpr int D = NPL * 64;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)B * T) return;
  const int b = (int)(row / T), t = (int)(row - (int64_t)b * T);
  const int c0 = lane * NPL;
  TY* yr = y + row * D + c0;
  if (lens && t >= lens[b]) {
    float z[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < NPL; i += 4) store4(yr + i, z);
    return;
  }
  float v[NPL];
#pragma unroll
  for (int i = 0; i < NPL; i += 4) {
    float q[4];
    load4(x + row * D + c0 + i, q);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[i + e] = q[e];
    if (res) {
      load4(res + row * D + c0 + i, q);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[i + e] += q[e];
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) s += v[i];
  const float mean = wave_sum(s) * (1.0f / D);
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const float dlt = v[i] - mean;
    ss += dlt * dlt;
  }
  const float rstd = rsqrtf(wave_sum(ss) * (1.0f / D) + eps);
#pragma unroll
  for (int i = 0; i < NPL; i += 4) {
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (v[i + e] - mean) * rstd * gamma[c0 + i + e] + beta[c0 + i + e];
    store4(yr + i, o);
  }
}

template <typename TX, typename TR, typename TY>
static int ln_launch(const void* x, const void* res, const float* g, const float* bt, const int32_t* lens,
                     int B, int T, int D, float eps, void* y, hipStream_t st) {
  const int64_t rows = (int64_t)B * T;
  dim3 grid((unsigned)((rows + 3) / 4));
  if (D == 256)
    hipLaunchKernelGGL((layernorm_kernel<TX, TR, TY, 4>), grid, dim3(256), 0, st, (const TX*)x, (const TR*)res,
                       g, bt, lens, B, T, eps, (TY*)y);
  else
    hipLaunchKernelGGL((layernorm_kernel<TX, TR, TY, 8>), grid, dim3(256), 0, st, (const TX*)x, (const TR*)res,
                       g, bt, lens, B, T, eps, (TY*)y);
  VO_RETURN_LAUNCH();
}

}  // namespace vo

using namespace vo;

extern "C" int vo_layernorm(const void* x, int x_dtype, const void* res, int res_dtype, const float* gamma,
                            const float* beta, const int32_t* lens, int B, int T, int D, float eps, void* y,
                            int y_dtype, void* stream) {
  VO_CHECK_ARG(x && gamma && beta && y, "layernorm: null pointer");
  VO_CHECK_ARG(D == 256 || D == 512, "layernorm: D=%d unsupported (256 or 512)", D);
  VO_CHECK_ARG(B > 0 && T > 0, "layernorm: empty");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (!res) res_dtype = x_dtype;
#define VO_LN(TX, TR, TY) return ln_launch<TX, TR, TY>(x, res, gamma, beta, lens, B, T, D, eps, y, st)
  if (x_dtype == VO_BF16 && res_dtype == VO_BF16 && y_dtype == VO_BF16) VO_LN(bf16_t, bf16_t, bf16_t);
  if (x_dtype == VO_F32 && res_dtype == VO_F32 && y_dtype == VO_F32) VO_LN(float, float, float);
  if (x_dtype == VO_BF16 && res_dtype == VO_BF16 && y_dtype == VO_F32) VO_LN(bf16_t, bf16_t, float);
  if (x_dtype == VO_F32 && res_dtype == VO_F32 && y_dtype == VO_BF16) VO_LN(float, float, bf16_t);
#undef VO_LN
  vo_set_error("layernorm: unsupported dtype combination");
  return VO_ERR_INVALID;
}
