// Residual + LayerNorm + pad-mask over channels-last rows, one wave per row.
// Replaces: LayerNorm(out + residual) of MultiHeadAttention / PositionwiseFeedForward
// (scripts/transformer/SubLayers.py:55,91) fused with FFTBlock.masked_fill(mask, 0)
// (scripts/transformer/Layers.py:25,28), and the VariancePredictor LayerNorms
// (scripts/model/modules.py:197-206).  HBM-bound: reads x (+res), writes y.

#include <algorithm>

#include "vo_common.h"

namespace vo {

// DUAL (round 4): a bf16 copy of y beside it (y16) -- the next conv of the "mixed" decoder, whose
// residual stream is fp32, reads the copy: half the bytes per re-read of its input tiles, and the same
// bits as the conv's own fp32 -> bf16 staging (round to nearest even)
// Dropout of x in the same pass (round 6, training: the sublayer output's nn.Dropout before the residual add,
// scripts/transformer/SubLayers.py:51,88): x_i kept iff drop_hash(seed, salt, i) >= thr (i = the flat element
// index -- the mask vo_dropout would draw for the same (seed, salt)), then scaled by 1 / (1 - p).
struct LnDrop {
  const int64_t* seed;  // nullptr: no dropout
  uint32_t salt, thr;
  float scale;
};

template <typename TX, typename TR, typename TY, int NPL, bool DUAL = false>
__global__ void __launch_bounds__(256) layernorm_kernel(const TX* __restrict__ x, const TR* __restrict__ res,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta,
                                                        const int32_t* __restrict__ lens, int B, int T,
                                                        float eps, TY* __restrict__ y, bf16_t* __restrict__ y16,
                                                        LnDrop dr = LnDrop{nullptr, 0u, 0u, 1.f}) {
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
    for (int i = 0; i < NPL; i += 4) {
      store4(yr + i, z);
      if constexpr (DUAL) store4(y16 + row * D + c0 + i, z);
    }
    return;
  }
  float v[NPL];
  uint32_t s0 = 0, s1 = 0;
  if (dr.seed) drop_keys(dr.seed, dr.salt, s0, s1);
#pragma unroll
  for (int i = 0; i < NPL; i += 4) {
    float q[4];
    load4(x + row * D + c0 + i, q);
    if (dr.seed) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        q[e] = drop_hash(s0, s1, (uint32_t)(row * D + c0 + i + e)) >= dr.thr ? q[e] * dr.scale : 0.f;
    }
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
    if constexpr (DUAL) store4(y16 + row * D + c0 + i, o);
  }
}

template <typename TX, typename TR, typename TY, bool DUAL = false>
static int ln_launch(const void* x, const void* res, const float* g, const float* bt, const int32_t* lens,
                     int B, int T, int D, float eps, void* y, hipStream_t st, void* y16 = nullptr,
                     LnDrop dr = LnDrop{nullptr, 0u, 0u, 1.f}) {
  const int64_t rows = (int64_t)B * T;
  dim3 grid((unsigned)((rows + 3) / 4));
  if (D == 256)
    hipLaunchKernelGGL((layernorm_kernel<TX, TR, TY, 4, DUAL>), grid, dim3(256), 0, st, (const TX*)x,
                       (const TR*)res, g, bt, lens, B, T, eps, (TY*)y, (bf16_t*)y16, dr);
  else
    hipLaunchKernelGGL((layernorm_kernel<TX, TR, TY, 8, DUAL>), grid, dim3(256), 0, st, (const TX*)x,
                       (const TR*)res, g, bt, lens, B, T, eps, (TY*)y, (bf16_t*)y16, dr);
  VO_RETURN_LAUNCH();
}

// ---------------------------------------------------------------- backward (training, C4)
// Gradient of y = pad ? 0 : LN(x + res) * gamma + beta (the forward above).  One wave per row
// recomputes mean / rstd from x (+ res) and writes
//   gh = rstd * (g*gy - mean(g*gy) - xhat * mean(g*gy * xhat))      (pad rows: 0)
// which is the gradient of both x and res.  gamma / beta gradients are column sums over the
// unmasked rows: each workgroup (16 waves x LN_BWD_RPW rows) reduces its rows in registers, then
// across its waves through LDS, and writes one partial row [2][D] to the workspace; a second
// kernel adds the partials in workgroup order (deterministic, no atomics).  A wave issues the
// loads of all its rows before the first reduction (the row chain is latency-, not
// bandwidth-bound at 16 rows per wave: 37 us at C2 -> see DESIGN.md).
// Replaces the PyTorch autograd recomputation of LayerNorm backward (SubLayers.py:55,91,
// Layers.py:25,28 under 04_train.py:128-141).  HBM-bound: reads x, res, gy, writes gh.
constexpr int LN_BWD_RPW = 4;   // rows per wave
constexpr int LN_BWD_NW = 16;   // waves per workgroup: 64 rows, 256 partials at C2

// Round 6 (vo_layernorm_bwd_ex): res may be fp32 beside a bf16 x (the mixed decoder's fp32 residual stream,
// vo_layernorm_dual's forward), a second incoming gradient gy2 (bf16: the gradient of y16, the copy the convs
// read) is added to gy in registers, and gh32 (optional) receives the fp32 gradient of res beside gh.
template <typename TX, typename TR, typename TG, int NPL>
__global__ void __launch_bounds__(1024) layernorm_bwd_kernel(const TX* __restrict__ x, const TR* __restrict__ res,
                                                             const TG* __restrict__ gy,
                                                             const bf16_t* __restrict__ gy2,
                                                             const float* __restrict__ gamma,
                                                             const int32_t* __restrict__ lens, int B, int T,
                                                             float eps, TX* __restrict__ gh,
                                                             TR* __restrict__ gres,
                                                             float* __restrict__ partial,
                                                             LnDrop dr = LnDrop{nullptr, 0u, 0u, 1.f}) {
  constexpr int D = NPL * 64;
  __shared__ float red[LN_BWD_NW][2][D];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = lane * NPL;
  const int64_t rows = (int64_t)B * T;
  float g[NPL], accg[NPL], accb[NPL];
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    g[i] = gamma[c0 + i];
    accg[i] = 0.f;
    accb[i] = 0.f;
  }
  const int64_t row0 = ((int64_t)blockIdx.x * LN_BWD_NW + wv) * LN_BWD_RPW;
  float v[LN_BWD_RPW][NPL], dy[LN_BWD_RPW][NPL];
  // (the dropout keys are named apart from the row sums s1 / s2 below: shadowed, the first version of this
  // fusion drew the x gradient's mask with a row sum as its key -- right forward, wrong zero pattern backward)
  uint32_t dk0 = 0, dk1 = 0;
  if (dr.seed) drop_keys(dr.seed, dr.salt, dk0, dk1);
  bool live[LN_BWD_RPW];
#pragma unroll
  for (int r = 0; r < LN_BWD_RPW; ++r) {
    const int64_t row = row0 + r;
    bool ok = row < rows;
    if (ok && lens) {
      const int b = (int)(row / T), t = (int)(row - (int64_t)b * T);
      ok = t < lens[b];
    }
    live[r] = ok;
    const int64_t rr = ok ? row : 0;
#pragma unroll
    for (int i = 0; i < NPL; i += 4) {
      float q[4], e[4], d[4];
      load4(x + rr * D + c0 + i, q);
      if (dr.seed) {  // the forward's dropout of x, recomputed
#pragma unroll
        for (int k = 0; k < 4; ++k)
          q[k] = drop_hash(dk0, dk1, (uint32_t)(rr * D + c0 + i + k)) >= dr.thr ? q[k] * dr.scale : 0.f;
      }
      if (res)
        load4(res + rr * D + c0 + i, e);
      else
        e[0] = e[1] = e[2] = e[3] = 0.f;
      load4(gy + rr * D + c0 + i, d);
      if (gy2) {
        float d2[4];
        load4(gy2 + rr * D + c0 + i, d2);
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] += d2[k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[r][i + k] = q[k] + e[k];
        dy[r][i + k] = ok ? d[k] : 0.f;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < LN_BWD_RPW; ++r) {
    const int64_t row = row0 + r;
    if (row >= rows) break;
    TX* gr = gh + row * D + c0;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) s += v[r][i];
    const float mean = wave_sum(s) * (1.0f / D);
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      v[r][i] -= mean;
      ss += v[r][i] * v[r][i];
    }
    const float rstd = rsqrtf(wave_sum(ss) * (1.0f / D) + eps);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      v[r][i] *= rstd;  // xhat
      const float gd = g[i] * dy[r][i];
      s1 += gd;
      s2 += gd * v[r][i];
      accg[i] += dy[r][i] * v[r][i];
      accb[i] += dy[r][i];
    }
    const float m1 = wave_sum(s1) * (1.0f / D), m2 = wave_sum(s2) * (1.0f / D);
    const float sc = live[r] ? rstd : 0.f;  // pad rows: zero gradient
#pragma unroll
    for (int i = 0; i < NPL; i += 4) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = sc * (g[i + e] * dy[r][i + e] - m1 - v[r][i + e] * m2);
      if (gres) store4(gres + row * D + c0 + i, o);  // res: the gradient of x + res as it is
      if (dr.seed) {  // x: through its dropout
#pragma unroll
        for (int e = 0; e < 4; ++e)
          o[e] = drop_hash(dk0, dk1, (uint32_t)(row * D + c0 + i + e)) >= dr.thr ? o[e] * dr.scale : 0.f;
      }
      store4(gr + i, o);
    }
  }
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    red[wv][0][c0 + i] = accg[i];
    red[wv][1][c0 + i] = accb[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * D; c += 1024) {
    const int k = c / D, col = c - k * D;
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < LN_BWD_NW; ++w) t += red[w][k][col];
    partial[(int64_t)blockIdx.x * 2 * D + c] = t;
  }
}

// dgamma / dbeta: sum the per-workgroup partials [nblk][2][D] column-wise in a fixed order.
// Workgroup = 64 columns x 16 row phases; phase s adds partials s, s + 16, ... (4 loads in
// flight per thread), then the 16 phases are added in LDS.
__global__ void __launch_bounds__(1024) ln_partial_sum_kernel(const float* __restrict__ partial, int nblk, int D2,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float red[16][64];
  const int cl = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (c < D2) {
    int k = ph;
    for (; k + 48 < nblk; k += 64) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = partial[(int64_t)(k + 16 * u) * D2 + c];
#pragma unroll
      for (int u = 0; u < 4; ++u) s += v[u];
    }
    for (; k < nblk; k += 16) s += partial[(int64_t)k * D2 + c];
  }
  red[ph][cl] = s;
  __syncthreads();
  if (ph == 0 && c < D2) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += red[w][cl];
    const int D = D2 / 2;
    if (c < D)
      dgamma[c] = t;
    else
      dbeta[c - D] = t;
  }
}

template <typename TX, typename TG, typename TR = TX>
static int ln_bwd_launch(const void* x, const void* res, const void* gy, const float* g, const int32_t* lens,
                         int B, int T, int D, float eps, void* gh, float* dgamma, float* dbeta, float* ws,
                         hipStream_t st, const void* gy2 = nullptr, void* gres = nullptr,
                         LnDrop dr = LnDrop{nullptr, 0u, 0u, 1.f}) {
  const int64_t rows = (int64_t)B * T;
  const int nblk = (int)((rows + LN_BWD_NW * LN_BWD_RPW - 1) / (LN_BWD_NW * LN_BWD_RPW));
  if (D == 256)
    hipLaunchKernelGGL((layernorm_bwd_kernel<TX, TR, TG, 4>), dim3(nblk), dim3(1024), 0, st, (const TX*)x,
                       (const TR*)res, (const TG*)gy, (const bf16_t*)gy2, g, lens, B, T, eps, (TX*)gh, (TR*)gres,
                       ws, dr);
  else
    hipLaunchKernelGGL((layernorm_bwd_kernel<TX, TR, TG, 8>), dim3(nblk), dim3(1024), 0, st, (const TX*)x,
                       (const TR*)res, (const TG*)gy, (const bf16_t*)gy2, g, lens, B, T, eps, (TX*)gh, (TR*)gres,
                       ws, dr);
  hipLaunchKernelGGL(ln_partial_sum_kernel, dim3((2 * D + 63) / 64), dim3(1024), 0, st, (const float*)ws, nblk,
                     2 * D, dgamma, dbeta);
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

extern "C" int vo_layernorm_dual(const void* x, int x_dtype, const void* res, int res_dtype, const float* gamma,
                                 const float* beta, const int32_t* lens, int B, int T, int D, float eps, void* y,
                                 void* y16, void* stream) {
  VO_CHECK_ARG(x && gamma && beta && y && y16, "layernorm_dual: null pointer");
  VO_CHECK_ARG(D == 256 || D == 512, "layernorm_dual: D=%d unsupported (256 or 512)", D);
  VO_CHECK_ARG(B > 0 && T > 0, "layernorm_dual: empty");
  VO_CHECK_ARG(y16 != y && y16 != x && y16 != res, "layernorm_dual: y16 must not alias x, res or y");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (!res) res_dtype = x_dtype;
  if (x_dtype == VO_F32 && res_dtype == VO_F32)
    return ln_launch<float, float, float, true>(x, res, gamma, beta, lens, B, T, D, eps, y, st, y16);
  if (x_dtype == VO_BF16 && res_dtype == VO_BF16)
    return ln_launch<bf16_t, bf16_t, float, true>(x, res, gamma, beta, lens, B, T, D, eps, y, st, y16);
  if (x_dtype == VO_BF16 && res_dtype == VO_F32)  // round 6: bf16 sublayer output + fp32 residual stream (training)
    return ln_launch<bf16_t, float, float, true>(x, res, gamma, beta, lens, B, T, D, eps, y, st, y16);
  vo_set_error("layernorm_dual: unsupported dtype combination (fp32 y; fp32 / fp32, bf16 / bf16 or bf16 / fp32 x / res)");
  return VO_ERR_INVALID;
}

extern "C" int64_t vo_layernorm_bwd_workspace_size(int B, int T, int D) {
  const int64_t rows = (int64_t)B * T;
  return ((rows + LN_BWD_NW * LN_BWD_RPW - 1) / (LN_BWD_NW * LN_BWD_RPW)) * 2 * D * (int64_t)sizeof(float);
}

extern "C" int vo_layernorm_bwd(const void* x, const void* res, int x_dtype, const void* gy, int gy_dtype,
                                const float* gamma, const int32_t* lens, int B, int T, int D, float eps, void* gh,
                                float* dgamma, float* dbeta, void* workspace, void* stream) {
  VO_CHECK_ARG(x && gy && gamma && gh && dgamma && dbeta && workspace, "layernorm_bwd: null pointer");
  VO_CHECK_ARG(D == 256 || D == 512, "layernorm_bwd: D=%d unsupported (256 or 512)", D);
  VO_CHECK_ARG(B > 0 && T > 0, "layernorm_bwd: empty");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* ws = (float*)workspace;
#define VO_LNB(TX, TG) return ln_bwd_launch<TX, TG>(x, res, gy, gamma, lens, B, T, D, eps, gh, dgamma, dbeta, ws, st)
  if (x_dtype == VO_BF16 && gy_dtype == VO_BF16) VO_LNB(bf16_t, bf16_t);
  if (x_dtype == VO_BF16 && gy_dtype == VO_F32) VO_LNB(bf16_t, float);
  if (x_dtype == VO_F32 && gy_dtype == VO_F32) VO_LNB(float, float);
  if (x_dtype == VO_F32 && gy_dtype == VO_BF16) VO_LNB(float, bf16_t);
#undef VO_LNB
  vo_set_error("layernorm_bwd: unsupported dtype combination");
  return VO_ERR_INVALID;
}

extern "C" int vo_layernorm_bwd_ex(const void* x, int x_dtype, const void* res, int res_dtype, const void* gy,
                                   int gy_dtype, const void* gy2, const float* gamma, const int32_t* lens, int B,
                                   int T, int D, float eps, void* gh, float* gh32, float* dgamma, float* dbeta,
                                   void* workspace, void* stream) {
  VO_CHECK_ARG(x && gy && gamma && gh && dgamma && dbeta && workspace, "layernorm_bwd_ex: null pointer");
  VO_CHECK_ARG(D == 256 || D == 512, "layernorm_bwd_ex: D=%d unsupported (256 or 512)", D);
  VO_CHECK_ARG(B > 0 && T > 0, "layernorm_bwd_ex: empty");
  VO_CHECK_ARG(gh32 == nullptr || ((const void*)gh32 != x && (const void*)gh32 != gh), "layernorm_bwd_ex: gh32 aliases");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* ws = (float*)workspace;
  if (!res) res_dtype = x_dtype;
  if (x_dtype == VO_BF16 && res_dtype == VO_F32 && gy_dtype == VO_F32)
    return ln_bwd_launch<bf16_t, float, float>(x, res, gy, gamma, lens, B, T, D, eps, gh, dgamma, dbeta, ws, st, gy2,
                                               gh32);
  if (x_dtype == VO_BF16 && res_dtype == VO_F32 && gy_dtype == VO_BF16)
    return ln_bwd_launch<bf16_t, bf16_t, float>(x, res, gy, gamma, lens, B, T, D, eps, gh, dgamma, dbeta, ws, st,
                                                gy2, gh32);
  if (x_dtype == res_dtype && gy2 == nullptr && gh32 == nullptr)
    return vo_layernorm_bwd(x, res, x_dtype, gy, gy_dtype, gamma, lens, B, T, D, eps, gh, dgamma, dbeta, workspace,
                            stream);
  vo_set_error("layernorm_bwd_ex: unsupported dtype combination (bf16 x with fp32 res, or equal x / res without gy2 / gh32)");
  return VO_ERR_INVALID;
}

// ---- round 6: the training FFT blocks' dropout fused into their LayerNorms (x = the sublayer output before its
// dropout).  Forward: y = LN(dropout(x) + res) (+ its bf16 copy y16 when y is fp32 and y16 != NULL).  Backward:
// gh = d/dx (through the mask), gres = d/dres (both 0 on pad rows), the dropout mask recomputed from (seed, salt).
static LnDrop ln_drop(float p, const int64_t* seed, unsigned salt) {
  LnDrop d;
  d.seed = seed;
  d.salt = salt;
  d.thr = (uint32_t)std::min(4294967295.0, (double)p * 4294967296.0);
  d.scale = 1.f / (1.f - p);
  return d;
}

extern "C" int vo_layernorm_drop(const void* x, int x_dtype, const void* res, int res_dtype, const float* gamma,
                                 const float* beta, const int32_t* lens, int B, int T, int D, float eps, void* y,
                                 int y_dtype, void* y16, float p, const int64_t* seed, unsigned salt, void* stream) {
  VO_CHECK_ARG(x && res && gamma && beta && y && seed, "layernorm_drop: null pointer");
  VO_CHECK_ARG(D == 256 || D == 512, "layernorm_drop: D=%d unsupported (256 or 512)", D);
  VO_CHECK_ARG(B > 0 && T > 0 && (int64_t)B * T * D < (1LL << 32), "layernorm_drop: empty or > 2^32 elements");
  VO_CHECK_ARG(p >= 0.f && p < 1.f, "layernorm_drop: p = %g outside [0, 1)", p);
  VO_CHECK_ARG(y16 == nullptr || (y_dtype == VO_F32 && y16 != y && y16 != x && y16 != res),
               "layernorm_drop: y16 needs an fp32 y and its own buffer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const LnDrop dr = ln_drop(p, seed, salt);
  if (y16) {
    if (x_dtype == VO_BF16 && res_dtype == VO_F32)
      return ln_launch<bf16_t, float, float, true>(x, res, gamma, beta, lens, B, T, D, eps, y, st, y16, dr);
    if (x_dtype == VO_F32 && res_dtype == VO_F32)
      return ln_launch<float, float, float, true>(x, res, gamma, beta, lens, B, T, D, eps, y, st, y16, dr);
  } else {
    if (x_dtype == VO_F32 && res_dtype == VO_F32 && y_dtype == VO_F32)
      return ln_launch<float, float, float>(x, res, gamma, beta, lens, B, T, D, eps, y, st, nullptr, dr);
    if (x_dtype == VO_BF16 && res_dtype == VO_BF16 && y_dtype == VO_BF16)
      return ln_launch<bf16_t, bf16_t, bf16_t>(x, res, gamma, beta, lens, B, T, D, eps, y, st, nullptr, dr);
    if (x_dtype == VO_BF16 && res_dtype == VO_F32 && y_dtype == VO_F32)
      return ln_launch<bf16_t, float, float>(x, res, gamma, beta, lens, B, T, D, eps, y, st, nullptr, dr);
  }
  vo_set_error("layernorm_drop: unsupported dtype combination");
  return VO_ERR_INVALID;
}

extern "C" int vo_layernorm_bwd_drop(const void* x, int x_dtype, const void* res, int res_dtype, const void* gy,
                                     int gy_dtype, const void* gy2, const float* gamma, const int32_t* lens, int B,
                                     int T, int D, float eps, float p, const int64_t* seed, unsigned salt, void* gh,
                                     void* gres, float* dgamma, float* dbeta, void* workspace, void* stream) {
  VO_CHECK_ARG(x && res && gy && gamma && gh && gres && dgamma && dbeta && workspace && seed,
               "layernorm_bwd_drop: null pointer");
  VO_CHECK_ARG(D == 256 || D == 512, "layernorm_bwd_drop: D=%d unsupported (256 or 512)", D);
  VO_CHECK_ARG(B > 0 && T > 0 && (int64_t)B * T * D < (1LL << 32), "layernorm_bwd_drop: empty or > 2^32 elements");
  VO_CHECK_ARG(p >= 0.f && p < 1.f, "layernorm_bwd_drop: p = %g outside [0, 1)", p);
  VO_CHECK_ARG(gres != gh && gres != x && gh != x, "layernorm_bwd_drop: outputs alias");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* ws = (float*)workspace;
  const LnDrop dr = ln_drop(p, seed, salt);
  if (x_dtype == VO_BF16 && res_dtype == VO_F32 && gy_dtype == VO_F32)
    return ln_bwd_launch<bf16_t, float, float>(x, res, gy, gamma, lens, B, T, D, eps, gh, dgamma, dbeta, ws, st, gy2,
                                               gres, dr);
  if (x_dtype == VO_BF16 && res_dtype == VO_F32 && gy_dtype == VO_BF16)
    return ln_bwd_launch<bf16_t, bf16_t, float>(x, res, gy, gamma, lens, B, T, D, eps, gh, dgamma, dbeta, ws, st, gy2,
                                                gres, dr);
  if (x_dtype == VO_F32 && res_dtype == VO_F32 && gy_dtype == VO_F32 && gy2 == nullptr)
    return ln_bwd_launch<float, float, float>(x, res, gy, gamma, lens, B, T, D, eps, gh, dgamma, dbeta, ws, st, nullptr,
                                              gres, dr);
  if (x_dtype == VO_BF16 && res_dtype == VO_BF16 && gy_dtype == VO_BF16 && gy2 == nullptr)
    return ln_bwd_launch<bf16_t, bf16_t, bf16_t>(x, res, gy, gamma, lens, B, T, D, eps, gh, dgamma, dbeta, ws, st,
                                                 nullptr, gres, dr);
  vo_set_error("layernorm_bwd_drop: unsupported dtype combination");
  return VO_ERR_INVALID;
}
