// Flash-style scaled-dot-product attention with key padding (no probability matrix).
//
// Replaces MultiHeadAttention's head split + ScaledDotProductAttention
// (scripts/transformer/SubLayers.py:39-53, scripts/transformer/Modules.py:14-25):
//   softmax((Q K^T) / sqrt(d_k), masked_fill(key >= len, -inf), dim = keys) V
// for H heads of d_k = 128 read straight out of the fused qkv projection (B, L, 3D).
//
// Workgroup = 4 waves = 64 queries of one (batch, head); each wave owns 16 query rows.
// Per 64-key tile: K staged row-major and V staged transposed in LDS (shared by the 4
// waves), S = Q K^T on MFMA (16 x 64 per wave), online softmax on the accumulator
// (row r of a lane group lives in register r, so the running max/sum and the O rescale
// need no lane movement beyond a 16-lane xor reduction), P through a per-wave LDS tile
// into the A operand of O += P V.

#include "vo_common.h"

namespace vo {

constexpr int ATT_DK = 128;
constexpr int KT = 64;  // keys per tile

template <typename TC>
__global__ void __launch_bounds__(256) attention_kernel(const TC* __restrict__ qkv, const int32_t* __restrict__ lens,
                                                        int L, int H, float scale, TC* __restrict__ out) {
  constexpr int KP = ATT_DK + 8;  // K tile pitch
  constexpr int VP = KT + 8;      // V^T tile pitch
  constexpr int PP = KT + 8;      // P tile pitch
  __shared__ __attribute__((aligned(16))) TC k_lds[KT * KP];
  __shared__ __attribute__((aligned(16))) TC vt_lds[ATT_DK * VP];
  __shared__ __attribute__((aligned(16))) TC p_lds[4][16 * PP];

  const int D = H * ATT_DK;
  const int bh = blockIdx.y;
  const int b = bh / H, h = bh - b * H;
  const int q0 = blockIdx.x * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4, lk = g * 8;
  const int len = lens ? lens[b] : L;
  const int64_t row_stride = 3 * (int64_t)D;
  const TC* base = qkv + (int64_t)b * L * row_stride;

  // Q fragments (A operand): row q = q0 + 16*wave + lr, dk = 32*ks + lk
  Frag<TC> qf[4];
  {
    const int q = q0 + 16 * wave + lr;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (q < L)
        qf[ks].load(base + (int64_t)q * row_stride + h * ATT_DK + 32 * ks + lk);
      else
        qf[ks].zero();
    }
  }

  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[4], l_run[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { m_run[r] = -INFINITY; l_run[r] = 0.f; }

  const int n_tiles = (min(len, L) + KT - 1) / KT;
  for (int kt = 0; kt < n_tiles; ++kt) {
    const int key0 = kt * KT;
    // stage K (row-major) and V (transposed): 64 keys x 128 dk = 1024 vectors of 8
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int v = tid + 256 * s;
      const int kr = v >> 4, c8 = (v & 15) * 8;
      const int key = key0 + kr;
      float kv[8], vv[8];
      if (key < L) {
        const TC* rp = base + (int64_t)key * row_stride + h * ATT_DK + c8;
        load8(rp + D, kv);
        load8(rp + 2 * D, vv);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) kv[e] = vv[e] = 0.f;
      }
      store8(k_lds + kr * KP + c8, kv);
#pragma unroll
      for (int e = 0; e < 8; ++e) vt_lds[(c8 + e) * VP + kr] = from_f32<TC>(vv[e]);
    }
    __syncthreads();

    // S = Q K^T  (16 q x 64 keys per wave)
    f32x4 s_acc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      s_acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        Frag<TC> kf;
        kf.load(k_lds + (16 * nt + lr) * KP + 32 * ks + lk);
        s_acc[nt] = mfma(qf[ks], kf, s_acc[nt]);
      }
    }
    // scale, mask, online softmax. lane holds S[q = 4g + r][key = 16 nt + lr]
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mx = -INFINITY;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int key = key0 + 16 * nt + lr;
        float sv = s_acc[nt][r] * scale;
        if (key >= len) sv = -INFINITY;
        s_acc[nt][r] = sv;
        mx = fmaxf(mx, sv);
      }
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, 64));
      const float m_new = fmaxf(m_run[r], mx);
      alpha[r] = (m_run[r] == -INFINITY) ? 0.f : __expf(m_run[r] - m_new);
      float sum = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const float p = (s_acc[nt][r] == -INFINITY) ? 0.f : __expf(s_acc[nt][r] - m_new);
        s_acc[nt][r] = p;
        sum += p;
      }
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) sum += __shfl_xor(sum, o2, 64);
      l_run[r] = l_run[r] * alpha[r] + sum;
      m_run[r] = m_new;
    }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[dt][r] *= alpha[r];
    // P -> LDS (per wave) in [q][key] order
    TC* pw = p_lds[wave];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) pw[(4 * g + r) * PP + 16 * nt + lr] = from_f32<TC>(s_acc[nt][r]);
    __syncthreads();
    // O += P V  : A = P[q = lr][key = 32 ks + lk + j], B = V[key][d = 16 dt + lr] = Vt[d][key]
    Frag<TC> pf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) pf[ks].load(pw + lr * PP + 32 * ks + lk);
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        Frag<TC> vf;
        vf.load(vt_lds + (16 * dt + lr) * VP + 32 * ks + lk);
        o[dt] = mfma(pf[ks], vf, o[dt]);
      }
    }
    __syncthreads();
  }

  // write O / l : lane holds O[q = 4g + r][d = 16 dt + lr]
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = q0 + 16 * wave + 4 * g + r;
    if (q >= L) continue;
    const float inv = l_run[r] > 0.f ? 1.0f / l_run[r] : 0.f;
    TC* orow = out + ((int64_t)b * L + q) * D + h * ATT_DK;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) orow[16 * dt + lr] = from_f32<TC>(o[dt][r] * inv);
  }
}

}  // namespace vo

using namespace vo;

extern "C" int vo_attention(const void* qkv, int dtype, const int32_t* lens, int B, int L, int H, int dk,
                            float scale, void* out, void* stream) {
  VO_CHECK_ARG(qkv && out, "attention: null pointer");
  VO_CHECK_ARG(dk == ATT_DK, "attention: d_k=%d unsupported (128)", dk);
  VO_CHECK_ARG(B > 0 && L > 0 && H > 0, "attention: empty");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((unsigned)((L + 63) / 64), (unsigned)(B * H));
  if (dtype == VO_BF16)
    hipLaunchKernelGGL(attention_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)qkv, lens, L, H, scale,
                       (bf16_t*)out);
  else if (dtype == VO_F32)
    hipLaunchKernelGGL(attention_kernel<float>, grid, dim3(256), 0, st, (const float*)qkv, lens, L, H, scale,
                       (float*)out);
  else {
    vo_set_error("attention: bad dtype");
    return VO_ERR_INVALID;
  }
  VO_RETURN_LAUNCH();
}
