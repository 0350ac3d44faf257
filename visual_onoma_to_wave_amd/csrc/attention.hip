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
                                                        int L, int H, float scale, TC* __restrict__ out, int xcd,
                                                        float* __restrict__ lse) {
  constexpr int KP = ATT_DK + 8;  // K tile pitch
  constexpr int VP = KT + 8;      // V^T tile pitch
  constexpr int PP = KT + 8;      // P tile pitch
  __shared__ __attribute__((aligned(16))) TC k_lds[KT * KP];
  __shared__ __attribute__((aligned(16))) TC vt_lds[ATT_DK * VP];
  __shared__ __attribute__((aligned(16))) TC p_lds[4][16 * PP];

  const int D = H * ATT_DK;
  // the query tiles of one (b, h) read the same K / V: consecutive logical ids, one XCD's L2
  const int nq = gridDim.x, wid = blockIdx.x + nq * blockIdx.y;
  const int lid = xcd ? xcd_grouped_id(wid, nq * gridDim.y) : wid;
  const int bh = lid / nq;
  const int b = bh / H, h = bh - b * H;
  const int q0 = (lid - bh * nq) * 64;
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
    if (lse && lr == 0) lse[(int64_t)bh * L + q] = l_run[r] > 0.f ? m_run[r] + __logf(l_run[r]) : INFINITY;
    const float inv = l_run[r] > 0.f ? 1.0f / l_run[r] : 0.f;
    TC* orow = out + ((int64_t)b * L + q) * D + h * ATT_DK;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) orow[16 * dt + lr] = from_f32<TC>(o[dt][r] * inv);
  }
}

// bf16 version 2: S^T = K Q^T instead of S = Q K^T, so a lane's accumulator column is ONE
// query (lane & 15) over 16 keys: the running max / sum are per lane, the O^T rescale is a
// per-lane scalar, and P^T feeds the B operand of O^T += V^T P^T straight from registers (the
// keys of a 32-deep k-step taken in the order the accumulator holds them; the V^T operand is
// read with the same key order by two ds_read_b64_tr_b16 per fragment from row-major V) -- no P
// round trip through LDS, no transposed scalar V stores.  K / V tiles are double-buffered:
// the next tile is fetched into registers while the current one is consumed (one barrier per
// tile).
template <int NONE = 0>
__global__ void __launch_bounds__(256) attention2_kernel(const bf16_t* __restrict__ qkv, const int32_t* __restrict__ lens,
                                                         int L, int H, float scale, bf16_t* __restrict__ out,
                                                         int xcd, float* __restrict__ lse) {
  constexpr int P = ATT_DK + 16;  // row pitch (elements): 72 dwords = 8 mod 64 banks
  __shared__ __attribute__((aligned(16))) bf16_t kv_lds[2][2][KT * P];  // [buf][K | V][key][dk]
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  typedef short v4s __attribute__((ext_vector_type(4)));
  typedef short v8s __attribute__((ext_vector_type(8)));
  typedef __attribute__((address_space(3))) v4s lds_v4s;

  const int D = H * ATT_DK;
  // the query tiles of one (b, h) read the same K / V: consecutive logical ids, one XCD's L2
  const int nq = gridDim.x, wid = blockIdx.x + nq * blockIdx.y;
  const int lid = xcd ? xcd_grouped_id(wid, nq * gridDim.y) : wid;
  const int bh = lid / nq;
  const int b = bh / H, h = bh - b * H;
  const int q0 = (lid - bh * nq) * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4;
  const int len = min(lens ? lens[b] : L, L);
  const int64_t row_stride = 3 * (int64_t)D;
  const bf16_t* base = qkv + (int64_t)b * L * row_stride + h * ATT_DK;

  // Q^T fragments (B operand): lane (g, lr) holds Q[q = q0 + 16 wave + lr][dk = 32 ks + 8 g + j]
  Frag<bf16_t> qf[4];
  const int qrow = q0 + 16 * wave + lr;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    if (qrow < L)
      qf[ks].load(base + (int64_t)qrow * row_stride + 32 * ks + 8 * g);
    else
      qf[ks].zero();
  }

  // staging: 64 keys x 128 dk = 1024 16-byte vectors per matrix, 4 per thread
  u4 kreg[4], vreg[4];
  auto fetch = [&](int key0) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int v = tid + 256 * s, kr = v >> 4, c8 = (v & 15) * 8;
      const int key = min(key0 + kr, L - 1);  // rows past L are masked by len <= L
      const bf16_t* rp = base + (int64_t)key * row_stride + c8;
      kreg[s] = *reinterpret_cast<const u4*>(rp + D);
      vreg[s] = *reinterpret_cast<const u4*>(rp + 2 * D);
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int v = tid + 256 * s, kr = v >> 4, c8 = (v & 15) * 8;
      *reinterpret_cast<u4*>(&kv_lds[buf][0][kr * P + c8]) = kreg[s];
      *reinterpret_cast<u4*>(&kv_lds[buf][1][kr * P + c8]) = vreg[s];
    }
  };

  f32x4 o[8];  // O^T: lane (g, lr) holds O[q = lr][d = 16 dt + 4 g + r]
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  const int n_tiles = (len + KT - 1) / KT;
  if (n_tiles > 0) {
    fetch(0);
    stash(0);
  }
  __syncthreads();
  const int tq = lane >> 2 & 3, tp = lane & 3;  // transposed-read lane roles within 16 lanes
  for (int kt = 0; kt < n_tiles; ++kt) {
    const int buf = kt & 1;
    const int key0 = kt * KT;
    if (kt + 1 < n_tiles) fetch(key0 + KT);
    const bf16_t* K = kv_lds[buf][0];
    const bf16_t* V = kv_lds[buf][1];
    // S^T = K Q^T: 64 keys x 16 queries; s[nt] lane (g, lr): key 16 nt + 4 g + r, query lr
    f32x4 sacc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      sacc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        Frag<bf16_t> kf;
        kf.load(K + (16 * nt + lr) * P + 32 * ks + 8 * g);
        sacc[nt] = mfma(kf, qf[ks], sacc[nt]);
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = key0 + 16 * nt + 4 * g + r;
        const float sv = key < len ? sacc[nt][r] * scale : -INFINITY;
        sacc[nt][r] = sv;
        mx = fmaxf(mx, sv);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = m_run == -INFINITY ? 0.f : __expf(m_run - m_new);
    float sum = 0.f;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = sacc[nt][r] == -INFINITY ? 0.f : __expf(sacc[nt][r] - m_new);
        sacc[nt][r] = pv;
        sum += pv;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    l_run = l_run * alpha + sum;
    m_run = m_new;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[dt][r] *= alpha;
    // O^T += V^T P^T over two 32-key steps; k index 8 g + j <-> key 32 ks + 4 g + j (j < 4),
    // 32 ks + 16 + 4 g + j - 4 (j >= 4): exactly the keys this lane's sacc[2 ks], sacc[2 ks + 1] hold
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // whole-vector bit cast of packed words (per-element __bf16 inserts are mis-lowered by hipcc)
      auto pk = [](float lo, float hi) {
        return (unsigned)pk_bf16(lo, hi);
      };
      const u4 pw = u4{pk(sacc[2 * ks][0], sacc[2 * ks][1]), pk(sacc[2 * ks][2], sacc[2 * ks][3]),
                       pk(sacc[2 * ks + 1][0], sacc[2 * ks + 1][1]), pk(sacc[2 * ks + 1][2], sacc[2 * ks + 1][3])};
      Frag<bf16_t> pf;
      pf.v = __builtin_bit_cast(bf16x8, pw);
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        const bf16_t* vb = V + (32 * ks + 4 * g + tq) * P + 16 * dt + 4 * tp;
        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)vb);
        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(vb + 16 * P));
        Frag<bf16_t> vf;
        vf.v = __builtin_bit_cast(bf16x8, (v8s)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        o[dt] = mfma(vf, pf, o[dt]);
      }
    }
    if (kt + 1 < n_tiles) stash(buf ^ 1);  // the other buffer was last read before the previous barrier
    __syncthreads();
  }

  if (qrow >= L) return;
  // the row log-sum-exp for the backward (vo_attention_bwd_lse): +inf for a row with no key (P = 0)
  if (lse && g == 0) lse[(int64_t)bh * L + qrow] = l_run > 0.f ? m_run + __logf(l_run) : INFINITY;
  const float inv = l_run > 0.f ? 1.0f / l_run : 0.f;
  bf16_t* orow = out + ((int64_t)b * L + qrow) * D + h * ATT_DK;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    uint32_t w0 = pk_bf16(o[dt][0] * inv, o[dt][1] * inv);
    uint32_t w1 = pk_bf16(o[dt][2] * inv, o[dt][3] * inv);
    *reinterpret_cast<uint2*>(orow + 16 * dt + 4 * g) = make_uint2(w0, w1);
  }
}

}  // namespace vo

using namespace vo;

static int attention_launch(const void* qkv, int dtype, const int32_t* lens, int B, int L, int H, int dk,
                            float scale, void* out, float* lse, void* stream) {
  VO_CHECK_ARG(qkv && out, "attention: null pointer");
  VO_CHECK_ARG(dk == ATT_DK, "attention: d_k=%d unsupported (128)", dk);
  VO_CHECK_ARG(B > 0 && L > 0 && H > 0, "attention: empty");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((unsigned)((L + 63) / 64), (unsigned)(B * H));
  const int xcd = vo_tune_get("att_xcd") != 1;  // att_xcd 1: plain (tile, head) order (A/B)
  if (dtype == VO_BF16 && vo_tune_get("att_cfg") != 1)
    hipLaunchKernelGGL(attention2_kernel<0>, grid, dim3(256), 0, st, (const bf16_t*)qkv, lens, L, H, scale,
                       (bf16_t*)out, xcd, lse);
  else if (dtype == VO_BF16)
    hipLaunchKernelGGL(attention_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)qkv, lens, L, H, scale,
                       (bf16_t*)out, xcd, lse);
  else if (dtype == VO_F32)
    hipLaunchKernelGGL(attention_kernel<float>, grid, dim3(256), 0, st, (const float*)qkv, lens, L, H, scale,
                       (float*)out, xcd, lse);
  else {
    vo_set_error("attention: bad dtype");
    return VO_ERR_INVALID;
  }
  VO_RETURN_LAUNCH();
}

extern "C" int vo_attention(const void* qkv, int dtype, const int32_t* lens, int B, int L, int H, int dk,
                            float scale, void* out, void* stream) {
  return attention_launch(qkv, dtype, lens, B, L, H, dk, scale, out, nullptr, stream);
}

extern "C" int vo_attention_lse(const void* qkv, int dtype, const int32_t* lens, int B, int L, int H, int dk,
                                float scale, void* out, float* lse, void* stream) {
  VO_CHECK_ARG(lse, "attention_lse: null lse");
  return attention_launch(qkv, dtype, lens, B, L, H, dk, scale, out, lse, stream);
}
