// Flash-style backward of the key-padded scaled-dot-product attention (training, config C4).
//
// Replaces the PyTorch autograd recomputation of MultiHeadAttention's head split +
// ScaledDotProductAttention (scripts/transformer/SubLayers.py:39-53, Modules.py:14-25) under
// scripts/04_train.py:128-141.  With S = Q K^T * scale (keys >= len at -inf), P = softmax(S):
//   dV = P^T dO,  dP = dO V^T,  dS = P o (dP - rowsum(dO o O)),  dQ = dS K * scale,
//   dK = dS^T Q * scale
// Nothing of size L x L reaches HBM.  Two kernels, no atomics:
//   attn_bwd_dq_kernel   -- one workgroup per 64 queries of one (batch, head): pass 1 rebuilds
//                           the row log-sum-exp over the key tiles, pass 2 forms P, dP, dS and
//                           accumulates dQ; writes LSE and D = rowsum(dO o O) to the workspace.
//   attn_bwd_dkdv_kernel -- one workgroup per 64 keys: loops over query tiles in transposed
//                           form (S^T = K Q^T, dP^T = V dO^T; the key-side operands stay in
//                           registers) and accumulates dK, dV.
// The MFMA operand convention is the forward's (vo_common.h Frag / mfma): A = lane row lr,
// k = lk..lk+7; B = lane column lr, k = lk..lk+7; C = lane rows 4g + r, column lr.  P / dS
// go through a per-wave LDS tile to become A operands; the operands that need their
// reduction index along keys / queries are staged transposed in LDS.
// bf16 (P / dS rounded to bf16 as operands, fp32 accumulation) or fp32 (parity mode).

#include "vo_common.h"

namespace vo {

constexpr int AB_DK = 128;
constexpr int AB_KT = 64;  // keys per tile (dq kernel) / keys per workgroup (dkdv kernel)

// stage ROWS rows of 128 channels (channel offset `col` in rows of pitch `ld` starting at `row0`)
// row-major into dst (pitch AB_DK + 8) and, if dst_t, transposed into dst_t[c][row] (pitch TP)
template <typename TC, int ROWS, int TP>
__device__ __forceinline__ void ab_stage(const TC* __restrict__ src, int64_t ld, int row0, int nrows, int tid,
                                         TC* __restrict__ dst, TC* __restrict__ dst_t) {
  constexpr int P = AB_DK + 8;
#pragma unroll
  for (int s = 0; s < ROWS * 16 / 256; ++s) {
    const int v = tid + 256 * s;
    const int r = v >> 4, c8 = (v & 15) * 8;
    float x[8];
    if (row0 + r < nrows)
      load8(src + (int64_t)(row0 + r) * ld + c8, x);
    else
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = 0.f;
    if (dst) store8(dst + r * P + c8, x);
    if (dst_t)
#pragma unroll
      for (int e = 0; e < 8; ++e) dst_t[(c8 + e) * TP + r] = from_f32<TC>(x[e]);
  }
}

template <typename TC>
__global__ void __launch_bounds__(256) attn_bwd_dq_kernel(const TC* __restrict__ qkv, const TC* __restrict__ o,
                                                          const TC* __restrict__ dout,
                                                          const int32_t* __restrict__ lens, int L, int H,
                                                          float scale, TC* __restrict__ dqkv,
                                                          float* __restrict__ lse_ws, float* __restrict__ dd_ws,
                                                          int xcd) {
  constexpr int KP = AB_DK + 8;
  constexpr int TP = AB_KT + 8;
  __shared__ __attribute__((aligned(16))) TC k_lds[AB_KT * KP];
  __shared__ __attribute__((aligned(16))) TC v_lds[AB_KT * KP];
  __shared__ __attribute__((aligned(16))) TC kt_lds[AB_DK * TP];
  __shared__ __attribute__((aligned(16))) TC p_lds[4][16 * TP];
  __shared__ float dd_lds[4][16];

  const int D = H * AB_DK;
  // the query tiles of one (b, h) read the same K / V: consecutive logical ids, one XCD's L2
  const int nq = gridDim.x, wid = blockIdx.x + nq * blockIdx.y;
  const int lid = xcd ? xcd_grouped_id(wid, nq * gridDim.y) : wid;
  const int bh = lid / nq;
  const int b = bh / H, h = bh - b * H;
  const int q0 = (lid - bh * nq) * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4, lk = g * 8;
  const int len = lens ? min(lens[b], L) : L;
  const int64_t rs = 3 * (int64_t)D;
  const TC* base = qkv + (int64_t)b * L * rs;
  const TC* kbase = base + D + h * AB_DK;
  const TC* vbase = base + 2 * D + h * AB_DK;

  // Q and dO fragments (A operands: row q, k = channel), D = rowsum(dO o O)
  Frag<TC> qf[4], df[4];
  float dpart = 0.f;
  {
    const int q = q0 + 16 * wave + lr;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (q < L) {
        const int c = h * AB_DK + 32 * ks + lk;
        qf[ks].load(base + (int64_t)q * rs + c);
        df[ks].load(dout + ((int64_t)b * L + q) * D + c);
        float ov[8], dv[8];
        load8(o + ((int64_t)b * L + q) * D + c, ov);
        load8(dout + ((int64_t)b * L + q) * D + c, dv);
#pragma unroll
        for (int e = 0; e < 8; ++e) dpart += ov[e] * dv[e];
      } else {
        qf[ks].zero();
        df[ks].zero();
      }
    }
  }
  dpart += __shfl_xor(dpart, 16, 64);
  dpart += __shfl_xor(dpart, 32, 64);
  if (g == 0) dd_lds[wave][lr] = dpart;

  // pass 1: row max / sum over the key tiles -> log-sum-exp
  const int n_tiles = (len + AB_KT - 1) / AB_KT;
  float m_run[4], l_run[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m_run[r] = -INFINITY;
    l_run[r] = 0.f;
  }
  for (int kt = 0; kt < n_tiles; ++kt) {
    const int key0 = kt * AB_KT;
    __syncthreads();
    ab_stage<TC, AB_KT, TP>(kbase, rs, key0, L, tid, k_lds, (TC*)nullptr);
    __syncthreads();
    f32x4 s[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      s[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        Frag<TC> kf;
        kf.load(k_lds + (16 * nt + lr) * KP + 32 * ks + lk);
        s[nt] = mfma(qf[ks], kf, s[nt]);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mx = -INFINITY;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const float sv = (key0 + 16 * nt + lr < len) ? s[nt][r] * scale : -INFINITY;
        s[nt][r] = sv;
        mx = fmaxf(mx, sv);
      }
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, 64));
      const float m_new = fmaxf(m_run[r], mx);
      float sum = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) sum += (s[nt][r] == -INFINITY) ? 0.f : __expf(s[nt][r] - m_new);
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) sum += __shfl_xor(sum, o2, 64);
      l_run[r] = l_run[r] * ((m_run[r] == -INFINITY) ? 0.f : __expf(m_run[r] - m_new)) + sum;
      m_run[r] = m_new;
    }
  }
  float lse[4], ddr[4];
  __syncthreads();  // dd_lds visible
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    lse[r] = l_run[r] > 0.f ? m_run[r] + __logf(l_run[r]) : INFINITY;  // +inf: the row has no keys -> P = 0
    ddr[r] = dd_lds[wave][4 * g + r];
    const int q = q0 + 16 * wave + 4 * g + r;
    if (lr == 0 && q < L) {
      lse_ws[(int64_t)bh * L + q] = lse[r];
      dd_ws[(int64_t)bh * L + q] = ddr[r];
    }
  }

  // pass 2: P, dP, dS; dQ += dS K
  f32x4 acc[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  TC* pw = p_lds[wave];
  for (int kt = 0; kt < n_tiles; ++kt) {
    const int key0 = kt * AB_KT;
    __syncthreads();
    ab_stage<TC, AB_KT, TP>(kbase, rs, key0, L, tid, k_lds, kt_lds);
    ab_stage<TC, AB_KT, TP>(vbase, rs, key0, L, tid, v_lds, (TC*)nullptr);
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      s[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        Frag<TC> kf, vf;
        kf.load(k_lds + (16 * nt + lr) * KP + 32 * ks + lk);
        vf.load(v_lds + (16 * nt + lr) * KP + 32 * ks + lk);
        s[nt] = mfma(qf[ks], kf, s[nt]);
        dp[nt] = mfma(df[ks], vf, dp[nt]);
      }
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool valid = key0 + 16 * nt + lr < len;
        const float p = valid ? __expf(s[nt][r] * scale - lse[r]) : 0.f;
        pw[(4 * g + r) * TP + 16 * nt + lr] = from_f32<TC>(p * (dp[nt][r] - ddr[r]));
      }
    __syncthreads();
    Frag<TC> sf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) sf[ks].load(pw + lr * TP + 32 * ks + lk);
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        Frag<TC> kf;
        kf.load(kt_lds + (16 * dt + lr) * TP + 32 * ks + lk);
        acc[dt] = mfma(sf[ks], kf, acc[dt]);
      }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = q0 + 16 * wave + 4 * g + r;
    if (q >= L) continue;
    TC* row = dqkv + ((int64_t)b * L + q) * rs + h * AB_DK;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) row[16 * dt + lr] = from_f32<TC>(acc[dt][r] * scale);
  }
}

template <typename TC, int QT>
__global__ void __launch_bounds__(256) attn_bwd_dkdv_kernel(const TC* __restrict__ qkv, const TC* __restrict__ dout,
                                                            const int32_t* __restrict__ lens, int L, int H,
                                                            float scale, TC* __restrict__ dqkv,
                                                            const float* __restrict__ lse_ws,
                                                            const float* __restrict__ dd_ws, int xcd) {
  constexpr int NT = QT / 16, KS = QT / 32;
  constexpr int QP = AB_DK + 8;
  constexpr int TP = QT + 8;
  __shared__ __attribute__((aligned(16))) TC q_lds[QT * QP];
  __shared__ __attribute__((aligned(16))) TC do_lds[QT * QP];
  __shared__ __attribute__((aligned(16))) TC qt_lds[AB_DK * TP];
  __shared__ __attribute__((aligned(16))) TC dot_lds[AB_DK * TP];
  __shared__ __attribute__((aligned(16))) TC pt_lds[4][16 * TP];
  __shared__ __attribute__((aligned(16))) TC st_lds[4][16 * TP];
  __shared__ float lse_s[QT], dd_s[QT];

  const int D = H * AB_DK;
  // the key tiles of one (b, h) read the same Q / dO: consecutive logical ids, one XCD's L2
  const int nk = gridDim.x, wid = blockIdx.x + nk * blockIdx.y;
  const int lid = xcd ? xcd_grouped_id(wid, nk * gridDim.y) : wid;
  const int bh = lid / nk;
  const int b = bh / H, h = bh - b * H;
  const int k0 = (lid - bh * nk) * AB_KT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4, lk = g * 8;
  const int len = lens ? min(lens[b], L) : L;
  const int64_t rs = 3 * (int64_t)D;
  const TC* base = qkv + (int64_t)b * L * rs;

  f32x4 dk[8], dv[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (k0 < len) {  // workgroup-uniform: a tile of padded keys only gets zero gradients
    Frag<TC> kf[4], vf[4];
    {
      const int key = k0 + 16 * wave + lr;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        if (key < L) {
          kf[ks].load(base + (int64_t)key * rs + D + h * AB_DK + 32 * ks + lk);
          vf[ks].load(base + (int64_t)key * rs + 2 * D + h * AB_DK + 32 * ks + lk);
        } else {
          kf[ks].zero();
          vf[ks].zero();
        }
      }
    }
    TC* pw = pt_lds[wave];
    TC* sw = st_lds[wave];
    const TC* dob = dout + (int64_t)b * L * D + h * AB_DK;
    const int n_qt = (L + QT - 1) / QT;
    for (int qt = 0; qt < n_qt; ++qt) {
      const int qb = qt * QT;
      __syncthreads();
      ab_stage<TC, QT, TP>(base + h * AB_DK, rs, qb, L, tid, q_lds, qt_lds);
      ab_stage<TC, QT, TP>(dob, D, qb, L, tid, do_lds, dot_lds);
      if (tid < QT) {
        const int q = qb + tid;
        lse_s[tid] = q < L ? lse_ws[(int64_t)bh * L + q] : INFINITY;
        dd_s[tid] = q < L ? dd_ws[(int64_t)bh * L + q] : 0.f;
      }
      __syncthreads();
      // S^T = K Q^T, dP^T = V dO^T : lane holds [key = 4g + r][q = 16 nt + lr]
      f32x4 st[NT], dpt[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        st[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        dpt[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          Frag<TC> qf, df;
          qf.load(q_lds + (16 * nt + lr) * QP + 32 * ks + lk);
          df.load(do_lds + (16 * nt + lr) * QP + 32 * ks + lk);
          st[nt] = mfma(kf[ks], qf, st[nt]);
          dpt[nt] = mfma(vf[ks], df, dpt[nt]);
        }
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int qq = 16 * nt + lr;
        const float lq = lse_s[qq], dq = dd_s[qq];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool valid = k0 + 16 * wave + 4 * g + r < len;
          const float p = valid ? __expf(st[nt][r] * scale - lq) : 0.f;
          pw[(4 * g + r) * TP + qq] = from_f32<TC>(p);
          sw[(4 * g + r) * TP + qq] = from_f32<TC>(p * (dpt[nt][r] - dq));
        }
      }
      __syncthreads();
      // dV += P^T dO, dK += dS^T Q : A = [key = lr][q = 32 ks + lk], B = [d = 16 dt + lr][q]
      Frag<TC> pf[KS], sf[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        pf[ks].load(pw + lr * TP + 32 * ks + lk);
        sf[ks].load(sw + lr * TP + 32 * ks + lk);
      }
#pragma unroll
      for (int dt = 0; dt < 8; ++dt)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          Frag<TC> a, c;
          a.load(dot_lds + (16 * dt + lr) * TP + 32 * ks + lk);
          c.load(qt_lds + (16 * dt + lr) * TP + 32 * ks + lk);
          dv[dt] = mfma(pf[ks], a, dv[dt]);
          dk[dt] = mfma(sf[ks], c, dk[dt]);
        }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int key = k0 + 16 * wave + 4 * g + r;
    if (key >= L) continue;
    TC* row = dqkv + ((int64_t)b * L + key) * rs + h * AB_DK;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      row[D + 16 * dt + lr] = from_f32<TC>(dk[dt][r] * scale);
      row[2 * D + 16 * dt + lr] = from_f32<TC>(dv[dt][r]);
    }
  }
}

// ---------------------------------------------------------------------------------- bf16 version 2
// (round 5) The row log-sum-exp comes from the forward (vo_attention_lse: attention2_kernel writes it),
// so the dQ kernel has no first pass over the keys; and every product is formed transposed, as in
// attention2_kernel, so that no P / dS tile goes through LDS and no operand is staged transposed:
//   dQ kernel (64 queries): S^T = K Q^T, dP^T = V dO^T   (lane: key 16 nt + 4 g + r, query lr)
//                            dQ^T += K^T dS^T            (A = K^T by ds_read_tr16_b64 of row-major K;
//                                                          B = dS^T from the lane's own accumulators)
//   dK/dV kernel (64 keys):  S = Q K^T, dP = dO V^T     (lane: query 16 nt + 4 g + r, key lr)
//                            dV^T += dO^T P, dK^T += Q^T dS
// The 32-deep k-steps take the keys (queries) in the order a lane's two accumulator tiles hold them
// (k index 8 g + j <-> 32 ks + 4 g + j, j < 4; 32 ks + 16 + 4 g + j - 4, j >= 4), and the transposed
// reads use the same order -- exactly attention2_kernel's O^T += V^T P^T.  K / V (Q / dO) tiles are
// double-buffered in LDS, the next tile fetched into registers during the current one (one barrier).
constexpr int AB2_P = AB_DK + 16;  // LDS row pitch (elements): 72 dwords = 8 mod 64 banks

typedef unsigned int ab_u4 __attribute__((ext_vector_type(4)));
typedef short ab_v4s __attribute__((ext_vector_type(4)));
typedef short ab_v8s __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) ab_v4s ab_lds_v4s;

// A fragment of X^T (rows d = 16 dt + lane row, k = the 32 rows 32 ks .. of the row-major LDS tile X, in
// the accumulator order above)
__device__ __forceinline__ Frag<bf16_t> ab_tr_frag(const bf16_t* X, int ks, int dt, int g, int tq, int tp) {
  const bf16_t* vb = X + (32 * ks + 4 * g + tq) * AB2_P + 16 * dt + 4 * tp;
  const ab_v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ab_lds_v4s*)vb);
  const ab_v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ab_lds_v4s*)(vb + 16 * AB2_P));
  Frag<bf16_t> f;
  f.v = __builtin_bit_cast(bf16x8, (ab_v8s)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  return f;
}

// B fragment from two accumulator tiles (k-step ks: tiles 2 ks, 2 ks + 1)
__device__ __forceinline__ Frag<bf16_t> ab_acc_frag(const f32x4& a, const f32x4& b) {
  const ab_u4 w = ab_u4{pk_bf16(a[0], a[1]), pk_bf16(a[2], a[3]), pk_bf16(b[0], b[1]), pk_bf16(b[2], b[3])};
  Frag<bf16_t> f;
  f.v = __builtin_bit_cast(bf16x8, w);
  return f;
}

template <int NONE = 0>
__global__ void __launch_bounds__(256) attn2_bwd_dq_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ o,
                                                           const bf16_t* __restrict__ dout,
                                                           const int32_t* __restrict__ lens, int L, int H, float scale,
                                                           const float* __restrict__ lse, bf16_t* __restrict__ dqkv,
                                                           float* __restrict__ dd_ws, int xcd) {
  constexpr int P = AB2_P, KT = AB_KT;
  __shared__ __attribute__((aligned(16))) bf16_t kv_lds[2][2][KT * P];  // [buf][K | V][key][dk]
  const int D = H * AB_DK;
  const int nq = gridDim.x, wid = blockIdx.x + nq * blockIdx.y;
  const int lid = xcd ? xcd_grouped_id(wid, nq * gridDim.y) : wid;
  const int bh = lid / nq;
  const int b = bh / H, h = bh - b * H;
  const int q0 = (lid - bh * nq) * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4;
  const int len = min(lens ? lens[b] : L, L);
  const int64_t rs = 3 * (int64_t)D;
  const bf16_t* base = qkv + (int64_t)b * L * rs + h * AB_DK;

  // Q^T / dO^T fragments (B operands): lane (g, lr) holds X[q = q0 + 16 wave + lr][32 ks + 8 g + j]
  const int qrow = q0 + 16 * wave + lr;
  const bool qok = qrow < L;
  Frag<bf16_t> qf[4], df[4];
  float dpart = 0.f;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    if (qok) {
      const int64_t off = ((int64_t)b * L + qrow) * D + h * AB_DK + 32 * ks + 8 * g;
      qf[ks].load(base + (int64_t)qrow * rs + 32 * ks + 8 * g);
      df[ks].load(dout + off);
      float ov[8], dv[8];
      load8(o + off, ov);
      load8(dout + off, dv);
#pragma unroll
      for (int e = 0; e < 8; ++e) dpart += ov[e] * dv[e];
    } else {
      qf[ks].zero();
      df[ks].zero();
    }
  }
  dpart += __shfl_xor(dpart, 16, 64);
  dpart += __shfl_xor(dpart, 32, 64);  // D = rowsum(dO o O) of query lr, in all four lane groups
  const float ddr = dpart;
  const float lq = qok ? lse[(int64_t)bh * L + qrow] : INFINITY;
  if (qok && g == 0) dd_ws[(int64_t)bh * L + qrow] = ddr;

  ab_u4 kreg[4], vreg[4];
  auto fetch = [&](int key0) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int v = tid + 256 * s, kr = v >> 4, c8 = (v & 15) * 8;
      const int key = min(key0 + kr, L - 1);  // rows past L are masked by len <= L
      const bf16_t* rp = base + (int64_t)key * rs + c8;
      kreg[s] = *reinterpret_cast<const ab_u4*>(rp + D);
      vreg[s] = *reinterpret_cast<const ab_u4*>(rp + 2 * D);
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int v = tid + 256 * s, kr = v >> 4, c8 = (v & 15) * 8;
      *reinterpret_cast<ab_u4*>(&kv_lds[buf][0][kr * P + c8]) = kreg[s];
      *reinterpret_cast<ab_u4*>(&kv_lds[buf][1][kr * P + c8]) = vreg[s];
    }
  };

  f32x4 dq[8];  // dQ^T: lane (g, lr) holds dQ[q = lr][d = 16 dt + 4 g + r]
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int n_tiles = (len + KT - 1) / KT;
  if (n_tiles > 0) {
    fetch(0);
    stash(0);
  }
  __syncthreads();
  const int tq = lane >> 2 & 3, tp = lane & 3;
  for (int kt = 0; kt < n_tiles; ++kt) {
    const int buf = kt & 1, key0 = kt * KT;
    if (kt + 1 < n_tiles) fetch(key0 + KT);
    const bf16_t* K = kv_lds[buf][0];
    const bf16_t* V = kv_lds[buf][1];
    f32x4 st[4], dpt[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      st[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      dpt[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        Frag<bf16_t> kf, vf;
        kf.load(K + (16 * nt + lr) * P + 32 * ks + 8 * g);
        vf.load(V + (16 * nt + lr) * P + 32 * ks + 8 * g);
        st[nt] = mfma(kf, qf[ks], st[nt]);
        dpt[nt] = mfma(vf, df[ks], dpt[nt]);
      }
    }
    // dS^T = P^T o (dP^T - D), P^T = exp(S^T * scale - lse): lane's key 16 nt + 4 g + r, query lr
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool valid = key0 + 16 * nt + 4 * g + r < len;
        const float p = valid ? __expf(st[nt][r] * scale - lq) : 0.f;
        st[nt][r] = p * (dpt[nt][r] - ddr);
      }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const Frag<bf16_t> sf = ab_acc_frag(st[2 * ks], st[2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) dq[dt] = mfma(ab_tr_frag(K, ks, dt, g, tq, tp), sf, dq[dt]);
    }
    if (kt + 1 < n_tiles) stash(buf ^ 1);  // the other buffer was last read before the previous barrier
    __syncthreads();
  }
  if (!qok) return;
  bf16_t* row = dqkv + ((int64_t)b * L + qrow) * rs + h * AB_DK;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
    *reinterpret_cast<uint2*>(row + 16 * dt + 4 * g) =
        make_uint2(pk_bf16(dq[dt][0] * scale, dq[dt][1] * scale), pk_bf16(dq[dt][2] * scale, dq[dt][3] * scale));
}

template <int V = 0>  // V = 2: the per-element lse / D reads under the padded-key branch (A/B, att_cfg 2)
__global__ void __launch_bounds__(256) attn2_bwd_dkdv_kernel(const bf16_t* __restrict__ qkv,
                                                             const bf16_t* __restrict__ dout,
                                                             const int32_t* __restrict__ lens, int L, int H,
                                                             float scale, const float* __restrict__ lse,
                                                             const float* __restrict__ dd_ws, bf16_t* __restrict__ dqkv,
                                                             int xcd) {
  constexpr int P = AB2_P, QT = 64;
  __shared__ __attribute__((aligned(16))) bf16_t qd_lds[2][2][QT * P];  // [buf][Q | dO][query][dk]
  __shared__ __attribute__((aligned(16))) float ld_s[2][2][QT];        // [buf][lse | D][query]
  const int D = H * AB_DK;
  const int nk = gridDim.x, wid = blockIdx.x + nk * blockIdx.y;
  const int lid = xcd ? xcd_grouped_id(wid, nk * gridDim.y) : wid;
  const int bh = lid / nk;
  const int b = bh / H, h = bh - b * H;
  const int k0 = (lid - bh * nk) * AB_KT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4;
  const int len = min(lens ? lens[b] : L, L);
  const int64_t rs = 3 * (int64_t)D;
  const bf16_t* base = qkv + (int64_t)b * L * rs + h * AB_DK;
  const bf16_t* dob = dout + (int64_t)b * L * D + h * AB_DK;
  const int krow = k0 + 16 * wave + lr;

  f32x4 dk[8], dv[8];  // dK^T / dV^T: lane (g, lr) holds [key = lr][d = 16 dt + 4 g + r]
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (k0 < len) {  // workgroup-uniform: a tile of padded keys only gets zero gradients
    Frag<bf16_t> kf[4], vf[4];  // K / V of key krow (B operands): [32 ks + 8 g + j]
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (krow < L) {
        kf[ks].load(base + (int64_t)krow * rs + D + 32 * ks + 8 * g);
        vf[ks].load(base + (int64_t)krow * rs + 2 * D + 32 * ks + 8 * g);
      } else {
        kf[ks].zero();
        vf[ks].zero();
      }
    }
    const bool kok = krow < len;
    ab_u4 qreg[4], dreg[4];
    float lreg = 0.f, dsreg = 0.f;
    auto fetch = [&](int qb) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int v = tid + 256 * s, qr = v >> 4, c8 = (v & 15) * 8;
        const int q = min(qb + qr, L - 1);  // rows past L: P = 0 through lse = +inf below
        qreg[s] = *reinterpret_cast<const ab_u4*>(base + (int64_t)q * rs + c8);
        dreg[s] = *reinterpret_cast<const ab_u4*>(dob + (int64_t)q * D + c8);
      }
      if (tid < QT) {
        const int q = qb + tid;
        lreg = q < L ? lse[(int64_t)bh * L + q] : INFINITY;
        dsreg = q < L ? dd_ws[(int64_t)bh * L + q] : 0.f;
      }
    };
    auto stash = [&](int buf) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int v = tid + 256 * s, qr = v >> 4, c8 = (v & 15) * 8;
        *reinterpret_cast<ab_u4*>(&qd_lds[buf][0][qr * P + c8]) = qreg[s];
        *reinterpret_cast<ab_u4*>(&qd_lds[buf][1][qr * P + c8]) = dreg[s];
      }
      if (tid < QT) {
        ld_s[buf][0][tid] = lreg;
        ld_s[buf][1][tid] = dsreg;
      }
    };
    const int n_qt = (L + QT - 1) / QT;
    fetch(0);
    stash(0);
    __syncthreads();
    const int tq = lane >> 2 & 3, tp = lane & 3;
    for (int qt = 0; qt < n_qt; ++qt) {
      const int buf = qt & 1;
      if (qt + 1 < n_qt) fetch((qt + 1) * QT);
      const bf16_t* Q = qd_lds[buf][0];
      const bf16_t* dO = qd_lds[buf][1];
      f32x4 sc[4], dp[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        sc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          Frag<bf16_t> qf, df;
          qf.load(Q + (16 * nt + lr) * P + 32 * ks + 8 * g);
          df.load(dO + (16 * nt + lr) * P + 32 * ks + 8 * g);
          sc[nt] = mfma(qf, kf[ks], sc[nt]);
          dp[nt] = mfma(df, vf[ks], dp[nt]);
        }
      }
      // P = exp(S * scale - lse[q]), dS = P o (dP - D[q]): lane's query 16 nt + 4 g + r, key lr.  The
      // lane's four lse / D values per nt come as one 16-byte LDS read each and every exp is computed
      // before the padded-key select: `kok ? exp(.. ld_s ..) : 0` became a branch per element with its
      // own LDS read and lgkmcnt(0) wait -- 16 serialised LDS round trips per query tile
      if constexpr (V == 2) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int qq = 16 * nt + 4 * g + r;
            const float p = kok ? __expf(sc[nt][r] * scale - ld_s[buf][0][qq]) : 0.f;
            sc[nt][r] = p;
            dp[nt][r] = p * (dp[nt][r] - ld_s[buf][1][qq]);
          }
      }
#pragma unroll
      for (int nt = 0; nt < (V == 2 ? 0 : 4); ++nt) {
        const float4 lv = *reinterpret_cast<const float4*>(&ld_s[buf][0][16 * nt + 4 * g]);
        const float4 dv4 = *reinterpret_cast<const float4*>(&ld_s[buf][1][16 * nt + 4 * g]);
        const float lq4[4] = {lv.x, lv.y, lv.z, lv.w}, dq4[4] = {dv4.x, dv4.y, dv4.z, dv4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __expf(sc[nt][r] * scale - lq4[r]);
          const float p = kok ? e : 0.f;
          sc[nt][r] = p;
          dp[nt][r] = p * (dp[nt][r] - dq4[r]);
        }
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const Frag<bf16_t> pf = ab_acc_frag(sc[2 * ks], sc[2 * ks + 1]);
        const Frag<bf16_t> sf = ab_acc_frag(dp[2 * ks], dp[2 * ks + 1]);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          dv[dt] = mfma(ab_tr_frag(dO, ks, dt, g, tq, tp), pf, dv[dt]);
          dk[dt] = mfma(ab_tr_frag(Q, ks, dt, g, tq, tp), sf, dk[dt]);
        }
      }
      if (qt + 1 < n_qt) stash(buf ^ 1);
      __syncthreads();
    }
  }
  if (krow >= L) return;
  bf16_t* row = dqkv + ((int64_t)b * L + krow) * rs + h * AB_DK;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    *reinterpret_cast<uint2*>(row + D + 16 * dt + 4 * g) =
        make_uint2(pk_bf16(dk[dt][0] * scale, dk[dt][1] * scale), pk_bf16(dk[dt][2] * scale, dk[dt][3] * scale));
    *reinterpret_cast<uint2*>(row + 2 * D + 16 * dt + 4 * g) =
        make_uint2(pk_bf16(dv[dt][0], dv[dt][1]), pk_bf16(dv[dt][2], dv[dt][3]));
  }
}

}  // namespace vo

using namespace vo;

extern "C" int64_t vo_attention_bwd_workspace_size(int B, int L, int H) {
  return 2 * (int64_t)B * H * L * (int64_t)sizeof(float);
}

extern "C" int vo_attention_bwd(const void* qkv, const void* out, const void* dout, int dtype, const int32_t* lens,
                                int B, int L, int H, int dk, float scale, void* dqkv, void* workspace,
                                void* stream) {
  VO_CHECK_ARG(qkv && out && dout && dqkv && workspace, "attention_bwd: null pointer");
  VO_CHECK_ARG(dk == AB_DK, "attention_bwd: d_k=%d unsupported (128)", dk);
  VO_CHECK_ARG(B > 0 && L > 0 && H > 0, "attention_bwd: empty");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* lse = (float*)workspace;
  float* dd = lse + (int64_t)B * H * L;
  dim3 grid((unsigned)((L + 63) / 64), (unsigned)(B * H));
  const int xcd = vo_tune_get("att_xcd") != 1;  // att_xcd 1: plain (tile, head) order (A/B)
  if (dtype == VO_BF16) {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)qkv, (const bf16_t*)out,
                       (const bf16_t*)dout, lens, L, H, scale, (bf16_t*)dqkv, lse, dd, xcd);
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<bf16_t, 64>), grid, dim3(256), 0, st, (const bf16_t*)qkv,
                       (const bf16_t*)dout, lens, L, H, scale, (bf16_t*)dqkv, (const float*)lse, (const float*)dd, xcd);
  } else if (dtype == VO_F32) {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<float>, grid, dim3(256), 0, st, (const float*)qkv, (const float*)out,
                       (const float*)dout, lens, L, H, scale, (float*)dqkv, lse, dd, xcd);
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<float, 32>), grid, dim3(256), 0, st, (const float*)qkv,
                       (const float*)dout, lens, L, H, scale, (float*)dqkv, (const float*)lse, (const float*)dd, xcd);
  } else {
    vo_set_error("attention_bwd: bad dtype");
    return VO_ERR_INVALID;
  }
  VO_RETURN_LAUNCH();
}

// Backward with the forward's row log-sum-exp (vo_attention_lse): bf16 -> the version-2 kernels (no key
// pass to rebuild it); fp32 -> the version-1 kernels (which rebuild it; lse unused).  workspace:
// vo_attention_bwd_workspace_size(B, L, H) bytes.
extern "C" int vo_attention_bwd_lse(const void* qkv, const void* out, const void* dout, int dtype, const int32_t* lens,
                                    int B, int L, int H, int dk, float scale, const float* lse, void* dqkv,
                                    void* workspace, void* stream) {
  VO_CHECK_ARG(qkv && out && dout && dqkv && workspace && lse, "attention_bwd_lse: null pointer");
  VO_CHECK_ARG(dk == AB_DK, "attention_bwd_lse: d_k=%d unsupported (128)", dk);
  VO_CHECK_ARG(B > 0 && L > 0 && H > 0, "attention_bwd_lse: empty");
  if (dtype != VO_BF16 || vo_tune_get("att_cfg") == 1)  // att_cfg 1: the version-1 kernels (A/B)
    return vo_attention_bwd(qkv, out, dout, dtype, lens, B, L, H, dk, scale, dqkv, workspace, stream);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* dd = (float*)workspace;
  dim3 grid((unsigned)((L + 63) / 64), (unsigned)(B * H));
  const int xcd = vo_tune_get("att_xcd") != 1;
  hipLaunchKernelGGL(attn2_bwd_dq_kernel<0>, grid, dim3(256), 0, st, (const bf16_t*)qkv, (const bf16_t*)out,
                     (const bf16_t*)dout, lens, L, H, scale, lse, (bf16_t*)dqkv, dd, xcd);
  auto dkdv = vo_tune_get("att_cfg") == 2 ? attn2_bwd_dkdv_kernel<2> : attn2_bwd_dkdv_kernel<0>;
  hipLaunchKernelGGL(dkdv, grid, dim3(256), 0, st, (const bf16_t*)qkv, (const bf16_t*)dout, lens,
                     L, H, scale, lse, (const float*)dd, (bf16_t*)dqkv, xcd);
  VO_RETURN_LAUNCH();
}
