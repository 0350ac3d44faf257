// Training-step glue that round 1 left on PyTorch-ROCm (config C4 / C5 backward):
//
//  * BatchNorm with batch statistics over channels-last rows (x: M rows x C channels), forward
//    (Welford partials per row block merged in a fixed order -> mean / biased var, the running
//    statistics update of nn.BatchNorm*, normalize + affine) and backward
//    (dx = g rstd (dy - mean(dy) - xhat mean(dy xhat)), dgamma = sum dy xhat, dbeta = sum dy):
//    PostNet's BatchNorm1d on (B, T, C) activations (scripts/transformer/Layers.py:67-137) and the
//    glyph encoder's single-channel BatchNorm2d (scripts/model/visual_feature_extractor.py:40-47,
//    C = 1: rows = every pixel);
//  * the glyph encoder's 1 -> 1 channel 3 x 3 Conv2d (pad 1) forward and backward (input, weight
//    and bias gradients; the weight / bias sums as per-block partials added in a fixed order);
//  * the backward of the HiFi-GAN training log-mel (vo_stft_mel_ex with mag_eps): per frame the
//    forward spectrum is recomputed, dL/d|X| = fb (g / melsum) on the bins whose mel sum passed the
//    log floor, dX = dL/d|X| X / |X|, the one-sided inverse DFT of dX (a 1024-point complex FFT
//    in LDS) times the window gives the frame gradient; a second kernel gathers the (<= n_fft / hop)
//    overlapping frames and the reflect-padded mirror positions of every sample in a fixed order.
// Everything deterministic (no atomics).

#include <algorithm>

#include "vo_common.h"

namespace vo {

// ------------------------------------------------------------------------------- BatchNorm

struct Welford {
  float n, mean, m2;
};

__device__ __forceinline__ Welford wf_merge(Welford a, Welford b) {
  if (b.n == 0.f) return a;
  if (a.n == 0.f) return b;
  const float n = a.n + b.n;
  const float d = b.mean - a.mean;
  const float fb = b.n / n;
  return Welford{n, a.mean + d * fb, a.m2 + b.m2 + d * d * a.n * fb};
}

// block: 256 threads = CT channels x (256 / CT) row lanes; rows [blockIdx.x * RB, +RB)
template <typename TX, int CT>
__global__ void __launch_bounds__(256) bn_stats_kernel(const TX* __restrict__ x, int M, int C, int RB,
                                                       float* __restrict__ part) {
  constexpr int RS = 256 / CT;
  __shared__ float sn[256], sm[256], s2[256];
  const int tid = threadIdx.x;
  const int cl = tid % CT, rl = tid / CT;
  const int c = blockIdx.y * CT + cl;
  const int r0 = blockIdx.x * RB;
  const int r1 = min(r0 + RB, M);
  Welford w{0.f, 0.f, 0.f};
  if (c < C) {
    for (int r = r0 + rl; r < r1; r += RS) {
      const float v = to_f32(x[(int64_t)r * C + c]);
      w.n += 1.f;
      const float d = v - w.mean;
      w.mean += d / w.n;
      w.m2 += d * (v - w.mean);
    }
  }
  sn[tid] = w.n; sm[tid] = w.mean; s2[tid] = w.m2;
  __syncthreads();
  if (rl == 0 && c < C) {
    for (int k = 1; k < RS; ++k) w = wf_merge(w, Welford{sn[k * CT + cl], sm[k * CT + cl], s2[k * CT + cl]});
    float* p = part + ((int64_t)blockIdx.x * C + c) * 3;
    p[0] = w.n; p[1] = w.mean; p[2] = w.m2;
  }
}

// per channel: merge the row-block partials in order; mean / rstd for the normalisation and the
// backward; running statistics: (1 - m) r + m stat, the variance unbiased (n / (n - 1))
__global__ void bn_finalize_kernel(const float* __restrict__ part, int nb, int C, float eps, float momentum,
                                   float* __restrict__ mean_rstd, float* __restrict__ run_mean,
                                   float* __restrict__ run_var, int64_t* __restrict__ nbt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt) nbt[0] += 1;
  if (c >= C) return;
  Welford w{0.f, 0.f, 0.f};
  for (int b = 0; b < nb; ++b) {
    const float* p = part + ((int64_t)b * C + c) * 3;
    w = wf_merge(w, Welford{p[0], p[1], p[2]});
  }
  const float var = w.n > 0.f ? w.m2 / w.n : 0.f;
  mean_rstd[c] = w.mean;
  mean_rstd[C + c] = rsqrtf(var + eps);
  if (run_mean) {
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * w.mean;
    const float unb = w.n > 1.f ? w.m2 / (w.n - 1.f) : var;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
  }
}

template <typename TX>
__global__ void __launch_bounds__(256) bn_apply_kernel(const TX* __restrict__ x, int64_t total, int C,
                                                       const float* __restrict__ mean_rstd,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       TX* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    float v = (to_f32(x[i]) - mean_rstd[c]) * mean_rstd[C + c];
    if (gamma) v = v * gamma[c] + beta[c];
    y[i] = from_f32<TX>(v);
  }
}

// backward partial sums per row block: [sum dy, sum dy * xhat] per channel
template <typename TX, typename TG, int CT>
__global__ void __launch_bounds__(256) bn_bwd_stats_kernel(const TX* __restrict__ x, const TG* __restrict__ dy,
                                                           int M, int C, int RB, const float* __restrict__ mean_rstd,
                                                           float* __restrict__ part) {
  constexpr int RS = 256 / CT;
  __shared__ float sa[256], sb[256];
  const int tid = threadIdx.x;
  const int cl = tid % CT, rl = tid / CT;
  const int c = blockIdx.y * CT + cl;
  const int r0 = blockIdx.x * RB;
  const int r1 = min(r0 + RB, M);
  float a = 0.f, bsum = 0.f;
  if (c < C) {
    const float mu = mean_rstd[c], rs = mean_rstd[C + c];
    for (int r = r0 + rl; r < r1; r += RS) {
      const int64_t i = (int64_t)r * C + c;
      const float g = to_f32(dy[i]);
      a += g;
      bsum += g * (to_f32(x[i]) - mu) * rs;
    }
  }
  sa[tid] = a; sb[tid] = bsum;
  __syncthreads();
  if (rl == 0 && c < C) {
    for (int k = 1; k < RS; ++k) {
      a += sa[k * CT + cl];
      bsum += sb[k * CT + cl];
    }
    float* p = part + ((int64_t)blockIdx.x * C + c) * 2;
    p[0] = a; p[1] = bsum;
  }
}

__global__ void bn_bwd_finalize_kernel(const float* __restrict__ part, int nb, int C, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float a = 0.f, b = 0.f;
  for (int k = 0; k < nb; ++k) {
    a += part[((int64_t)k * C + c) * 2];
    b += part[((int64_t)k * C + c) * 2 + 1];
  }
  dbeta[c] = a;
  dgamma[c] = b;
}

template <typename TX, typename TG>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const TX* __restrict__ x, const TG* __restrict__ dy,
                                                           int64_t total, int C, float inv_m,
                                                           const float* __restrict__ mean_rstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ dgamma,
                                                           const float* __restrict__ dbeta, TX* __restrict__ dx) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    const float rs = mean_rstd[C + c];
    const float xh = (to_f32(x[i]) - mean_rstd[c]) * rs;
    const float g = gamma ? gamma[c] : 1.f;
    const float v = g * rs * (to_f32(dy[i]) - dbeta[c] * inv_m - xh * dgamma[c] * inv_m);
    dx[i] = from_f32<TX>(v);
  }
}

// ---- vectorised BatchNorm (16-byte vectors: 8 bf16 / 4 fp32 channels per lane).  The scalar kernels
// above read 2-4 bytes per lane and run a division per element (Welford) and serial partial merges:
// at PostNet's 16384 x 512 bf16 a forward took 71 us and a backward 75 us (C4 trace, round 5).  Here
// each lane sums (v - k) and (v - k)^2 against the first value it read (k), converted to a Welford
// triple once; the row lanes of a block, the blocks and (FLAT: C = 1, every element one channel) the
// lanes of a vector merge in a fixed order, so results stay deterministic.
template <typename TX> struct BnVec;
template <> struct BnVec<float> {
  static constexpr int V = 4;
  __device__ static __forceinline__ void load(const float* p, float (&v)[4]) {
    const float4 u = *reinterpret_cast<const float4*>(p);
    v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w;
  }
  __device__ static __forceinline__ void store(float* p, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct BnVec<bf16_t> {
  static constexpr int V = 8;
  __device__ static __forceinline__ void load(const bf16_t* p, float (&v)[8]) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ static __forceinline__ void store(bf16_t* p, const float (&v)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = pk_bf16(v[2 * i], v[2 * i + 1]);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};

constexpr int BN_NB = 128;  // row blocks (partials per channel) of the vectorised kernels
constexpr int BN_CMAX = 2048;  // channels of the vectorised kernels (C / V <= 256 vector columns)

// part[block][c] = (n, mean, m2).  Non-FLAT: CV = C / V vector columns, RL = 256 / CV row lanes, rows
// [blockIdx.x RB, +RB) of M.  FLAT (C = 1): the M elements as M / V rows of one vector.
template <typename TX, bool FLAT>
__global__ void __launch_bounds__(256) bn_stats_v_kernel(const TX* __restrict__ x, int rows, int C, int RB,
                                                         float* __restrict__ part) {
  using VT = BnVec<TX>;
  constexpr int V = VT::V;
  __shared__ float sn[256], sm[256 * V], s2[256 * V];
  const int CV = FLAT ? 1 : C / V, RL = 256 / CV;
  const int tid = threadIdx.x, vc = tid % CV, rl = tid / CV;
  const int r0 = blockIdx.x * RB, r1 = min(r0 + RB, rows);
  float k[V], a1[V], a2[V];
  int n = 0;
#pragma unroll
  for (int e = 0; e < V; ++e) k[e] = a1[e] = a2[e] = 0.f;
  if (rl < RL && r0 + rl < r1) {
    VT::load(x + ((int64_t)(r0 + rl) * CV + vc) * V, k);
    for (int r = r0 + rl; r < r1; r += RL) {
      float v[V];
      VT::load(x + ((int64_t)r * CV + vc) * V, v);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float d = v[e] - k[e];
        a1[e] += d;
        a2[e] = fmaf(d, d, a2[e]);
      }
      ++n;
    }
  }
  // the lane's Welford triple per vector element
  const float fn = (float)n, inv = n ? 1.f / fn : 0.f;
  if (FLAT) {  // merge the V elements (one channel) in order
    Welford w{0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < V; ++e) w = wf_merge(w, Welford{fn, k[e] + a1[e] * inv, a2[e] - a1[e] * a1[e] * inv});
    sn[tid] = w.n; sm[tid] = w.mean; s2[tid] = w.m2;
    __syncthreads();
    for (int h = 128; h >= 1; h >>= 1) {  // pairwise tree over the 256 lanes (fixed order)
      if (tid < h) {
        const Welford m = wf_merge(Welford{sn[tid], sm[tid], s2[tid]}, Welford{sn[tid + h], sm[tid + h], s2[tid + h]});
        sn[tid] = m.n; sm[tid] = m.mean; s2[tid] = m.m2;
      }
      __syncthreads();
    }
    if (tid == 0) {
      float* p = part + (int64_t)blockIdx.x * 3;
      p[0] = sn[0]; p[1] = sm[0]; p[2] = s2[0];
    }
    return;
  }
  sn[tid] = fn;
#pragma unroll
  for (int e = 0; e < V; ++e) {
    sm[tid * V + e] = k[e] + a1[e] * inv;
    s2[tid * V + e] = a2[e] - a1[e] * a1[e] * inv;
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {  // channel c = vector column c / V, element c % V: merge the row lanes
    const int cv = c / V, e = c % V;
    Welford w{0.f, 0.f, 0.f};
    for (int l = 0; l < RL; ++l) {
      const int t = l * CV + cv;
      w = wf_merge(w, Welford{sn[t], sm[t * V + e], s2[t * V + e]});
    }
    float* p = part + ((int64_t)blockIdx.x * C + c) * 3;
    p[0] = w.n; p[1] = w.mean; p[2] = w.m2;
  }
}

// finalize: 8 lanes per channel, lane s merging partials s, s + 8, .. (loads issued ahead), then the 8
// lane results merged in lane order -- a fixed order (deterministic).  One lane walking all 128
// partials took 17 us (serial merges with a division each, behind one load latency per step).
constexpr int BN_FL = 8;
__global__ void __launch_bounds__(256) bn_finalize_v_kernel(const float* __restrict__ part, int nb, int C, float eps,
                                                            float momentum, float* __restrict__ mean_rstd,
                                                            float* __restrict__ run_mean, float* __restrict__ run_var,
                                                            int64_t* __restrict__ nbt) {
  __shared__ float sn[256], sm[256], s2[256];
  const int tid = threadIdx.x, sl = tid % BN_FL;
  const int c = blockIdx.x * (256 / BN_FL) + tid / BN_FL;
  if (blockIdx.x == 0 && tid == 0 && nbt) nbt[0] += 1;
  Welford w{0.f, 0.f, 0.f};
  if (c < C) {
    for (int b0 = sl; b0 < nb; b0 += 4 * BN_FL) {
      float q[4][3];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = min(b0 + i * BN_FL, nb - 1);
        const float* p = part + ((int64_t)b * C + c) * 3;
        q[i][0] = p[0]; q[i][1] = p[1]; q[i][2] = p[2];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (b0 + i * BN_FL < nb) w = wf_merge(w, Welford{q[i][0], q[i][1], q[i][2]});
    }
  }
  sn[tid] = w.n; sm[tid] = w.mean; s2[tid] = w.m2;
  __syncthreads();
  if (sl != 0 || c >= C) return;
  for (int k = 1; k < BN_FL; ++k) w = wf_merge(w, Welford{sn[tid + k], sm[tid + k], s2[tid + k]});
  const float var = w.n > 0.f ? w.m2 / w.n : 0.f;
  mean_rstd[c] = w.mean;
  mean_rstd[C + c] = rsqrtf(var + eps);
  if (run_mean) {
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * w.mean;
    const float unb = w.n > 1.f ? w.m2 / (w.n - 1.f) : var;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
  }
}

// apply: the grid's thread count is a multiple of CV (the launcher rounds it), so a thread's vector
// column -- and its channels' parameters, loaded once -- stays the same over the grid-stride loop
// (per-element parameter loads, 8 channels 32 bytes apart per lane, ran the kernel at 59 us)
template <typename TX, bool FLAT>
__global__ void __launch_bounds__(256) bn_apply_v_kernel(const TX* __restrict__ x, int nvec, int C,
                                                         const float* __restrict__ mean_rstd,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, TX* __restrict__ y) {
  using VT = BnVec<TX>;
  constexpr int V = VT::V;
  const int CV = FLAT ? 1 : C / V;
  const int i0 = blockIdx.x * 256 + threadIdx.x;
  const int c0 = FLAT ? 0 : (i0 % CV) * V;
  // the block's copy of the per-channel parameters (coalesced), then 8 consecutive per thread from LDS
  // (each thread loading its own 8-channel run from global was the kernel's cost: 32 scattered loads)
  __shared__ float sp[4][BN_CMAX];
  for (int c = threadIdx.x; c < C; c += 256) {
    sp[0][c] = mean_rstd[c]; sp[1][c] = mean_rstd[C + c];
    sp[2][c] = gamma ? gamma[c] : 1.f; sp[3][c] = gamma ? beta[c] : 0.f;
  }
  __syncthreads();
  float mu[V], rs[V], ga[V], be[V];
#pragma unroll
  for (int e = 0; e < V; ++e) {
    const int c = FLAT ? 0 : c0 + e;
    mu[e] = sp[0][c]; rs[e] = sp[1][c]; ga[e] = sp[2][c]; be[e] = sp[3][c];
  }
  // four vectors in flight per thread (one load, wait, compute, store at a time ran at 0.9 TB/s)
  const int stride = gridDim.x * 256;
  for (int i = i0; i < nvec; i += 4 * stride) {
    float v[4][V];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * stride < nvec) VT::load(x + (int64_t)(i + u * stride) * V, v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float t = (v[u][e] - mu[e]) * rs[e];
        v[u][e] = gamma ? t * ga[e] + be[e] : t;
      }
      if (i + u * stride < nvec) VT::store(y + (int64_t)(i + u * stride) * V, v[u]);
    }
  }
}

// backward partials per row block: part[block][c] = (sum dy, sum dy xhat)
template <typename TX, typename TG, bool FLAT>
__global__ void __launch_bounds__(256) bn_bwd_stats_v_kernel(const TX* __restrict__ x, const TG* __restrict__ dy,
                                                             int rows, int C, int RB,
                                                             const float* __restrict__ mean_rstd,
                                                             float* __restrict__ part) {
  constexpr int V = BnVec<TX>::V;
  static_assert(BnVec<TG>::V >= V, "dy vector at least as wide as x's");
  __shared__ float sa[256 * V], sb[256 * V];
  const int CV = FLAT ? 1 : C / V, RL = 256 / CV;
  const int tid = threadIdx.x, vc = tid % CV, rl = tid / CV;
  const int r0 = blockIdx.x * RB, r1 = min(r0 + RB, rows);
  float mu[V], rs[V], a[V], b[V];
#pragma unroll
  for (int e = 0; e < V; ++e) {
    const int c = FLAT ? 0 : vc * V + e;
    mu[e] = mean_rstd[c]; rs[e] = mean_rstd[C + c];
    a[e] = b[e] = 0.f;
  }
  if (rl < RL)
    for (int r = r0 + rl; r < r1; r += RL) {
      const int64_t o = ((int64_t)r * CV + vc) * V;
      float xv[V], gv[V];
      BnVec<TX>::load(x + o, xv);
      if constexpr (sizeof(TG) == sizeof(TX)) {
        BnVec<TG>::load(dy + o, gv);
      } else {  // x fp32 (4 per vector), dy bf16: 8-byte loads
        const uint2 u = *reinterpret_cast<const uint2*>(dy + o);
        gv[0] = __uint_as_float(u.x << 16); gv[1] = __uint_as_float(u.x & 0xffff0000u);
        gv[2] = __uint_as_float(u.y << 16); gv[3] = __uint_as_float(u.y & 0xffff0000u);
      }
#pragma unroll
      for (int e = 0; e < V; ++e) {
        a[e] += gv[e];
        b[e] = fmaf(gv[e], (xv[e] - mu[e]) * rs[e], b[e]);
      }
    }
  if (FLAT) {
    float ta = 0.f, tb = 0.f;
#pragma unroll
    for (int e = 0; e < V; ++e) { ta += a[e]; tb += b[e]; }
    sa[tid] = ta; sb[tid] = tb;
    __syncthreads();
    for (int h = 128; h >= 1; h >>= 1) {
      if (tid < h) { sa[tid] += sa[tid + h]; sb[tid] += sb[tid + h]; }
      __syncthreads();
    }
    if (tid == 0) {
      float* p = part + (int64_t)blockIdx.x * 2;
      p[0] = sa[0]; p[1] = sb[0];
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < V; ++e) { sa[tid * V + e] = a[e]; sb[tid * V + e] = b[e]; }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    const int cv = c / V, e = c % V;
    float ta = 0.f, tb = 0.f;
    for (int l = 0; l < RL; ++l) {
      const int t = (l * CV + cv) * V + e;
      ta += sa[t]; tb += sb[t];
    }
    float* p = part + ((int64_t)blockIdx.x * C + c) * 2;
    p[0] = ta; p[1] = tb;
  }
}

__global__ void __launch_bounds__(256) bn_bwd_finalize_v_kernel(const float* __restrict__ part, int nb, int C,
                                                                float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float sa[256], sb[256];
  const int tid = threadIdx.x, sl = tid % BN_FL;
  const int c = blockIdx.x * (256 / BN_FL) + tid / BN_FL;
  float a = 0.f, b = 0.f;
  if (c < C) {
    for (int k0 = sl; k0 < nb; k0 += 4 * BN_FL) {
      float q[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = min(k0 + i * BN_FL, nb - 1);
        q[i][0] = part[((int64_t)k * C + c) * 2];
        q[i][1] = part[((int64_t)k * C + c) * 2 + 1];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (k0 + i * BN_FL < nb) { a += q[i][0]; b += q[i][1]; }
    }
  }
  sa[tid] = a; sb[tid] = b;
  __syncthreads();
  if (sl != 0 || c >= C) return;
  for (int k = 1; k < BN_FL; ++k) { a += sa[tid + k]; b += sb[tid + k]; }
  dbeta[c] = a;
  dgamma[c] = b;
}

template <typename TX, typename TG, bool FLAT>
__global__ void __launch_bounds__(256) bn_bwd_apply_v_kernel(const TX* __restrict__ x, const TG* __restrict__ dy,
                                                             int nvec, int C, float inv_m,
                                                             const float* __restrict__ mean_rstd,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ dgamma,
                                                             const float* __restrict__ dbeta, TX* __restrict__ dx) {
  constexpr int V = BnVec<TX>::V;
  const int CV = FLAT ? 1 : C / V;
  const int i0 = blockIdx.x * 256 + threadIdx.x;
  const int c0 = FLAT ? 0 : (i0 % CV) * V;
  __shared__ float sp[5][BN_CMAX];  // per-channel parameters staged once per block (see bn_apply_v_kernel)
  for (int c = threadIdx.x; c < C; c += 256) {
    sp[0][c] = mean_rstd[c]; sp[1][c] = mean_rstd[C + c];
    sp[2][c] = (gamma ? gamma[c] : 1.f) * mean_rstd[C + c];
    sp[3][c] = dbeta[c] * inv_m; sp[4][c] = dgamma[c] * inv_m;
  }
  __syncthreads();
  float mu[V], rs[V], gr[V], db[V], dg[V];  // gr = gamma rstd, db / dg = dbeta / M, dgamma / M
#pragma unroll
  for (int e = 0; e < V; ++e) {
    const int c = FLAT ? 0 : c0 + e;
    mu[e] = sp[0][c]; rs[e] = sp[1][c]; gr[e] = sp[2][c]; db[e] = sp[3][c]; dg[e] = sp[4][c];
  }
  const int stride = gridDim.x * 256;
  for (int i = i0; i < nvec; i += 2 * stride) {  // two vectors of x and dy in flight per thread
    float xv[2][V], gv[2][V];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (i + u * stride >= nvec) continue;
      const int64_t o = (int64_t)(i + u * stride) * V;
      BnVec<TX>::load(x + o, xv[u]);
      if constexpr (sizeof(TG) == sizeof(TX)) {
        BnVec<TG>::load(dy + o, gv[u]);
      } else {
        const uint2 q = *reinterpret_cast<const uint2*>(dy + o);
        gv[u][0] = __uint_as_float(q.x << 16); gv[u][1] = __uint_as_float(q.x & 0xffff0000u);
        gv[u][2] = __uint_as_float(q.y << 16); gv[u][3] = __uint_as_float(q.y & 0xffff0000u);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (i + u * stride >= nvec) continue;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float xh = (xv[u][e] - mu[e]) * rs[e];
        xv[u][e] = gr[e] * (gv[u][e] - db[e] - xh * dg[e]);
      }
      BnVec<TX>::store(dx + (int64_t)(i + u * stride) * V, xv[u]);
    }
  }
}

// ------------------------------------------------------------------------------- dropout
// Counter-based dropout (nn.Dropout / F.dropout in training, scripts/transformer/SubLayers.py:38,87,
// scripts/transformer/Layers.py:129-131, scripts/model/modules.py:52-56): element i is kept iff
// hash(seed, i) >= p 2^32, y = keep ? x / (1 - p) : 0.  The mask is a pure function of (seed, i), so
// the backward is the same call on dy -- no mask tensor is written or read (ATen's fused_dropout writes
// one byte per element and its masked_scale reads it back).  seed: a device int64 drawn per call from
// torch's generator (graph-safe: every replay draws a new one).
// (drop_mix / drop_hash / drop_keys: vo_common.h -- the LayerNorm kernels apply the same mask in-pass)

template <typename T>
__global__ void __launch_bounds__(256) dropout_kernel(const T* __restrict__ x, int64_t n, uint32_t thr, float scale,
                                                      const int64_t* __restrict__ seed, uint32_t salt,
                                                      T* __restrict__ y) {
  using VT = BnVec<T>;
  constexpr int V = VT::V;
  uint32_t s0, s1;
  drop_keys(seed, salt, s0, s1);
  const int64_t nv = n / V;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += 4 * stride) {  // 4 vectors in flight
    float v[4][V];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * stride < nv) VT::load(x + (i + u * stride) * V, v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t iv = i + u * stride;
      if (iv >= nv) continue;
#pragma unroll
      for (int e = 0; e < V; ++e) v[u][e] = drop_hash(s0, s1, (uint32_t)(iv * V + e)) >= thr ? v[u][e] * scale : 0.f;
      VT::store(y + iv * V, v[u]);
    }
  }
  const int64_t t = nv * V + threadIdx.x;  // the n % V tail, one element a thread of block 0
  if (blockIdx.x == 0 && t < n) y[t] = from_f32<T>(drop_hash(s0, s1, (uint32_t)t) >= thr ? to_f32(x[t]) * scale : 0.f);
}

// ------------------------------------------------------------------------------- 3 x 3 single-channel conv

constexpr int VC_TILE = 256;  // pixels per block (the weight / bias partials: one row per block)

__global__ void __launch_bounds__(VC_TILE) vfe_conv_fwd_kernel(const float* __restrict__ x, int N, int H, int W,
                                                               const float* __restrict__ w, float* __restrict__ y) {
  const int64_t total = (int64_t)N * H * W;
  const int64_t i = (int64_t)blockIdx.x * VC_TILE + threadIdx.x;
  if (i >= total) return;
  const int wq = (int)(i % W), hq = (int)((i / W) % H);
  const int64_t base = i - (int64_t)hq * W - wq;
  float s = w[9];  // bias
#pragma unroll
  for (int di = -1; di <= 1; ++di)
#pragma unroll
    for (int dj = -1; dj <= 1; ++dj) {
      const int h = hq + di, ww = wq + dj;
      if (h >= 0 && h < H && ww >= 0 && ww < W) s += w[(di + 1) * 3 + (dj + 1)] * x[base + (int64_t)h * W + ww];
    }
  y[i] = s;
}

// dx = correlation of dy with the flipped kernel; per block: the 10 weight / bias partial sums
__global__ void __launch_bounds__(VC_TILE) vfe_conv_bwd_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ dy, int N, int H, int W,
                                                               const float* __restrict__ w, float* __restrict__ dx,
                                                               float* __restrict__ part) {
  __shared__ float red[10][VC_TILE / 64];
  const int64_t total = (int64_t)N * H * W;
  const int64_t i = (int64_t)blockIdx.x * VC_TILE + threadIdx.x;
  float pw[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) pw[k] = 0.f;
  if (i < total) {
    const int wq = (int)(i % W), hq = (int)((i / W) % H);
    const int64_t base = i - (int64_t)hq * W - wq;
    float s = 0.f;
    const float g = dy[i];
#pragma unroll
    for (int di = -1; di <= 1; ++di)
#pragma unroll
      for (int dj = -1; dj <= 1; ++dj) {
        const int h = hq + di, ww = wq + dj;
        if (h >= 0 && h < H && ww >= 0 && ww < W) {
          // y[h, ww] used x[hq, wq] with kernel tap (-di, -dj): dx += w[1 - di][1 - dj] dy[h, ww]
          s += w[(1 - di) * 3 + (1 - dj)] * dy[base + (int64_t)h * W + ww];
          // dW[di + 1][dj + 1] += dy[hq, wq] x[hq + di, wq + dj]
          pw[(di + 1) * 3 + (dj + 1)] = g * x[base + (int64_t)h * W + ww];
        }
      }
    pw[9] = g;
    dx[i] = s;
  }
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    const float v = wave_sum(pw[k]);
    if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = v;
  }
  __syncthreads();
  if (threadIdx.x < 10) {
    float v = 0.f;
    for (int q = 0; q < VC_TILE / 64; ++q) v += red[threadIdx.x][q];
    part[(int64_t)blockIdx.x * 10 + threadIdx.x] = v;
  }
}

__global__ void vfe_conv_wgrad_finalize_kernel(const float* __restrict__ part, int nb, float* __restrict__ dw) {
  // one wave per weight: lanes stride over blocks in order, a fixed-shape tree inside the wave
  const int k = blockIdx.x;
  float s = 0.f;
  for (int b = threadIdx.x; b < nb; b += 64) s += part[(int64_t)b * 10 + k];
  s = wave_sum(s);
  if (threadIdx.x == 0) dw[k] = s;
}

// ------------------------------------------------------------------------------- STFT log-mel backward

constexpr int SMB_MAX_N = 2048;

__device__ __forceinline__ int reflect_idx(int i, int n) {
  if (i < 0) i = -i;
  if (i >= n) i = 2 * (n - 1) - i;
  return i;
}

// in-place-free radix-2 Stockham FFT of length L (power of two) on buf[src]; sign -1 forward,
// +1 inverse (unnormalised); returns the buffer holding the result
__device__ int fft_stockham(float2 (*buf)[SMB_MAX_N], int L, float sign, int tid, int nthreads) {
  int src = 0;
  for (int ns = 1; ns < L; ns <<= 1) {
    for (int j = tid; j < L / 2; j += nthreads) {
      const int k = j & (ns - 1);
      const float2 u = buf[src][j];
      const float2 v = buf[src][j + L / 2];
      float s, c;
      sincospif(sign * (float)k / (float)ns, &s, &c);
      const float2 tv = make_float2(v.x * c - v.y * s, v.x * s + v.y * c);
      const int out = (j - k) * 2 + k;
      buf[src ^ 1][out] = make_float2(u.x + tv.x, u.y + tv.y);
      buf[src ^ 1][out + ns] = make_float2(u.x - tv.x, u.y - tv.y);
    }
    __syncthreads();
    src ^= 1;
  }
  return src;
}

// one workgroup per (frame, utterance): gframe[b][f][n] = d loss / d x_frame[n] (after the window)
__global__ void __launch_bounds__(256) stft_mel_bwd_frame_kernel(const float* __restrict__ wav, int N, int F,
                                                                 const float* __restrict__ window,
                                                                 const float* __restrict__ fb, int n_fft, int hop,
                                                                 int n_mels, int pad, float mag_eps, float log_floor,
                                                                 const float* __restrict__ gmel,
                                                                 float* __restrict__ gframe) {
  __shared__ float2 buf[2][SMB_MAX_N];
  __shared__ float mag[SMB_MAX_N / 2 + 1];
  __shared__ float xre[SMB_MAX_N / 2 + 1], xim[SMB_MAX_N / 2 + 1];
  __shared__ float dm[256];  // d loss / d melsum per mel bin (n_mels <= 256)
  const int f = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int n = n_fft, half = n / 2;
  const float* x = wav + (int64_t)b * N;
  const int start = f * hop - pad;

  // forward: full n-point complex FFT of the windowed real frame
  for (int m = tid; m < n; m += 256) buf[0][m] = make_float2(x[reflect_idx(start + m, N)] * window[m], 0.f);
  __syncthreads();
  int s = fft_stockham(buf, n, -1.f, tid, 256);
  for (int k = tid; k <= half; k += 256) {
    const float2 z = buf[s][k];
    xre[k] = z.x;
    xim[k] = z.y;
    mag[k] = sqrtf(z.x * z.x + z.y * z.y + mag_eps);
  }
  __syncthreads();
  // mel sums and their log-floor derivative
  const int lane = tid & 63, wave = tid >> 6;
  const int nf = half + 1;
  for (int m = wave; m < n_mels; m += 4) {
    float acc = 0.f;
    for (int k = lane; k < nf; k += 64) acc += fb[(int64_t)k * n_mels + m] * mag[k];
    acc = wave_sum(acc);
    if (lane == 0) dm[m] = acc >= log_floor ? gmel[((int64_t)b * n_mels + m) * F + f] / acc : 0.f;
  }
  __syncthreads();
  // dX[k] = (fb dm)[k] X[k] / |X[k]| for k <= n/2, zero above: the inverse DFT's real part is the
  // gradient w.r.t. the windowed frame (Re sum_k conj-free D_k e^{+2 pi i k t / n})
  for (int k = tid; k < n; k += 256) {
    float2 d = make_float2(0.f, 0.f);
    if (k <= half) {
      float g = 0.f;
      for (int m = 0; m < n_mels; ++m) g += fb[(int64_t)k * n_mels + m] * dm[m];
      const float sc = g / mag[k];
      d = make_float2(sc * xre[k], sc * xim[k]);
    }
    buf[0][k] = d;
  }
  __syncthreads();
  s = fft_stockham(buf, n, 1.f, tid, 256);
  float* out = gframe + ((int64_t)b * F + f) * n;
  for (int m = tid; m < n; m += 256) out[m] = buf[s][m].x * window[m];
}

// dwav[b][i] = sum over padded positions p with reflect(p - pad) == i and frames f covering p
// (f hop <= p < f hop + n_fft) of gframe[b][f][p - f hop], in a fixed order
__global__ void __launch_bounds__(256) stft_mel_bwd_gather_kernel(const float* __restrict__ gframe, int N, int F,
                                                                  int n_fft, int hop, int pad,
                                                                  float* __restrict__ dwav) {
  const int i = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (i >= N) return;
  const float* gf = gframe + (int64_t)b * F * n_fft;
  float s = 0.f;
  int ps[3];
  int np = 0;
  ps[np++] = i + pad;                                    // the sample itself
  if (i >= 1 && i <= pad) ps[np++] = pad - i;            // mirrored into the left pad
  if (i <= N - 2 && i >= N - 1 - pad) ps[np++] = pad + 2 * (N - 1) - i;  // mirrored into the right pad
  for (int q = 0; q < np; ++q) {
    const int p = ps[q];
    int f0 = p - n_fft + 1;
    f0 = f0 <= 0 ? 0 : (f0 + hop - 1) / hop;
    const int f1 = min(p / hop, F - 1);
    for (int f = f0; f <= f1; ++f) s += gf[(int64_t)f * n_fft + (p - f * hop)];
  }
  dwav[(int64_t)b * N + i] = s;
}

// ------------------------------------------------------------------------------- STFT magnitude
// torch.stft(center=True, reflect pad n_fft / 2, onesided) of a window zero-padded to n_fft, and
// mag = sqrt(max(|X|^2, eps)): the multi-resolution STFT loss of Parallel WaveGAN-style vocoder
// training.  One workgroup per (frame, utterance); mag laid out (B, F, n_fft / 2 + 1).
__global__ void __launch_bounds__(256) stft_mag_kernel(const float* __restrict__ wav, int N, int F,
                                                       const float* __restrict__ window, int n_fft, int hop,
                                                       float eps, float* __restrict__ mag) {
  __shared__ float2 buf[2][SMB_MAX_N];
  const int f = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int n = n_fft, half = n / 2;
  const float* x = wav + (int64_t)b * N;
  const int start = f * hop - half;
  for (int m = tid; m < n; m += 256) buf[0][m] = make_float2(x[reflect_idx(start + m, N)] * window[m], 0.f);
  __syncthreads();
  const int s = fft_stockham(buf, n, -1.f, tid, 256);
  float* out = mag + ((int64_t)b * F + f) * (half + 1);
  for (int k = tid; k <= half; k += 256) {
    const float2 z = buf[s][k];
    out[k] = sqrtf(fmaxf(z.x * z.x + z.y * z.y, eps));
  }
}

// frame gradient of the magnitude: dX = gmag X / |X| where |X|^2 > eps (the clamp passes no
// gradient below it), zero above n / 2; the inverse DFT's real part times the window
__global__ void __launch_bounds__(256) stft_mag_bwd_frame_kernel(const float* __restrict__ wav, int N, int F,
                                                                 const float* __restrict__ window, int n_fft,
                                                                 int hop, float eps, const float* __restrict__ gmag,
                                                                 float* __restrict__ gframe) {
  __shared__ float2 buf[2][SMB_MAX_N];
  const int f = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int n = n_fft, half = n / 2;
  const float* x = wav + (int64_t)b * N;
  const int start = f * hop - half;
  for (int m = tid; m < n; m += 256) buf[0][m] = make_float2(x[reflect_idx(start + m, N)] * window[m], 0.f);
  __syncthreads();
  int s = fft_stockham(buf, n, -1.f, tid, 256);
  const float* gm = gmag + ((int64_t)b * F + f) * (half + 1);
  float2 d[SMB_MAX_N / 256];
#pragma unroll
  for (int u = 0; u < SMB_MAX_N / 256; ++u) {
    const int k = tid + u * 256;
    d[u] = make_float2(0.f, 0.f);
    if (k <= half) {
      const float2 z = buf[s][k];
      const float p = z.x * z.x + z.y * z.y;
      const float sc = p > eps ? gm[k] * rsqrtf(p) : 0.f;
      d[u] = make_float2(sc * z.x, sc * z.y);
    }
  }
  __syncthreads();  // every spectrum read done before the buffer is reused
#pragma unroll
  for (int u = 0; u < SMB_MAX_N / 256; ++u) {
    const int k = tid + u * 256;
    if (k < n) buf[0][k] = d[u];
  }
  __syncthreads();
  s = fft_stockham(buf, n, 1.f, tid, 256);
  float* out = gframe + ((int64_t)b * F + f) * n;
  for (int m = tid; m < n; m += 256) out[m] = buf[s][m].x * window[m];
}

// multi-resolution STFT loss terms of one resolution over n magnitudes (x = generated, y =
// target): part[block] = (sum (y - x)^2, sum y^2, sum |log y - log x|); one wave adds the block
// partials in order into out[0..3)
__global__ void __launch_bounds__(256) stft_loss_reduce_kernel(const float* __restrict__ xm,
                                                               const float* __restrict__ ym, int64_t n,
                                                               float* __restrict__ part) {
  __shared__ float red[3][4];
  float a = 0.f, c = 0.f, l = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float x = xm[i], y = ym[i];
    a += (y - x) * (y - x);
    c += y * y;
    l += fabsf(__logf(y) - __logf(x));
  }
  a = wave_sum(a);
  c = wave_sum(c);
  l = wave_sum(l);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = a;
    red[1][threadIdx.x >> 6] = c;
    red[2][threadIdx.x >> 6] = l;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const float* r = red[threadIdx.x];
    part[(int64_t)blockIdx.x * 3 + threadIdx.x] = r[0] + r[1] + r[2] + r[3];
  }
}

__global__ void __launch_bounds__(64) stft_loss_final_kernel(const float* __restrict__ part, int nb,
                                                             float* __restrict__ out) {
  for (int k = 0; k < 3; ++k) {
    float v = 0.f;
    for (int i = threadIdx.x; i < nb; i += 64) v += part[(int64_t)i * 3 + k];
    v = wave_sum(v);
    if (threadIdx.x == 0) out[k] = v;
  }
}

// d/dx of w_sc * sqrt(A) / sqrt(C) + w_mag * L / n, A / C / L the sums above:
//   w_sc (x - y) / (sqrt(A) sqrt(C)) + w_mag sign(log x - log y) / (n x)
__global__ void __launch_bounds__(256) stft_loss_grad_kernel(const float* __restrict__ xm,
                                                             const float* __restrict__ ym, int64_t n,
                                                             const float* __restrict__ sums,
                                                             const float* __restrict__ w, float* __restrict__ gx) {
  const float w_sc = w[0], w_mag = w[1];  // device scalars: the incoming loss gradients (graph-safe)
  const float sa = sqrtf(sums[0]), sc = sqrtf(sums[1]);
  const float k_sc = sa > 0.f && sc > 0.f ? w_sc / (sa * sc) : 0.f;
  const float k_mag = w_mag / (float)n;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float x = xm[i], y = ym[i];
    const float dl = __logf(x) - __logf(y);
    gx[i] = k_sc * (x - y) + (dl > 0.f ? k_mag : (dl < 0.f ? -k_mag : 0.f)) / x;
  }
}

}  // namespace vo

using namespace vo;

// ---- BatchNorm: x (M, C) channels-last, dtype VO_F32 / VO_BF16; workspace: bn workspace size
// the vectorised kernels cover C % V == 0 with C / V <= 256 vector columns (V = 8 bf16 / 4 fp32), and
// C = 1 with M % V == 0 (FLAT); other shapes take the scalar kernels
static bool bn_vec_ok(int M, int C, int dtype, bool* flat) {
  const int V = dtype == VO_BF16 ? 8 : 4;
  *flat = C == 1;
  if (C == 1) return M % V == 0;
  return C % V == 0 && C / V <= 256;
}

// apply grid: at most 2048 blocks, the thread count a multiple of the CV vector columns (so that every
// thread keeps one column: bn_apply_v_kernel)
static unsigned bn_apply_blocks(int nvec, int CV) {
  int g = 256, c = CV;
  while (c) { const int t = g % c; g = c; c = t; }  // gcd(256, CV)
  const int step = CV / g;
  int64_t blk = std::min<int64_t>((nvec + 1023) / 1024, 1024);  // ~4 vectors per thread (4096 blocks: 3x slower)
  blk = (blk + step - 1) / step * step;
  return (unsigned)std::max<int64_t>(blk, step);
}

static void bn_vec_geometry(int M, int C, int dtype, bool flat, int* rows, int* RB, int* nb) {
  const int V = dtype == VO_BF16 ? 8 : 4;
  *rows = flat ? M / V : M;
  const int RL = flat ? 256 : 256 / (C / V);
  int rb = (*rows + BN_NB - 1) / BN_NB;
  rb = (rb + RL - 1) / RL * RL;  // whole passes of the block's row lanes
  *RB = rb > 0 ? rb : RL;
  *nb = (*rows + *RB - 1) / *RB;
}

extern "C" int64_t vo_bn_workspace_size(int M, int C) {
  const int CT = C == 1 ? 1 : 64;
  const int RB = C == 1 ? 8192 : 512;
  const int64_t nb = (M + RB - 1) / RB;
  (void)CT;
  // (the vectorised kernels use at most BN_NB partials per channel)
  return std::max<int64_t>(nb, BN_NB) * C * 3 * (int64_t)sizeof(float);
}

static void bn_geometry(int M, int C, int* CT, int* RB, int* nb) {
  *CT = C == 1 ? 1 : 64;
  *RB = C == 1 ? 8192 : 512;
  *nb = (M + *RB - 1) / *RB;
}

extern "C" int vo_bn_train_fwd(const void* x, int dtype, int M, int C, const float* gamma, const float* beta,
                               float eps, float momentum, float* run_mean, float* run_var, int64_t* nbt,
                               float* mean_rstd, float* workspace, void* y, void* stream) {
  VO_CHECK_ARG(x && y && mean_rstd && workspace && M > 0 && C > 0, "bn_train_fwd: bad arguments");
  VO_CHECK_ARG(dtype == VO_F32 || dtype == VO_BF16, "bn_train_fwd: dtype");
  VO_CHECK_ARG((gamma == nullptr) == (beta == nullptr), "bn_train_fwd: gamma and beta together");
  VO_CHECK_ARG((run_mean == nullptr) == (run_var == nullptr), "bn_train_fwd: running stats together");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  bool flat = false;
  if (bn_vec_ok(M, C, dtype, &flat)) {
    int rows, RBv, nbv;
    bn_vec_geometry(M, C, dtype, flat, &rows, &RBv, &nbv);
    const int V = dtype == VO_BF16 ? 8 : 4;
    const int nvec = (int)((int64_t)M * C / V);
    const unsigned ablk = bn_apply_blocks(nvec, flat ? 1 : C / V);
#define VO_BN_FWD(TX, FL)                                                                                          \
  do {                                                                                                             \
    hipLaunchKernelGGL((bn_stats_v_kernel<TX, FL>), dim3((unsigned)nbv), dim3(256), 0, st, (const TX*)x, rows, C, RBv, \
                       workspace);                                                                                 \
    hipLaunchKernelGGL(bn_finalize_v_kernel, dim3((unsigned)((C + 31) / 32)), dim3(256), 0, st, workspace, nbv, C,    \
                       eps, momentum, mean_rstd, run_mean, run_var, nbt);                                          \
    hipLaunchKernelGGL((bn_apply_v_kernel<TX, FL>), dim3(ablk), dim3(256), 0, st, (const TX*)x, nvec, C, mean_rstd,  \
                       gamma, beta, (TX*)y);                                                                       \
  } while (0)
    if (dtype == VO_F32) {
      if (flat) VO_BN_FWD(float, true); else VO_BN_FWD(float, false);
    } else {
      if (flat) VO_BN_FWD(bf16_t, true); else VO_BN_FWD(bf16_t, false);
    }
#undef VO_BN_FWD
    VO_RETURN_LAUNCH();
  }
  int CT, RB, nb;
  bn_geometry(M, C, &CT, &RB, &nb);
  const dim3 grid((unsigned)nb, (unsigned)((C + CT - 1) / CT));
  if (dtype == VO_F32) {
    if (CT == 1) hipLaunchKernelGGL((bn_stats_kernel<float, 1>), grid, dim3(256), 0, st, (const float*)x, M, C, RB, workspace);
    else hipLaunchKernelGGL((bn_stats_kernel<float, 64>), grid, dim3(256), 0, st, (const float*)x, M, C, RB, workspace);
  } else {
    if (CT == 1) hipLaunchKernelGGL((bn_stats_kernel<bf16_t, 1>), grid, dim3(256), 0, st, (const bf16_t*)x, M, C, RB, workspace);
    else hipLaunchKernelGGL((bn_stats_kernel<bf16_t, 64>), grid, dim3(256), 0, st, (const bf16_t*)x, M, C, RB, workspace);
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, workspace, nb, C, eps,
                     momentum, mean_rstd, run_mean, run_var, nbt);
  const int64_t total = (int64_t)M * C;
  const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 4096);
  if (dtype == VO_F32)
    hipLaunchKernelGGL((bn_apply_kernel<float>), dim3(blocks), dim3(256), 0, st, (const float*)x, total, C, mean_rstd,
                       gamma, beta, (float*)y);
  else
    hipLaunchKernelGGL((bn_apply_kernel<bf16_t>), dim3(blocks), dim3(256), 0, st, (const bf16_t*)x, total, C,
                       mean_rstd, gamma, beta, (bf16_t*)y);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_bn_bwd(const void* x, int x_dtype, const void* dy, int dy_dtype, int M, int C, const float* gamma,
                         const float* mean_rstd, float* workspace, float* dgamma, float* dbeta, void* dx, void* stream) {
  VO_CHECK_ARG(x && dy && mean_rstd && workspace && dgamma && dbeta && dx && M > 0 && C > 0, "bn_bwd: bad arguments");
  VO_CHECK_ARG((x_dtype == VO_F32 || x_dtype == VO_BF16) && (dy_dtype == VO_F32 || dy_dtype == VO_BF16),
               "bn_bwd: dtypes");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  bool flat = false;
  // vectorised: x's vector width sets the layout; dy bf16 under fp32 x is read 4 per lane (8 bytes)
  if (bn_vec_ok(M, C, x_dtype, &flat) && !(x_dtype == VO_BF16 && dy_dtype == VO_F32)) {
    int rows, RBv, nbv;
    bn_vec_geometry(M, C, x_dtype, flat, &rows, &RBv, &nbv);
    const int V = x_dtype == VO_BF16 ? 8 : 4;
    const int nvec = (int)((int64_t)M * C / V);
    const unsigned ablk = bn_apply_blocks(nvec, flat ? 1 : C / V);
    const float inv_m = 1.f / (float)M;
#define VO_BNB_V(TX, TG, FL)                                                                                        \
  do {                                                                                                              \
    hipLaunchKernelGGL((bn_bwd_stats_v_kernel<TX, TG, FL>), dim3((unsigned)nbv), dim3(256), 0, st, (const TX*)x,     \
                       (const TG*)dy, rows, C, RBv, mean_rstd, workspace);                                          \
    hipLaunchKernelGGL(bn_bwd_finalize_v_kernel, dim3((unsigned)((C + 31) / 32)), dim3(256), 0, st, workspace, nbv,   \
                       C, dgamma, dbeta);                                                                           \
    hipLaunchKernelGGL((bn_bwd_apply_v_kernel<TX, TG, FL>), dim3(ablk), dim3(256), 0, st, (const TX*)x,             \
                       (const TG*)dy, nvec, C, inv_m, mean_rstd, gamma, dgamma, dbeta, (TX*)dx);                    \
  } while (0)
    if (x_dtype == VO_F32 && dy_dtype == VO_F32) {
      if (flat) VO_BNB_V(float, float, true); else VO_BNB_V(float, float, false);
    } else if (x_dtype == VO_F32) {
      if (flat) VO_BNB_V(float, bf16_t, true); else VO_BNB_V(float, bf16_t, false);
    } else {
      if (flat) VO_BNB_V(bf16_t, bf16_t, true); else VO_BNB_V(bf16_t, bf16_t, false);
    }
#undef VO_BNB_V
    VO_RETURN_LAUNCH();
  }
  int CT, RB, nb;
  bn_geometry(M, C, &CT, &RB, &nb);
  const dim3 grid((unsigned)nb, (unsigned)((C + CT - 1) / CT));
#define VO_BNB_STATS(TX, TG)                                                                                     \
  do {                                                                                                           \
    if (CT == 1)                                                                                                 \
      hipLaunchKernelGGL((bn_bwd_stats_kernel<TX, TG, 1>), grid, dim3(256), 0, st, (const TX*)x, (const TG*)dy, M, \
                         C, RB, mean_rstd, workspace);                                                           \
    else                                                                                                         \
      hipLaunchKernelGGL((bn_bwd_stats_kernel<TX, TG, 64>), grid, dim3(256), 0, st, (const TX*)x, (const TG*)dy, M, \
                         C, RB, mean_rstd, workspace);                                                           \
  } while (0)
  if (x_dtype == VO_F32 && dy_dtype == VO_F32) VO_BNB_STATS(float, float);
  else if (x_dtype == VO_F32) VO_BNB_STATS(float, bf16_t);
  else if (dy_dtype == VO_F32) VO_BNB_STATS(bf16_t, float);
  else VO_BNB_STATS(bf16_t, bf16_t);
#undef VO_BNB_STATS
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, workspace, nb, C,
                     dgamma, dbeta);
  const int64_t total = (int64_t)M * C;
  const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 4096);
  const float inv_m = 1.f / (float)M;
#define VO_BNB_APPLY(TX, TG)                                                                                      \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<TX, TG>), dim3(blocks), dim3(256), 0, st, (const TX*)x, (const TG*)dy, total, \
                     C, inv_m, mean_rstd, gamma, dgamma, dbeta, (TX*)dx)
  if (x_dtype == VO_F32 && dy_dtype == VO_F32) VO_BNB_APPLY(float, float);
  else if (x_dtype == VO_F32) VO_BNB_APPLY(float, bf16_t);
  else if (dy_dtype == VO_F32) VO_BNB_APPLY(bf16_t, float);
  else VO_BNB_APPLY(bf16_t, bf16_t);
#undef VO_BNB_APPLY
  VO_RETURN_LAUNCH();
}

// ---- glyph-encoder conv: x (N, H, W) fp32, w[10] = 3 x 3 kernel (row-major) + bias
extern "C" int64_t vo_vfe_conv_workspace_size(int N, int H, int W) {
  const int64_t nb = ((int64_t)N * H * W + VC_TILE - 1) / VC_TILE;
  return nb * 10 * (int64_t)sizeof(float);
}

extern "C" int vo_vfe_conv_fwd(const float* x, int N, int H, int W, const float* w, float* y, void* stream) {
  VO_CHECK_ARG(x && w && y && N > 0 && H > 0 && W > 0, "vfe_conv_fwd: bad arguments");
  const int64_t total = (int64_t)N * H * W;
  hipLaunchKernelGGL(vfe_conv_fwd_kernel, dim3((unsigned)((total + VC_TILE - 1) / VC_TILE)), dim3(VC_TILE), 0,
                     reinterpret_cast<hipStream_t>(stream), x, N, H, W, w, y);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_vfe_conv_bwd(const float* x, const float* dy, int N, int H, int W, const float* w, float* dx,
                               float* dw, float* workspace, void* stream) {
  VO_CHECK_ARG(x && dy && w && dx && dw && workspace && N > 0 && H > 0 && W > 0, "vfe_conv_bwd: bad arguments");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t total = (int64_t)N * H * W;
  const int nb = (int)((total + VC_TILE - 1) / VC_TILE);
  hipLaunchKernelGGL(vfe_conv_bwd_kernel, dim3((unsigned)nb), dim3(VC_TILE), 0, st, x, dy, N, H, W, w, dx, workspace);
  hipLaunchKernelGGL(vfe_conv_wgrad_finalize_kernel, dim3(10), dim3(64), 0, st, workspace, nb, dw);
  VO_RETURN_LAUNCH();
}

// ---- log-mel backward (the framing of vo_stft_mel_ex, clip off): gmel (B, n_mels, F) -> dwav (B, N)
extern "C" int64_t vo_stft_mel_bwd_workspace_size(int B, int N, int n_fft, int hop, int pad) {
  const int64_t F = 1 + (N + 2 * (int64_t)pad - n_fft) / hop;
  return (int64_t)B * F * n_fft * (int64_t)sizeof(float);
}

extern "C" int vo_stft_mel_bwd(const float* wav, int B, int N, const float* window, const float* fb, int n_fft, int hop,
                               int n_mels, int pad, float mag_eps, float log_floor, const float* gmel, float* dwav,
                               float* workspace, void* stream) {
  VO_CHECK_ARG(wav && window && fb && gmel && dwav && workspace, "stft_mel_bwd: null pointer");
  VO_CHECK_ARG(n_fft >= 8 && n_fft <= SMB_MAX_N && (n_fft & (n_fft - 1)) == 0, "stft_mel_bwd: n_fft=%d", n_fft);
  VO_CHECK_ARG(hop > 0 && n_mels > 0 && n_mels <= 256 && B > 0 && pad >= 0 && N > pad && N + 2 * pad >= n_fft,
               "stft_mel_bwd: bad sizes");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int F = 1 + (N + 2 * pad - n_fft) / hop;
  hipLaunchKernelGGL(stft_mel_bwd_frame_kernel, dim3((unsigned)F, (unsigned)B), dim3(256), 0, st, wav, N, F, window,
                     fb, n_fft, hop, n_mels, pad, mag_eps, log_floor, gmel, workspace);
  hipLaunchKernelGGL(stft_mel_bwd_gather_kernel, dim3((unsigned)((N + 255) / 256), (unsigned)B), dim3(256), 0, st,
                     workspace, N, F, n_fft, hop, pad, dwav);
  VO_RETURN_LAUNCH();
}

// ---- STFT magnitude (multi-resolution STFT loss): wav (B, N) -> mag (B, 1 + N / hop, n_fft / 2 + 1)
extern "C" int vo_stft_mag(const float* wav, int B, int N, const float* window, int n_fft, int hop, float eps,
                           float* mag, void* stream) {
  VO_CHECK_ARG(wav && window && mag, "stft_mag: null pointer");
  VO_CHECK_ARG(n_fft >= 8 && n_fft <= SMB_MAX_N && (n_fft & (n_fft - 1)) == 0, "stft_mag: n_fft=%d", n_fft);
  VO_CHECK_ARG(B > 0 && hop > 0 && N > n_fft / 2, "stft_mag: bad sizes (reflect padding needs N > n_fft / 2)");
  const int F = 1 + N / hop;
  hipLaunchKernelGGL(stft_mag_kernel, dim3((unsigned)F, (unsigned)B), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), wav, N, F, window, n_fft, hop, eps, mag);
  VO_RETURN_LAUNCH();
}

extern "C" int64_t vo_stft_mag_bwd_workspace_size(int B, int N, int n_fft, int hop) {
  const int64_t F = 1 + N / hop;
  return (int64_t)B * F * n_fft * (int64_t)sizeof(float);
}

extern "C" int vo_stft_mag_bwd(const float* wav, int B, int N, const float* window, int n_fft, int hop, float eps,
                               const float* gmag, float* dwav, float* workspace, void* stream) {
  VO_CHECK_ARG(wav && window && gmag && dwav && workspace, "stft_mag_bwd: null pointer");
  VO_CHECK_ARG(n_fft >= 8 && n_fft <= SMB_MAX_N && (n_fft & (n_fft - 1)) == 0, "stft_mag_bwd: n_fft=%d", n_fft);
  VO_CHECK_ARG(B > 0 && hop > 0 && N > n_fft / 2, "stft_mag_bwd: bad sizes");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int F = 1 + N / hop;
  hipLaunchKernelGGL(stft_mag_bwd_frame_kernel, dim3((unsigned)F, (unsigned)B), dim3(256), 0, st, wav, N, F, window,
                     n_fft, hop, eps, gmag, workspace);
  hipLaunchKernelGGL(stft_mel_bwd_gather_kernel, dim3((unsigned)((N + 255) / 256), (unsigned)B), dim3(256), 0, st,
                     workspace, N, F, n_fft, hop, n_fft / 2, dwav);
  VO_RETURN_LAUNCH();
}

// ---- one resolution's loss sums: out[3] = (sum (y-x)^2, sum y^2, sum |log y - log x|); workspace >= 3 * 512 floats
extern "C" int vo_stft_loss(const float* xm, const float* ym, int64_t n, float* out, float* workspace, void* stream) {
  VO_CHECK_ARG(xm && ym && out && workspace && n > 0, "stft_loss: bad arguments");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nb = (int)std::min<int64_t>((n + 255) / 256, 512);
  hipLaunchKernelGGL(stft_loss_reduce_kernel, dim3((unsigned)nb), dim3(256), 0, st, xm, ym, n, workspace);
  hipLaunchKernelGGL(stft_loss_final_kernel, dim3(1), dim3(64), 0, st, workspace, nb, out);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_stft_loss_grad(const float* xm, const float* ym, int64_t n, const float* sums, const float* w,
                                 float* gx, void* stream) {
  VO_CHECK_ARG(xm && ym && sums && w && gx && n > 0, "stft_loss_grad: bad arguments");
  const unsigned nb = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(stft_loss_grad_kernel, dim3(nb), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), xm, ym, n,
                     sums, w, gx);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_dropout(const void* x, int dtype, int64_t n, float p, const int64_t* seed, unsigned salt, void* y,
                          void* stream) {
  VO_CHECK_ARG(x && y && seed && n >= 0, "dropout: bad arguments");
  VO_CHECK_ARG(dtype == VO_F32 || dtype == VO_BF16, "dropout: dtype");
  VO_CHECK_ARG(p >= 0.f && p < 1.f, "dropout: p = %g outside [0, 1)", p);
  VO_CHECK_ARG(n < (1LL << 32), "dropout: %lld elements (the mask index is 32-bit)", (long long)n);
  VO_CHECK_ARG(((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0, "dropout: x / y must be 16-byte aligned");
  if (n == 0) return VO_OK;
  const uint32_t thr = (uint32_t)std::min(4294967295.0, (double)p * 4294967296.0);
  const float scale = 1.f / (1.f - p);
  const int V = dtype == VO_BF16 ? 8 : 4;
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n / V + 255) / 256, 8192));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == VO_BF16)
    hipLaunchKernelGGL(dropout_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)x, n, thr, scale, seed,
                       (uint32_t)salt, (bf16_t*)y);
  else
    hipLaunchKernelGGL(dropout_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)x, n, thr, scale, seed,
                       (uint32_t)salt, (float*)y);
  VO_RETURN_LAUNCH();
}
