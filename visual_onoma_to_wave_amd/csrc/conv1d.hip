// Channels-last implicit-GEMM Conv1d on gfx950 MFMA.
//
// GEMM view of one launch:  C[co][pos] = sum_{tap k, ci} W[k][co][ci] * X[pos + k*dil - pad][ci]
//   M = output channels (A operand = packed weights, rows read from LDS),
//   N = output positions of one batch element (B operand = the input window in LDS),
//   reduction = (input-channel chunk of 32) x (tap).
// One workgroup owns a BCO x BT output tile.  For every 32-channel chunk it stages the
// input WINDOW (BT + (K-1)*dil rows) once and reuses it for all K taps by shifting the
// row index -- a dilated conv costs no extra HBM/L2 traffic over a 1x1 conv.  The weight
// tile of the next (chunk, tap) step and the next chunk's window are fetched into
// registers before the current step's MFMAs and written to the other LDS buffer after
// them (issue-early / write-late), so there is one barrier per step.
//
// Accumulator -> output mapping: MFMA row m of co-tile i is channel NI*4*(m>>2) + 4*i +
// (m&3), so lane (g = lane>>4, n = lane&15) ends up holding 4*NI CONTIGUOUS channels of
// ONE position -> vector stores of whole channel runs (channels-last).
//
// The lrelu/relu prologue is applied while staging (replaces F.leaky_relu before every
// HiFi-GAN conv), and the epilogue fuses bias, post-activation (relu/tanh), residual add,
// scale and MRF accumulate (y = (post(acc + b) + res1) * scale + res2).
//
// References: PositionwiseFeedForward (scripts/transformer/SubLayers.py:85-93), PostNet
// (scripts/transformer/Layers.py:129-137), VariancePredictor.Conv (scripts/model/
// modules.py:216-259), ResBlock (scripts/hifigan/models.py:96-103), Generator conv_pre /
// ups (models.py:149-160).

#include "vo_common.h"

namespace vo {

constexpr int KC = 32;        // reduction chunk = one bf16 MFMA k-depth
constexpr int HALO_MAX = 64;  // (K-1)*dil supported by the register staging arrays

struct ConvArgs {
  const void* x; int64_t xbs; int ldx;
  const void* w; const float* bias;
  void* y; int64_t ybs; int ldy;
  const void* res1; const void* res2;
  int T_in, T_out, Ci, Co, K, dil, pad;
  int pre_act; float pre_slope; int post_act; float post_slope; float out_scale;
  int transposed, up_stride, up_pad, up_cout, up_tout;
  int tiles_per_b;
};

template <typename T> struct Raw8;  // 8 elements of T held in registers
template <> struct Raw8<bf16_t> {
  uint4 u;
  __device__ __forceinline__ void load(const bf16_t* p) { u = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void zero() { u = make_uint4(0, 0, 0, 0); }
  __device__ __forceinline__ void to_f32(float (&v)[8]) const {
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
};
template <> struct Raw8<float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const float4*>(p);
    b = *reinterpret_cast<const float4*>(p + 4);
  }
  __device__ __forceinline__ void zero() { a = b = make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ __forceinline__ void to_f32(float (&v)[8]) const {
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
};

// write 8 floats to LDS as TC
__device__ __forceinline__ void lds_store8(bf16_t* p, const float (&v)[8]) { store8(p, v); }
__device__ __forceinline__ void lds_store8(float* p, const float (&v)[8]) { store8(p, v); }

// ROLE only names the instantiation (0 = generic, 1..4 = HiFi-GAN MRF stage 0..3), so a
// profiler attributes the vocoder's stages to distinct kernels; the code is identical.
template <typename TIN, typename TC, typename TOUT, int NI, int NJ, int WCO, int WT, int ROLE>
__global__ void __launch_bounds__(WCO * WT * 64)
conv1d_kernel(ConvArgs a) {
  constexpr int NT = WCO * WT * 64;
  constexpr int BCO = 16 * NI * WCO;
  constexpr int BT = 16 * NJ * WT;
  constexpr int RP = KC + 8;                  // LDS row pitch (elements)
  constexpr int VPR = KC / 8;                 // 8-element vectors per row
  constexpr int MAXV = ((BT + HALO_MAX) * VPR + NT - 1) / NT;
  constexpr int WV = (BCO * VPR + NT - 1) / NT;

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  TC* smem = reinterpret_cast<TC*>(smem_raw);

  const int halo = (a.K - 1) * a.dil;
  const int win_rows = BT + halo;
  TC* win_buf[2] = {smem, smem + win_rows * RP};
  TC* w_buf[2] = {smem + 2 * win_rows * RP, smem + 2 * win_rows * RP + BCO * RP};

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_co0 = (wave % WCO) * 16 * NI;
  const int wave_t0 = (wave / WCO) * 16 * NJ;

  const int b = blockIdx.x / a.tiles_per_b;
  const int t0 = (blockIdx.x % a.tiles_per_b) * BT;
  const int co_blk = blockIdx.y * BCO;

  const TIN* __restrict__ X = reinterpret_cast<const TIN*>(a.x) + (int64_t)b * a.xbs;
  const TC* __restrict__ Wp = reinterpret_cast<const TC*>(a.w);
  const int in_row0 = t0 - a.pad;
  const int n_chunks = (a.Ci + KC - 1) / KC;
  const int n_steps = n_chunks * a.K;

  Raw8<TIN> win_r[MAXV];
  Raw8<TC> w_r[WV];

  auto load_window = [&](int c) {
    const int c0 = c * KC;
#pragma unroll
    for (int s = 0; s < MAXV; ++s) {
      const int v = tid + s * NT;
      const int r = v / VPR, q = v % VPR;
      const int t_in = in_row0 + r;
      const int ci = c0 + q * 8;
      if (r < win_rows && t_in >= 0 && t_in < a.T_in && ci < a.Ci)
        win_r[s].load(X + (int64_t)t_in * a.ldx + ci);
      else
        win_r[s].zero();
    }
  };
  auto store_window = [&](int buf) {
#pragma unroll
    for (int s = 0; s < MAXV; ++s) {
      const int v = tid + s * NT;
      const int r = v / VPR, q = v % VPR;
      if (r < win_rows) {
        float f[8];
        win_r[s].to_f32(f);
        if (a.pre_act != VO_ACT_NONE) {
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = act(a.pre_act, f[e], a.pre_slope);
        }
        lds_store8(win_buf[buf] + r * RP + q * 8, f);
      }
    }
  };
  auto load_w = [&](int c, int k) {
    const int c0 = c * KC;
#pragma unroll
    for (int s = 0; s < WV; ++s) {
      const int v = tid + s * NT;
      const int r = v / VPR, q = v % VPR;
      const int co = co_blk + r;
      const int ci = c0 + q * 8;
      if (r < BCO && co < a.Co && ci < a.Ci)
        w_r[s].load(Wp + ((int64_t)k * a.Co + co) * a.Ci + ci);
      else
        w_r[s].zero();
    }
  };
  auto store_w = [&](int buf) {
#pragma unroll
    for (int s = 0; s < WV; ++s) {
      const int v = tid + s * NT;
      const int r = v / VPR, q = v % VPR;
      if (r < BCO) {
        float f[8];
        w_r[s].to_f32(f);
        lds_store8(w_buf[buf] + r * RP + q * 8, f);
      }
    }
  };

  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue
  load_window(0);
  load_w(0, 0);
  store_window(0);
  store_w(0);
  __syncthreads();

  const int lr = lane & 15;
  const int lk = (lane >> 4) * 8;
  // A row (weights) for co-tile i:  NI*4*(lr>>2) + 4*i + (lr&3)
  const int a_row_base = wave_co0 + NI * 4 * (lr >> 2) + (lr & 3);

  for (int s = 0; s < n_steps; ++s) {
    const int c = s / a.K;
    const int k = s - c * a.K;
    const bool has_next = (s + 1) < n_steps;
    const int cn = (s + 1) / a.K;
    const int kn = (s + 1) - cn * a.K;
    if (has_next) {
      load_w(cn, kn);
      if (kn == 0) load_window(cn);
    }

    const TC* wb = w_buf[s & 1];
    const TC* xb = win_buf[c & 1];
    Frag<TC> af[NI], bfr[NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i) af[i].load(wb + (a_row_base + 4 * i) * RP + lk);
    const int brow = wave_t0 + lr + k * a.dil;
#pragma unroll
    for (int j = 0; j < NJ; ++j) bfr[j].load(xb + (brow + 16 * j) * RP + lk);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma(af[i], bfr[j], acc[i][j]);

    if (has_next) {
      store_w((s + 1) & 1);
      if (kn == 0) store_window(cn & 1);
    }
    __syncthreads();
  }

  // epilogue: lane holds channels [co0, co0 + 4*NI) of position pos
  const int g = lane >> 4;
  const int n0 = co_blk + wave_co0 + NI * 4 * g;
  if (n0 >= a.Co) return;
  TOUT* Y = reinterpret_cast<TOUT*>(a.y) + (int64_t)b * a.ybs;
  const TOUT* R1 = a.res1 ? reinterpret_cast<const TOUT*>(a.res1) + (int64_t)b * a.ybs : nullptr;
  const TOUT* R2 = a.res2 ? reinterpret_cast<const TOUT*>(a.res2) + (int64_t)b * a.ybs : nullptr;

  int col = n0, trow_shift = 0;
  if (a.transposed) {
    const int phase = n0 / a.up_cout;
    col = n0 - phase * a.up_cout;
    trow_shift = phase - a.up_pad;
  }
  float bias[4 * NI];
#pragma unroll
  for (int e = 0; e < 4 * NI; ++e) bias[e] = a.bias ? a.bias[(a.transposed ? col : n0) + e] : 0.f;

#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int pos = t0 + wave_t0 + 16 * j + lr;
    if (pos >= a.T_out) continue;
    int trow = pos;
    if (a.transposed) {
      trow = pos * a.up_stride + trow_shift;
      if (trow < 0 || trow >= a.up_tout) continue;
    }
    const int64_t off = (int64_t)trow * a.ldy + col;
    float v[4 * NI];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[4 * i + r] = act(a.post_act, acc[i][j][r] + bias[4 * i + r], a.post_slope);
#pragma unroll
    for (int h = 0; h < NI; ++h) {
      float q[4] = {v[4 * h], v[4 * h + 1], v[4 * h + 2], v[4 * h + 3]};
      if (R1) {
        float rr[4];
        load4(R1 + off + 4 * h, rr);
#pragma unroll
        for (int e = 0; e < 4; ++e) q[e] += rr[e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) q[e] *= a.out_scale;
      if (R2) {
        float rr[4];
        load4(R2 + off + 4 * h, rr);
#pragma unroll
        for (int e = 0; e < 4; ++e) q[e] += rr[e];
      }
      store4(Y + off + 4 * h, q);
    }
  }
}

// ------------------------------------------------------------------ host dispatch
template <typename TIN, typename TC, typename TOUT, int NI, int NJ, int WCO, int WT, int ROLE = 0>
static int launch_cfg(const vo_conv1d_desc* d, hipStream_t st) {
  constexpr int BCO = 16 * NI * WCO;
  constexpr int BT = 16 * NJ * WT;
  ConvArgs a;
  a.x = d->x; a.xbs = d->x_bstride; a.ldx = d->ldx;
  a.w = d->w; a.bias = d->bias;
  a.y = d->y; a.ybs = d->y_bstride; a.ldy = d->ldy;
  a.res1 = d->res1; a.res2 = d->res2;
  a.T_in = d->T_in; a.T_out = d->T_out; a.Ci = d->Ci; a.Co = d->Co;
  a.K = d->K; a.dil = d->dil; a.pad = d->pad;
  a.pre_act = d->pre_act; a.pre_slope = d->pre_slope;
  a.post_act = d->post_act; a.post_slope = d->post_slope; a.out_scale = d->out_scale;
  a.transposed = d->transposed; a.up_stride = d->up_stride; a.up_pad = d->up_pad;
  a.up_cout = d->up_cout; a.up_tout = d->up_tout;
  a.tiles_per_b = (d->T_out + BT - 1) / BT;
  const int win_rows = BT + (d->K - 1) * d->dil;
  const size_t lds = (size_t)(2 * win_rows + 2 * BCO) * (KC + 8) * sizeof(TC);
  if (lds > 160 * 1024) {
    vo_set_error("conv1d: LDS request %zu B exceeds 160 KiB", lds);
    return VO_ERR_INVALID;
  }
  dim3 grid((unsigned)(a.tiles_per_b * d->B), (unsigned)((d->Co + BCO - 1) / BCO));
  hipLaunchKernelGGL((conv1d_kernel<TIN, TC, TOUT, NI, NJ, WCO, WT, ROLE>), grid, dim3(WCO * WT * 64),
                     lds, st, a);
  VO_RETURN_LAUNCH();
}

template <typename TIN, typename TC, typename TOUT>
static int launch_types(const vo_conv1d_desc* d, hipStream_t st) {
  const int64_t rows = (int64_t)d->B * d->T_out;
  if (d->Co <= 32) return launch_cfg<TIN, TC, TOUT, 2, 4, 1, 4>(d, st);   // 32 x 256
  if (d->Co <= 64 || d->Co == 80) return launch_cfg<TIN, TC, TOUT, 4, 4, 1, 4>(d, st);  // 64 x 256
  if (rows <= 2048) return launch_cfg<TIN, TC, TOUT, 2, 2, 2, 2>(d, st);  // 64 x 64
  return launch_cfg<TIN, TC, TOUT, 4, 4, 2, 2>(d, st);                    // 128 x 128
}

}  // namespace vo

using namespace vo;

extern "C" int vo_conv1d(const vo_conv1d_desc* d, void* stream) {
  VO_CHECK_ARG(d != nullptr, "conv1d: null descriptor");
  VO_CHECK_ARG(d->x && d->w && d->y, "conv1d: null tensor pointer");
  VO_CHECK_ARG(d->B > 0 && d->T_in > 0 && d->T_out > 0 && d->Ci > 0 && d->Co > 0 && d->K > 0,
               "conv1d: non-positive size (B=%d T_in=%d T_out=%d Ci=%d Co=%d K=%d)", d->B,
               d->T_in, d->T_out, d->Ci, d->Co, d->K);
  VO_CHECK_ARG(d->Ci % 8 == 0 && d->ldx % 8 == 0 && d->ldx >= d->Ci,
               "conv1d: Ci (%d) and ldx (%d) must be multiples of 8, ldx >= Ci", d->Ci, d->ldx);
  VO_CHECK_ARG(d->Co % 4 == 0 && d->ldy % 4 == 0, "conv1d: Co (%d) and ldy (%d) must be multiples of 4",
               d->Co, d->ldy);
  VO_CHECK_ARG(d->dil >= 1 && (d->K - 1) * d->dil <= HALO_MAX,
               "conv1d: (K-1)*dil = %d exceeds the supported halo %d", (d->K - 1) * d->dil, HALO_MAX);
  VO_CHECK_ARG(d->variant == 0 || (d->variant == 1 && d->Co >= 128) || (d->variant == 2 && d->Co >= 128) ||
                   (d->variant == 3 && d->Co <= 64 && d->Co % 16 == 0) || (d->variant == 4 && d->Co <= 32),
               "conv1d: variant %d does not fit Co=%d", d->variant, d->Co);
  if (d->transposed) {
    VO_CHECK_ARG(d->up_stride >= 1 && d->up_cout > 0 && d->Co == d->up_stride * d->up_cout &&
                     d->up_cout % 16 == 0 && d->K == 2 && d->pad == 1,
                 "conv1d: bad polyphase ConvTranspose1d descriptor");
  } else {
    VO_CHECK_ARG(d->Co % 16 == 0 || d->Co == 80 || d->Co <= 32, "conv1d: unsupported Co %d", d->Co);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(const_cast<void*>(stream));
  const int xi = d->x_dtype, yo = d->y_dtype;
  if (d->compute_dtype == VO_F32) {
    VO_CHECK_ARG(xi == VO_F32 && yo == VO_F32, "conv1d: fp32 compute needs fp32 I/O");
    return launch_types<float, float, float>(d, st);
  }
  VO_CHECK_ARG(d->compute_dtype == VO_BF16, "conv1d: bad compute dtype");
  if (xi == VO_BF16 && yo == VO_BF16) {
    switch (d->variant) {  // HiFi-GAN MRF stages: own instantiations (same tiles as generic)
      case 1: return launch_cfg<bf16_t, bf16_t, bf16_t, 4, 4, 2, 2, 1>(d, st);
      case 2: return launch_cfg<bf16_t, bf16_t, bf16_t, 4, 4, 2, 2, 2>(d, st);
      case 3: return launch_cfg<bf16_t, bf16_t, bf16_t, 4, 4, 1, 4, 3>(d, st);
      case 4: return launch_cfg<bf16_t, bf16_t, bf16_t, 2, 4, 1, 4, 4>(d, st);
      default: return launch_types<bf16_t, bf16_t, bf16_t>(d, st);
    }
  }
  if (xi == VO_F32 && yo == VO_BF16) return launch_types<float, bf16_t, bf16_t>(d, st);
  if (xi == VO_BF16 && yo == VO_F32) return launch_types<bf16_t, bf16_t, float>(d, st);
  if (xi == VO_F32 && yo == VO_F32) return launch_types<float, bf16_t, float>(d, st);
  vo_set_error("conv1d: bad dtypes");
  return VO_ERR_INVALID;
}
