// Fused HiFi-GAN ResBlock1 pair for the narrow MRF stages (C = 32 / 64):
//   y = (x + c2(lrelu(c1_d(lrelu(x), slope), slope))) * out_scale (+ acc)
// (scripts/hifigan/models.py:96-103, one (c1, c2) iteration; the Generator's MRF sum and
// 1/num_kernels scale, models.py:155-160, ride in the epilogue).
//
// One workgroup = R1 = 256 consecutive c1-output rows = BT = R1 - (K-1) output positions:
//   phase 1: T1 = lrelu(c1(window) + b1) for positions [t0 - h2, t0 - h2 + R1) straight into
//            LDS (rows outside [0, T) forced to 0 = c2's zero padding); the input window
//            (R1 + (K-1)*dil rows, lrelu applied once while staging) is loaded ONCE for all
//            channel chunks and taps;
//   phase 2: y = c2(T1) + b2 + x (residual re-read from global, L2-hot), scaled/accumulated.
// The intermediate never touches HBM: per position the pair reads x ~1.2x (halo) + once for
// the residual and writes y once (bf16), against 5 activation passes for two separate
// conv launches.  Both GEMMs run on v_mfma_f32_16x16x32_bf16 with the conflict-free
// XOR-swizzled 64-byte LDS rows of conv1d.hip; weights stream through a double buffer,
// TPS taps per barrier.

#include "vo_common.h"

namespace vo {

// c1 rows per workgroup = R1 (template): 4 waves x 16*NJ positions

struct PairArgs {
  const bf16_t* x; const bf16_t* w1; const float* b1; const bf16_t* w2; const float* b2;
  bf16_t* y; const bf16_t* acc;
  int T, K, dil, tiles_per_b;
  float slope, out_scale;
};

__device__ __forceinline__ int rb_off(int r, int q, int sh) { return r * 32 + 8 * (q ^ ((r >> (sh - 1)) & 2)); }

template <int C, int TPS, int RB_R1>
__global__ void __launch_bounds__(256) resblock_pair_kernel(PairArgs a) {
  constexpr int NC = C / 32;              // 32-channel planes
  constexpr int NI = C / 16;              // co tiles per wave (all channels in one wave)
  constexpr int NJ = RB_R1 / 64;          // 16*NJ positions per wave
  constexpr int SHW = NI == 4 ? 4 : 3;    // log2(4 * NI)
  constexpr int WVEC = TPS * C * 4;       // 8-element weight vectors per step (TPS taps x C co x 32 ci)
  constexpr int WV = (WVEC + 255) / 256;

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* smem = reinterpret_cast<bf16_t*>(smem_raw);
  const int K = a.K, dil = a.dil;
  const int h1 = dil * (K - 1) / 2, h2 = (K - 1) / 2;
  const int win_rows = RB_R1 + 2 * h1;
  const int t1_rows = RB_R1 + 16;          // phase-2 reads up to row 255 + K - 1 (garbage rows feed discarded outputs)
  bf16_t* win = smem;                                   // [NC][win_rows][32]
  bf16_t* t1 = win + NC * win_rows * 32;                // [NC][t1_rows][32]
  bf16_t* wbuf = t1 + NC * t1_rows * 32;                // [2][TPS][C][32]
  constexpr int WSTRIDE = TPS * C * 32;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  const int BT = RB_R1 - 2 * h2;
  const int b = blockIdx.x / a.tiles_per_b;
  const int t0 = (blockIdx.x - b * a.tiles_per_b) * BT;
  const bf16_t* X = a.x + (int64_t)b * a.T * C;
  const float slope = a.slope;

  // ---- stage the lrelu'd input window, all planes (positions t0 - h2 - h1 + r).  Every
  // load is issued before the first one is consumed (compile-time-bounded register array):
  // a runtime-trip-count load->store loop serialises one HBM round trip per iteration.
  {
    constexpr int MAXW = (NC * (RB_R1 + 128) * 4 + 255) / 256;
    const int row0 = t0 - h2 - h1;
    const int nvec = NC * win_rows * 4;
    uint4 buf[MAXW];
#pragma unroll
    for (int i = 0; i < MAXW; ++i) {
      const int v = tid + i * 256;
      const int pl = v / (win_rows * 4);
      const int rem = v - pl * win_rows * 4;
      const int t = row0 + (rem >> 2);
      buf[i] = make_uint4(0, 0, 0, 0);
      if (v < nvec && t >= 0 && t < a.T)
        buf[i] = *reinterpret_cast<const uint4*>(X + (int64_t)t * C + pl * 32 + (rem & 3) * 8);
    }
#pragma unroll
    for (int i = 0; i < MAXW; ++i) {
      const int v = tid + i * 256;
      if (v >= nvec) break;
      const int pl = v / (win_rows * 4);
      const int rem = v - pl * win_rows * 4;
      const int r = rem >> 2, q = rem & 3;
      const uint4 u = buf[i];
      float f[8];
      uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f[2 * i] = __uint_as_float(w[i] << 16);
        f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = f[e] > 0.f ? f[e] : f[e] * slope;
      store8(win + pl * win_rows * 32 + rb_off(r, q, 2), f);
    }
  }

  // ---- weight streaming: step s covers (phase, plane c, taps k0..k0+TPS-1)
  const int tsteps = (K + TPS - 1) / TPS;
  const int S1 = NC * tsteps;
  const int S = 2 * S1;
  int wg[WV], wl[WV], wk[WV];
  bool wv_ok[WV];
#pragma unroll
  for (int s = 0; s < WV; ++s) {
    const int v = tid + s * 256;
    const int r = v >> 2, q = v & 3;  // r = t * C + co
    const int t = r / C, co = r - t * C;
    wv_ok[s] = v < WVEC;
    wk[s] = t;
    wg[s] = co * C + q * 8;
    wl[s] = t * C * 32 + rb_off(co, q, SHW);
  }
  uint4 w_r[WV];
  auto load_w = [&](int s) {
    const int ph = s >= S1;
    const int ss = s - ph * S1;
    const int c = ss / tsteps, k0 = (ss - c * tsteps) * TPS;
    const bf16_t* W = ph ? a.w2 : a.w1;
#pragma unroll
    for (int i = 0; i < WV; ++i) {
      const int k = min(k0 + wk[i], K - 1);
      if (wv_ok[i]) w_r[i] = *reinterpret_cast<const uint4*>(W + (int64_t)k * C * C + wg[i] + c * 32);
    }
  };
  auto store_w = [&](int buf) {
#pragma unroll
    for (int i = 0; i < WV; ++i)
      if (wv_ok[i]) *reinterpret_cast<uint4*>(wbuf + buf * WSTRIDE + wl[i]) = w_r[i];
  };

  int a_off[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) a_off[i] = rb_off(NI * 4 * (lr >> 2) + 4 * i + (lr & 3), lq, SHW);
  const int brow0 = wave * 16 * NJ + lr;

  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_w(0);
  store_w(0);
  __syncthreads();

  const int g = lane >> 4;
  const int n0 = NI * 4 * g;  // this lane's first output channel (4*NI contiguous channels)
  for (int s = 0; s < S; ++s) {
    if (s + 1 < S) load_w(s + 1);
    const int ph = s >= S1;
    const int ss = s - ph * S1;
    const int c = ss / tsteps, k0 = (ss - c * tsteps) * TPS;
    const bf16_t* wb = wbuf + (s & 1) * WSTRIDE;
    const bf16_t* src = ph ? (t1 + c * t1_rows * 32) : (win + c * win_rows * 32);
    const int step = ph ? 1 : dil;
#pragma unroll
    for (int t = 0; t < TPS; ++t) {
      if (k0 + t < K) {
        Frag<bf16_t> af[NI], bfr[NJ];
#pragma unroll
        for (int i = 0; i < NI; ++i) af[i].load(wb + t * C * 32 + a_off[i]);
        const int br = brow0 + (k0 + t) * step;
        const int boff = rb_off(br, lq, 2);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[j].load(src + boff + 16 * j * 32);
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = mfma(af[i], bfr[j], acc[i][j]);
      }
    }
    if (s + 1 < S) store_w((s + 1) & 1);

    if (s == S1 - 1) {
      // phase-1 epilogue: T1 = lrelu(acc + b1), zero outside [0, T) (c2's zero padding)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = wave * 16 * NJ + 16 * j + lr;
        const int pos = t0 - h2 + r;
        const bool inside = pos >= 0 && pos < a.T;
        float v[4 * NI];
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float z = acc[i][j][e] + a.b1[n0 + 4 * i + e];
            v[4 * i + e] = inside ? (z > 0.f ? z : z * slope) : 0.f;
          }
#pragma unroll
        for (int h = 0; h < NI / 2; ++h) {  // 8-channel chunks
          const int ch = n0 + 8 * h;
          float f[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = v[8 * h + e];
          store8(t1 + (ch / 32) * t1_rows * 32 + rb_off(r, (ch & 31) / 8, 2), f);
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    __syncthreads();
  }

  // ---- phase-2 epilogue: y = (c2 + b2 + x) * out_scale (+ acc)
  bf16_t* Y = a.y + (int64_t)b * a.T * C;
  const bf16_t* A = a.acc ? a.acc + (int64_t)b * a.T * C : nullptr;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int r = wave * 16 * NJ + 16 * j + lr;
    const int pos = t0 + r;
    if (r >= BT || pos >= a.T) continue;
    const int64_t off = (int64_t)pos * C + n0;
#pragma unroll
    for (int h = 0; h < NI; ++h) {
      float xr[4], q[4];
      load4(X + off + 4 * h, xr);
#pragma unroll
      for (int e = 0; e < 4; ++e) q[e] = (acc[h][j][e] + a.b2[n0 + 4 * h + e] + xr[e]) * a.out_scale;
      if (A) {
        float ar[4];
        load4(A + off + 4 * h, ar);
#pragma unroll
        for (int e = 0; e < 4; ++e) q[e] += ar[e];
      }
      store4(Y + off + 4 * h, q);
    }
  }
}

template <int C, int TPS, int RB_R1>
static int pair_launch(const PairArgs& a0, int B, int T, int K, int dil, hipStream_t st) {
  PairArgs a = a0;
  const int h1 = dil * (K - 1) / 2, h2 = (K - 1) / 2;
  const int BT = RB_R1 - 2 * h2;
  a.tiles_per_b = (T + BT - 1) / BT;
  const size_t lds = ((size_t)(C / 32) * (RB_R1 + 2 * h1) * 32 + (size_t)(C / 32) * (RB_R1 + 16) * 32 +
                      2 * (size_t)TPS * C * 32) * sizeof(bf16_t);
  if (lds > 160 * 1024) {
    vo_set_error("resblock_pair: LDS %zu B exceeds 160 KiB", lds);
    return VO_ERR_INVALID;
  }
  hipLaunchKernelGGL((resblock_pair_kernel<C, TPS, RB_R1>), dim3((unsigned)(a.tiles_per_b * B)), dim3(256), lds, st, a);
  VO_RETURN_LAUNCH();
}

}  // namespace vo

using namespace vo;

extern "C" int vo_resblock_pair(const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                                void* y, const void* acc, int B, int T, int C, int K, int dil, float slope,
                                float out_scale, void* stream) {
  VO_CHECK_ARG(x && w1 && b1 && w2 && b2 && y, "resblock_pair: null pointer");
  VO_CHECK_ARG(C == 32 || C == 64, "resblock_pair: C=%d unsupported (32 or 64)", C);
  VO_CHECK_ARG(K % 2 == 1 && K >= 1 && dil >= 1 && dil * (K - 1) <= 128 && K <= 15,
               "resblock_pair: K=%d dil=%d unsupported", K, dil);
  VO_CHECK_ARG(B > 0 && T > 0, "resblock_pair: empty");
  VO_CHECK_ARG(y != x, "resblock_pair: y must not alias x (the residual is re-read)");
  PairArgs a;
  a.x = (const bf16_t*)x; a.w1 = (const bf16_t*)w1; a.b1 = b1; a.w2 = (const bf16_t*)w2; a.b2 = b2;
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)acc;
  a.T = T; a.K = K; a.dil = dil; a.slope = slope; a.out_scale = out_scale;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int cfg = vo_tune_get("pair_cfg");
  if (C == 32) return cfg == 1 ? pair_launch<32, 8, 256>(a, B, T, K, dil, st) : pair_launch<32, 4, 256>(a, B, T, K, dil, st);
  return cfg == 1 ? pair_launch<64, 4, 128>(a, B, T, K, dil, st) : pair_launch<64, 2, 128>(a, B, T, K, dil, st);
}
