// HiFi-GAN MRF at C = 32 (the widest-in-time, narrowest-in-channels stage: B x 131072 x 32) with
// WAVE-PRIVATE frames (round 3): every wave owns a whole time frame of its own -- window, halo and
// all -- and runs its convs on it with no workgroup barrier after the one that publishes the
// resident weights.  The k = 3 ResBlock (three (c1, c2) pairs, dilations 1 / 3 / 5,
// scripts/hifigan/models.py:96-103) runs as one launch (MODE 0), a k = 7 / 11 pair as another
// (MODE 1); the MRF sum / 1 / num_kernels scale (models.py:155-160) rides in the last epilogue.
//
// Why: the round-2 C = 32 kernels shared one frame per 8-wave workgroup, so every conv ended in a
// workgroup barrier and all waves ran their epilogues (VALU) at the same moment, their MFMAs at
// another and their window fetch at a third: the SQ counters showed 7-9 VALU instructions per
// MFMA, 45 % of wave cycles waiting and the MFMA pipes 25 % busy (profiles/r03/counters).  Here
// the two waves of a SIMD drift apart freely: one's epilogue or window wait overlaps the other's
// MFMAs.  The price is a halo per wave (frame F yields F - 24 rows for the k = 3 block, F - 2 h2
// for a pair) -- the same redundancy a workgroup frame pays, at wave granularity.
//
// Per wave tile: the window lands in the wave's LDS region by LDS-DMA (swizzle on the source
// address), the residual x rows are read from it, it is lrelu'd in place (rows outside [0, T)
// zeroed), then each conv's MFMAs read the region and its epilogue writes the next input over it
// (T1 = lrelu(c1 + b1); x_{s+1} stays in registers, its lrelu'd copy goes to LDS).  The next
// tile's window DMA is issued before the last epilogue's stores.  Biases enter as the C operand of
// each conv's first MFMA; leaky ReLU in packed fp32.  All weights stay resident in LDS.

// Measured-and-dropped (round 3): compiled only into the A/B library (make abl, -DVO_ABLATIONS).
#ifdef VO_ABLATIONS
#include <algorithm>
#include <type_traits>

#include "mrf_common.h"  // visual_onoma_to_wave_amd/csrc (make abl adds it to the include path)

namespace vo {

struct WaveArgs {
  const bf16_t* x;
  const bf16_t* w[6]; const float* b[6];  // MODE 0: c1_0 c2_0 c1_1 c2_1 c1_2 c2_2; MODE 1: c1 c2
  bf16_t* y; const bf16_t* acc;
  int T, tiles_per_b, ntiles;
  float slope, out_scale;
};

typedef __attribute__((address_space(3))) void w5_lds_void;
typedef const __attribute__((address_space(1))) void w5_g_void;

template <int MODE, int K, int D1, int NJ>
__global__ void __launch_bounds__(512, 1) mrf_wave_kernel(WaveArgs a) {
  constexpr int C = 32, NI = 2, SHW = 3;
  constexpr int NW = 8, NT = NW * 64;
  constexpr int NCV = MODE == 0 ? 6 : 2;                  // convs per tile
  constexpr int H2 = (K - 1) / 2;
  constexpr int HP = MODE == 0 ? 8 : (D1 * H2 + 7) / 8 * 8;  // region pad rows per side
  constexpr int F = 16 * NJ;                              // frame rows (one wave)
  constexpr int RR = F + 2 * HP;                          // region rows
  static_assert(RR % 16 == 0, "window DMA pieces are 16 rows");
  constexpr int HALO = MODE == 0 ? 12 : H2;               // invalid frame rows per side of the output
  constexpr int BT = F - 2 * HALO;                        // output rows per tile
  constexpr int TAPE = C * 32;                            // LDS elements per weight tap (1 plane)
  constexpr int NTAP = NCV * K;
  constexpr int PIECES = RR / 16;
  constexpr int LV = RR * 4 / 64;                         // lrelu-pass vectors per lane

  const int T = a.T;
  const float slope = a.slope;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* wls = reinterpret_cast<bf16_t*>(smem_raw);      // [NTAP][TAPE] resident weights
  float* sbias = reinterpret_cast<float*>(wls + NTAP * TAPE);  // [NCV][C]
  bf16_t* regions = reinterpret_cast<bf16_t*>(sbias + NCV * C);  // [NW][RR][32]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  const int n0 = NI * 4 * lq;
  bf16_t* reg = regions + __builtin_amdgcn_readfirstlane(wave) * (RR * 32);

  // ---- resident weights and biases: the only workgroup barrier
  for (int v = tid; v < NTAP * C * 4; v += NT) {
    const int tp = v / (C * 4), vv = v - tp * (C * 4);
    const int co = vv >> 2, q = vv & 3;
    const bf16_t* W = a.w[tp / K] + (tp % K) * (C * C);
    *reinterpret_cast<u32x4*>(wls + tp * TAPE + rb_off(co, q, SHW)) = *reinterpret_cast<const u32x4*>(W + vv * 8);
  }
  for (int i = tid; i < NCV * C; i += NT) sbias[i] = a.b[i / C][i % C];
  __syncthreads();

  const int W = gridDim.x * NW;
  const int gw = blockIdx.x * NW + wave;
  int tile = (int)(((int64_t)gw * a.ntiles) / W);
  const int tile_end = (int)(((int64_t)(gw + 1) * a.ntiles) / W);
  if (tile >= tile_end) return;  // uniform per wave; no barrier follows

  int a_off[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) a_off[i] = rb_off(NI * 4 * (lr >> 2) + 4 * i + (lr & 3), lq, SHW);

  // window DMA: piece p = region rows [16 p, 16 p + 16); lane l -> row 16 p + l / 4, slot l % 4,
  // which holds chunk (l % 4) ^ swz(row)
  const int wrow = lane >> 2, wq = (lane & 3) ^ ((wrow >> 1) & 2);
  auto frame0 = [&](int tl, int& b) {  // position of frame row 0
    b = tl / a.tiles_per_b;
    return (tl - b * a.tiles_per_b) * BT - HALO;
  };
  auto issue_window = [&](int tl) {
    int b;
    const int P0 = frame0(tl, b);
    const bf16_t* xb = a.x + (int64_t)b * T * C + wq * 8;
#pragma unroll
    for (int p = 0; p < PIECES; ++p) {
      const int t = min(max(P0 - HP + 16 * p + wrow, 0), T - 1);  // clamped; zeroed by the lrelu pass
      __builtin_amdgcn_global_load_lds((w5_g_void*)(xb + (int64_t)t * C), (w5_lds_void*)(reg + p * 512), 16, 0, 0);
    }
  };
  constexpr int NST = NJ;  // y stores per tile (one 16-byte vector per row-fragment and lane)

  issue_window(tile);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the first window (the loop-top wait counts stores)
  f32x4 acc[NI][NJ];
  for (; tile < tile_end; ++tile) {
    int b;
    const int P0 = frame0(tile, b);
    const bool has_next = tile + 1 < tile_end;
    // opaque per tile: the per-tap / per-slot LDS addresses are recomputed where they are used
    // instead of all being hoisted out of the tile loop and held in registers (that spilled)
    int lane_v = lane;
    asm volatile("" : "+v"(lane_v));
    const int lr_t = lane_v & 15;
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");  // this tile's window landed; the
                                                                // previous tile's y stores may fly
    // ---- residual rows: raw x at frame row f = 16 j + lr (region row f + HP), epilogue layout
    u32x4 xres[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      xres[j] = *reinterpret_cast<const u32x4*>(reg + rb_off(16 * j + lr_t + HP, lq, 2));
    // ---- lrelu the window in place; rows outside [0, T) -> 0 (c1's zero padding)
#pragma unroll
    for (int s = 0; s < LV; ++s) {
      const int v = lane_v + 64 * s;  // 16-byte slot v of the region (row v / 4)
      const int t = P0 - HP + (v >> 2);
      bf16_t* p = reg + v * 8;
      const u32x4 u = lrelu8_pk(*reinterpret_cast<const u32x4*>(p), slope);
      *reinterpret_cast<u32x4*>(p) = (t >= 0 && t < T) ? u : u32x4{0u, 0u, 0u, 0u};
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const bool interior = P0 >= 0 && P0 + F <= T;

    u32x4 ares[NJ];
    const bf16_t* accp = a.acc ? a.acc : a.x;
    auto load_acc = [&]() {  // MRF accumulator rows of the output positions (clamped)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int pos = min(max(P0 + 16 * j + lr, 0), T - 1);
        ares[j] = *reinterpret_cast<const u32x4*>(accp + ((int64_t)b * T + pos) * C + n0);
      }
    };

#pragma unroll
    for (int cv = 0; cv < NCV; ++cv) {
      const int dil = MODE == 0 ? ((cv & 1) ? 1 : 2 * (cv >> 1) + 1) : (cv == 0 ? D1 : 1);
      if (cv == NCV - 1) load_acc();
      // ---- MFMAs: frame row f reads region rows f + HP + (k - H2) * dil
      const bf16_t* wc = wls + cv * K * TAPE;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        Frag<bf16_t> af[NI], bfr[NJ];
#pragma unroll
        for (int i = 0; i < NI; ++i) af[i].load(wc + k * TAPE + a_off[i]);
        const int row = lr_t + HP + (k - H2) * dil;
        const int boff = rb_off(row, lq, 2);  // + 16 j rows keep the swizzle
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[j].load(reg + boff + 16 * j * 32);
        if (k == 0) {  // the conv's bias is the C operand of its first MFMAs
#pragma unroll
          for (int i = 0; i < NI; ++i) {
            const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + cv * C + n0 + 4 * i);
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] = mfma(af[i], bfr[j], bv);
          }
        } else {
#pragma unroll
          for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] = mfma(af[i], bfr[j], acc[i][j]);
        }
        // keep the taps apart: hoisting later taps' fragment reads above these MFMAs spills
        __builtin_amdgcn_sched_barrier(0);
      }
      if (cv == NCV - 1) break;
      // ---- epilogue into the region (this wave's reads of it are all issued: LDS runs them in order)
      const bool c1 = MODE == 1 || (cv & 1) == 0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int f = 16 * j + lr_t;
        const int pos = P0 + f;
        const uint32_t km = (interior || (pos >= 0 && pos < T)) ? 0xffffffffu : 0u;
        uint32_t l[4];
        if (c1) {  // T1 = lrelu(c1 + b1), zero outside [0, T) (c2's zero padding)
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) {
            const int e = 2 * e2;
            l[e2] = lrelu_pk(acc[e / 4][j][e & 3], acc[(e + 1) / 4][j][(e + 1) & 3], slope);
          }
        } else {  // x_{s+1} = x_s + c2 + b2 (bf16 in registers), lrelu(x_{s+1}) into the region
          float xf[8];
          unpack8(xres[j], xf);
          uint32_t w[4];
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) {
            const int e = 2 * e2;
            const f32x2v v = f32x2v{acc[e / 4][j][e & 3], acc[(e + 1) / 4][j][(e + 1) & 3]} + f32x2v{xf[e], xf[e + 1]};
            w[e2] = pk_bf16(v.x, v.y);
            l[e2] = lrelu_pk(v.x, v.y, slope);
          }
          xres[j] = u32x4{w[0], w[1], w[2], w[3]};
        }
        if (!interior) {
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) l[e2] &= km;
        }
        *reinterpret_cast<u32x4*>(reg + rb_off(f + HP, lq, 2)) = u32x4{l[0], l[1], l[2], l[3]};
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // visible to this wave's next reads
    }

    // ---- last epilogue: y = (x + c2 + b2) * out_scale (+ acc) on the valid rows.  The loaded rows are
    // consumed first (empty asm uses: hipcc waits for them here), then the next window's DMA is issued
    // (the region's last reads are done), then the stores (the next tile's wait leaves them in flight)
#pragma unroll
    for (int j = 0; j < NJ; ++j) asm volatile("" ::"v"(ares[j]));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the last conv's region reads have returned
    if (has_next) issue_window(tile + 1);
    const int t0 = P0 + HALO;
    const int valid = min(BT, T - t0);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.y + ((int64_t)b * T + t0) * C), (short)0, valid * C * (int)sizeof(bf16_t), 0x00020000);
    auto store_rows = [&](auto with_acc) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float xf[8], af8[8];
        unpack8(xres[j], xf);
        if constexpr (decltype(with_acc)::value) unpack8(ares[j], af8);
        uint32_t w[4];
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          float q[2];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int e = 2 * e2 + u;
            q[u] = (acc[e / 4][j][e & 3] + xf[e]) * a.out_scale;
            if constexpr (decltype(with_acc)::value) q[u] += af8[e];
          }
          w[e2] = pk_bf16(q[0], q[1]);
        }
        const int r = 16 * j + lr - HALO;  // row within the resource; rows before it: past any resource
        const int roff = r >= 0 ? r * C * (int)sizeof(bf16_t) : 0x40000000;
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{w[0], w[1], w[2], w[3]}, yrs, roff + n0 * (int)sizeof(bf16_t), 0, 0);
      }
    };
    if (a.acc)
      store_rows(std::true_type{});
    else
      store_rows(std::false_type{});
  }
}

template <int MODE, int K, int D1, int NJ>
static int wave_launch(WaveArgs a, int B, hipStream_t st) {
  constexpr int C = 32, NW = 8;
  constexpr int NCV = MODE == 0 ? 6 : 2;
  constexpr int H2 = (K - 1) / 2;
  constexpr int HP = MODE == 0 ? 8 : (D1 * H2 + 7) / 8 * 8;
  constexpr int F = 16 * NJ;
  constexpr int RR = F + 2 * HP;
  constexpr int BT = F - 2 * (MODE == 0 ? 12 : H2);
  a.tiles_per_b = (a.T + BT - 1) / BT;
  a.ntiles = a.tiles_per_b * B;
  const size_t lds = (size_t)NCV * K * C * C * sizeof(bf16_t) + NCV * C * sizeof(float) +
                     (size_t)NW * RR * C * sizeof(bf16_t);
  if (lds > 160 * 1024) {
    vo_set_error("mrf wave kernel: LDS %zu B exceeds 160 KiB", lds);
    return VO_ERR_INVALID;
  }
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  const int grid = (int)std::min<int64_t>((int64_t)cus, ((int64_t)a.ntiles + NW - 1) / NW);
  hipLaunchKernelGGL((mrf_wave_kernel<MODE, K, D1, NJ>), dim3((unsigned)grid), dim3(NW * 64), lds, st, a);
  VO_RETURN_LAUNCH();
}

}  // namespace vo

using namespace vo;

// k = 3 ResBlock at C = 32, dilations (1, 3, 5) (vo_resblock3's shape); *handled = 0 otherwise
int vo_rb3_wave_try(const void* x, const void* const* w1, const float* const* b1, const void* const* w2,
                    const float* const* b2, const int* dil, void* y, const void* acc, int B, int T, int C, float slope,
                    float out_scale, int cfg, hipStream_t st, int* handled) {
  *handled = 0;
  if (C != 32 || dil[0] != 1 || dil[1] != 3 || dil[2] != 5) return VO_OK;
  WaveArgs a;
  a.x = (const bf16_t*)x;
  for (int s = 0; s < 3; ++s) {
    a.w[2 * s] = (const bf16_t*)w1[s]; a.b[2 * s] = b1[s];
    a.w[2 * s + 1] = (const bf16_t*)w2[s]; a.b[2 * s + 1] = b2[s];
  }
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)acc;
  a.T = T; a.slope = slope; a.out_scale = out_scale;
  *handled = 1;
  if (cfg == 31) return wave_launch<0, 3, 1, 10>(a, B, st);   // 160-row frames (136 output rows)
  return wave_launch<0, 3, 1, 8>(a, B, st);                   // 128-row frames (104 output rows)
}

// k = 7 / 11 pair at C = 32, dilation 1 / 3 / 5
int vo_pair_wave_try(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                     const void* acc, int B, int T, int C, int K, int dil, float slope, float out_scale, int cfg,
                     hipStream_t st, int* handled) {
  *handled = 0;
  if (C != 32 || !(K == 7 || K == 11) || !(dil == 1 || dil == 3 || dil == 5)) return VO_OK;
  WaveArgs a;
  a.x = (const bf16_t*)x;
  a.w[0] = (const bf16_t*)w1; a.b[0] = b1; a.w[1] = (const bf16_t*)w2; a.b[1] = b2;
  for (int s = 2; s < 6; ++s) { a.w[s] = nullptr; a.b[s] = nullptr; }
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)acc;
  a.T = T; a.slope = slope; a.out_scale = out_scale;
  *handled = 1;
  (void)cfg;
  // frames: 160 rows (region 160 + 2 x 32 pad at k = 11, d = 5)
  if (K == 7) {
    if (dil == 1) return wave_launch<1, 7, 1, 10>(a, B, st);
    if (dil == 3) return wave_launch<1, 7, 3, 10>(a, B, st);
    return wave_launch<1, 7, 5, 10>(a, B, st);
  }
  if (dil == 1) return wave_launch<1, 11, 1, 10>(a, B, st);
  if (dil == 3) return wave_launch<1, 11, 3, 10>(a, B, st);
  return wave_launch<1, 11, 5, 10>(a, B, st);
}
#endif  // VO_ABLATIONS
