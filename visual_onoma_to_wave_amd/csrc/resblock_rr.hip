// Register-resident HiFi-GAN ResBlock1, kernel size 3 (round 4): the whole block
//   x1 = x  + c2_0(lrelu(c1_1(lrelu x )))
//   x2 = x1 + c2_1(lrelu(c1_3(lrelu x1)))
//   y  = (x2 + c2_2(lrelu(c1_5(lrelu x2)))) * out_scale (+ acc)
// (scripts/hifigan/models.py:96-103 with dilations (1, 3, 5); the MRF sum / num_kernels scale of
// :155-160 in the epilogue) for the narrow stages, C = 32 and C = 64, with NO workgroup barrier
// after the weights are staged.
//
// Why: the LDS-frame kernel (resblock3.hip) spends 36-49 % of its wave cycles at the six per-conv
// barriers and 4.5-7 VALU instructions per MFMA rewriting the LDS frame (round-3 counters).  Here
// each wave owns a frame of NB 16-row blocks and keeps every activation in registers:
//
// * Layout.  A conv is D = W . X with M = output channels, N = 16 time rows, K = 32 input
//   channels (v_mfma_f32_16x16x32_bf16).  The packed weights' output channels are permuted so that
//   co-block b, accumulator row 4g + r is channel 32 (b / 2) + 8 g + 4 (b % 2) + r: lane l of the
//   two co-blocks 2s, 2s + 1 then holds channels 32 s + 8 (l / 16) + 0..7 of time row l % 16 --
//   exactly the B operand of K-step s of the next conv, and exactly 16 contiguous bytes of a
//   channels-last row in HBM.  A conv's output becomes the next conv's input with no data
//   movement: lrelu, one packed convert, done.
// * Taps.  Tap k of a conv with dilation d reads rows t + (k - 1) d: a lane shift inside each
//   16-lane row of the B operand, two DPP moves per dword (row_shl from the block, row_shr from
//   its neighbour for the lanes that cross the block edge).
// * Halo.  Every conv runs over the whole frame and the valid rows shrink by the halo (12 per
//   side for dilations 1, 3, 5); a frame of 16 NB rows yields 16 NB - 24 output rows.
// * Weights.  All 18 taps of the block live in LDS, fragment-major (each A fragment is 1 KiB,
//   lane l at byte 16 l: conflict-free ds_read_b128), staged once per workgroup: C = 64 144 KiB,
//   C = 32 36 KiB.  One A fragment feeds NB MFMAs.
// * Memory.  The next frame is requested at the start of a tile and the MRF accumulator rows at
//   the start of the last conv, through buffer resources whose range checks return 0 for rows
//   outside the utterance (the convs' zero padding) and drop the stores of halo rows.
//
// Accumulation order per output: bias, then tap-major, K-steps inner -- the order of the
// LDS-frame kernel is plane-major within a tap as well, so results agree to fp32 summation order.

#include <algorithm>
#include <type_traits>
#include <utility>

#include "mrf_common.h"

namespace vo {

struct RrArgs {
  const bf16_t* x;
  const bf16_t* w[6];  // c1_0, c2_0, c1_1, c2_1, c1_2, c2_2: packed (3, C, C) bf16
  const float* bias[6];
  bf16_t* y;
  const bf16_t* acc;
  int T, tiles_per_b, ntiles;
  float slope, out_scale;
};

constexpr int RR_HALO = 12;  // rows lost per side over the six convs (dilations 1, 3, 5)

// a copy the compiler cannot see through: the residual's unpack in an epilogue must not be CSE'd with
// the unpack inside the lrelu that made the conv input from the same registers (that kept the
// unpacked fp32 copy -- twice the residual's registers -- live through the whole conv)
__device__ __forceinline__ u32x4 opaque(u32x4 v) {
  asm volatile("" : "+v"(v));
  return v;
}

// f(integral_constant<int, i>) for i = 0 .. N - 1, unrolled at compile time
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// Frame layout ("lane-major"): lane column c (= lane % 16) of block n holds frame row c * NB + n, so a
// shift by O rows moves block n to block n + O when that stays in [0, NB) -- a register rename --
// and otherwise to block n + O -+ NB one lane over (one DPP move per dword, zero at the frame edge)
template <int O, int NB, int NS, int n>
__device__ __forceinline__ u32x4 shifted(const u32x4 (&in)[NB][NS], int s) {
  constexpr int m = n + O;
  constexpr int q = m >= 0 ? m / NB : -((-m + NB - 1) / NB);  // floor(m / NB)
  constexpr int r = m - q * NB;
  static_assert(q > -16 && q < 16, "shift");
  if constexpr (q == 0) {
    return in[r][s];
  } else {
    // row_shl:q (lane i reads lane i + q) / row_shr:-q (lane i reads i + q); bound_ctrl: 0 past the edge
    constexpr int ctrl = q > 0 ? 0x100 + q : 0x110 - q;
    u32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (unsigned)__builtin_amdgcn_mov_dpp((int)in[r][s][i], ctrl, 0xf, 0xf, true);
    return v;
  }
}

// NWV waves per workgroup (NWV / 4 per SIMD); PF: the next frame requested at the start of a tile
// (registers permitting; otherwise the partner wave covers the latency)
template <int C, int NB, int NWV, bool PF, bool PA = false, bool PL = false>
__global__ void __launch_bounds__(NWV * 64, 1) mrf_rr3_kernel(RrArgs a) {
  constexpr int NS = C / 32;   // K-steps (32-channel planes)
  constexpr int NCB = C / 16;  // 16-channel output blocks
  constexpr int NT = NWV * 64;
  constexpr int F = 16 * NB;   // frame rows
  constexpr int OR = F - 2 * RR_HALO;
  constexpr int NFR = 6 * 3 * NS * NCB;  // A fragments
  constexpr int NST = 3 * NS;            // (tap, K-step) steps per conv
  static_assert(C == 32 || C == 64, "narrow stages");
  static_assert((6 * NST) % 2 == 0, "fragment double buffer parity repeats per tile");

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  u32x4* wfr = reinterpret_cast<u32x4*>(smem_raw);              // [NFR][64 lanes]
  float* sb = reinterpret_cast<float*>(smem_raw + NFR * 1024);  // [6][C]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: the buffer resources stay scalar
  const int lr = lane & 15, lq = lane >> 4;
  const int T = a.T;
  const float slope = a.slope;

  // ---- weights (fragment-major, output channels permuted) and biases, once per workgroup
  for (int i = tid; i < NFR * 64; i += NT) {
    const int f = i >> 6, l = i & 63;
    const int b = f % NCB, s = (f / NCB) % NS, k = (f / (NCB * NS)) % 3, cv = f / (NCB * NS * 3);
    const int m = l & 15;
    const int co = 32 * (b >> 1) + 8 * (m >> 2) + 4 * (b & 1) + (m & 3);
    wfr[i] = *reinterpret_cast<const u32x4*>(a.w[cv] + k * C * C + co * C + 32 * s + 8 * (l >> 4));
  }
  for (int i = tid; i < 6 * C; i += NT) sb[i] = a.bias[i / C][i % C];
  __syncthreads();

  const int gw = blockIdx.x * NWV + wave, nw = gridDim.x * NWV;
  int tile = (int)(((int64_t)gw * a.ntiles) / nw);
  const int tile_end = (int)(((int64_t)(gw + 1) * a.ntiles) / nw);
  if (tile >= tile_end) return;  // per wave: no barrier follows

  const int lane_off = 2 * (lr * NB * C + 8 * lq);  // bytes: frame row lr * NB, channels 8 lq.. of plane 0
  auto utt_rsrc = [&](const bf16_t* base, int b) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (int64_t)b * T * C), (short)0, T * C * 2, 0x00020000);
  };
  // frame of tile tl: rows w0 .. w0 + F - 1 of utterance b (rows outside it read as 0)
  auto load_rows = [&](const bf16_t* base, int tl, u32x4 (&fr)[NB][NS]) {
    const int b = tl / a.tiles_per_b;
    const int w0 = (tl - b * a.tiles_per_b) * OR - RR_HALO;
    const __amdgpu_buffer_rsrc_t rs = utt_rsrc(base, b);
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int s = 0; s < NS; ++s)
        fr[n][s] = __builtin_amdgcn_raw_buffer_load_b128(rs, (w0 + n) * C * 2 + lane_off, 64 * s, 0);
  };

  // PF: the next frame requested at the start of a tile; PL: after the last conv's MFMAs, into the
  // registers its input has just freed (in flight during the final epilogue and stores)
  u32x4 xn[(PF || PL) ? NB : 1][NS];
  if constexpr (PF || PL) load_rows(a.x, tile, xn);
  u32x4 af[2][NCB];  // A fragments: step g of a tile uses af[g & 1]
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) af[0][cb] = wfr[(NS * NCB + cb) * 64 + lane];  // (conv 0, tap 1, K-step 0)

  for (; tile < tile_end; ++tile) {
    const int b = tile / a.tiles_per_b;
    const int t0 = (tile - b * a.tiles_per_b) * OR;  // first output row
    const int w0 = t0 - RR_HALO;
    const bool interior = w0 >= 0 && w0 + F <= T;
    u32x4 xb[NB][NS], in[NB][NS];
    if constexpr (PF || PL) {
#pragma unroll
      for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int s = 0; s < NS; ++s) xb[n][s] = xn[n][s];
      if constexpr (PF) load_rows(a.x, tile + 1 < tile_end ? tile + 1 : tile, xn);  // unconditional
    } else {
      load_rows(a.x, tile, xb);
    }
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int s = 0; s < NS; ++s) in[n][s] = lrelu8_pk(xb[n][s], slope);  // rows outside [0, T): 0

    // the fragment reads depend on the tile (opaque to the compiler): otherwise they are
    // loop-invariant and hoisted out of the tile loop, 4 registers per fragment for all 18 taps
    int fl = lane;
    asm volatile("" : "+v"(fl));
    const u32x4* wl = wfr + fl;
    f32x4 acc[NB][NCB];

    auto conv = [&](auto cvc) {
      constexpr int cv = decltype(cvc)::value;
      constexpr int d = (cv & 1) ? 1 : (cv == 0 ? 1 : (cv == 2 ? 3 : 5));
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {  // bias: the C operand of the first MFMA
        const f32x4 bv = *reinterpret_cast<const f32x4*>(sb + cv * C + 32 * (cb >> 1) + 8 * lq + 4 * (cb & 1));
#pragma unroll
        for (int n = 0; n < NB; ++n) acc[n][cb] = bv;
      }
      // (tap, K-step) steps, centre tap first (its operands need no shift); the A fragments of the
      // next step -- across convs and tiles -- are requested before the MFMAs of this one
      auto tap = [&](auto kc, auto jc) {
        constexpr int k = decltype(kc)::value;
        constexpr int j0 = decltype(jc)::value;  // step of the conv at K-step 0
        constexpr int O = (k - 1) * d;
        constexpr int kn = k == 1 ? 0 : (k == 0 ? 2 : 1);  // the next tap (after tap 2: the next conv)
        constexpr int cvn = k == 2 ? (cv + 1) % 6 : cv;
        auto ks = [&](auto sc) {
          constexpr int s = decltype(sc)::value;
          constexpr int g = cv * NST + j0 + s;  // step of the tile
          constexpr int fn = s + 1 < NS ? (((cv * 3 + k) * NS + s + 1) * NCB) : (((cvn * 3 + kn) * NS) * NCB);
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb) af[(g + 1) & 1][cb] = wl[(fn + cb) * 64];
          __builtin_amdgcn_sched_barrier(0);
          auto blk = [&](auto nc) {
            constexpr int n = decltype(nc)::value;
            const bf16x8 bv = __builtin_bit_cast(bf16x8, shifted<O, NB, NS, n>(in, s));
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb)
              acc[n][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[g & 1][cb]), bv,
                                                                  acc[n][cb], 0, 0, 0);
          };
          static_for<NB>(blk);
        };
        static_for<NS>(ks);
      };
      tap(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{});
      tap(std::integral_constant<int, 0>{}, std::integral_constant<int, NS>{});
      tap(std::integral_constant<int, 2>{}, std::integral_constant<int, 2 * NS>{});

      // epilogues; masks (rows outside [0, T) -> 0: the next conv's zero padding) in edge tiles only
      auto epi = [&](auto edge) {
        constexpr bool EDGE = decltype(edge)::value;
#pragma unroll
        for (int n = 0; n < NB; ++n) {
          uint32_t km = 0xffffffffu;
          if constexpr (EDGE) {
            const int pos = w0 + lr * NB + n;
            km = (pos >= 0 && pos < T) ? 0xffffffffu : 0u;
          }
#pragma unroll
          for (int s = 0; s < NS; ++s) {
            const f32x4 lo = acc[n][2 * s], hi = acc[n][2 * s + 1];
            const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            if constexpr ((cv & 1) == 0) {  // T1 = lrelu(c1 + b1)
              uint32_t w[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                w[e] = pk_bf16(lrelu_max(v[2 * e], slope), lrelu_max(v[2 * e + 1], slope));
                if constexpr (EDGE) w[e] &= km;
              }
              in[n][s] = u32x4{w[0], w[1], w[2], w[3]};
            } else {  // x_{s+1} = x_s + c2 + b2 (bf16), lrelu from the fp32 sum
              float xf[8];
              unpack8(opaque(xb[n][s]), xf);
              uint32_t w[4], l[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float z0 = v[2 * e] + xf[2 * e], z1 = v[2 * e + 1] + xf[2 * e + 1];
                w[e] = pk_bf16(z0, z1);
                l[e] = pk_bf16(lrelu_max(z0, slope), lrelu_max(z1, slope));
                if constexpr (EDGE) l[e] &= km;
              }
              xb[n][s] = u32x4{w[0], w[1], w[2], w[3]};
              in[n][s] = u32x4{l[0], l[1], l[2], l[3]};
            }
          }
        }
      };
      if constexpr (cv < 5) {
        if (interior)
          epi(std::false_type{});
        else
          epi(std::true_type{});
      }
    };
    conv(std::integral_constant<int, 0>{});
    conv(std::integral_constant<int, 1>{});
    conv(std::integral_constant<int, 2>{});
    conv(std::integral_constant<int, 3>{});
    conv(std::integral_constant<int, 4>{});
    // PA: the MRF accumulator rows requested before the last conv (in flight during its MFMAs)
    u32x4 ainp[PA ? NB : 1][NS];
    if constexpr (PA) load_rows(a.acc ? a.acc : a.x, tile, ainp);
    conv(std::integral_constant<int, 5>{});
    if constexpr (PL) load_rows(a.x, tile + 1 < tile_end ? tile + 1 : tile, xn);

    // y = (x2 + c2 + b2) * out_scale (+ acc) on rows t0 .. t0 + valid - 1 = frame rows HALO ..: a
    // resource over exactly those rows drops the halo rows' stores (rows before it: an offset past
    // any resource)
    const int valid = min(OR, T - t0);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.y + ((int64_t)b * T + t0) * C), (short)0, valid * C * 2, 0x00020000);
    auto fin = [&](auto with_acc) {
      constexpr bool ACC = decltype(with_acc)::value;
      u32x4 ain[ACC ? NB : 1][NS];
      if constexpr (ACC) {
        if constexpr (PA) {
#pragma unroll
          for (int n = 0; n < NB; ++n)
#pragma unroll
            for (int s = 0; s < NS; ++s) ain[n][s] = ainp[n][s];
        } else {
          load_rows(a.acc, tile, ain);
        }
      }
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const int r = lr * NB + n - RR_HALO;
        const int off = r >= 0 ? r * C * 2 + 16 * lq : 0x40000000;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const f32x4 lo = acc[n][2 * s], hi = acc[n][2 * s + 1];
          const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          float xf[8], af8[8];
          unpack8(opaque(xb[n][s]), xf);
          if constexpr (ACC) unpack8(ain[n][s], af8);
          uint32_t w[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float z0 = (v[2 * e] + xf[2 * e]) * a.out_scale, z1 = (v[2 * e + 1] + xf[2 * e + 1]) * a.out_scale;
            if constexpr (ACC) {
              z0 += af8[2 * e];
              z1 += af8[2 * e + 1];
            }
            w[e] = pk_bf16(z0, z1);
          }
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{w[0], w[1], w[2], w[3]}, yrs, off, 64 * s, 0);
        }
      }
    };
    if (a.acc)
      fin(std::true_type{});
    else
      fin(std::false_type{});
  }
}

// ------------------------------------------------------------------------------------------------
// The same block on v_mfma_f32_32x32x16_bf16 ("w"): 32-row blocks, 16-channel K-steps, 32-channel
// output blocks.  A 32x32x16 MFMA holds the SIMD's vector issue for 8 of its 32 cycles, so one wave
// hides ~6 VALU instructions behind each (16x16x32: ~2 per 16 cycles) -- the epilogues' leaky ReLU /
// residual / convert work is what binds these narrow blocks.
//   B operand (K-step s): lane l = 32 h + c holds channels 16 s + 8 h + 0..7 of frame row c NB + n.
//   D (co-block cb): lane (h, c), register r = 8 u + j holds D row (j & 3) + 16 u + 8 (j >> 2) + 4 h,
//   which the weight pack maps to channel 32 cb + 16 u + 8 h + j: registers 8u .. 8u + 7 ARE the B
//   operand of K-step 2 cb + u.
//   Bias: one extra MFMA per (block, co-block) and conv, A = the bias split into bf16 hi + lo in K
//   columns 0 and 1, B = ones there, C = 0 -- no accumulator initialisation by VALU.
//   Shifts: a lane step crosses the 16-lane DPP rows: wave_shl:1 / wave_shr:1 (lanes 31 / 32 then
//   mix the two K halves: frame-edge rows, invalid by then anyway).
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int O, int NB, int NK, int n>
__device__ __forceinline__ u32x4 shifted_w(const u32x4 (&in)[NB][NK], int s) {
  constexpr int m = n + O;
  constexpr int q = m >= 0 ? m / NB : -((-m + NB - 1) / NB);  // floor(m / NB): lanes to move
  constexpr int r = m - q * NB;
  static_assert(q >= -2 && q <= 2, "|shift| <= 2 NB");
  if constexpr (q == 0) {
    return in[r][s];
  } else {
    constexpr int ctrl = q > 0 ? 0x130 : 0x138;  // wave_shl:1 (lane i reads i + 1) / wave_shr:1
    u32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int t = __builtin_amdgcn_mov_dpp((int)in[r][s][i], ctrl, 0xf, 0xf, true);
      if constexpr (q == 2 || q == -2) t = __builtin_amdgcn_mov_dpp(t, ctrl, 0xf, 0xf, true);
      v[i] = (unsigned)t;
    }
    return v;
  }
}

__device__ __forceinline__ int rrw_perm(int cb, int m) {  // D row m of co-block cb -> output channel
  return 32 * cb + 16 * (m >> 4) + 8 * ((m >> 2) & 1) + (m & 3) + 4 * ((m >> 3) & 1);
}

template <int C, int NB, int NWV, bool PF, bool RM>
__global__ void __launch_bounds__(NWV * 64, 1) mrf_rr3w_kernel(RrArgs a) {
  constexpr int NK = C / 16;   // 16-channel K-steps
  constexpr int NCB = C / 32;  // 32-channel output blocks
  constexpr int NT = NWV * 64;
  constexpr int F = 32 * NB;
  constexpr int OR = F - 2 * RR_HALO;
  constexpr int NFR = 6 * 3 * NK * NCB;  // weight fragments; then 6 * NCB bias fragments
  constexpr int NST = 3 * NK;
  static_assert(C == 32 || C == 64, "narrow stages");
  static_assert(2 * NB >= 5, "dilation 5 shifts by at most two lanes");

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  u32x4* wfr = reinterpret_cast<u32x4*>(smem_raw);  // [NFR + 6 NCB][64 lanes]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lc = lane & 31, lh = lane >> 5;
  const int T = a.T;
  const float slope = a.slope;

  for (int i = tid; i < (NFR + 6 * NCB) * 64; i += NT) {
    const int f = i >> 6, l = i & 63;
    const int m = l & 31, hh = l >> 5;
    if (f < NFR) {
      const int cb = f % NCB, s = (f / NCB) % NK, k = (f / (NCB * NK)) % 3, cv = f / (NCB * NK * 3);
      wfr[i] = *reinterpret_cast<const u32x4*>(a.w[cv] + k * C * C + rrw_perm(cb, m) * C + 16 * s + 8 * hh);
    } else {
      const int cb = (f - NFR) % NCB, cv = (f - NFR) / NCB;
      u32x4 v = u32x4{0u, 0u, 0u, 0u};
      if (hh == 0) {  // K columns 0 / 1: the fp32 bias as bf16 hi + lo
        const float bvv = a.bias[cv][rrw_perm(cb, m)];
        const uint32_t hi = __float_as_uint(bvv) & 0xffff0000u;
        const float lo = bvv - __uint_as_float(hi);
        v.x = (hi >> 16) | (pk_bf16(lo, 0.f) << 16);
      }
      wfr[i] = v;
    }
  }
  __syncthreads();

  const int gw = blockIdx.x * NWV + wave, nw = gridDim.x * NWV;
  int tile = (int)(((int64_t)gw * a.ntiles) / nw);
  const int tile_end = (int)(((int64_t)(gw + 1) * a.ntiles) / nw);
  if (tile >= tile_end) return;

  const int lane_off = 2 * (lc * NB * C + 8 * lh);
  auto utt_rsrc = [&](const bf16_t* base, int b) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (int64_t)b * T * C), (short)0, T * C * 2, 0x00020000);
  };
  auto load_rows = [&](const bf16_t* base, int tl, u32x4 (&fr)[NB][NK]) {
    const int b = tl / a.tiles_per_b;
    const int w0 = (tl - b * a.tiles_per_b) * OR - RR_HALO;
    const __amdgpu_buffer_rsrc_t rs = utt_rsrc(base, b);
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int s = 0; s < NK; ++s)
        fr[n][s] = __builtin_amdgcn_raw_buffer_load_b128(rs, (w0 + n) * C * 2 + lane_off, 32 * s, 0);
  };
  const u32x4 ones = u32x4{lh == 0 ? 0x3f803f80u : 0u, 0u, 0u, 0u};  // B: 1.0 in K rows 0 and 1
  const bf16x8 onesv = __builtin_bit_cast(bf16x8, ones);
  // RM: the residual x_s enters a c2 conv's accumulator through two more MFMAs per (block, co-block)
  // with permuted-identity A fragments (K-step 2 cb + v, v = 0 / 1; the same for every cb): exact
  // (x * 1.0 summed in fp32), and the epilogue needs no bf16 unpack and add (2 VALU per value)
  bf16x8 idf[2];
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int m = lane & 31;
    const int um = m >> 4, hm = (m >> 2) & 1, jm = (m & 3) + 4 * ((m >> 3) & 1);
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (um == v && lh == hm) w[jm >> 1] = (jm & 1) ? 0x3f800000u : 0x00003f80u;
    idf[v] = __builtin_bit_cast(bf16x8, u32x4{w[0], w[1], w[2], w[3]});
  }

  u32x4 xn[PF ? NB : 1][NK];
  if constexpr (PF) load_rows(a.x, tile, xn);
  u32x4 af[2][NCB];
  u32x4 abias[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    af[0][cb] = wfr[(NK * NCB + cb) * 64 + lane];  // (conv 0, tap 1, K-step 0)
    abias[cb] = wfr[(NFR + cb) * 64 + lane];
  }

  for (; tile < tile_end; ++tile) {
    const int b = tile / a.tiles_per_b;
    const int t0 = (tile - b * a.tiles_per_b) * OR;
    const int w0 = t0 - RR_HALO;
    const bool interior = w0 >= 0 && w0 + F <= T;
    u32x4 xb[NB][NK], in[NB][NK];
    if constexpr (PF) {
#pragma unroll
      for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int s = 0; s < NK; ++s) xb[n][s] = xn[n][s];
      load_rows(a.x, tile + 1 < tile_end ? tile + 1 : tile, xn);
    } else {
      load_rows(a.x, tile, xb);
    }
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int s = 0; s < NK; ++s) in[n][s] = lrelu8_pk(xb[n][s], slope);

    int fl = lane;
    asm volatile("" : "+v"(fl));
    const u32x4* wl = wfr + fl;
    f32x16 acc[NB][NCB];

    auto conv = [&](auto cvc) {
      constexpr int cv = decltype(cvc)::value;
      constexpr int d = (cv & 1) ? 1 : (cv == 0 ? 1 : (cv == 2 ? 3 : 5));
      const f32x16 zero = {};
#pragma unroll
      for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
          acc[n][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, abias[cb]), onesv, zero, 0, 0, 0);
      if constexpr (RM && (cv & 1)) {
#pragma unroll
        for (int n = 0; n < NB; ++n)
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
            for (int v = 0; v < 2; ++v)
              acc[n][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(idf[v], __builtin_bit_cast(bf16x8, xb[n][2 * cb + v]),
                                                                  acc[n][cb], 0, 0, 0);
      }
      auto tap = [&](auto kc, auto jc) {
        constexpr int k = decltype(kc)::value;
        constexpr int j0 = decltype(jc)::value;
        constexpr int O = (k - 1) * d;
        constexpr int kn = k == 1 ? 0 : (k == 0 ? 2 : 1);
        constexpr int cvn = k == 2 ? (cv + 1) % 6 : cv;
        auto ks = [&](auto sc) {
          constexpr int s = decltype(sc)::value;
          constexpr int g = cv * NST + j0 + s;
          constexpr bool last = k == 2 && s + 1 == NK;  // the conv's last step: fetch the next conv's bias too
          constexpr int fn = s + 1 < NK ? (((cv * 3 + k) * NK + s + 1) * NCB) : (((cvn * 3 + kn) * NK) * NCB);
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb) {
            af[(g + 1) & 1][cb] = wl[(fn + cb) * 64];
            if constexpr (last) abias[cb] = wl[(NFR + cvn * NCB + cb) * 64];
          }
          __builtin_amdgcn_sched_barrier(0);
          auto blk = [&](auto nc) {
            constexpr int n = decltype(nc)::value;
            const bf16x8 bv = __builtin_bit_cast(bf16x8, shifted_w<O, NB, NK, n>(in, s));
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb)
              acc[n][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[g & 1][cb]), bv,
                                                                  acc[n][cb], 0, 0, 0);
          };
          static_for<NB>(blk);
        };
        static_for<NK>(ks);
      };
      tap(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{});
      tap(std::integral_constant<int, 0>{}, std::integral_constant<int, NK>{});
      tap(std::integral_constant<int, 2>{}, std::integral_constant<int, 2 * NK>{});

      auto epi = [&](auto edge) {
        constexpr bool EDGE = decltype(edge)::value;
#pragma unroll
        for (int n = 0; n < NB; ++n) {
          uint32_t km = 0xffffffffu;
          if constexpr (EDGE) {
            const int pos = w0 + lc * NB + n;
            km = (pos >= 0 && pos < T) ? 0xffffffffu : 0u;
          }
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const int s = 2 * cb + u;
              const f32x16 av = acc[n][cb];
              if constexpr ((cv & 1) == 0) {
                uint32_t w[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  w[e] = pk_bf16(lrelu_max(av[8 * u + 2 * e], slope), lrelu_max(av[8 * u + 2 * e + 1], slope));
                  if constexpr (EDGE) w[e] &= km;
                }
                in[n][s] = u32x4{w[0], w[1], w[2], w[3]};
              } else {
                float xf[8];
                if constexpr (RM) {
#pragma unroll
                  for (int e = 0; e < 8; ++e) xf[e] = 0.f;
                } else {
                  unpack8(opaque(xb[n][s]), xf);
                }
                uint32_t w[4], l[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const float z0 = RM ? av[8 * u + 2 * e] : av[8 * u + 2 * e] + xf[2 * e];
                  const float z1 = RM ? av[8 * u + 2 * e + 1] : av[8 * u + 2 * e + 1] + xf[2 * e + 1];
                  w[e] = pk_bf16(z0, z1);
                  l[e] = pk_bf16(lrelu_max(z0, slope), lrelu_max(z1, slope));
                  if constexpr (EDGE) l[e] &= km;
                }
                xb[n][s] = u32x4{w[0], w[1], w[2], w[3]};
                in[n][s] = u32x4{l[0], l[1], l[2], l[3]};
              }
            }
        }
      };
      if constexpr (cv < 5) {
        if (interior)
          epi(std::false_type{});
        else
          epi(std::true_type{});
      }
    };
    conv(std::integral_constant<int, 0>{});
    conv(std::integral_constant<int, 1>{});
    conv(std::integral_constant<int, 2>{});
    conv(std::integral_constant<int, 3>{});
    conv(std::integral_constant<int, 4>{});
    conv(std::integral_constant<int, 5>{});

    const int valid = min(OR, T - t0);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.y + ((int64_t)b * T + t0) * C), (short)0, valid * C * 2, 0x00020000);
    auto fin = [&](auto with_acc) {
      constexpr bool ACC = decltype(with_acc)::value;
      u32x4 ain[ACC ? NB : 1][NK];
      if constexpr (ACC) load_rows(a.acc, tile, ain);
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const int r = lc * NB + n - RR_HALO;
        const int off = r >= 0 ? r * C * 2 + 16 * lh : 0x40000000;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int s = 2 * cb + u;
            const f32x16 av = acc[n][cb];
            float xf[8], af8[8];
            if constexpr (RM) {
#pragma unroll
              for (int e = 0; e < 8; ++e) xf[e] = 0.f;
            } else {
              unpack8(opaque(xb[n][s]), xf);
            }
            if constexpr (ACC) unpack8(ain[n][s], af8);
            uint32_t w[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float z0 = (RM ? av[8 * u + 2 * e] : av[8 * u + 2 * e] + xf[2 * e]) * a.out_scale;
              float z1 = (RM ? av[8 * u + 2 * e + 1] : av[8 * u + 2 * e + 1] + xf[2 * e + 1]) * a.out_scale;
              if constexpr (ACC) {
                z0 += af8[2 * e];
                z1 += af8[2 * e + 1];
              }
              w[e] = pk_bf16(z0, z1);
            }
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{w[0], w[1], w[2], w[3]}, yrs, off, 32 * s, 0);
          }
      }
    };
    if (a.acc)
      fin(std::true_type{});
    else
      fin(std::false_type{});
  }
}

template <int C, int NB, int NWV, bool PF, bool RM = true>
static int rr3w_launch(RrArgs a, int B, hipStream_t st) {
  constexpr int OR = 32 * NB - 2 * RR_HALO;
  constexpr size_t lds = (size_t)(6 * 3 * (C / 16) * (C / 32) + 6 * (C / 32)) * 1024;
  static_assert(lds <= 160 * 1024, "LDS");
  a.tiles_per_b = (a.T + OR - 1) / OR;
  a.ntiles = a.tiles_per_b * B;
  auto kern = mrf_rr3w_kernel<C, NB, NWV, PF, RM>;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  const int grid = (int)std::min<int64_t>(cus, (a.ntiles + NWV - 1) / NWV);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NWV * 64), lds, st, a);
  VO_RETURN_LAUNCH();
}

template <int C, int NB, int NWV, bool PF, bool PA = false, bool PL = false>
static int rr3_launch(RrArgs a, int B, hipStream_t st) {
  constexpr int OR = 16 * NB - 2 * RR_HALO;
  constexpr size_t lds = (size_t)6 * 3 * (C / 32) * (C / 16) * 1024 + 6 * C * sizeof(float);
  static_assert(lds <= 160 * 1024, "LDS");
  a.tiles_per_b = (a.T + OR - 1) / OR;
  a.ntiles = a.tiles_per_b * B;
  auto kern = mrf_rr3_kernel<C, NB, NWV, PF, PA, PL>;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  const int grid = (int)std::min<int64_t>(cus, (a.ntiles + NWV - 1) / NWV);  // one workgroup per CU
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NWV * 64), lds, st, a);
  VO_RETURN_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// The same formulation for a k = 7 / 11 ResBlock iteration (vo_resblock_pair):
//   y = (x + c2(lrelu(c1_D(lrelu x)))) * out_scale (+ acc)
// c1 (dilation D) and c2 (dilation 1) run over the whole 16 NB-row frame; the valid rows shrink by
// the halo (K - 1) / 2 * (D + 1) per side.  Tap shifts of up to 15 lanes are one DPP row_shl /
// row_shr per dword (lane-major frames).  Both convs' weights live in LDS (C = 32: 2 K KiB).  x is
// read twice: the frame at the start (its leaky ReLU is the c1 input) and the output rows again for
// the residual at the end (L2 / MALL hits: the frame was fetched one tile earlier).
struct RrpArgs {
  const bf16_t* x;
  const bf16_t* w[2];
  const float* bias[2];
  bf16_t* y;
  const bf16_t* acc;
  int T, tiles_per_b, ntiles;
  float slope, out_scale;
};

// RT: each conv's centre tap held in registers (loaded once per kernel) and only the other K - 1 taps in
// LDS -- C = 64, K = 11: 160 instead of 176 KiB of fragments
template <int C, int K, int D, int NB, int NWV, bool RT = false>
__global__ void __launch_bounds__(NWV * 64, 1) mrf_rrp_kernel(RrpArgs a) {
  constexpr int NS = C / 32, NCB = C / 16, NT = NWV * 64, F = 16 * NB;
  constexpr int HK = (K - 1) / 2;
  constexpr int HALO = HK * (D + 1);
  constexpr int OR = F - 2 * HALO;
  constexpr int KL = RT ? K - 1 : K;       // taps per conv in LDS
  constexpr int NFR = 2 * KL * NS * NCB;   // LDS fragments
  static_assert(OR > 0 && HK * D < 16 * NB, "frame too small for the halo");
  static_assert((2 * KL * NS) % 2 == 0, "fragment parity repeats per tile");
  // LDS fragment of (conv, tap, K-step, co-block) (RT: never the centre tap)
  auto lfi = [](int cv, int k, int s, int cb) constexpr {
    const int kl = RT ? (k < (K - 1) / 2 ? k : k - 1) : k;
    return ((cv * KL + kl) * NS + s) * NCB + cb;
  };

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  u32x4* wfr = reinterpret_cast<u32x4*>(smem_raw);
  float* sb = reinterpret_cast<float*>(smem_raw + NFR * 1024);  // (RT: the biases live in registers)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lq = lane >> 4;
  const int T = a.T;
  const float slope = a.slope;

  for (int i = tid; i < NFR * 64; i += NT) {
    const int f = i >> 6, l = i & 63;
    const int b = f % NCB, s = (f / NCB) % NS, kl = (f / (NCB * NS)) % KL, cv = f / (NCB * NS * KL);
    const int k = RT ? (kl < HK ? kl : kl + 1) : kl;
    const int m = l & 15;
    const int co = 32 * (b >> 1) + 8 * (m >> 2) + 4 * (b & 1) + (m & 3);
    wfr[i] = *reinterpret_cast<const u32x4*>(a.w[cv] + k * C * C + co * C + 32 * s + 8 * (l >> 4));
  }
  if constexpr (!RT)
    for (int i = tid; i < 2 * C; i += NT) sb[i] = a.bias[i / C][i % C];
  __syncthreads();

  const int gw = blockIdx.x * NWV + wave, nw = gridDim.x * NWV;
  int tile = (int)(((int64_t)gw * a.ntiles) / nw);
  const int tile_end = (int)(((int64_t)(gw + 1) * a.ntiles) / nw);
  if (tile >= tile_end) return;

  const int lane_off = 2 * (lr * NB * C + 8 * lq);
  auto utt_rsrc = [&](const bf16_t* base, int b) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (int64_t)b * T * C), (short)0, T * C * 2, 0x00020000);
  };
  auto load_rows = [&](const bf16_t* base, int tl, u32x4 (&fr)[NB][NS]) {
    const int b = tl / a.tiles_per_b;
    const int w0 = (tl - b * a.tiles_per_b) * OR - HALO;
    const __amdgpu_buffer_rsrc_t rs = utt_rsrc(base, b);
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int s = 0; s < NS; ++s)
        fr[n][s] = __builtin_amdgcn_raw_buffer_load_b128(rs, (w0 + n) * C * 2 + lane_off, 64 * s, 0);
  };
  // tap of step j of a conv: the centre tap first (no shift), then 0 .. K - 1 without it
  auto tap_of = [](int j) constexpr { return j == 0 ? (K - 1) / 2 : (j <= (K - 1) / 2 ? j - 1 : j); };

  // the centre taps (RT), straight from the packed weights: lane layout of an A fragment
  u32x4 ctap[RT ? 2 : 1][NS][NCB];
  if constexpr (RT) {
#pragma unroll
    for (int cv = 0; cv < 2; ++cv)
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          const int m = lane & 15;
          const int co = 32 * (cb >> 1) + 8 * (m >> 2) + 4 * (cb & 1) + (m & 3);
          ctap[cv][s][cb] = *reinterpret_cast<const u32x4*>(a.w[cv] + HK * C * C + co * C + 32 * s + 8 * lq);
        }
  }
  f32x4 breg[RT ? 2 : 1][NCB];  // RT: the lane's bias values of both convs (the LDS is full)
  if constexpr (RT) {
#pragma unroll
    for (int cv = 0; cv < 2; ++cv)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        breg[cv][cb] = *reinterpret_cast<const f32x4*>(a.bias[cv] + 32 * (cb >> 1) + 8 * lq + 4 * (cb & 1));
  }
  u32x4 af[2][NCB];
  // the first LDS step of c1: the centre tap (or, RT, tap 0)
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) af[0][cb] = wfr[lfi(0, RT ? 0 : HK, 0, cb) * 64 + lane];

  for (; tile < tile_end; ++tile) {
    const int b = tile / a.tiles_per_b;
    const int t0 = (tile - b * a.tiles_per_b) * OR;
    const int w0 = t0 - HALO;
    const bool interior = w0 >= 0 && w0 + F <= T;
    u32x4 in[NB][NS];
    load_rows(a.x, tile, in);
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int s = 0; s < NS; ++s) in[n][s] = lrelu8_pk(in[n][s], slope);

    int fl = lane;
    asm volatile("" : "+v"(fl));
    const u32x4* wl = wfr + fl;
    f32x4 acc[NB][NCB];

    auto conv = [&](auto cvc) {
      constexpr int cv = decltype(cvc)::value;
      constexpr int d = cv == 0 ? D : 1;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        f32x4 bv;
        if constexpr (RT)
          bv = breg[cv][cb];
        else
          bv = *reinterpret_cast<const f32x4*>(sb + cv * C + 32 * (cb >> 1) + 8 * lq + 4 * (cb & 1));
#pragma unroll
        for (int n = 0; n < NB; ++n) acc[n][cb] = bv;
      }
      auto step = [&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr int k = tap_of(j);
        constexpr int O = (k - HK) * d;
        constexpr bool REG = RT && j == 0;  // the centre tap from registers
        auto ks = [&](auto sc) {
          constexpr int s = decltype(sc)::value;
          // LDS step index within the tile (its parity picks the fragment buffer) and the next LDS step
          constexpr int g = cv * KL * NS + (RT ? j - 1 : j) * NS + s;
          constexpr int fn = s + 1 < NS ? lfi(cv, k, s + 1, 0)
                                        : (j + 1 < K ? lfi(cv, tap_of(j + 1), 0, 0)
                                                     : lfi((cv + 1) % 2, tap_of(RT ? 1 : 0), 0, 0));
          if constexpr (!REG) {
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) af[(g + 1) & 1][cb] = wl[(fn + cb) * 64];
          }
          __builtin_amdgcn_sched_barrier(0);
          auto blk = [&](auto nc) {
            constexpr int n = decltype(nc)::value;
            const bf16x8 bv = __builtin_bit_cast(bf16x8, shifted<O, NB, NS, n>(in, s));
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
              u32x4 A;
              if constexpr (REG)
                A = ctap[RT ? cv : 0][s][cb];
              else
                A = af[g & 1][cb];
              acc[n][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, A), bv, acc[n][cb], 0,
                                                                  0, 0);
            }
          };
          static_for<NB>(blk);
        };
        static_for<NS>(ks);
      };
      static_for<K>(step);
    };
    conv(std::integral_constant<int, 0>{});
    // T1 = lrelu(c1 + b1), zero outside [0, T) (c2's padding), over the c1 input
    auto epi1 = [&](auto edge) {
      constexpr bool EDGE = decltype(edge)::value;
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        uint32_t km = 0xffffffffu;
        if constexpr (EDGE) {
          const int pos = w0 + lr * NB + n;
          km = (pos >= 0 && pos < T) ? 0xffffffffu : 0u;
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const f32x4 lo = acc[n][2 * s], hi = acc[n][2 * s + 1];
          const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          uint32_t w[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            w[e] = pk_bf16(lrelu_max(v[2 * e], slope), lrelu_max(v[2 * e + 1], slope));
            if constexpr (EDGE) w[e] &= km;
          }
          in[n][s] = u32x4{w[0], w[1], w[2], w[3]};
        }
      }
    };
    if (interior)
      epi1(std::false_type{});
    else
      epi1(std::true_type{});
    // the residual rows and the MRF accumulator rows, in flight during c2
    u32x4 xr[NB][NS], ain[NB][NS];
    load_rows(a.x, tile, xr);
    load_rows(a.acc ? a.acc : a.x, tile, ain);
    conv(std::integral_constant<int, 1>{});

    const int valid = min(OR, T - t0);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.y + ((int64_t)b * T + t0) * C), (short)0, valid * C * 2, 0x00020000);
    auto fin = [&](auto with_acc) {
      constexpr bool ACC = decltype(with_acc)::value;
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const int r = lr * NB + n - HALO;
        const int off = r >= 0 ? r * C * 2 + 16 * lq : 0x40000000;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const f32x4 lo = acc[n][2 * s], hi = acc[n][2 * s + 1];
          const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          float xf[8], af8[8];
          unpack8(xr[n][s], xf);
          if constexpr (ACC) unpack8(ain[n][s], af8);
          uint32_t w[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float z0 = (v[2 * e] + xf[2 * e]) * a.out_scale, z1 = (v[2 * e + 1] + xf[2 * e + 1]) * a.out_scale;
            if constexpr (ACC) {
              z0 += af8[2 * e];
              z1 += af8[2 * e + 1];
            }
            w[e] = pk_bf16(z0, z1);
          }
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{w[0], w[1], w[2], w[3]}, yrs, off, 64 * s, 0);
        }
      }
    };
    if (a.acc)
      fin(std::true_type{});
    else
      fin(std::false_type{});
  }
}

template <int C, int K, int D, int NB, int NWV, bool RT = false>
static int rrp_launch(RrpArgs a, int B, hipStream_t st) {
  constexpr int OR = 16 * NB - 2 * ((K - 1) / 2) * (D + 1);
  constexpr size_t lds = (size_t)2 * (RT ? K - 1 : K) * (C / 32) * (C / 16) * 1024 + (RT ? 0 : 2 * C * sizeof(float));
  static_assert(lds <= 160 * 1024, "LDS");
  a.tiles_per_b = (a.T + OR - 1) / OR;
  a.ntiles = a.tiles_per_b * B;
  auto kern = mrf_rrp_kernel<C, K, D, NB, NWV, RT>;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  const int grid = (int)std::min<int64_t>(cus, (a.ntiles + NWV - 1) / NWV);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NWV * 64), lds, st, a);
  VO_RETURN_LAUNCH();
}

template <int C, int K, int NB, int NWV, bool RT = false>
static int rrp_launch_d(RrpArgs a, int B, int dil, hipStream_t st) {
  if (dil == 1) return rrp_launch<C, K, 1, NB, NWV, RT>(a, B, st);
  if (dil == 3) return rrp_launch<C, K, 3, NB, NWV, RT>(a, B, st);
  return rrp_launch<C, K, 5, NB, NWV, RT>(a, B, st);
}

}  // namespace vo

using namespace vo;

// vo_resblock3's register-resident path (C = 32 / 64, dilations (1, 3, 5)); *handled = 0 leaves
// the call to the LDS-frame kernel
int vo_rb3_rr_try(const void* x, const void* const* w1, const float* const* b1, const void* const* w2,
                  const float* const* b2, const int* dil, void* y, const void* acc, int B, int T, int C, float slope,
                  float out_scale, int cfg, hipStream_t st, int* handled) {
  *handled = 0;
  if (!(C == 32 || C == 64) || dil[0] != 1 || dil[1] != 3 || dil[2] != 5) return VO_OK;
  if ((int64_t)T * C * 2 >= (int64_t)1 << 31) return VO_OK;  // buffer ranges are 32-bit
  RrArgs a;
  a.x = (const bf16_t*)x;
  for (int s = 0; s < 3; ++s) {
    a.w[2 * s] = (const bf16_t*)w1[s]; a.bias[2 * s] = b1[s];
    a.w[2 * s + 1] = (const bf16_t*)w2[s]; a.bias[2 * s + 1] = b2[s];
  }
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)acc;
  a.T = T; a.slope = slope; a.out_scale = out_scale;
#ifdef VO_ABLATIONS  // the other frame shapes / MFMA forms, measured
  *handled = 1;
  if (C == 32) {
    if (cfg == 80) return rr3_launch<32, 12, 4, true>(a, B, st);
    if (cfg == 82) return rr3w_launch<32, 4, 8, false>(a, B, st);
    if (cfg == 83) return rr3w_launch<32, 8, 4, true>(a, B, st);
    if (cfg == 84) return rr3_launch<32, 8, 8, true>(a, B, st);
    if (cfg == 85) return rr3_launch<32, 7, 8, true>(a, B, st);
    if (cfg == 86) return rr3_launch<32, 6, 12, false>(a, B, st);
    if (cfg == 87) return rr3_launch<32, 10, 8, false>(a, B, st);
    if (cfg == 88) return rr3_launch<32, 8, 8, false, true>(a, B, st);
    if (cfg == 89) return rr3_launch<32, 8, 8, false, true, true>(a, B, st);
    if (cfg == 79) return rr3_launch<32, 8, 8, false, false, true>(a, B, st);
  } else {
    if (cfg == 80) return rr3_launch<64, 6, 4, false>(a, B, st);
    if (cfg == 81) return rr3_launch<64, 6, 4, true>(a, B, st);
    if (cfg == 82) return rr3w_launch<64, 4, 4, false>(a, B, st);
    if (cfg == 83) return rr3w_launch<64, 4, 4, true>(a, B, st);
    if (cfg == 78) return rr3_launch<64, 6, 4, false, true>(a, B, st);
    if (cfg == 77) return rr3_launch<64, 6, 4, false, true, true>(a, B, st);
  }
  *handled = 0;
#endif
  // shipped: C = 32, 16x16x32, 128-row frames (8 blocks), two waves per SIMD: 0.300 -> 0.254 ms
  // (tools/mrf_bench.py --stages 3 --tune rb3_cfg=0,81 before the switch); C = 64 keeps the LDS-frame
  // kernel (no register-resident variant beat it)
  if (C != 32 || cfg != 0) return VO_OK;
  *handled = 1;
  return rr3_launch<32, 8, 8, false>(a, B, st);
}

// vo_resblock_pair's register-resident path (C = 32, K = 7 / 11, dilations 1 / 3 / 5)
int vo_pair_rr_try(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                   const void* acc, int B, int T, int C, int K, int dil, float slope, float out_scale, int cfg,
                   hipStream_t st, int* handled) {
  *handled = 0;
  if (!(C == 32 || C == 64) || !(K == 7 || K == 11) || !(dil == 1 || dil == 3 || dil == 5)) return VO_OK;
  if ((int64_t)T * C * 2 >= (int64_t)1 << 31) return VO_OK;
  RrpArgs a;
  a.x = (const bf16_t*)x;
  a.w[0] = (const bf16_t*)w1; a.bias[0] = b1; a.w[1] = (const bf16_t*)w2; a.bias[1] = b2;
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)acc;
  a.T = T; a.slope = slope; a.out_scale = out_scale;
#ifdef VO_ABLATIONS  // other frame shapes
  *handled = C == 32;
  if (C == 32 && cfg == 90) return K == 7 ? rrp_launch_d<32, 7, 12, 8>(a, B, dil, st) : rrp_launch_d<32, 11, 12, 8>(a, B, dil, st);
  if (C == 32 && cfg == 91) return K == 7 ? rrp_launch_d<32, 7, 16, 4>(a, B, dil, st) : rrp_launch_d<32, 11, 16, 4>(a, B, dil, st);
  if (C == 32 && cfg == 92) return K == 7 ? rrp_launch_d<32, 7, 8, 8>(a, B, dil, st) : rrp_launch_d<32, 11, 10, 8>(a, B, dil, st);
  if (C == 32 && cfg == 93) return K == 7 ? rrp_launch_d<32, 7, 8, 8>(a, B, dil, st) : rrp_launch_d<32, 11, 8, 8>(a, B, dil, st);
  if (C == 32 && cfg == 99) return K == 7 ? rrp_launch<32, 7, 1, 8, 8>(a, B, st) : rrp_launch<32, 11, 1, 8, 8>(a, B, st);
  *handled = 0;
  if (C == 64) {  // k = 7 (k = 11's two convs, 176 KiB, do not fit the LDS)
    *handled = 1;
    if (K == 7 && cfg == 94) return rrp_launch_d<64, 7, 10, 4>(a, B, dil, st);
    if (K == 7 && cfg == 95) return rrp_launch_d<64, 7, 8, 4>(a, B, dil, st);
    if (K == 7 && cfg == 96) return rrp_launch_d<64, 7, 12, 4>(a, B, dil, st);
    if (K == 7 && cfg == 97) return rrp_launch_d<64, 7, 7, 4>(a, B, dil, st);
    if (K == 11 && cfg == 94) return rrp_launch_d<64, 11, 8, 4, true>(a, B, dil, st);
    if (K == 11 && cfg == 95) return rrp_launch_d<64, 11, 10, 4, true>(a, B, dil, st);
    // 98: 128-row frames for k = 7 at d = 1 / 3, 144-row at d = 5; k = 11 d = 1 with the centre taps in registers
    if (cfg == 98) {
      if (K == 7) return dil == 5 ? rrp_launch_d<64, 7, 9, 4>(a, B, dil, st) : rrp_launch_d<64, 7, 8, 4>(a, B, dil, st);
      if (dil == 1) return rrp_launch<64, 11, 1, 8, 4, true>(a, B, st);
    }
    *handled = 0;
  }
#endif
  if (cfg != 0) return VO_OK;
  if (C == 64) {
    // k = 7, one wave per SIMD, 144-row frames (9 blocks): 0.326 -> 0.264 / 0.293 / 0.313 ms at d = 1 / 3 / 5
    // (pair_cfg 0 / 98 before the switch; 128-row frames, pair_cfg 95: 0.262 / 0.289 / 0.328)
    if (K != 7) return VO_OK;
    *handled = 1;
    return rrp_launch_d<64, 7, 9, 4>(a, B, dil, st);
  }
  // C = 32 keeps the LDS-tile kernels: at d = 1 the frames (pair_cfg 93 in the A/B library) measure
  // faster alone (k = 7 0.197 -> 0.187 ms, k = 11 0.238 -> 0.217) but ~9 us per launch slower inside the
  // bench step (tools/bench_ab.sh: s3 0.1947 vs 0.1921 ms per launch, two rounds); at d = 3 / 5 the
  // halo, (K - 1) / 2 * (d + 1) rows per side, costs more than the frames save
  return VO_OK;
}
