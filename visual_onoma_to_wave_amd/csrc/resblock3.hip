// Fused HiFi-GAN ResBlock1 with kernel size 3: all three (c1_d, c2) iterations of one
// ResBlock in ONE persistent launch (scripts/hifigan/models.py:96-103, dilations (1, 3, 5)),
// with the Generator's MRF sum / num_kernels scale in the last epilogue (models.py:155-160):
//   x1 = x  + c2_0(lrelu(c1_1(lrelu x )))          (each rounded to bf16, as between the
//   x2 = x1 + c2_1(lrelu(c1_3(lrelu x1)))           per-pair launches of resblock.hip)
//   y  = (x2 + c2_2(lrelu(c1_5(lrelu x2)))) * out_scale (+ acc)
//
// Why: at k = 3 a per-pair launch moves ~4 activation passes (window, residual, MRF
// accumulator, output) for little MFMA work, and every CU fetches its next window at the same
// moment (the pair kernels' timing ablation: 26 % of a k = 3 launch).  Here a tile's window is
// fetched once for three pairs; x1 / x2 never leave the chip (bf16 in registers, lrelu'd copy
// in LDS).  Cost: every conv is evaluated on the whole F-row frame and the valid rows shrink by
// the halos, 1+1+3+1+5+1 = 12 per side, so a tile yields F - 24 output rows (9 % more MFMA work
// at F = 256).
//
// LDS: one activation region of F + 2*HPC rows per 32-channel plane (frame row f lives at
// region row f + HPC; the pad rows only feed frame rows whose outputs are discarded), used in
// place: lrelu(x_s) -> (P1) -> T1 over it -> (P2) -> lrelu(x_{s+1}) over it; weights either all
// 18 taps resident (C = 32) or streamed one tap at a time through a double buffer by LDS-DMA.
// Accumulation order per conv: tap-major, planes inner (as the streamed pair kernels).

#include <algorithm>
#include <type_traits>

#include "mrf_common.h"

namespace vo {

struct Rb3Args {
  const bf16_t* x;
  const bf16_t* w1[3]; const float* b1[3]; const bf16_t* w2[3]; const float* b2[3];
  bf16_t* y; const bf16_t* acc;
  int T, dil[3], tiles_per_b, ntiles;
  float slope, out_scale;
};

constexpr int RB3_HPC = 8;    // region pad rows per side (dilation <= 8)
constexpr int RB3_HALO = 12;  // valid rows lost per side: sum over the six convs of (k-1)/2 * dil

// Streamed weights: a group is 1 / SPLIT of a tap (NC / SPLIT planes); NBUF group buffers form
// a ring and each group's LDS-DMA is issued NBUF - 1 groups ahead (vmcnt is in-order, so the
// wait at a group's end leaves the younger NBUF - 2 groups in flight).
// 4-wave workgroups (WC * WT = 4) are sized for two per CU: one workgroup's epilogues, window
// fetch and barriers overlap the other's MFMAs
// VD (round 3, "VALU diet"; the round-2 epilogues ran 6-9 VALU instructions per MFMA): each conv's
// bias enters as the C operand of its first MFMA (no accumulator zeroing, no bias adds), leaky ReLU
// and the residual update in packed fp32 (v_pk_mul / v_pk_add), x_{s+1}'s lrelu'd copy taken from
// the fp32 sum instead of re-unpacking the rounded bf16, boundary masks only in boundary tiles.
// TPG (round 3): taps per streamed group -- 3 = a whole conv per group, so the group's wait and
// barrier coincide with the conv-end barrier the region rewrite needs anyway (6 barriers per tile
// instead of 24, 96 MFMAs per wave between them at C = 64)
// PIPE (round 3, whole-conv groups only): the conv's 3 x NC (tap, plane) steps software-pipelined --
// the fragments of step st + 1 are read before the MFMAs of step st (two register sets, pinned by
// sched_barrier; hipcc otherwise issues each A fragment right before its MFMAs and waits for it)
template <int C, int WC, int WT, int NJ, bool RESW, int SPLIT = 1, int NBUF = 2, bool VD = true, int TPG = 1,
          bool PIPE = false>
__global__ void __launch_bounds__(WC * WT * 64, WC * WT == 4 ? 2 : 1) mrf_rb3_kernel(Rb3Args a) {
  // streamed-weight blocks: bare LDS barriers (the fence of __syncthreads drains the window
  // prefetch and the y stores at every group); resident-weight (C = 32) blocks keep
  // __syncthreads -- without its vmcnt(0) that kernel ran 0.29 -> 0.40 ms (the next tile's loads
  // queued behind the previous tile's y stores)
  auto bar = [&]() {
    if constexpr (RESW)
      __syncthreads();
    else
      lds_barrier();
  };
  constexpr int NW = WC * WT;
  constexpr int NT = NW * 64;
  constexpr int NC = C / 32;               // 32-channel planes
  constexpr int NI = C / (16 * WC);        // co tiles per wave
  constexpr int F = WT * 16 * NJ;          // frame rows per tile
  constexpr int RR = F + 2 * RB3_HPC;      // region rows per plane
  constexpr int BT = F - 2 * RB3_HALO;     // valid output rows per tile
  constexpr int SHW = NI >= 8 ? 5 : (NI == 4 ? 4 : 3);
  constexpr int VPR = NC * 4;              // 16-byte vectors per activation row
  constexpr int TAPV = C * VPR;            // 16-byte vectors per weight tap
  constexpr int TAPE = NC * C * 32;        // LDS elements per weight tap
  constexpr int NH = NI / 2;               // 8-channel vectors per lane in epilogue layout
  constexpr int NG = 18;                   // taps per tile: 3 stages x 2 convs x 3 taps
  constexpr int D = NBUF - 1;              // DMA prefetch distance in groups
  static_assert(TPG == 1 || (TPG == 3 && SPLIT == 1 && !RESW), "whole-conv groups: 3 taps, unsplit");
  static_assert(!PIPE || (!RESW && SPLIT == 1), "PIPE: streamed whole taps / convs");
  constexpr int NGR = TPG > 1 ? NG / TPG : NG * SPLIT;  // streamed groups per tile
  constexpr int GE = TPG > 1 ? TPG * TAPE : TAPE / SPLIT;  // LDS elements per group buffer
  constexpr int GPL = NC / SPLIT;          // planes per group tap
  static_assert(RESW || (NC % SPLIT == 0 && (TPG * TAPV / SPLIT) % NT == 0 && NBUF >= 2),
                "streamed groups split into whole wave-KiB DMA instructions");
  static_assert(NT % VPR == 0 && (NT / VPR) % 8 == 0, "window slot stride must keep the swizzle");
  constexpr int RSTEP = NT / VPR;
  constexpr int MAXW = (RR + RSTEP - 1) / RSTEP;  // window vectors per thread

  const int T = a.T;
  const float slope = a.slope;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* reg = reinterpret_cast<bf16_t*>(smem_raw);  // [NC][RR][32]
  bf16_t* wls = reg + NC * RR * 32;                   // RESW: [18] taps; else [2] tap buffers
  float* sbias = reinterpret_cast<float*>(wls + (RESW ? NG * TAPE : NBUF * GE));  // [6][C]: b1_0 b2_0 b1_1 ...
  bf16_t* spare = reinterpret_cast<bf16_t*>(sbias + 6 * C);               // sink for idle slots

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  const int wc = wave % WC, wt = wave / WC;
  const int cw0 = wc * (C / WC);
  const int n0 = cw0 + NI * 4 * lq;

  const int G = gridDim.x;
  int tile = (int)(((int64_t)blockIdx.x * a.ntiles) / G);
  const int tile_end = (int)(((int64_t)(blockIdx.x + 1) * a.ntiles) / G);
  if (tile >= tile_end) return;  // uniform per workgroup

  for (int i = tid; i < 6 * C; i += NT) {
    const int s = i / (2 * C), ph = (i / C) & 1, c = i % C;
    sbias[i] = ph ? a.b2[s][c] : a.b1[s][c];
  }

  // ---- weights.  Tap g of a tile: stage g / 6, conv (g / 3) & 1, tap g % 3.
  auto tap_src = [&](int g) -> const bf16_t* {
    const int s = g / 6, ph = (g / 3) & 1, k = g % 3;
    return (ph ? a.w2[s] : a.w1[s]) + k * (C * C);
  };
  constexpr int GLN = RESW ? 1 : TPG * TAPV / SPLIT / NT;  // DMA instructions per wave per group
  int gl_off[GLN];
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  if constexpr (!RESW) {
#pragma unroll
    for (int s = 0; s < GLN; ++s) {  // LDS slot p holds (plane, co, chunk q ^ swz(co)): swizzle on the source
      const int p0 = (s * NW + wave) * 64 + lane;
      const int t = p0 / TAPV, p = p0 - t * TAPV;  // TPG > 1: tap t of the group (contiguous in W)
      const int pl = p / (C * 4), rem = p - pl * C * 4;
      const int co = rem >> 2, q = (rem & 3) ^ ((co >> (SHW - 1)) & 2);
      gl_off[s] = t * (C * C) + co * C + pl * 32 + q * 8;
    }
  }
  auto load_grp = [&](int h, int buf) {  // LDS-DMA of group h (planes of tap h / SPLIT) into buffer buf
    typedef __attribute__((address_space(3))) void lds_void;
    typedef const __attribute__((address_space(1))) void g_void;
    const bf16_t* W = TPG > 1 ? tap_src(h * TPG) : tap_src(h / SPLIT) + (h % SPLIT) * GPL * 32;
#pragma unroll
    for (int s = 0; s < GLN; ++s)
      __builtin_amdgcn_global_load_lds((g_void*)(W + gl_off[s]),
                                       (lds_void*)(wls + buf * GE + (s * NW + wave_u) * 64 * 8), 16, 0, 0);
  };
  if constexpr (RESW) {  // all 18 taps, once per kernel (tap loop uniform: the source is a kernel argument)
    for (int g = 0; g < NG; ++g) {
      const bf16_t* W = tap_src(g);
      for (int vv = tid; vv < TAPV; vv += NT) {
        const int co = vv / VPR, rem = vv - co * VPR;
        *reinterpret_cast<u32x4*>(wls + g * TAPE + (rem >> 2) * C * 32 + rb_off(co, rem & 3, SHW)) =
            *reinterpret_cast<const u32x4*>(W + vv * 8);
      }
    }
  } else {
    for (int h = 0; h < D; ++h) load_grp(h, h);
  }

  // ---- window staging: region rows [0, RR) = positions p0 - HPC + row, p0 = t0 - HALO
  const int xr0 = tid / VPR, xrem = tid - xr0 * VPR;
  const int xg0 = xrem * 8;
  const int xl0 = (xrem >> 2) * RR * 32 + rb_off(xr0, xrem & 3, 2);
  u32x4 xw[MAXW];
  bool xw_ok[MAXW];
  auto load_win = [&](int tl) {
    const int b = tl / a.tiles_per_b;
    const int R0 = (tl - b * a.tiles_per_b) * BT - RB3_HALO - RB3_HPC;
    const bf16_t* base = a.x + (int64_t)b * T * C;
#pragma unroll
    for (int s = 0; s < MAXW; ++s) {
      const int t = R0 + xr0 + s * RSTEP;
      xw_ok[s] = t >= 0 && t < T && xr0 + s * RSTEP < RR;
      xw[s] = *reinterpret_cast<const u32x4*>(base + (int64_t)min(max(t, 0), T - 1) * C + xg0);
    }
  };
  auto store_win = [&]() {
#pragma unroll
    for (int s = 0; s < MAXW; ++s) {
      const u32x4 v = VD ? lrelu8_pk(xw[s], slope) : lrelu8(xw[s], slope);
      *reinterpret_cast<u32x4*>(xr0 + s * RSTEP < RR ? reg + xl0 + s * RSTEP * 32 : spare) =
          xw_ok[s] ? v : u32x4{0u, 0u, 0u, 0u};
    }
  };

  int a_off[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) a_off[i] = rb_off(cw0 + NI * 4 * (lr >> 2) + 4 * i + (lr & 3), lq, SHW);
  const int brow0 = wt * 16 * NJ + lr + RB3_HPC;  // region row of the lane's first B-fragment row

  load_win(tile);
  store_win();
  if constexpr (!RESW) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();

  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto lane_bias = [&](int which, float (&bz)[8 * NH]) {
    const float4* bp = reinterpret_cast<const float4*>(sbias + which * C + n0);
#pragma unroll
    for (int u = 0; u < 2 * NH; ++u) {
      const float4 v = bp[u];
      bz[4 * u] = v.x; bz[4 * u + 1] = v.y; bz[4 * u + 2] = v.z; bz[4 * u + 3] = v.w;
    }
  };

  int gcount = 0;  // streamed groups consumed (position in the buffer ring)
  for (; tile < tile_end; ++tile) {
    const int b = tile / a.tiles_per_b;
    const int p0 = (tile - b * a.tiles_per_b) * BT - RB3_HALO;  // position of frame row 0
    const bool has_next = tile + 1 < tile_end;
    u32x4 xres[NJ][NH];  // x_s of the lane's frame rows (bf16), the next stage's residual

    for (int cv = 0; cv < 6; ++cv) {  // conv cv: stage cv / 2, c1 (even) or c2 (odd)
      const int s = cv >> 1, ph = cv & 1;
      const int step = ph ? 1 : a.dil[s];
      if constexpr (PIPE) {
        static_assert((TPG == 3 || TPG == 1) && !RESW && SPLIT == 1, "PIPE: streamed whole taps / convs");
        constexpr int NKG = 3 / TPG;  // groups per conv
#pragma unroll
        for (int kg = 0; kg < NKG; ++kg) {
          const int g = cv * NKG + kg;  // group of the tile
          load_grp(g + D < NGR ? g + D : g + D - NGR, (gcount + D) % NBUF);
          const bf16_t* wb0 = wls + (gcount % NBUF) * GE;
          if (g == 0) {  // the tile's x rows (see below)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
              const int pos = min(max(p0 + wt * 16 * NJ + 16 * j + lr, 0), T - 1);
              const int64_t off = ((int64_t)b * T + pos) * C + n0;
#pragma unroll
              for (int h = 0; h < NH; ++h) xres[j][h] = *reinterpret_cast<const u32x4*>(a.x + off + 8 * h);
            }
          }
          constexpr int S = TPG * NC;
          Frag<bf16_t> fa[2][NI], fb[2][NJ];
          auto ld = [&](int st, int set) {
            const int t = st / NC, c = st - t * NC, k = kg * TPG + t;
#pragma unroll
            for (int i = 0; i < NI; ++i) fa[set][i].load(wb0 + t * TAPE + c * C * 32 + a_off[i]);
            const int boff = c * RR * 32 + rb_off(brow0 + (k - 1) * step, lq, 2);
#pragma unroll
            for (int j = 0; j < NJ; ++j) fb[set][j].load(reg + boff + 16 * j * 32);
          };
          // the next step's reads go out after the step's first MFMA: the wait before it then covers
          // only reads issued a whole step earlier (16 outstanding reads exceed the 4-bit lgkmcnt, and
          // with both sets in flight hipcc waited for all of them, the just-issued ones included)
          f32x4 bz4[NI];
          if (VD && kg == 0) {
#pragma unroll
            for (int i = 0; i < NI; ++i) bz4[i] = *reinterpret_cast<const f32x4*>(sbias + cv * C + n0 + 4 * i);
          }
          ld(0, 0);
#pragma unroll
          for (int st = 0; st < S; ++st) {
            const int set = st & 1;
#pragma unroll
            for (int q = 0; q < NI * NJ; ++q) {
              const int i = q / NJ, j = q - i * NJ;
              acc[i][j] = mfma(fa[set][i], fb[set][j], VD && kg == 0 && st == 0 ? bz4[i] : acc[i][j]);
              if (q == 0) {
                __builtin_amdgcn_sched_barrier(0);
                if (st + 1 < S) ld(st + 1, (st + 1) & 1);
                __builtin_amdgcn_sched_barrier(0);
              }
            }
            __builtin_amdgcn_sched_barrier(0);
          }
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * GLN) : "memory");
          bar();
          ++gcount;
        }
      }
#pragma unroll
      for (int k = 0; k < (PIPE ? 0 : 3); ++k) {  // taps (compile-time: the conv's first step is known statically)
      const int g = cv * 3 + k;
      const int row = brow0 + (k - 1) * step;
#pragma unroll
      for (int part = 0; part < (RESW ? 1 : SPLIT); ++part) {
        const bf16_t* wb;
        if constexpr (RESW) {
          wb = wls + g * TAPE;
        } else if constexpr (TPG > 1) {  // the conv's group; the next conv's issued at its first tap
          if (k == 0) load_grp(cv + D < NGR ? cv + D : cv + D - NGR, (gcount + D) % NBUF);
          wb = wls + (gcount % NBUF) * GE + k * TAPE;
        } else {  // group D ahead (wrapping into the next tile's first groups)
          const int h = g * SPLIT + part;
          load_grp(h + D < NGR ? h + D : h + D - NGR, (gcount + D) % NBUF);
          wb = wls + (gcount % NBUF) * GE;
        }
        if (g == 0 && part == 0) {
          // the tile's x rows (stage 0's residual, epilogue layout), requested with the first
          // group (after its weight DMA: the group-end wait then covers both) instead of at the
          // end of stage 0's c2, where each load's latency was exposed; xres is live across the
          // tap loop anyway (x1 / x2)
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int pos = min(max(p0 + wt * 16 * NJ + 16 * j + lr, 0), T - 1);
            const int64_t off = ((int64_t)b * T + pos) * C + n0;
#pragma unroll
            for (int h = 0; h < NH; ++h) xres[j][h] = *reinterpret_cast<const u32x4*>(a.x + off + 8 * h);
          }
        }
#pragma unroll
        for (int cl = 0; cl < (RESW ? NC : GPL); ++cl) {
          const int c = part * GPL + cl;
          Frag<bf16_t> af[NI], bfr[NJ];
#pragma unroll
          for (int i = 0; i < NI; ++i) af[i].load(wb + cl * C * 32 + a_off[i]);
          const int boff = c * RR * 32 + rb_off(row, lq, 2);
#pragma unroll
          for (int j = 0; j < NJ; ++j) bfr[j].load(reg + boff + 16 * j * 32);
          if (VD && k == 0 && part == 0 && cl == 0) {  // the conv's first step: its bias is the C operand
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
        }
        if constexpr (!RESW) {
          // the next group's DMA (issued D - 1 groups ago) has landed for this wave; younger ones
          // stay in flight; the barrier publishes it and frees this group's buffer
          if (TPG == 1 || k == TPG - 1) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * GLN) : "memory");
            bar();
            ++gcount;
          }
        }
      }
      }  // taps
      // ---- end of a conv: every wave is past its reads of the region
      if constexpr (RESW) bar();
      if (s == 2 && ph == 1) break;  // the last conv's epilogue follows the loop (its window
                                     // registers must not be live around the loop)
      float bz[8 * NH];
      if constexpr (VD) {
#pragma unroll
        for (int u = 0; u < 8 * NH; ++u) bz[u] = 0.f;  // the bias is in the accumulators
      } else {
        lane_bias(2 * s + ph, bz);
      }
      // frame rows outside [0, T) exist only in an utterance's first / last tile
      const bool interior = p0 >= 0 && p0 + F <= T;
      if (VD && ph == 0) {  // T1 = lrelu(c1 + b1), zero outside [0, T) (c2's zero padding)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int r = wt * 16 * NJ + 16 * j + lr;
          const int pos = p0 + r;
          const uint32_t km = (interior || (pos >= 0 && pos < T)) ? 0xffffffffu : 0u;
#pragma unroll
          for (int h = 0; h < NH; ++h) {
            uint32_t w[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2) {
              const int e = 2 * e2;
              w[e2] = lrelu_pk(acc[2 * h + e / 4][j][e & 3], acc[2 * h + (e + 1) / 4][j][(e + 1) & 3], slope);
            }
            if (!interior) {
#pragma unroll
              for (int e2 = 0; e2 < 4; ++e2) w[e2] &= km;
            }
            const int ch = n0 + 8 * h;
            *reinterpret_cast<u32x4*>(reg + (ch >> 5) * RR * 32 + rb_off(r + RB3_HPC, (ch & 31) >> 3, 2)) = u32x4{w[0], w[1], w[2], w[3]};
          }
        }
      } else if (VD && s < 2) {  // x_{s+1} = x_s + c2 + b2 (bf16) and lrelu(x_{s+1}) from the fp32 sum
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int r = wt * 16 * NJ + 16 * j + lr;
          const int pos = p0 + r;
          const uint32_t km = (interior || (pos >= 0 && pos < T)) ? 0xffffffffu : 0u;
#pragma unroll
          for (int h = 0; h < NH; ++h) {
            float xf[8];
            unpack8(xres[j][h], xf);
            uint32_t w[4], l[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2) {
              const int e = 2 * e2;
              const f32x2v v = f32x2v{acc[2 * h + e / 4][j][e & 3], acc[2 * h + (e + 1) / 4][j][(e + 1) & 3]} +
                               f32x2v{xf[e], xf[e + 1]};
              w[e2] = pk_bf16(v.x, v.y);
              l[e2] = lrelu_pk(v.x, v.y, slope);
            }
            if (!interior) {
#pragma unroll
              for (int e2 = 0; e2 < 4; ++e2) l[e2] &= km;
            }
            xres[j][h] = u32x4{w[0], w[1], w[2], w[3]};
            const int ch = n0 + 8 * h;
            *reinterpret_cast<u32x4*>(reg + (ch >> 5) * RR * 32 + rb_off(r + RB3_HPC, (ch & 31) >> 3, 2)) = u32x4{l[0], l[1], l[2], l[3]};
          }
        }
      } else if (ph == 0) {  // T1 = lrelu(c1 + b1), zero outside [0, T) (c2's zero padding)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int r = wt * 16 * NJ + 16 * j + lr;
          const int pos = p0 + r;
          // c2's zero padding: one AND per packed dword (rows outside [0, T) -> +0)
          const uint32_t km = (interior || (pos >= 0 && pos < T)) ? 0xffffffffu : 0u;
#pragma unroll
          for (int h = 0; h < NH; ++h) {
            uint32_t w[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2) {
              const int e = 2 * e2;
              const float z0 = acc[2 * h + e / 4][j][e & 3] + bz[8 * h + e];
              const float z1 = acc[2 * h + (e + 1) / 4][j][(e + 1) & 3] + bz[8 * h + e + 1];
              w[e2] = pk_bf16(lrelu_max(z0, slope), lrelu_max(z1, slope)) & km;
            }
            const int ch = n0 + 8 * h;
            *reinterpret_cast<u32x4*>(reg + (ch >> 5) * RR * 32 + rb_off(r + RB3_HPC, (ch & 31) >> 3, 2)) = u32x4{w[0], w[1], w[2], w[3]};
          }
        }
      } else if (s < 2) {  // x_{s+1} = x_s + c2 + b2 (bf16), its lrelu'd copy over the region
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int r = wt * 16 * NJ + 16 * j + lr;
          const int pos = p0 + r;
          const bool inside = interior || (pos >= 0 && pos < T);
#pragma unroll
          for (int h = 0; h < NH; ++h) {
            float xf[8];
            unpack8(xres[j][h], xf);
            uint32_t w[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2) {
              const int e = 2 * e2;
              w[e2] = pack_bf16x2(acc[2 * h + e / 4][j][e & 3] + bz[8 * h + e] + xf[e],
                                  acc[2 * h + (e + 1) / 4][j][(e + 1) & 3] + bz[8 * h + e + 1] + xf[e + 1]);
            }
            xres[j][h] = u32x4{w[0], w[1], w[2], w[3]};
            const int ch = n0 + 8 * h;
            u32x4 v = lrelu8(xres[j][h], slope);
            if (!interior) {
              const uint32_t km = inside ? 0xffffffffu : 0u;
              v = u32x4{v.x & km, v.y & km, v.z & km, v.w & km};
            }
            *reinterpret_cast<u32x4*>(reg + (ch >> 5) * RR * 32 + rb_off(r + RB3_HPC, (ch & 31) >> 3, 2)) = v;
          }
        }
      }
      if constexpr (!VD) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if (cv < 5) bar();  // region rewritten: visible before the next conv reads it
    }
    {  // y = (x2 + c2 + b2) * out_scale (+ acc) on the valid rows
      float bz[8 * NH];
      if constexpr (VD) {
#pragma unroll
        for (int u = 0; u < 8 * NH; ++u) bz[u] = 0.f;  // the bias is in the accumulators
      } else {
        lane_bias(5, bz);
      }
      // the accumulator rows for every (j, h) at once (clamped, unconditional: without acc the
      // x rows are read and not added) instead of one dependent load per store; the y values
      // are packed, the next tile's window is requested (before the y stores: vmcnt retires in
      // order), then the y rows go out through a buffer resource that covers exactly the
      // tile's valid rows -- the stores of the halo rows and of rows past T fall outside it and
      // are dropped by the hardware
      u32x4 ares[NJ][NH], yv[NJ][NH];
      const bf16_t* accp = a.acc ? a.acc : a.x;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int pos = min(max(p0 + wt * 16 * NJ + 16 * j + lr, 0), T - 1);
        const int64_t off = ((int64_t)b * T + pos) * C + n0;
#pragma unroll
        for (int h = 0; h < NH; ++h) ares[j][h] = *reinterpret_cast<const u32x4*>(accp + off + 8 * h);
      }
      auto epilogue = [&](auto with_acc) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
#pragma unroll
          for (int h = 0; h < NH; ++h) {
            float xf[8], af8[8];
            uint32_t w[4];
            unpack8(xres[j][h], xf);
            if constexpr (decltype(with_acc)::value) unpack8(ares[j][h], af8);
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2) {
              float q[2];
#pragma unroll
              for (int u = 0; u < 2; ++u) {
                const int e = 2 * e2 + u;
                q[u] = (acc[2 * h + e / 4][j][e & 3] + bz[8 * h + e] + xf[e]) * a.out_scale;
                if constexpr (decltype(with_acc)::value) q[u] += af8[e];
              }
              w[e2] = pk_bf16(q[0], q[1]);
            }
            yv[j][h] = u32x4{w[0], w[1], w[2], w[3]};
          }
        }
      };
      if (a.acc)
        epilogue(std::true_type{});
      else
        epilogue(std::false_type{});
      load_win(has_next ? tile + 1 : tile);  // unconditional (see load_win)
      const int t0 = p0 + RB3_HALO;  // the tile's first output position (frame row HALO)
      const int valid = min(BT, T - t0);
      const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.y + ((int64_t)b * T + t0) * C), (short)0, valid * C * (int)sizeof(bf16_t), 0x00020000);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = wt * 16 * NJ + 16 * j + lr - RB3_HALO;  // row within the resource
        // rows before it: an offset past any resource (dropped like the rows past it)
        const int roff = r >= 0 ? r * C * (int)sizeof(bf16_t) : 0x40000000;
#pragma unroll
        for (int h = 0; h < NH; ++h)
          __builtin_amdgcn_raw_buffer_store_b128(yv[j][h], yrs, roff + (n0 + 8 * h) * (int)sizeof(bf16_t), 0, 0);
      }
    }
    if constexpr (!VD) {
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // next window (requested in the last epilogue) over the region (P2 of stage 2 ended its
    // region reads at the last barrier)
    if (has_next) store_win();
    bar();
  }
}

template <int C, int WC, int WT, int NJ, bool RESW, int SPLIT = 1, int NBUF = 2, bool VD = true, int TPG = 1,
          bool PIPE = false>
static int rb3_launch(Rb3Args a, int B, hipStream_t st) {
  constexpr int NW = WC * WT;
  constexpr int F = WT * 16 * NJ;
  constexpr int BT = F - 2 * RB3_HALO;
  constexpr int RR = F + 2 * RB3_HPC;
  a.tiles_per_b = (a.T + BT - 1) / BT;
  a.ntiles = a.tiles_per_b * B;
  const size_t wel = RESW ? 18 * (size_t)C * C : (size_t)NBUF * TPG * C * C / SPLIT;
  const size_t lds = ((size_t)RR * C + wel) * sizeof(bf16_t) + 6 * C * sizeof(float) + 16;
  if (lds > 160 * 1024) {
    vo_set_error("resblock3: LDS %zu B exceeds 160 KiB", lds);
    return VO_ERR_INVALID;
  }
  auto kern = mrf_rb3_kernel<C, WC, WT, NJ, RESW, SPLIT, NBUF, VD, TPG, PIPE>;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, NW * 64, lds) != hipSuccess || per_cu < 1) per_cu = 1;
  const int grid = (int)std::min<int64_t>((int64_t)cus * per_cu, a.ntiles);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NW * 64), lds, st, a);
  VO_RETURN_LAUNCH();
}

}  // namespace vo

using namespace vo;

int vo_rb3_wave_try(const void* x, const void* const* w1, const float* const* b1, const void* const* w2,
                    const float* const* b2, const int* dil, void* y, const void* acc, int B, int T, int C, float slope,
                    float out_scale, int cfg, hipStream_t st, int* handled);  // resblock5.hip
int vo_rb3_rr_try(const void* x, const void* const* w1, const float* const* b1, const void* const* w2,
                  const float* const* b2, const int* dil, void* y, const void* acc, int B, int T, int C, float slope,
                  float out_scale, int cfg, hipStream_t st, int* handled);  // resblock_rr.hip
int vo_rb3_pb_try(const void* x, const void* const* w1, const float* const* b1, const void* const* w2,
                  const float* const* b2, const int* dil, void* y, const void* acc, int B, int T, int C, float slope,
                  float out_scale, hipStream_t st, int* handled, int frag);  // resblock_pb3.hip

extern "C" int vo_resblock3(const void* x, const void* const* w1, const float* const* b1, const void* const* w2,
                            const float* const* b2, const int* dil, void* y, const void* acc, int B, int T, int C,
                            float slope, float out_scale, void* stream) {
  VO_CHECK_ARG(x && w1 && b1 && w2 && b2 && dil && y, "resblock3: null pointer");
  VO_CHECK_ARG(C == 32 || C == 64 || C == 128, "resblock3: C=%d unsupported (32, 64 or 128)", C);
  VO_CHECK_ARG(B > 0 && T > 0, "resblock3: empty");
  VO_CHECK_ARG(slope >= 0.f && slope <= 1.f, "resblock3: slope %g outside [0, 1]", slope);
  VO_CHECK_ARG(y != x, "resblock3: y must not alias x (neighbouring tiles re-read x)");
  VO_CHECK_ARG(acc == nullptr || acc == y || acc != x, "resblock3: acc must not alias x");
  Rb3Args a;
  a.x = (const bf16_t*)x;
  int halo = 0;
  for (int s = 0; s < 3; ++s) {
    VO_CHECK_ARG(w1[s] && b1[s] && w2[s] && b2[s], "resblock3: null weight of stage %d", s);
    VO_CHECK_ARG(dil[s] >= 1 && dil[s] <= RB3_HPC, "resblock3: dilation %d outside [1, %d]", dil[s], RB3_HPC);
    a.w1[s] = (const bf16_t*)w1[s]; a.b1[s] = b1[s]; a.w2[s] = (const bf16_t*)w2[s]; a.b2[s] = b2[s];
    a.dil[s] = dil[s];
    halo += dil[s] + 1;
  }
  VO_CHECK_ARG(halo <= RB3_HALO, "resblock3: dilations (%d, %d, %d) exceed the 12-row halo", dil[0], dil[1], dil[2]);
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)acc;
  a.T = T; a.slope = slope; a.out_scale = out_scale;
  a.tiles_per_b = a.ntiles = 0;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // measured on MI355X at B = 32 (tools/ab_rb3.py, with the MRF accumulator), against three
  // vo_resblock_pair launches: C = 128 0.84 vs 1.02 ms, C = 64 0.61 vs 0.67, C = 32 0.39 vs 0.52.
  // rb3_cfg (A/B): 1 = 128-row frames (C = 32: 512-row), 4 = a 3-deep LDS-DMA ring of half / whole
  // taps (C = 128 / 64; within 2 % of double buffering: the DMA latency is not what binds).
  const int cfg = vo_tune_get("rb3_cfg");
  if (cfg == 0) {  // round 6: wave-owned output planes (resblock_pb3.hip) for C = 64 / 128; rb3_cfg 90: the LDS-tile block
    int handled = 0;
    const int rc = vo_rb3_pb_try(x, w1, b1, w2, b2, dil, y, acc, B, T, C, slope, out_scale, st, &handled, 0);
    if (handled) return rc;
  }
  {  // round 4: register-resident frames (resblock_rr.hip) for C = 32, dilations (1, 3, 5); rb3_cfg 77-89 (A/B)
    int handled = 0;
    const int rc = vo_rb3_rr_try(x, w1, b1, w2, b2, dil, y, acc, B, T, C, slope, out_scale, cfg, st, &handled);
    if (handled) return rc;
  }
#ifdef VO_ABLATIONS  // measured-and-dropped variants (A/B builds only: make abl)
  if (C == 32 && (cfg == 30 || cfg == 31)) {  // round 3: wave-private frames (resblock5.hip)
    int handled = 0;
    const int rc = vo_rb3_wave_try(x, w1, b1, w2, b2, dil, y, acc, B, T, C, slope, out_scale, cfg, st, &handled);
    if (handled) return rc;
  }
  if (cfg == 20) {  // the round-2 kernels (epilogues without the VALU diet), for A/B
    if (C == 32) return rb3_launch<32, 1, 8, 2, true, 1, 2, false>(a, B, st);
    if (C == 64) return rb3_launch<64, 1, 8, 4, false, 1, 2, false>(a, B, st);
    return rb3_launch<128, 2, 4, 4, false, 1, 2, false>(a, B, st);
  }
  if (C == 32 && cfg == 1) return rb3_launch<32, 1, 8, 4, true>(a, B, st);
  if (C == 64) {
    if (cfg == 1) return rb3_launch<64, 1, 8, 2, false>(a, B, st);
    if (cfg == 4) return rb3_launch<64, 1, 8, 4, false, 1, 4>(a, B, st);
    if (cfg == 5) return rb3_launch<64, 1, 4, 4, false>(a, B, st);
    if (cfg == 7) return rb3_launch<64, 1, 4, 4, false, 1, 4>(a, B, st);
    // cfg 6 / 7: two 4-wave workgroups of 256-row frames per CU with a 3- / 4-deep weight ring
    // (round 2, bare LDS barriers): 0.53 -> 0.50 ms alone with the MRF accumulator
    // (tools/ab_pair2.py), the same 12.40 / 12.46 ms bench step (s2 within noise) -- not default
    if (cfg == 6) return rb3_launch<64, 1, 4, 4, false, 1, 3>(a, B, st);
    if (cfg == 40) return rb3_launch<64, 1, 8, 4, false>(a, B, st);  // one tap per group (round 2 / 3)
    if (cfg == 41) return rb3_launch<64, 1, 8, 3, false, 1, 2, true, 3>(a, B, st);
    if (cfg == 43) return rb3_launch<64, 1, 8, 3, false, 1, 2, true, 3, true>(a, B, st);
    if (cfg == 44) return rb3_launch<64, 1, 8, 4, false, 1, 2, true, 1, true>(a, B, st);
    if (cfg == 45) return rb3_launch<64, 1, 8, 4, false, 1, 2, true, 3>(a, B, st);
  }
  if (C == 128) {
    if (cfg == 1) return rb3_launch<128, 2, 4, 2, false>(a, B, st);
    if (cfg == 4) return rb3_launch<128, 2, 4, 4, false, 2, 4>(a, B, st);
    if (cfg == 42) return rb3_launch<128, 2, 4, 4, false>(a, B, st);  // without the PIPE steps
  }
#else
  (void)cfg;
#endif
  // C = 32: 256-row frames, all weights resident: 2 workgroups (4 waves / SIMD) per CU
  if (C == 32) return rb3_launch<32, 1, 8, 2, true>(a, B, st);
  // C = 64: a whole conv (3 taps, 24 KB) per streamed group: 6 barriers per tile instead of 24, 0.476
  // -> 0.448 ms (tools/mrf_bench.py --stages 2 --tune rb3_cfg=0,40, round 3, bit-identical); with the
  // software-pipelined steps (PIPE) 0.443 -> 0.437 ms
  if (C == 64) return rb3_launch<64, 1, 8, 4, false, 1, 2, true, 3, true>(a, B, st);
  // C = 128: software-pipelined steps (PIPE: the next (tap, plane) step's fragments read during the
  // current step's MFMAs): 0.720 -> 0.686 ms, bit-identical (tools/mrf_bench.py --tune rb3_cfg=0,42)
  return rb3_launch<128, 2, 4, 4, false, 1, 2, true, 1, true>(a, B, st);
}
