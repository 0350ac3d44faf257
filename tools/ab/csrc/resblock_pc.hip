// HiFi-GAN ResBlock1 pair for the C = 128 MRF stage with the tile-boundary loads taken off the
// MFMA waves' critical path (round 4):
//   y = (x + c2(lrelu(c1_d(lrelu(x), slope), slope))) * out_scale (+ acc)
// (scripts/hifigan/models.py:96-103, one (c1, c2) iteration; the MRF sum and 1/num_kernels
// scale of models.py:155-160 ride in the epilogue).
//
// Same tile geometry as mrf_pair_kernel<128> (resblock.hip: 8 waves of 64 co x 64 rows, 256-row
// tiles, T1 written over the dead window), but the work is ordered so that no HBM round trip is
// waited for at a tile boundary (the round-3 kernel waited for two there: the residual /
// accumulator rows, then the next tile's window, 17-21 % of its time by ablation):
//  * plane-major slice order: a conv is NC x K slices (input plane c, tap k) of 8 KiB of weights,
//    streamed four per group through an LDS double buffer.  In P2 the T1 plane c is dead once its
//    K slices are done, so the NEXT tile's window plane c is DMA'd into that plane while P2 goes
//    on; the last plane(s) are DMA'd at the start of the next P1, which reads them last.
//  * producer roles: waves 0-3 issue the weight DMA (one slice each per group), waves 4-7 the
//    window DMA and the leaky-ReLU / zero-padding pass over each landed plane.  vmcnt is per wave
//    and in order, so the weight waves' per-group waits never drain a window load.
//  * the DMAs are inline asm: hipcc cannot tell an LDS-DMA destination from the buffer the next
//    ds_read uses and would wait for every DMA before the next fragment read; the kernel waits
//    itself, with counts that are lower bounds of the younger vector-memory operations (an
//    under-count only over-waits).
//  * the residual rows are loaded during the last P1 group and folded into P2's accumulator init
//    (acc = b2 + x); the MRF accumulator rows are requested in the P1 epilogue and added after
//    P2's first group (acc += acc_in / out_scale); y = acc * out_scale -- no loads after P2, no
//    residual registers live through P2.
// The fold rounds differently from (c2 + b2 + x) * s + acc_in in the last fp32 bits only.

#ifdef VO_ABLATIONS  // round-4 C = 128 candidate (producer roles): measured slower, A/B builds only
#include <type_traits>

#include "mrf_common.h"  // visual_onoma_to_wave_amd/csrc (make abl adds it to the include path)

namespace vo {

struct PcArgs {
  const bf16_t* x; const bf16_t* w1; const float* b1; const bf16_t* w2; const float* b2;
  bf16_t* y; const bf16_t* acc;
  int T, dil, tiles_per_b, ntiles;
  float slope, out_scale, inv_scale;
};

// 16 B per lane, global -> LDS at lds + 16 * lane (wave-uniform lds), invisible to hipcc's
// waitcnt insertion (the caller waits)
// (saddr form: wave-uniform base in SGPRs + 32-bit per-lane byte offset)
__device__ __forceinline__ void dma16(const void* base, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(base),
               "s"(__builtin_amdgcn_readfirstlane(lds))
               : "memory", "m0");
}
template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

#ifdef VO_ABLATIONS
// diagnostic stamps (ABL bit 2, ablation library only): s_memtime at group start / MFMA end for
// waves 0 and 4 of workgroups 0-7, first 4 tiles: [wg][role][tile][slot 0..63][2]
__device__ unsigned long long g_pc_stamp[8 * 2 * 4 * 64 * 2];
#endif

// constexpr schedule of the window planes (K taps, NC planes, SPG slices per group)
template <int K, int NC, int SPG> struct PcPlan {
  static constexpr int NS = NC * K, NG = (NS + SPG - 1) / SPG;
  // last P2 group reading T1 plane c, first P1 group reading window plane c
  static constexpr int gf(int c) { return (c * K + K - 1) / SPG; }
  static constexpr int gn(int c) { return (c * K) / SPG; }
  // early planes: DMA'd during P2 of the previous tile (after gf(c)); late: at the start of P1
  static constexpr bool early(int c) { return gf(c) + 1 < NG; }
  static constexpr int n_early_after(int c) {
    int n = 0;
    for (int d = c + 1; d < NC; ++d) n += early(d) ? 1 : 0;
    return n;
  }
  static constexpr int n_late_after(int c) {  // late planes after late plane c
    int n = 0;
    for (int d = c + 1; d < NC; ++d) n += early(d) ? 0 : 1;
    return n;
  }
  static constexpr int n_late() { return n_late_after(-1); }
};

// MODE 0: waves 0-3 issue the whole weight stream (one slice each per group), waves 4-7 the window;
// MODE 1: every wave issues half a slice per group, waves 4-7 also the window (their group-end wait
// leaves that group's window pieces in flight; the next group's wait drains them).
// ABL (timing ablations, garbage results; VO_ABLATIONS builds only): bit 0 = no window DMA / pass,
// bit 1 = no weight DMA.
// VAR (A/B): 1 = waves 4-7 at s_setprio 1 for the whole kernel; 2 = slices without the pinned
// fragment pipeline (hipcc schedules the reads)
template <int K, bool HAS_ACC, int MODE = 0, int ABL = 0, int VAR = 0>
__global__ void __launch_bounds__(512, 2) mrf_pair_pc_kernel(PcArgs a) {
  constexpr int C = 128, NC = 4, WC = 2, WT = 4, NJ = 4, NI = 4, NT = 512;
  constexpr int R1 = WT * 16 * NJ;     // 256 c1 rows per tile
  constexpr int SHW = 4;               // weight-row swizzle (rb_off)
  constexpr int PSR = 320;             // rows per activation plane (window <= 320 rows, T1 272)
  constexpr int PLANE_E = PSR * 32;    // elements per plane
  constexpr int SLICE_E = C * 32;      // elements per weight slice (8 KiB)
  constexpr int SPG = 4;               // slices per group (one per weight wave)
  using P = PcPlan<K, NC, SPG>;
  constexpr int NS = P::NS, NG = P::NG;
  constexpr int h2 = (K - 1) / 2;
  constexpr int BT = R1 - 2 * h2;
  constexpr int WPW = PSR / 16 / 4;    // window DMA pieces (1 KiB) per window wave per plane
  constexpr int NH = 2;
  static_assert(NS % SPG == 0, "whole groups");
  static_assert(NC * PLANE_E * 2 + 2 * SPG * SLICE_E * 2 + 2 * C * 4 <= 160 * 1024, "LDS");

  const int T = a.T, dil = a.dil;
  const int h1 = dil * (K - 1) / 2;
  const float slope = a.slope;

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* act = reinterpret_cast<bf16_t*>(smem_raw);            // [NC][PSR][32]: window / T1
  bf16_t* wls = act + NC * PLANE_E;                              // [2][SPG][C][32]
  float* sbias = reinterpret_cast<float*>(wls + 2 * SPG * SLICE_E);  // [b1 | b2]
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem_raw);
  const uint32_t lds_act = lds0, lds_w = lds0 + NC * PLANE_E * 2;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lq = lane >> 4;
  const int wc = wave % WC, wt = wave / WC;
  const int cw0 = wc * (C / WC);
  const int n0 = cw0 + NI * 4 * lq;
  const bool wrole = wave < 4;             // weight-DMA waves (one per SIMD); 4-7: window waves
  const int rw = wave & 3;                 // index within the role

  const int G = gridDim.x;
  int tile = (int)(((int64_t)blockIdx.x * a.ntiles) / G);
  const int tile_end = (int)(((int64_t)(blockIdx.x + 1) * a.ntiles) / G);
  if (tile >= tile_end) return;

  for (int i = tid; i < 2 * C; i += NT) sbias[i] = i < C ? a.b1[i] : a.b2[i - C];

  // ---- weight DMA: weight wave rw owns slot rw of every group; piece pp (0..7) = 16 co rows.
  // LDS slot (co, q') of a slice holds source chunk q = q' ^ swz(co), swz(co) = 2 * (pp & 1)
  uint32_t wsrc[2];  // per-lane byte offsets of even / odd pieces
#pragma unroll
  for (int odd = 0; odd < 2; ++odd) wsrc[odd] = 2u * ((lane >> 2) * C + 8 * ((lane & 3) ^ (2 * odd)));
  constexpr int WPP = MODE == 0 ? 8 : 4;  // weight pieces per issuing wave per group
  const int wpp0 = MODE == 0 ? 0 : (wave >> 2) * 4;
  auto issue_group = [&](int gi, int buf) {  // gi in [0, 2 NG): phase gi / NG
    if constexpr ((ABL & 2) != 0) return;
    const int ph = gi >= NG;
    const int s = (gi - ph * NG) * SPG + rw;
    const int c = s / K, k = s - c * K;
    const bf16_t* W = (ph ? a.w2 : a.w1) + k * (C * C) + c * 32;
    const uint32_t dst = lds_w + (uint32_t)((buf * SPG + rw) * SLICE_E * 2);
#pragma unroll
    for (int u = 0; u < WPP; ++u) {
      const int pp = wpp0 + u;
      dma16(W + pp * 16 * C, wsrc[u & 1], dst + pp * 1024);  // wpp0 is even: pp & 1 == u & 1
    }
  };
  const bool wissue = MODE == 0 ? wrole : true;  // this wave issues weight pieces

  // ---- window DMA: window wave rw owns pieces rw * WPW .. + WPW - 1 of a plane (16 rows each);
  // lane -> row 16 p + lane / 4, LDS chunk q' = lane & 3, source chunk q' ^ ((row >> 1) & 2)
  const uint32_t wq = 16u * ((lane & 3) ^ (2 * ((lane >> 4) & 1)));  // byte offset in the row
  auto issue_plane = [&](int c, int b, int R0) {
    if constexpr ((ABL & 1) != 0) return;
    const bf16_t* base = a.x + (int64_t)b * T * C + c * 32;  // utterance b is < 2 GiB (checked)
    const uint32_t dst = lds_act + (uint32_t)(c * PLANE_E * 2);
#pragma unroll
    for (int u = 0; u < WPW; ++u) {
      const int p = rw * WPW + u;
      const int t = min(max(R0 + 16 * p + (lane >> 2), 0), T - 1);
      dma16(base, (uint32_t)t * (C * 2) + wq, dst + p * 1024);
    }
  };
  // leaky ReLU in place over this wave's pieces of plane c; rows outside [0, T) -> 0 (c1's padding)
  auto relu_plane = [&](int c, int R0) {
    if constexpr ((ABL & 1) != 0) return;
#pragma unroll
    for (int u = 0; u < WPW; ++u) {
      const int p = rw * WPW + u;
      const int t = R0 + 16 * p + (lane >> 2);
      u32x4* q = reinterpret_cast<u32x4*>(act + c * PLANE_E + p * 512 + lane * 8);
      const u32x4 v = lrelu8_pk(*q, slope);
      *q = (t >= 0 && t < T) ? v : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto tile_geo = [&](int tl, int& b, int& t0) {
    b = tl / a.tiles_per_b;
    t0 = (tl - b * a.tiles_per_b) * BT;
  };

  // ---- prologue: the first tile's whole window and the first weight group
  {
    int b, t0;
    tile_geo(tile, b, t0);
    const int R0 = t0 - h2 - h1;
    if (wissue) issue_group(0, 0);
    if (!wrole) {
#pragma unroll
      for (int c = 0; c < NC; ++c) issue_plane(c, b, R0);
    }
    wait_vm<0>();
    if (!wrole) {
      // only the planes a steady-state tile finds already activated (leaky ReLU'd at the previous
      // P2's end); the others are activated by the tile loop itself (late planes after their
      // re-DMA at P1 start, early ones in the group before their first use)
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (P::early(c) && P::gn(c) == 0) relu_plane(c, R0);
    }
  }
  lds_barrier();

  int a_off[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) a_off[i] = rb_off(cw0 + NI * 4 * (lr >> 2) + 4 * i + (lr & 3), lq, SHW);
  const int brow0 = wt * 16 * NJ + lr;

  f32x4 acc[NI][NJ];
  u32x4 xres[NJ][NH], ares[NJ][NH];
  if constexpr (VAR == 1)
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  int gcount = 0;
  int titer = 0;  // tiles done by this workgroup (diagnostic stamps)
  auto stamp = [&](int slot, int which) {
#ifdef VO_ABLATIONS
    if constexpr ((ABL & 4) != 0) {
      if (blockIdx.x < 8 && titer < 4 && (wave & 3) == 0 && lane == 0) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        g_pc_stamp[(((blockIdx.x * 2 + (wave >> 2)) * 4 + titer) * 64 + slot) * 2 + which] = t;
      }
    }
#endif
    (void)slot; (void)which;
  };

  for (; tile < tile_end; ++tile) {
    int b, t0;
    tile_geo(tile, b, t0);
    const int R0 = t0 - h2 - h1;
    int nb, nt0;
    tile_geo(min(tile + 1, a.ntiles - 1), nb, nt0);  // next window (a valid dummy after the run)
    const int nR0 = nt0 - h2 - h1;

    // P1 accumulators start at b1
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + n0 + 4 * i);
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = bv;
    }

    auto group = [&](const int ph, const int g) {
      stamp(ph * NG + g, 0);
      const int gi = ph * NG + g;
      const bf16_t* wb = wls + (gcount & 1) * SPG * SLICE_E;
      if (wissue) issue_group(gi + 1 == 2 * NG ? 0 : gi + 1, (gcount + 1) & 1);
      int wpieces = 0;  // window pieces issued in this group (MODE 1's group-end wait leaves them in flight)
      if (wrole) {
      } else if (ph == 0) {
        if (g == 0) {  // late planes of this tile's window (their T1 planes died at the last P2 group)
#pragma unroll
          for (int c = 0; c < NC; ++c)
            if (!P::early(c)) issue_plane(c, b, R0);
          wpieces = P::n_late();
        }
        // leaky ReLU of plane c one group before P1 first reads it
#pragma unroll
        for (int c = 1; c < NC; ++c) {
          if (P::gn(c) >= 1 && g == P::gn(c) - 1) {
            // vector-memory operations issued after plane c's DMA: for an early plane the later
            // early planes, the previous tile's y stores and this tile's late planes; for a late
            // plane the later late planes
            if (P::early(c)) {
              switch (P::n_early_after(c) + P::n_late()) {  // wait_vm needs an immediate
                case 0: wait_vm<NJ * NH>(); break;
                case 1: wait_vm<WPW + NJ * NH>(); break;
                case 2: wait_vm<2 * WPW + NJ * NH>(); break;
                default: wait_vm<3 * WPW + NJ * NH>(); break;
              }
            } else {
              switch (P::n_late_after(c)) {
                case 0: wait_vm<0>(); break;
                case 1: wait_vm<WPW>(); break;
                default: wait_vm<2 * WPW>(); break;
              }
            }
            relu_plane(c, R0);
          }
        }
      } else {
        // P2: the next tile's early planes go into the T1 planes that just died
#pragma unroll
        for (int c = 0; c < NC; ++c)
          if (P::early(c) && g == P::gf(c) + 1) {
            issue_plane(c, nb, nR0);
            wpieces = 1;
          }
      }
      if (ph == 0 && g == NG - 1) {  // residual (and accumulator) rows, folded into P2's init
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int pos = min(t0 + wt * 16 * NJ + 16 * j + lr, T - 1);
          const int64_t off = ((int64_t)b * T + pos) * C + n0;
#pragma unroll
          for (int h = 0; h < NH; ++h) xres[j][h] = *reinterpret_cast<const u32x4*>(a.x + off + 8 * h);
        }
      }

      // SPG slices, software-pipelined: slice st + 1's fragments are read right after slice st's
      // first MFMA
      const bf16_t* src_base = act;
      const int step = ph ? 1 : dil;
      Frag<bf16_t> af[2][NI], bq[2][NJ];
      auto ld = [&](int st, int set) {
        const int s = g * SPG + st;
        const int c = s / K, k = s - c * K;
        const bf16_t* wt_ = wb + st * SLICE_E;
#pragma unroll
        for (int i = 0; i < NI; ++i) af[set][i].load(wt_ + a_off[i]);
        const int boff = c * PLANE_E + rb_off(brow0 + k * step, lq, 2);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bq[set][j].load(src_base + boff + 16 * j * 32);
      };
      if constexpr (VAR == 2) {
#pragma unroll
        for (int st = 0; st < SPG; ++st) {
          ld(st, 0);
#pragma unroll
          for (int q = 0; q < NI * NJ; ++q) acc[q / NJ][q % NJ] = mfma(af[0][q / NJ], bq[0][q % NJ], acc[q / NJ][q % NJ]);
        }
      }
      if (VAR != 2) ld(0, 0);
#pragma unroll
      for (int st = 0; st < (VAR == 2 ? 0 : SPG); ++st) {
#pragma unroll
        for (int q = 0; q < NI * NJ; ++q) {
          const int i = q / NJ, j = q - i * NJ;
          acc[i][j] = mfma(af[st & 1][i], bq[st & 1][j], acc[i][j]);
          if (q == 0) {
            __builtin_amdgcn_sched_barrier(0);
            if (st + 1 < SPG) ld(st + 1, (st + 1) & 1);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (HAS_ACC && ph == 1 && g == 0) {  // the MRF accumulator rows (requested in the P1 epilogue)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int h = 0; h < NH; ++h) {
            float af8[8];
            unpack8(ares[j][h], af8);
#pragma unroll
            for (int e8 = 0; e8 < 8; ++e8) acc[2 * h + e8 / 4][j][e8 & 3] += af8[e8] * a.inv_scale;
          }
      }
      stamp(ph * NG + g, 1);
      if (MODE == 0 && wrole) wait_vm<0>();  // this wave's slice of the next group landed
      if (MODE == 1) {  // this wave's weight pieces landed; this group's window pieces may not have
        if (wpieces == 0) wait_vm<0>();
        else if (wpieces == 1) wait_vm<WPW>();
        else wait_vm<2 * WPW>();
      }
      lds_barrier();
      ++gcount;
    };

    for (int g = 0; g < NG; ++g) group(0, g);
    stamp(60, 0);

    // the MRF accumulator rows: requested here, added after P2's first group (registers are short
    // during P1's last group, which holds the residual rows)
    if constexpr (HAS_ACC) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int pos = min(t0 + wt * 16 * NJ + 16 * j + lr, T - 1);
        const int64_t off = ((int64_t)b * T + pos) * C + n0;
#pragma unroll
        for (int h = 0; h < NH; ++h) ares[j][h] = *reinterpret_cast<const u32x4*>(a.acc + off + 8 * h);
      }
    }
    // P1 epilogue: T1 = lrelu(acc) over the dead window, zero outside [0, T) (c2's padding).  The
    // lane's row / channel are re-derived from an opaque copy of the thread id: hoisted out of the
    // tile loop, the eight store addresses were spilled to scratch (and each reload's vmcnt(0)
    // waited for the accumulator rows just requested)
    {
      int tv = tid;
      asm volatile("" : "+v"(tv));
      const int lr_ = tv & 15, n0_ = cw0 + NI * 4 * ((tv & 63) >> 4);
      const bool interior = t0 - h2 >= 0 && t0 - h2 + R1 <= T;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = wt * 16 * NJ + 16 * j + lr_;
        const int pos = t0 - h2 + r;
        const uint32_t km = (interior || (pos >= 0 && pos < T)) ? 0xffffffffu : 0u;
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          uint32_t w[4];
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) {
            const int e = 2 * e2;
            w[e2] = lrelu_pk(acc[2 * h + e / 4][j][e & 3], acc[2 * h + (e + 1) / 4][j][(e + 1) & 3], slope) & km;
          }
          const int ch = n0_ + 8 * h;
          *reinterpret_cast<u32x4*>(act + (ch >> 5) * PLANE_E + rb_off(r, (ch & 31) >> 3, 2)) = u32x4{w[0], w[1], w[2], w[3]};
        }
      }
    }
    // P2 accumulators start at b2 + x (+ acc_in / out_scale)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        float xf[8];
        unpack8(xres[j][h], xf);
#pragma unroll
        for (int e8 = 0; e8 < 8; ++e8) {
          const int i = 2 * h + e8 / 4, e = e8 & 3;
          acc[i][j][e] = sbias[C + n0 + 4 * i + e] + xf[e8];
        }
      }
    }
    lds_barrier();  // T1 complete
    stamp(60, 1);

    for (int g = 0; g < NG; ++g) group(1, g);
    stamp(61, 0);

    // window waves: leaky ReLU of the next window's planes that P1 reads in its first group
    if (!wrole) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (P::early(c) && P::gn(c) == 0) {
          switch (P::n_early_after(c)) {
            case 0: wait_vm<0>(); break;
            case 1: wait_vm<WPW>(); break;
            case 2: wait_vm<2 * WPW>(); break;
            default: wait_vm<3 * WPW>(); break;
          }
          relu_plane(c, nR0);
        }
      }
    }
    // P2 epilogue: y = acc * out_scale; rows past the tile / past T fall outside the buffer
    // resource and their stores are dropped
    const int valid = min(BT, T - t0);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.y + ((int64_t)b * T + t0) * C), (short)0, valid * C * (int)sizeof(bf16_t), 0x00020000);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int r = wt * 16 * NJ + 16 * j + lr;
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        uint32_t w[4];
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          const int e = 2 * e2;
          w[e2] = pk_bf16(acc[2 * h + e / 4][j][e & 3] * a.out_scale, acc[2 * h + (e + 1) / 4][j][(e + 1) & 3] * a.out_scale);
        }
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{w[0], w[1], w[2], w[3]}, yrs,
                                               (r * C + n0 + 8 * h) * (int)sizeof(bf16_t), 0, 0);
      }
    }
    lds_barrier();  // plane-0 leaky ReLU visible before the next P1
    stamp(63, 0);
    ++titer;
  }
  wait_vm<0>();  // no LDS-DMA may land after the workgroup's LDS is released
}

template <int K, bool HAS_ACC, int MODE, int ABL, int VAR = 0>
static int pc_launch(PcArgs a, int B, hipStream_t st) {
  constexpr int R1 = 256;
  constexpr int h2 = (K - 1) / 2;
  constexpr int BT = R1 - 2 * h2;
  a.tiles_per_b = (a.T + BT - 1) / BT;
  a.ntiles = a.tiles_per_b * B;
  constexpr size_t lds = 4 * 320 * 64 + 2 * 4 * 128 * 64 + 2 * 128 * 4;
  auto kern = mrf_pair_pc_kernel<K, HAS_ACC, MODE, ABL, VAR>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  const int grid = (int)std::min<int64_t>((int64_t)cus, a.ntiles);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(512), lds, st, a);
  VO_RETURN_LAUNCH();
}

}  // namespace vo

using namespace vo;

// C = 128, K in {7, 11}, dil * (K - 1) <= 64, out_scale > 0: the round-4 producer-role pair.
// *handled = 0 when the shape is not covered (the caller falls back).
int vo_pair_pc_try(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                   const void* acc, int B, int T, int C, int K, int dil, float slope, float out_scale,
                   hipStream_t st, int* handled) {
  *handled = 0;
  if (C != 128 || (K != 7 && K != 11) || dil < 1 || dil * (K - 1) > 64 || !(out_scale > 0.f) ||
      (int64_t)T * C * 2 >= (int64_t)1 << 31)
    return VO_OK;
  *handled = 1;
  PcArgs a;
  a.x = (const bf16_t*)x; a.w1 = (const bf16_t*)w1; a.b1 = b1; a.w2 = (const bf16_t*)w2; a.b2 = b2;
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)acc;
  a.T = T; a.dil = dil; a.slope = slope; a.out_scale = out_scale; a.inv_scale = 1.f / out_scale;
  a.tiles_per_b = a.ntiles = 0;
  const int mode = vo_tune_get("pc_cfg");
#ifdef VO_ABLATIONS
  if (mode == 8) return K == 7 ? pc_launch<7, true, 0, 1>(a, B, st) : pc_launch<11, true, 0, 1>(a, B, st);
  if (mode == 9) return K == 7 ? pc_launch<7, true, 0, 2>(a, B, st) : pc_launch<11, true, 0, 2>(a, B, st);
  if (mode == 10) return K == 7 ? pc_launch<7, true, 0, 3>(a, B, st) : pc_launch<11, true, 0, 3>(a, B, st);
  if (mode == 12) return K == 7 ? pc_launch<7, true, 0, 4>(a, B, st) : pc_launch<11, true, 0, 4>(a, B, st);
  if (mode == 13) return K == 7 ? pc_launch<7, true, 0, 7>(a, B, st) : pc_launch<11, true, 0, 7>(a, B, st);
  if (mode == 14) return K == 7 ? pc_launch<7, true, 0, 4, 1>(a, B, st) : pc_launch<11, true, 0, 4, 1>(a, B, st);
  if (mode == 15) return K == 7 ? pc_launch<7, true, 0, 4, 2>(a, B, st) : pc_launch<11, true, 0, 4, 2>(a, B, st);
#endif
  if (mode == 2 || mode == 3) {
    if (K == 7) return mode == 2 ? pc_launch<7, true, 0, 0, 1>(a, B, st) : pc_launch<7, true, 0, 0, 2>(a, B, st);
    return mode == 2 ? pc_launch<11, true, 0, 0, 1>(a, B, st) : pc_launch<11, true, 0, 0, 2>(a, B, st);
  }
  if (mode == 1) {
    if (K == 7) return acc ? pc_launch<7, true, 1, 0>(a, B, st) : pc_launch<7, false, 1, 0>(a, B, st);
    return acc ? pc_launch<11, true, 1, 0>(a, B, st) : pc_launch<11, false, 1, 0>(a, B, st);
  }
  if (K == 7) return acc ? pc_launch<7, true, 0, 0>(a, B, st) : pc_launch<7, false, 0, 0>(a, B, st);
  return acc ? pc_launch<11, true, 0, 0>(a, B, st) : pc_launch<11, false, 0, 0>(a, B, st);
}

#ifdef VO_ABLATIONS
// copies the diagnostic stamps (see g_pc_stamp) to host memory: n 64-bit values
extern "C" int vo_pc_stamps(unsigned long long* host, int n) {
  const int cap = (int)(sizeof(g_pc_stamp) / sizeof(g_pc_stamp[0]));
  if (n > cap) n = cap;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pc_stamp), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
#endif

#endif  // VO_ABLATIONS
