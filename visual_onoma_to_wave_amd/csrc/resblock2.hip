// Fused HiFi-GAN ResBlock1 pair, version 2 (k = 7 / 11 at C = 64 / 128):
//   y = (x + c2(lrelu(c1_d(lrelu(x), slope), slope))) * out_scale (+ acc)
// (scripts/hifigan/models.py:96-103, one (c1, c2) iteration; the MRF sum and 1/num_kernels
// scale of models.py:155-160 ride in the epilogue).
//
// Same tiling as resblock.hip's in-place kernel (persistent workgroups walking contiguous tile
// runs; T1 = lrelu(c1) written over the dead window; weights streamed one group of TG taps at a
// time through a double buffer), with two changes measured on the bench shapes:
//  * the kernel size K is a template parameter, so the tap loops are straight-line code with
//    compile-time LDS offsets;
//  * the NEXT tile's input window is fetched DURING P2, a slot or two per tap group, into
//    registers, and written to LDS (lrelu'd) right after P2.  In resblock.hip every CU fetched
//    its whole next window after P2 at the same moment, with no MFMA work to overlap: the timing
//    ablation without window / residual loads ran 17-21 % faster (tools/ab_pair2.py, cfg 17).
//    The group-end wait is `s_waitcnt vmcnt(n)` with n = the window loads of this group: vmcnt
//    retires in issue order, so the group's weight DMA (issued first) has landed while the
//    window loads may stay in flight for up to two groups.
// Dilation <= DMAX (5: the HiFi-GAN V1 MRF); the region rows are sized for it at compile time.

#include <algorithm>
#include <type_traits>

#include "mrf_common.h"

namespace vo {

struct Pair2Args {
  const bf16_t* x; const bf16_t* w1; const float* b1; const bf16_t* w2; const float* b2;
  bf16_t* y; const bf16_t* acc;
  int T, dil, tiles_per_b, ntiles;
  float slope, out_scale;
};

constexpr int PAIR2_DMAX = 5;

// VD (round 3, "VALU diet"): each conv's bias is the C operand of its first MFMAs (no accumulator
// zeroing, no bias adds), leaky ReLU in packed fp32, the T1 mask only in boundary tiles.
// PIPE (round 3): each group's (tap, plane) steps software-pipelined as in resblock3.hip -- the next
// step's fragments are read right after the current step's first MFMA (two register sets); bit 0: P1,
// bit 1: P2 (where the next tile's window slots are live too)
template <int C, int WC, int WT, int NJ, int K, bool GL, int TG, bool VD = true, int PIPE = 0>
__global__ void __launch_bounds__(WC * WT * 64, 2) mrf_pair2_kernel(Pair2Args a) {
  constexpr int NW = WC * WT;
  constexpr int NT = NW * 64;
  constexpr int NC = C / 32;              // 32-channel planes
  constexpr int NI = C / (16 * WC);       // co tiles per wave
  constexpr int R1 = WT * 16 * NJ;        // c1 rows per tile
  constexpr int SHW = NI >= 8 ? 5 : (NI == 4 ? 4 : 3);  // log2(4 * NI): weight-row swizzle
  constexpr int VPR = NC * 4;             // 16-byte vectors per activation row
  constexpr int H2 = (K - 1) / 2;
  constexpr int WRMAX = R1 + 2 * PAIR2_DMAX * H2;  // window rows at the largest dilation
  constexpr int T1R = R1 + 16;            // P2 reads up to row R1 + K - 2 (feeds discarded rows only)
  constexpr int WR = WRMAX > T1R ? WRMAX : T1R;  // region rows per plane (window, then T1 over it)
  constexpr int TAPV = C * VPR;           // 16-byte vectors per weight tap
  constexpr int TAPE = NC * C * 32;       // LDS elements per weight tap
  constexpr int NG = (K + TG - 1) / TG;   // weight groups per conv
  constexpr int GE = TG * TAPE;           // LDS elements per group buffer
  constexpr int GV = (TG * TAPV + NT - 1) / NT;  // register-staged vectors per thread per group
  constexpr int GLN = GL ? TG * TAPV / (64 * NW) : 1;  // DMA instructions per wave per group
  static_assert(!GL || (TG * TAPV) % (64 * NW) == 0, "DMA groups split into whole wave-KiB");
  static_assert(NT % VPR == 0 && (NT / VPR) % 8 == 0, "window slot stride must keep the swizzle");
  constexpr int RSTEP = NT / VPR;         // window rows between a thread's slots
  constexpr int MAXW = (WRMAX + RSTEP - 1) / RSTEP;  // window vectors per thread
  // window slots fetched per P2 group: two where the unrolled groups would otherwise spill (C = 128)
  constexpr int SPG = C >= 128 ? 2 : (MAXW + NG - 1) / NG;
  static_assert(SPG <= 3, "at most 3 window slots per group");
  constexpr int NGW = (MAXW + SPG - 1) / SPG;        // P2 groups that fetch window slots
  static_assert(NGW <= NG, "window slots must fit the P2 groups");
  constexpr int NH = NI / 2;              // 8-channel vectors per lane in epilogue layout
  constexpr int BT = R1 - 2 * H2;         // output rows per tile

  const int dil = a.dil, T = a.T;
  const int h1 = dil * H2;
  const int win_rows = R1 + 2 * h1;
  const float slope = a.slope;

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* reg = reinterpret_cast<bf16_t*>(smem_raw);   // [NC][WR][32]: window, then T1
  bf16_t* wls = reg + NC * WR * 32;                     // [2][GE] weight group buffers
  float* sbias = reinterpret_cast<float*>(wls + 2 * GE);  // [b1 | b2]
  bf16_t* spare = reinterpret_cast<bf16_t*>(sbias + 2 * C);  // 16 B sink for idle staging slots

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  const int wc = wave % WC, wt = wave / WC;
  const int cw0 = wc * (C / WC);
  const int n0 = cw0 + NI * 4 * lq;

  const int G = gridDim.x;
  int tile = (int)(((int64_t)blockIdx.x * a.ntiles) / G);
  const int tile_end = (int)(((int64_t)(blockIdx.x + 1) * a.ntiles) / G);
  if (tile >= tile_end) return;  // uniform per workgroup

  for (int i = tid; i < 2 * C; i += NT) sbias[i] = i < C ? a.b1[i] : a.b2[i - C];

  // ---- weight groups: group q in [0, 2 NG): conv q / NG, taps (q % NG) * TG + [0, TG)
  int wg_g[GV], wg_l[GV], wg_t[GV];
#pragma unroll
  for (int s = 0; s < GV; ++s) {
    const int v = tid + s * NT;
    const int t = v / TAPV, vv = v - t * TAPV;
    const int pl = vv / (C * 4), rem = vv - pl * C * 4;
    const int co = rem >> 2, q = rem & 3;
    wg_t[s] = v < TG * TAPV ? t : TG;  // TG marks an idle slot
    wg_g[s] = co * C + pl * 32 + q * 8;
    wg_l[s] = t * TAPE + pl * C * 32 + rb_off(co, q, SHW);
  }
  u32x4 wr[GV];
  int gl_t[GLN], gl_off[GLN];
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  if constexpr (GL) {
#pragma unroll
    for (int s = 0; s < GLN; ++s) {
      const int p = (s * NW + wave) * 64 + lane;
      const int t = p / TAPV, vv = p - t * TAPV;
      const int pl = vv / (C * 4), rem = vv - pl * C * 4;
      const int co = rem >> 2, q = (rem & 3) ^ ((co >> (SHW - 1)) & 2);
      gl_t[s] = t;
      gl_off[s] = co * C + pl * 32 + q * 8;
    }
  }
  auto load_group = [&](int q, int buf) {
    const int ph = q >= NG;
    const int k0 = (q - ph * NG) * TG;
    const bf16_t* W = ph ? a.w2 : a.w1;
    if constexpr (GL) {
      typedef __attribute__((address_space(3))) void lds_void;
      typedef const __attribute__((address_space(1))) void g_void;
      const bf16_t* Wk = W + k0 * (C * C);
#pragma unroll
      for (int s = 0; s < GLN; ++s) {
        const int dt = TG == 1 ? 0 : min(gl_t[s], K - 1 - k0);  // taps past K re-read K - 1 (unused)
        __builtin_amdgcn_global_load_lds((g_void*)(Wk + (dt * (C * C) + gl_off[s])),
                                         (lds_void*)(wls + buf * GE + (s * NW + wave_u) * 64 * 8), 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < GV; ++s) {
        const int k = k0 + (wg_t[s] < TG ? wg_t[s] : 0);
        wr[s] = *reinterpret_cast<const u32x4*>(W + (int64_t)min(k, K - 1) * C * C + wg_g[s]);
      }
    }
  };
  auto store_group = [&](int buf) {
    if constexpr (!GL) {
#pragma unroll
      for (int s = 0; s < GV; ++s)
        if (GV * NT == TG * TAPV || wg_t[s] < TG) *reinterpret_cast<u32x4*>(wls + buf * GE + wg_l[s]) = wr[s];
    }
  };

  // ---- window staging (row-major vectors; slot s of a thread = row xr0 + s * RSTEP)
  const int xr0 = tid / VPR, xrem = tid - xr0 * VPR;
  const int xg0 = xrem * 8;
  const int xl0 = (xrem >> 2) * WR * 32 + rb_off(xr0, xrem & 3, 2);
  u32x4 xw[MAXW];
  bool xw_ok[MAXW];
  auto load_slot = [&](int s, int tl) {  // s compile-time after unrolling
    const int b = tl / a.tiles_per_b;
    const int R0 = (tl - b * a.tiles_per_b) * BT - H2 - h1;
    const int t = R0 + xr0 + s * RSTEP;
    xw_ok[s] = t >= 0 && t < T && xr0 + s * RSTEP < win_rows;
    xw[s] = *reinterpret_cast<const u32x4*>(a.x + ((int64_t)b * T + min(max(t, 0), T - 1)) * C + xg0);
  };
  auto store_win = [&]() {
#pragma unroll
    for (int s = 0; s < MAXW; ++s) {
      const u32x4 v = lrelu8(xw[s], slope);
      *reinterpret_cast<u32x4*>(xr0 + s * RSTEP < win_rows ? reg + xl0 + s * RSTEP * 32 : spare) =
          xw_ok[s] ? v : u32x4{0u, 0u, 0u, 0u};
    }
  };

  int a_off[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) a_off[i] = rb_off(cw0 + NI * 4 * (lr >> 2) + 4 * i + (lr & 3), lq, SHW);
  const int brow0_ = wt * 16 * NJ + lr;

  load_group(0, 0);
  store_group(0);
#pragma unroll
  for (int s = 0; s < MAXW; ++s) load_slot(s, tile);
  store_win();
  if constexpr (GL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();

  f32x4 acc[NI][NJ];
  int gc = 0;  // groups consumed (double-buffer parity)

  auto lane_bias = [&](int which, float (&bz)[8 * NH]) {
    const float4* bp = reinterpret_cast<const float4*>(sbias + which * C + n0);
#pragma unroll
    for (int u = 0; u < 2 * NH; ++u) {
      const float4 v = bp[u];
      bz[4 * u] = v.x; bz[4 * u + 1] = v.y; bz[4 * u + 2] = v.z; bz[4 * u + 3] = v.w;
    }
  };

  // one (tap, plane) step: NI x NJ MFMAs; bias_row >= 0 (VD, a conv's first step): the bias of that
  // conv is the C operand
  auto tap = [&](const bf16_t* wt_, const bf16_t* src, int row, int bias_row = -1) {
    Frag<bf16_t> af[NI], bfr[NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i) af[i].load(wt_ + a_off[i]);
    const int boff = rb_off(row, lq, 2);
#pragma unroll
    for (int j = 0; j < NJ; ++j) bfr[j].load(src + boff + 16 * j * 32);
    if (bias_row >= 0) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + bias_row * C + n0 + 4 * i);
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma(af[i], bfr[j], bv);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma(af[i], bfr[j], acc[i][j]);
    }
    // keep the unrolled straight-line steps apart: hoisting the next steps' fragment reads
    // above these MFMAs blew the register budget (spills)
    __builtin_amdgcn_sched_barrier(0);
  };

  // S_c steps; aptr(st) / bptr(st): the step's A (weights) and B (activation rows) base addresses;
  // valid(st): the step's tap exists; bias_row >= 0 (compile-time after inlining): bias as C
  auto piped = [&](auto S_c, auto&& aptr, auto&& bptr, auto&& valid, int bias_row) {
    constexpr int S = decltype(S_c)::value;
    Frag<bf16_t> fa[2][NI], fb[2][NJ];
    auto ld = [&](int st, int set) {
      const bf16_t* pa = aptr(st);
      const bf16_t* pb = bptr(st);
#pragma unroll
      for (int i = 0; i < NI; ++i) fa[set][i].load(pa + a_off[i]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb[set][j].load(pb + 16 * j * 32);
    };
    f32x4 bz4[NI];
    if (bias_row >= 0) {
#pragma unroll
      for (int i = 0; i < NI; ++i) bz4[i] = *reinterpret_cast<const f32x4*>(sbias + bias_row * C + n0 + 4 * i);
    }
    ld(0, 0);
#pragma unroll
    for (int st = 0; st < S; ++st) {
      const int set = st & 1;
      const bool ok = valid(st), first = bias_row >= 0 && st == 0;
#pragma unroll
      for (int q = 0; q < NI * NJ; ++q) {
        const int i = q / NJ, j = q - i * NJ;
        if (ok) acc[i][j] = mfma(fa[set][i], fb[set][j], first ? bz4[i] : acc[i][j]);
        if (q == 0) {
          __builtin_amdgcn_sched_barrier(0);
          if (st + 1 < S) ld(st + 1, (st + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  for (; tile < tile_end; ++tile) {
    const int b = tile / a.tiles_per_b;
    const int t0 = (tile - b * a.tiles_per_b) * BT;
    const bool has_next = tile + 1 < tile_end;
    // opaque per tile: the per-step fragment addresses are recomputed inside their (sched-barrier
    // fenced) steps instead of all being hoisted out of the tile loop and held in registers
    int brow0 = brow0_;
    asm volatile("" : "+v"(brow0));

    if constexpr (!VD) {
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // ---- P1: c1 over the lrelu'd window (a runtime loop: unrolled, both phases spilled); the first
    // group is peeled so that its first step (bias as the C operand) is known statically
    auto p1_group = [&](int g, bool first) {
      load_group(g + 1, (gc + 1) & 1);  // g = NG - 1: P2's first group
      const bf16_t* wb = wls + (gc & 1) * GE;
      if constexpr ((PIPE & 1) != 0) {
        piped(std::integral_constant<int, TG * NC>{},
              [&](int st) { return wb + (st / NC) * TAPE + (st % NC) * C * 32; },
              [&](int st) { return reg + (st % NC) * WR * 32 + rb_off(brow0 + (g * TG + st / NC) * dil, lq, 2); },
              [&](int st) { return TG == 1 || g * TG + st / NC < K; }, VD && first ? 0 : -1);
      }
#pragma unroll
      for (int t = 0; t < ((PIPE & 1) ? 0 : TG); ++t) {
        if (g * TG + t >= K) continue;
#pragma unroll
        for (int c = 0; c < NC; ++c)
          tap(wb + t * TAPE + c * C * 32, reg + c * WR * 32, brow0 + (g * TG + t) * dil,
              VD && first && t == 0 && c == 0 ? 0 : -1);
      }
      store_group((gc + 1) & 1);
      if constexpr (GL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
      ++gc;
    };
    p1_group(0, true);
#pragma unroll 1
    for (int g = 1; g < NG; ++g) p1_group(g, false);

    // ---- P1 epilogue: T1 = lrelu(acc + b1) over the (dead) window; zero outside [0, T)
    if constexpr (VD) {  // the bias is in the accumulators
      const bool interior = t0 - H2 >= 0 && t0 - H2 + R1 <= T;  // uniform
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = wt * 16 * NJ + 16 * j + lr;
        const int pos = t0 - H2 + r;
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
          *reinterpret_cast<u32x4*>(reg + (ch >> 5) * WR * 32 + rb_off(r, (ch & 31) >> 3, 2)) = u32x4{w[0], w[1], w[2], w[3]};
        }
      }
    } else {
      float bz[8 * NH];
      lane_bias(0, bz);
      const bool interior = t0 - H2 >= 0 && t0 - H2 + R1 <= T;  // uniform
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = wt * 16 * NJ + 16 * j + lr;
        const int pos = t0 - H2 + r;
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
          *reinterpret_cast<u32x4*>(reg + (ch >> 5) * WR * 32 + rb_off(r, (ch & 31) >> 3, 2)) = u32x4{w[0], w[1], w[2], w[3]};
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    lds_barrier();

    // ---- P2: c2 over T1; the next tile's window slots [g SPG, (g + 1) SPG) are fetched in groups
    // g < NGW (unrolled: the slot registers need compile-time indices), the rest is a runtime loop
    auto p2_group = [&](int g, int s_lo, int s_hi) {
      load_group(g + 1 < NG ? NG + g + 1 : 0, (gc + 1) & 1);  // last group: the next tile's first
      __builtin_amdgcn_sched_barrier(0);  // the weight DMA stays older than the window loads
      // unconditional (the last tile of a run re-reads its own window): conditional loads kept
      // the window registers live around the tile loop (spills)
#pragma unroll
      for (int s = s_lo; s < s_hi; ++s) load_slot(s, has_next ? tile + 1 : tile);
      __builtin_amdgcn_sched_barrier(0);
      const bf16_t* wb = wls + (gc & 1) * GE;
      if constexpr ((PIPE & 2) != 0) {
        piped(std::integral_constant<int, TG * NC>{},
              [&](int st) { return wb + (st / NC) * TAPE + (st % NC) * C * 32; },
              [&](int st) { return reg + (st % NC) * WR * 32 + rb_off(brow0 + g * TG + st / NC, lq, 2); },
              [&](int st) { return TG == 1 || g * TG + st / NC < K; }, VD && g == 0 ? 1 : -1);
      }
#pragma unroll
      for (int t = 0; t < ((PIPE & 2) ? 0 : TG); ++t) {
        if (g * TG + t >= K) continue;
#pragma unroll
        for (int c = 0; c < NC; ++c)
          tap(wb + t * TAPE + c * C * 32, reg + c * WR * 32, brow0 + g * TG + t, VD && g == 0 && t == 0 && c == 0 ? 1 : -1);
      }
      store_group((gc + 1) & 1);
      if constexpr (GL) {
        // the DMA has landed; this group's window loads may stay in flight
        switch (s_hi - s_lo) {  // folds to one wait in the unrolled groups
          case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
          case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
          case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
          default: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        }
      }
      lds_barrier();
      ++gc;
    };
#pragma unroll
    for (int g = 0; g < NGW; ++g) p2_group(g, g * SPG, (g + 1) * SPG < MAXW ? (g + 1) * SPG : MAXW);
#pragma unroll 1
    for (int g = NGW; g < NG; ++g) p2_group(g, 0, 0);

    // ---- P2 epilogue: the residual rows are requested first, the window goes to LDS while
    // they are in flight (T1's reads ended at the last group barrier), then
    // y = (c2 + b2 + x) * out_scale (+ acc), stored through a buffer resource that covers exactly
    // the tile's valid rows (the stores of the rows past it are dropped: no per-lane branch)
    u32x4 xres[NJ][NH], ares[NJ][NH];
    const bf16_t* accp = a.acc ? a.acc : a.x;  // loaded either way (no branch), added only with acc
    if (C >= 128 && has_next) store_win();  // C = 128: no registers to spare for the early loads
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int pos = min(t0 + wt * 16 * NJ + 16 * j + lr, T - 1);
      const int64_t off = ((int64_t)b * T + pos) * C + n0;
#pragma unroll
      for (int h = 0; h < NH; ++h) xres[j][h] = *reinterpret_cast<const u32x4*>(a.x + off + 8 * h);
    }
    if (C < 128 && has_next) store_win();  // its registers are free before the accumulator rows are requested
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int pos = min(t0 + wt * 16 * NJ + 16 * j + lr, T - 1);
      const int64_t off = ((int64_t)b * T + pos) * C + n0;
#pragma unroll
      for (int h = 0; h < NH; ++h) ares[j][h] = *reinterpret_cast<const u32x4*>(accp + off + 8 * h);
    }
    float b2z[8 * NH];
    if constexpr (VD) {
#pragma unroll
      for (int u = 0; u < 8 * NH; ++u) b2z[u] = 0.f;  // the bias is in the accumulators
    } else {
      lane_bias(1, b2z);
    }
    const int valid = min(BT, T - t0);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.y + ((int64_t)b * T + t0) * C), (short)0, valid * C * (int)sizeof(bf16_t), 0x00020000);
    auto epilogue = [&](auto with_acc) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = wt * 16 * NJ + 16 * j + lr;
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
              q[u] = (acc[2 * h + e / 4][j][e & 3] + b2z[8 * h + e] + xf[e]) * a.out_scale;
              if constexpr (decltype(with_acc)::value) q[u] += af8[e];
            }
            w[e2] = pk_bf16(q[0], q[1]);
          }
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{w[0], w[1], w[2], w[3]}, yrs,
                                                 (r * C + n0 + 8 * h) * (int)sizeof(bf16_t), 0, 0);
        }
      }
    };
    if (a.acc)
      epilogue(std::true_type{});
    else
      epilogue(std::false_type{});
    lds_barrier();  // the next window is visible before the next P1
  }
}

template <int C, int WC, int WT, int NJ, int K, bool GL, int TG, bool VD = true, int PIPE = 0>
static int pair2_launch(Pair2Args a, int B, hipStream_t st) {
  constexpr int NW = WC * WT;
  constexpr int R1 = WT * 16 * NJ;
  constexpr int H2 = (K - 1) / 2;
  constexpr int WRMAX = R1 + 2 * PAIR2_DMAX * H2;
  constexpr int WR = WRMAX > R1 + 16 ? WRMAX : R1 + 16;
  constexpr int BT = R1 - 2 * H2;
  a.tiles_per_b = (a.T + BT - 1) / BT;
  a.ntiles = a.tiles_per_b * B;
  const size_t lds = ((size_t)WR * C + 2 * (size_t)TG * C * C) * sizeof(bf16_t) + 2 * C * sizeof(float) + 16;
  if (lds > 160 * 1024) {
    vo_set_error("resblock_pair (v2): LDS %zu B exceeds 160 KiB", lds);
    return VO_ERR_INVALID;
  }
  auto kern = mrf_pair2_kernel<C, WC, WT, NJ, K, GL, TG, VD, PIPE>;
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

// Entry from vo_resblock_pair (resblock.hip): returns 1 in *handled when this kernel covers the
// shape (C = 64 / 128, K = 7 / 11, dilation <= 5), else leaves the launch to the v1 kernels.
int vo_pair2_try(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                 const void* acc, int B, int T, int C, int K, int dil, float slope, float out_scale, int cfg,
                 hipStream_t st, int* handled) {
  *handled = 0;
#ifdef VO_ABLATIONS
  const bool c128 = C == 128;  // the C = 128 form is an A/B variant (pair_cfg 30 / 31)
#else
  const bool c128 = false;
#endif
  if (!((C == 64 || c128) && (K == 7 || K == 11) && dil >= 1 && dil <= PAIR2_DMAX)) return VO_OK;
  Pair2Args a;
  a.x = (const bf16_t*)x; a.w1 = (const bf16_t*)w1; a.b1 = b1; a.w2 = (const bf16_t*)w2; a.b2 = b2;
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)acc;
  a.T = T; a.dil = dil; a.slope = slope; a.out_scale = out_scale;
  a.tiles_per_b = a.ntiles = 0;
  *handled = 1;
#ifdef VO_ABLATIONS
  if (C == 128) {  // 2 x 4 waves of 64 channels, 256-row tiles, whole taps by LDS-DMA
    if (K == 7) return pair2_launch<128, 2, 4, 4, 7, true, 1>(a, B, st);
    return pair2_launch<128, 2, 4, 4, 11, true, 1>(a, B, st);
  }
  // C = 64: 8 waves of 64 rows, 512-row tiles, 2-tap register-staged groups (cfg 31: LDS-DMA).
  // Measured and dropped: two 4-wave workgroups of 256-row tiles per CU (LDS-DMA weights): 4-8 %
  // faster alone (tools/ab_pair2.py), but s2 -3.6 % / s3 +4 % and the same 13.75 ms in the bench step
  // VALU diet (VD) at C = 64: k = 11 0.408 -> 0.398 ms, k = 7 0.311 -> 0.318 (tools/mrf_bench.py
  // --tune pair_cfg=33,0, round 3): k = 11 ships with it, k = 7 without; cfg 33 swaps both, for A/B
  if (cfg == 33) {  // (A/B variants of the C = 64 kernel: VO_ABLATIONS builds only)
    if (K == 7) return pair2_launch<64, 1, 8, 4, 7, false, 2, true>(a, B, st);
    return pair2_launch<64, 1, 8, 4, 11, false, 2, false>(a, B, st);
  }
  if (cfg == 34 || cfg == 35) {  // software-pipelined steps (PIPE): 34 = both phases, 35 = P1 only
    if (cfg == 34) {
      if (K == 7) return pair2_launch<64, 1, 8, 4, 7, false, 2, false, 3>(a, B, st);
      return pair2_launch<64, 1, 8, 4, 11, false, 2, true, 3>(a, B, st);
    }
    if (K == 7) return pair2_launch<64, 1, 8, 4, 7, false, 2, false, 1>(a, B, st);
    return pair2_launch<64, 1, 8, 4, 11, false, 2, true, 1>(a, B, st);
  }
  if (cfg == 31) {
    if (K == 7) return pair2_launch<64, 1, 8, 4, 7, true, 2>(a, B, st);
    return pair2_launch<64, 1, 8, 4, 11, true, 2>(a, B, st);
  }
  if (cfg == 32) {  // two 4-wave workgroups of 256-row tiles per CU, register-staged weights:
                    // 7-18 % slower (the doubled window registers per thread spill), round 2
    if (K == 7) return pair2_launch<64, 1, 4, 4, 7, false, 2>(a, B, st);
    return pair2_launch<64, 1, 4, 4, 11, false, 2>(a, B, st);
  }
#else
  (void)cfg;
#endif
  if (K == 7) return pair2_launch<64, 1, 8, 4, 7, false, 2, false>(a, B, st);
  return pair2_launch<64, 1, 8, 4, 11, false, 2, true>(a, B, st);
}
