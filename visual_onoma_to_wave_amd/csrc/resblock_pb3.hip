// HiFi-GAN ResBlock1 with kernel size 3 -- the whole block (three (c1_d, c2) iterations, dilations
// (1, 3, 5)) in one launch, in the "wave-owned output planes" form of resblock_rw.hip:
//   x1 = x  + c2_0(lrelu(c1_1(lrelu x )))        (x1, x2 rounded to bf16 as between per-pair launches)
//   x2 = x1 + c2_1(lrelu(c1_3(lrelu x1)))
//   y  = (x2 + c2_2(lrelu(c1_5(lrelu x2)))) * out_scale (+ acc)
// (scripts/hifigan/models.py:96-103; the MRF sum and 1/num_kernels scale of models.py:155-160 ride in the
// last epilogue).
//
// Why (round 6).  The LDS-tile block (resblock3.hip) shares every streamed weight tap between its waves
// through LDS: 0.37 (C = 128) / 0.27 (C = 64) of the dense bf16 peak, and 13 M LDS bank conflicts at
// C = 64.  Here, as in the k = 7 / 11 pair kernel that lifted stage 1 to 0.50:
//   * 4 waves, one per SIMD; wave w owns the 32 output channels of plane w % NP for 256 frame rows, in
//     all six convs of the block.  Its weights (32 co x C ci per tap) stream from L2 straight into its
//     registers one tap ahead -- no weight goes through LDS, no tap needs a barrier;
//   * the activations are shared through LDS: the lrelu'd window (lrelu x, then lrelu x1, lrelu x2 written
//     over it) and c1's output T1.  6 barriers per tile (one per conv);
//   * x1 / x2 never leave the chip: a wave's P2 accumulators ARE the x_{s+1} rows of its plane, kept as
//     bf16 in registers (the next P2's residual, entered by identity MFMAs: exact) and written lrelu'd
//     into the window for the next c1;
//   * every conv runs on the whole F-row frame; the valid rows shrink by the halos (1+1+3+1+5+1 = 12 per
//     side), so a tile yields F - 24 output rows (F = 256 at C = 128: 9 % extra MFMA work; F = 512 at C = 64);
//   * LDS rows [plane][row][32 ch], 16-byte chunk q of row r at q ^ ((r >> 1) & 3) (rw_off): the B-fragment
//     reads at any row shift, the T1 / window stores of the epilogues and the window staging (odd plane
//     stride) are bank-conflict free.
// Weights: [K][C_out][C_in] bf16 packs (vo_pack_weight) or the fragment order of vo_pack_frag (FR);
// biases fp32.

#include <algorithm>
#include <cmath>

#include "mrf_common.h"

#ifndef VO_PB3_PK
#define VO_PB3_PK 0  // epilogue leaky ReLU with one packed multiply per value pair (A/B)
#endif

namespace vo {

struct Pb3Args {
  const bf16_t* x;
  const bf16_t* w[6];  // conv v = 2 s + ph: c1 of stage s (ph 0), c2 of stage s (ph 1)
  const float* b[6];
  bf16_t* y; const bf16_t* acc;
  int T, dil[3], tiles_per_b, ntiles;
  float slope, out_scale;
  unsigned long long* stamps;  // diagnostic builds only (-DVO_PB3_STAMPS, tools/probes/pb3_stamps.py)
};
constexpr int PB_NSTW = 16, PB_NSTT = 4, PB_NPT = 30;  // stamp geometry: workgroups, tiles, stamps per tile

constexpr int PB_HP = 8;     // LDS pad rows per side (dilation <= 8; a multiple of 8 keeps the swizzle)
constexpr int PB_HALO = 12;  // valid rows lost per side: sum over the six convs of dil * (k - 1) / 2
constexpr int pb_np(int C) { return C / 32; }
// row tiles (16 rows) per wave (even: phase 1 runs blocks of two): the frame is 16 NJ rows per row group.
// C = 128: 14 (224-row frames, 200 output rows: 89.3 % of the MFMA work kept); C = 64: 16 (512-row frames, 488
// output rows, 95.3 %).  One more block (C = 128: 16) exceeds 512 registers, and the spill reloads' vmcnt(0)
// waits drain every prefetch in flight (measured 1.5x slower in an earlier layout)
#ifndef VO_PB3_NJ128
#define VO_PB3_NJ128 14
#endif
#ifndef VO_PB3_NJ64
#define VO_PB3_NJ64 16
#endif
constexpr int pb_nj(int C) { return C == 128 ? VO_PB3_NJ128 : VO_PB3_NJ64; }
constexpr int pb_f(int C) { return 16 * pb_nj(C) * (4 / pb_np(C)); }  // frame rows per tile
constexpr int pb_rp(int C) { return pb_f(C) + 2 * PB_HP + 1; }    // LDS rows per plane (odd)
constexpr size_t pb_lds(int C) { return (size_t)2 * pb_np(C) * pb_rp(C) * 32 * sizeof(bf16_t) + 6 * C * sizeof(float); }

__device__ __forceinline__ int pb_off(int r, int q) { return r * 32 + 8 * (q ^ ((r >> 1) & 3)); }

template <int C, int ACC, bool FR, bool ST = false>
__global__ void __launch_bounds__(256, 1) mrf_pb3_kernel(Pb3Args a) {
  constexpr int NP = pb_np(C), F = pb_f(C), NJ = pb_nj(C), RP = pb_rp(C), PL = RP * 32;
  constexpr int BT = F - 2 * PB_HALO;
  constexpr int VPR = C / 8, RPS = 256 / VPR, NWV = F / RPS;  // window: 16-byte vectors per row, rows per slot, slots
  constexpr int NAP = 2 * NP;                                  // A pieces (KiB) per tap and wave
  constexpr int NST = NJ * NP;                                 // (row tile, plane) steps per tap
  constexpr int NB = 10, DB = 8;                               // B-fragment ring / prefetch distance (steps)
  constexpr int NU = 18;                                       // taps per tile (6 convs x 3)
  constexpr int BS = 4 * NP;                                   // phase-1 block: 2 taps x NP planes x 2 row tiles
  static_assert(RPS % 8 == 0 && NWV * RPS == F && NJ % 2 == 0 && NST >= 4 * NAP, "geometry");

  const int T = a.T;
  const float slope = a.slope;

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* win = reinterpret_cast<bf16_t*>(smem_raw);       // [NP][RP][32]: lrelu x_s
  bf16_t* t1 = win + NP * PL;                               // [NP][RP][32]: c1's output
  float* sbias = reinterpret_cast<float*>(t1 + NP * PL);    // [6][C]

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pw = w % NP, row0 = (w / NP) * 16 * NJ;  // the wave's plane and first frame row
  const int lr = lane & 15, lg = lane >> 4;

  // ST (diagnostic builds): s_memtime at conv v's barrier (5v), its phase 0 (5v + 1), phase 1 (5v + 2), the middle
  // of phase 1 (5v + 3) and its end (5v + 4), first PB_NSTT tiles of workgroups 0 .. PB_NSTW-1, written by lane 0
  // of each wave (vector stores)
  int st_tile = 0;
  auto stamp = [&](int idx) __attribute__((always_inline)) {
    if constexpr (ST) {
      if (blockIdx.x < PB_NSTW && st_tile < PB_NSTT && lane == 0)
        a.stamps[((blockIdx.x * 4 + w) * PB_NSTT + st_tile) * PB_NPT + idx] = __builtin_amdgcn_s_memtime();
    }
  };

  const int G = gridDim.x;
  int tile = (int)(((int64_t)blockIdx.x * a.ntiles) / G);
  const int tile_end = (int)(((int64_t)(blockIdx.x + 1) * a.ntiles) / G);
  if (tile >= tile_end) return;  // uniform per workgroup

  for (int i = tid; i < 6 * C; i += 256) sbias[i] = a.b[i / C][i % C];
  // pad rows (read only by taps of frame rows whose outputs the halo discards): zeros, never NaN
  for (int i = tid; i < 2 * NP * (2 * PB_HP + 1) * 4; i += 256) {
    const int q = i & 3, r0 = (i >> 2) % (2 * PB_HP + 1), pb = (i >> 2) / (2 * PB_HP + 1);
    const int r = r0 < PB_HP ? r0 : F + r0;
    *reinterpret_cast<u32x4*>(win + pb * PL + pb_off(r, q)) = u32x4{0u, 0u, 0u, 0u};
  }

  // ---- A fragments (as resblock_rw.hip): lane l holds W[tap][co][ci], co = 32pw + 8(lr>>2) + 4t + (lr&3),
  // ci = 32s + 8lg .. +7; accumulator register i of co tile t is then channel 32pw + 8lg + 4t + i.
  // Three tap slots (tap u in slot u % 3; 18 taps per tile): a conv's taps 1 and 2 run interleaved (phase 1),
  // so both are resident while the next conv's tap 0 is fetched into the slot tap 0 freed
  const int aoff = ((32 * pw + 8 * (lr >> 2) + (lr & 3)) * C + 8 * lg) * (int)sizeof(bf16_t);
  const int afr = pw * NAP * 1024 + lane * 16;
  __amdgpu_buffer_rsrc_t rw[6];
#pragma unroll
  for (int v = 0; v < 6; ++v) rw[v] = __builtin_amdgcn_make_buffer_rsrc((void*)a.w[v], (short)0, 3 * C * C * 2, 0x00020000);
  bf16x8 A[3][NP][2];
  auto loadA_piece = [&](int u, int i) __attribute__((always_inline)) {
    const int uu = u % NU, v = uu / 3, k = uu % 3;
    const int s = i >> 1, t = i & 1;
    const int lo = FR ? afr + i * 1024 : aoff + t * 4 * C * 2 + s * 64;
    A[uu % 3][s][t] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw[v], lo, k * (C * C * 2), 0));
  };
  auto utt = [&](const bf16_t* p, int b) __attribute__((always_inline)) {  // one utterance of a (B, T, C) tensor: rows outside read 0
    return __builtin_amdgcn_make_buffer_rsrc((void*)(p + (int64_t)b * T * C), (short)0, T * C * 2, 0x00020000);
  };
  // op i of n spread over the steps [lo, lo + span) of a phase: does step jj carry it?
  auto at = [](int jj, int lo, int span, int n, int i) __attribute__((always_inline)) { return jj == lo + i * span / n; };

  // ---- window staging: vector v = tid + 256 slot = (frame row xr + RPS slot, 16-byte column xc)
  const int xr = tid / VPR, xc = tid % VPR;
  const int xl = (xc >> 2) * PL + pb_off(xr + PB_HP, xc & 3);  // + slot * RPS rows (swizzle unchanged)
  u32x4 xw[NWV];
  auto load_win = [&](int tl, int sl) __attribute__((always_inline)) {
    const int b = tl / a.tiles_per_b;
    const int p0 = (tl - b * a.tiles_per_b) * BT - PB_HALO;
    // positions before 0 wrap to huge offsets and past T exceed the range: both read 0 (zero padding)
    xw[sl] = __builtin_amdgcn_raw_buffer_load_b128(utt(a.x, b), ((p0 + xr + RPS * sl) * C + xc * 8) * 2, 0, 0);
  };
  auto store_win = [&](int sl) __attribute__((always_inline)) { *reinterpret_cast<u32x4*>(win + xl + sl * RPS * 32) = lrelu8(xw[sl], slope); };

#pragma unroll
  for (int i = 0; i < NAP; ++i) loadA_piece(0, i);
#pragma unroll
  for (int sl = 0; sl < NWV; ++sl) load_win(tile, sl);
#pragma unroll
  for (int sl = 0; sl < NWV; ++sl) store_win(sl);

  f32x4 acc[2][NJ];
  bf16x8 Bq[NB];
  u32x4 xres[NJ];  // the wave's residual rows (x from HBM for stage 0, then x1, x2 from its own epilogues)
  u32x4 ares[NJ];
  bf16x8 aid[2], ais[2];  // identity A fragments (co tile t); ais scaled by 1 / out_scale (ACC == 2)
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool one = (lr >> 2) == lg && e == 4 * t + (lr & 3);
      aid[t][e] = (__bf16)(one ? 1.0f : 0.0f);
      ais[t][e] = (__bf16)(one ? 1.0f / a.out_scale : 0.0f);
    }

  // One conv of the block over the frame, in two phases:
  //   phase 0: tap 0, plane-major over the NJ row tiles (NST steps);
  //   phase 1: taps 1 and 2 interleaved, in blocks of 2 row tiles (plane, tap, row tile inner: the two row
  //            tiles alternate, so no MFMA depends on the one just issued); a block's accumulators are final
  //            after its BS steps and its epilogue (8 parts) runs under the next block's MFMAs -- twice the MFMA
  //            time a last-tap-only epilogue had (the k = 3 block's six epilogues per tile were VALU-bound:
  //            0.50 MFMA busy, 2.5 VALU per MFMA).
  // Each step: one B-fragment read (DB steps ahead), two MFMAs, and the side work (A pieces: taps 1 / 2 in
  // phase 0, the next conv's tap 0 in phase 1; the hook).
  auto conv = [&](auto vc, auto hook, auto post, auto extra) __attribute__((always_inline)) {
    constexpr int V = decltype(vc)::value, PH = V & 1, S = V >> 1;
    const bf16_t* src = PH ? t1 : win;
    const int step = PH ? 1 : a.dil[S];
    int lro = lr, lgo = lg;
    asm volatile("" : "+v"(lro), "+v"(lgo));
    // step q of the conv (0 .. 3 NST) -> (tap, row tile, plane)
    auto dk = [&](int q) __attribute__((always_inline)) { return q < NST ? 0 : 1 + (((q - NST) % BS) / 2) % 2; };
    auto dj = [&](int q) __attribute__((always_inline)) { return q < NST ? q % NJ : 2 * ((q - NST) / BS) + (q - NST) % 2; };
    auto ds = [&](int q) __attribute__((always_inline)) { return q < NST ? q / NJ : ((q - NST) % BS) / 4; };
    auto readB = [&](int q) __attribute__((always_inline)) {
      const int k = dk(q), j = dj(q), s = ds(q);
      const bf16_t* base = src + (s >> 1) * 2 * PL + pb_off(PB_HP + (k - 1) * step + row0 + lro, lgo);
      Bq[q % NB] = *reinterpret_cast<const bf16x8*>(base + (s & 1) * PL + j * 512);
    };
    const f32x4* bz = reinterpret_cast<const f32x4*>(sbias + V * C + 32 * pw + 8 * lg);
    const f32x4 bz0 = bz[0], bz1 = bz[1];
#pragma unroll
    for (int q = 0; q < DB; ++q) readB(q);
    auto phase = [&](auto phc) __attribute__((always_inline)) {
      constexpr int ph = decltype(phc)::value, n = ph ? 2 * NST : NST;
      stamp(5 * V + 1 + ph);
#pragma unroll
      for (int jj = 0; jj < n; ++jj) {
        const int q = ph * NST + jj;
        const int k = dk(q), j = dj(q), s = ds(q);
        if (ST && ph == 1 && jj == NST) stamp(5 * V + 3);
        if (q + DB < 3 * NST) readB(q + DB);
        if (jj % 2 == 0) {
          if (ph == 0 && jj < 4 * NAP) loadA_piece(3 * V + 1 + jj / (2 * NAP), (jj / 2) % NAP);
          if (ph == 1 && jj < 2 * NAP) loadA_piece(3 * V + 3, jj / 2);
        }
        hook(ph, jj);
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8 b = Bq[q % NB];
        const bf16x8(&Ak)[NP][2] = A[(3 * V + k) % 3];
        if (k == 0 && s == 0) {
          acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ak[s][0], b, bz0, 0, 0, 0);
          acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ak[s][1], b, bz1, 0, 0, 0);
        } else {
          acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ak[s][0], b, acc[0][j], 0, 0, 0);
          acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ak[s][1], b, acc[1][j], 0, 0, 0);
        }
        extra(k, j, s);
        if (ph == 1 && jj >= BS) {  // the previous block's epilogue: 8 parts over this block's BS steps
          const int bb = jj / BS - 1, r = jj % BS;
#pragma unroll
          for (int p = 0; p < 8; ++p)
            if (r == p * BS / 8) post(2 * bb + p / 4, p % 4);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    phase(std::integral_constant<int, 0>{});
    phase(std::integral_constant<int, 1>{});
#pragma unroll
    for (int p = 0; p < 8; ++p) post(NJ - 2 + p / 4, p % 4);
    stamp(5 * V + 4);
  };

  const int cofs = 32 * pw + 8 * lg;
  for (; tile < tile_end; ++tile) {
    const int b = tile / a.tiles_per_b;
    const int t0 = (tile - b * a.tiles_per_b) * BT;
    const int p0 = t0 - PB_HALO;  // position of frame row 0
    const int ntile = tile + 1 < tile_end ? tile + 1 : tile;
    // Zero padding: the epilogues write every frame row unmasked (a mask per row tile cost 5 of its ~38 vector
    // instructions, in the VALU-bound epilogue phase; a branch around it made hipcc copy eight accumulators out
    // of the AGPRs at every join); in the tiles whose frame crosses an utterance end, the rows outside [0, T) of
    // the wave's own plane are zeroed after the epilogue, before the barrier that publishes them
    const bool edge = p0 < 0 || p0 + F > T;
    const int zlo = p0 < 0 ? -p0 : 0, zhi = T - p0;  // frame rows [zlo, zhi) are inside the utterance
    auto zero_rows = [&](bf16_t* buf) __attribute__((always_inline)) {
      if (!edge) return;
      for (int f = row0 + lane; f < row0 + 16 * NJ; f += 64)
        if (f < zlo || f >= zhi)
#pragma unroll
          for (int q = 0; q < 4; ++q) *reinterpret_cast<u32x4*>(buf + pw * PL + pb_off(f + PB_HP, q)) = u32x4{0u, 0u, 0u, 0u};
    };
    const __amdgpu_buffer_rsrc_t rsx = utt(a.x, b);
    const __amdgpu_buffer_rsrc_t rsa = utt(ACC ? a.acc : a.x, b);

    stamp(0);
    lds_barrier();  // window staged; the previous tile's T1 reads are done

    uint32_t pv[4];
    // P1 epilogue: T1 = lrelu(acc) (bias in acc), frame rows outside [0, T) = 0 (c2's zero padding)
    auto p1_post = [&](int j, int p) __attribute__((always_inline)) {
      const int t = p >> 1, e = 2 * (p & 1);
#if VO_PB3_PK
      pv[p] = lrelu_pk(acc[t][j][e], acc[t][j][e + 1], slope);
#else
      pv[p] = pk_bf16(lrelu_max(acc[t][j][e], slope), lrelu_max(acc[t][j][e + 1], slope));
#endif
      if (p == 3) {
        const int f = row0 + 16 * j + lr;
        *reinterpret_cast<u32x4*>(t1 + pw * PL + pb_off(f + PB_HP, lg)) = u32x4{pv[0], pv[1], pv[2], pv[3]};
      }
    };
    // P2 epilogue of stages 0 / 1: x_{s+1} = bf16(acc) kept in xres; lrelu(x_{s+1}) into the window (rows
    // outside [0, T) = 0: the next c1's zero padding).  The lrelu'd copy is taken from the fp32 sum (one
    // multiply and max per value, no unpacking of the rounded bf16 -- as resblock3.hip's epilogues)
    uint32_t lv[4];
    auto p2_mid_post = [&](int j, int p) __attribute__((always_inline)) {
      const int e = 2 * p;
      const float a0 = acc[e >> 2][j][e & 3], a1 = acc[e >> 2][j][(e & 3) + 1];
      pv[p] = pk_bf16(a0, a1);
#if VO_PB3_PK
      lv[p] = lrelu_pk(a0, a1, slope);
#else
      lv[p] = pk_bf16(lrelu_max(a0, slope), lrelu_max(a1, slope));
#endif
      if (p == 3) {
        const int f = row0 + 16 * j + lr;
        xres[j] = u32x4{pv[0], pv[1], pv[2], pv[3]};
        *reinterpret_cast<u32x4*>(win + pw * PL + pb_off(f + PB_HP, lg)) = u32x4{lv[0], lv[1], lv[2], lv[3]};
      }
    };
    // the residual (and acc_in / out_scale) through identity MFMAs at plane 0's step of row tile j:
    // the lane's residual vector of row tile j IS a B fragment of its own plane
    auto res_extra = [&](int k, int j, int s) __attribute__((always_inline)) {
      if (s != 0 || k != 0) return;
#pragma unroll
      for (int t = 0; t < 2; ++t)
        acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aid[t], __builtin_bit_cast(bf16x8, xres[j]), acc[t][j], 0, 0, 0);
    };
    auto no_hook = [&](int, int) __attribute__((always_inline)) {};
    auto no_extra = [&](int, int, int) __attribute__((always_inline)) {};

    // ---- stage 0, c1 (dilation dil[0]) over lrelu x; x's rows of this wave's plane requested in phase 1 (L2
    // hits: the window staging just read them), the residual of stage 0's c2
    auto s0_hook = [&](int ph, int jj) __attribute__((always_inline)) {
      if (ph != 1 || jj < 2 * NAP) return;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        if (at(jj, 2 * NAP, 2 * NST - 2 * NAP, NJ, j))
          xres[j] = __builtin_amdgcn_raw_buffer_load_b128(rsx, ((p0 + row0 + 16 * j + lr) * C + cofs) * 2, 0, 0);
    };
    conv(std::integral_constant<int, 0>{}, s0_hook, p1_post, no_extra);
    zero_rows(t1);
    stamp(5);
    lds_barrier();
    conv(std::integral_constant<int, 1>{}, no_hook, p2_mid_post, res_extra);
    zero_rows(win);
    stamp(10);
    lds_barrier();
    conv(std::integral_constant<int, 2>{}, no_hook, p1_post, no_extra);
    zero_rows(t1);
    stamp(15);
    lds_barrier();
    conv(std::integral_constant<int, 3>{}, no_hook, p2_mid_post, res_extra);
    zero_rows(win);
    stamp(20);
    lds_barrier();

    // ---- stage 2: c1 loads the next tile's window into registers (phase 1, after the A pieces: vmcnt retires in
    // issue order, so a load issued before an A piece would hold up the next phase's first MFMAs)
    auto s2a_hook = [&](int ph, int jj) __attribute__((always_inline)) {
      if (ph != 1 || jj < 2 * NAP) return;
#pragma unroll
      for (int sl = 0; sl < NWV; ++sl)
        if (at(jj, 2 * NAP, 2 * NST - 2 * NAP, NWV, sl)) load_win(ntile, sl);
    };
    conv(std::integral_constant<int, 4>{}, s2a_hook, p1_post, no_extra);
    zero_rows(t1);
    stamp(25);
    lds_barrier();  // T1 complete; the window is dead until the next tile

    // ---- stage 2, c2: y = (x2 + c2) * out_scale (+ acc) -> HBM.  Phase 0, after its A pieces: the next window
    // written lrelu'd, and the MRF accumulator rows requested (x2's registers are free after the residual
    // MFMAs of plane 0); they enter in phase 1 (identity MFMA, ACC == 2) or the epilogue (ACC == 1)
    const int valid = min(BT, T - t0);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.y + ((int64_t)b * T + t0) * C), (short)0, valid * C * (int)sizeof(bf16_t), 0x00020000);
    auto s2b_hook = [&](int ph, int jj) __attribute__((always_inline)) {
      if (ph != 0 || jj < 4 * NAP) return;
#pragma unroll
      for (int sl = 0; sl < NWV; ++sl)
        if (at(jj, 4 * NAP, NST - 4 * NAP, NWV, sl)) store_win(sl);
      if constexpr (ACC != 0) {
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          if (at(jj, 4 * NAP, NST - 4 * NAP, NJ, j))
            ares[j] = __builtin_amdgcn_raw_buffer_load_b128(rsa, ((p0 + row0 + 16 * j + lr) * C + cofs) * 2, 0, 0);
      }
    };
    auto s2b_extra = [&](int k, int j, int s) __attribute__((always_inline)) {
      if (s != 0) return;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (k == 0)
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aid[t], __builtin_bit_cast(bf16x8, xres[j]), acc[t][j], 0, 0, 0);
        if constexpr (ACC == 2)
          if (k == 2)
            acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ais[t], __builtin_bit_cast(bf16x8, ares[j]), acc[t][j], 0, 0, 0);
      }
    };
    const float osc = a.out_scale;
    auto s2b_post = [&](int j, int p) __attribute__((always_inline)) {
      float q[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int e = 2 * p + u;
        q[u] = acc[e >> 2][j][e & 3] * osc;
        if constexpr (ACC == 1) {
          const uint32_t aw2 = ares[j][p];
          q[u] += __uint_as_float(u ? (aw2 & 0xffff0000u) : (aw2 << 16));
        }
      }
      pv[p] = pk_bf16(q[0], q[1]);
      if (p == 3)  // frame rows before the halo wrap to huge offsets, rows past `valid` exceed the range
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{pv[0], pv[1], pv[2], pv[3]}, yrs,
                                               ((row0 + 16 * j + lr - PB_HALO) * C + cofs) * (int)sizeof(bf16_t), 0, 0);
    };
    conv(std::integral_constant<int, 5>{}, s2b_hook, s2b_post, s2b_extra);
    ++st_tile;
  }
}

template <int C, int ACC, bool FR>
static int pb3_launch(Pb3Args a, int B, hipStream_t st) {
  constexpr int BT = pb_f(C) - 2 * PB_HALO;
  a.tiles_per_b = (a.T + BT - 1) / BT;
  a.ntiles = a.tiles_per_b * B;
  auto kern = mrf_pb3_kernel<C, ACC, FR>;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  const int grid = (int)std::min<int64_t>((int64_t)cus, a.ntiles);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), pb_lds(C), st, a);
  VO_RETURN_LAUNCH();
}

}  // namespace vo

using namespace vo;

// Entry from vo_resblock3 / vo_resblock3_frag: *handled = 1 when this kernel covers the shape (C = 64 / 128,
// every dilation <= 8 and their halo sum <= 12).
int vo_rb3_pb_try(const void* x, const void* const* w1, const float* const* b1, const void* const* w2,
                  const float* const* b2, const int* dil, void* y, const void* acc, int B, int T, int C, float slope,
                  float out_scale, hipStream_t st, int* handled, int frag) {
  *handled = 0;
  if (!(C == 64 || C == 128)) return VO_OK;
  int halo = 0;
  for (int s = 0; s < 3; ++s) {
    if (dil[s] < 1 || dil[s] > PB_HP) return VO_OK;
    halo += dil[s] + 1;
  }
  if (halo > PB_HALO) return VO_OK;
  Pb3Args a;
  a.x = (const bf16_t*)x;
  for (int s = 0; s < 3; ++s) {
    a.w[2 * s] = (const bf16_t*)w1[s]; a.b[2 * s] = b1[s];
    a.w[2 * s + 1] = (const bf16_t*)w2[s]; a.b[2 * s + 1] = b2[s];
    a.dil[s] = dil[s];
  }
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)acc;
  a.T = T; a.slope = slope; a.out_scale = out_scale;
  a.tiles_per_b = a.ntiles = 0;
  a.stamps = nullptr;
  *handled = 1;
  int accm = 0;
  if (acc) {  // acc_in / out_scale through the identity MFMA when 1 / out_scale is a bf16 value (3)
    const float inv = 1.0f / out_scale;
    const float invb = __bfloat162float(__float2bfloat16(inv));
    accm = (invb == inv && std::isfinite(inv) && inv * out_scale == 1.0f) ? 2 : 1;
  }
#define VO_PB3_DISPATCH(CC, FF) \
  return accm == 2 ? pb3_launch<CC, 2, FF>(a, B, st) : accm == 1 ? pb3_launch<CC, 1, FF>(a, B, st) \
                                                   : pb3_launch<CC, 0, FF>(a, B, st)
  if (C == 64) {
    if (frag) VO_PB3_DISPATCH(64, true);
    VO_PB3_DISPATCH(64, false);
  }
  if (frag) VO_PB3_DISPATCH(128, true);
  VO_PB3_DISPATCH(128, false);
#undef VO_PB3_DISPATCH
}

#ifdef VO_PB3_STAMPS
// Diagnostic entry (tools/probes/pb3_stamps.py builds its own library with -DVO_PB3_STAMPS): one stamped launch
// of the k = 3 block (dilations 1 / 3 / 5, MRF accumulator on, out_scale 1/3, [K][Co][Ci] weights) at C = 64 / 128;
// host_out receives PB_NSTW x 4 waves x PB_NSTT tiles x PB_NPT stamps.
extern "C" int vo_pb3_stamps(const void* x, const void* const* w1, const float* const* b1, const void* const* w2,
                             const float* const* b2, void* y, int B, int T, int C, unsigned long long* host_out) {
  const size_t n = (size_t)PB_NSTW * 4 * PB_NSTT * PB_NPT;
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, n * 8) != hipSuccess) return -1;
  (void)hipMemset(d, 0, n * 8);
  Pb3Args a;
  a.x = (const bf16_t*)x;
  for (int s = 0; s < 3; ++s) {
    a.w[2 * s] = (const bf16_t*)w1[s]; a.b[2 * s] = b1[s];
    a.w[2 * s + 1] = (const bf16_t*)w2[s]; a.b[2 * s + 1] = b2[s];
    a.dil[s] = 2 * s + 1;
  }
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)y;
  a.T = T; a.slope = 0.1f; a.out_scale = 1.f / 3; a.stamps = d;
  const int BT = pb_f(C) - 2 * PB_HALO;
  a.tiles_per_b = (T + BT - 1) / BT;
  a.ntiles = a.tiles_per_b * B;
  const int grid = std::min(256, a.ntiles);
  if (C == 64)
    hipLaunchKernelGGL((mrf_pb3_kernel<64, 2, false, true>), dim3(grid), dim3(256), pb_lds(64), 0, a);
  else
    hipLaunchKernelGGL((mrf_pb3_kernel<128, 2, false, true>), dim3(grid), dim3(256), pb_lds(128), 0, a);
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(host_out, d, n * 8, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  return 0;
}
#endif
