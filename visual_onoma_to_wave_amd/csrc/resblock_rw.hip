// HiFi-GAN ResBlock1 pair at C = 128 (MRF stage 1), k = 7 / 11 -- "wave-owned output planes":
//   y = (x + c2(lrelu(c1_d(lrelu(x), slope), slope))) * out_scale (+ acc)
// (scripts/hifigan/models.py:96-103, one (c1, c2) iteration; the MRF sum and 1/num_kernels scale of
// models.py:155-160 ride in the epilogue).
//
// Why a new kernel (round 5).  The LDS-tile pair (resblock.hip) shares every streamed weight tap
// between its 8 waves through LDS, so each of the 2K taps per tile ends in a workgroup barrier; with
// two waves per SIMD the younger one finishes each tap a tail later (oldest-first arbitration) and
// every wave waits for it -- 0.43 of the dense bf16 peak for three rounds.  Here the workgroup is 4
// waves, one per SIMD, and wave w owns the 32 output channels of plane w for ALL 256 rows of the tile:
//   * its weights (32 co x 128 ci per tap = 8 KiB) go straight from L2 into its own registers, two
//     taps ahead (a 3-slot ring) -- no wave reads another wave's weights, so no tap needs a barrier;
//   * the activations it multiplies them with (the lrelu'd input window in P1, c1's output T1 in P2)
//     are shared through LDS, and only those hand-offs synchronise: 2 barriers per tile, not 2K + 2;
//   * v_mfma_f32_16x16x32_bf16, 2 co tiles x 16 row tiles per wave: per MFMA 0.5 ds_read_b128 of B
//     (128 B/clk per CU, half the LDS array) and 1/16 of a global load of A;
//   * the next tile's window is fetched during P2 (the window is dead once P1 ends; T1 has its own
//     buffer) and written, lrelu'd, two taps after its loads were issued;
//   * LDS layout [plane][row][32 ch] with 16-byte chunk q of row r at q ^ ((r >> 1) & 3): the B-fragment
//     reads (16 rows x 4 chunks at ANY row offset -- the taps shift rows by k*dil), the T1 stores and
//     the window stores (plane stride of 321 rows: odd) are all bank-conflict free (checked exhaustively
//     over the lane groups of ds_read_b128 / ds_write_b128, MI355X_MICROARCH.md section LDS);
//   * output channels permuted in the A rows so that a lane's two accumulators of one row tile are the
//     8 consecutive channels 32w + 8(l>>4) .. +7 of row (l & 15): one 16-byte T1 store / y store per row
//     tile, in the layout the next conv's B fragments read.
// Weights: the ordinary [K][C_out][C_in] bf16 pack (vo_pack_weight); bias fp32.

#include <algorithm>
#include <cmath>
#include <type_traits>

#include "mrf_common.h"

namespace vo {

struct PrwArgs {
  const bf16_t* x; const bf16_t* w1; const float* b1; const bf16_t* w2; const float* b2;
  bf16_t* y; const bf16_t* acc;
  int T, dil, tiles_per_b, ntiles;
  float slope, out_scale;
  unsigned long long* stamps;  // diagnostic builds only (-DVO_PRW_STAMPS, tools/probes/prw_stamps.py)
};

// Geometry by channel count C (32, 64 or 128): NP = C / 32 planes; the 4 waves are NP output planes x RG = 4 / NP
// row groups of 256 rows, so a tile is R1 = 256 RG c1 rows and every wave owns 32 channels x 256 rows.
constexpr int rw_np(int C) { return C / 32; }
constexpr int rw_r1(int C) { return 256 * (4 / rw_np(C)); }
constexpr int rw_wp(int C) { return rw_r1(C) + 64 + 1; }  // window rows per plane: halo <= 64 (odd: conflict-free stores)
constexpr int rw_tp(int C) { return rw_r1(C) + 16; }      // T1 rows per plane: P2 reads up to row R1 + K - 2
constexpr size_t rw_lds(int C) {
  return (size_t)rw_np(C) * (rw_wp(C) + rw_tp(C)) * 32 * sizeof(bf16_t) + 2 * C * sizeof(float);
}
constexpr int RW_NSTW = 16, RW_NSTT = 4, RW_NPT = 2 * 11 + 6;  // stamp geometry (diagnostic builds)

__device__ __forceinline__ int rw_off(int r, int q) { return r * 32 + 8 * (q ^ ((r >> 1) & 3)); }

template <int C, int K, int ACC, bool FR = false, bool ST = false>
__global__ void __launch_bounds__(256, 1) mrf_prw_kernel(PrwArgs a) {
  constexpr int NP = rw_np(C), R1 = rw_r1(C), NJ = 16;  // planes, c1 rows per tile, row tiles per wave
  constexpr int WP = rw_wp(C), TP = rw_tp(C);
  constexpr int H2 = (K - 1) / 2, BT = R1 - 2 * H2;
  constexpr int VPR = C / 8, RPS = 256 / VPR;  // 16-byte vectors per row, rows per staging slot
  constexpr int NWV = (R1 + 64) * VPR / 256;  // window vectors (16 B) per thread
  constexpr int SPT = (NWV + K - 3) / (K - 2);  // window slots loaded per P2 tap (taps 0 .. K-3)
  constexpr int NAP = 2 * NP;                 // A pieces (KiB) per tap and wave
  constexpr int RD = 12 * NP;                 // MRF-accumulator prefetch distance (steps)
  constexpr int NST = NJ * NP;                // (row tile, plane) steps per tap
  constexpr int SP2 = (NST - 2 * NAP) / SPT;  // P2 staging: steps between a tap's window slots
#ifndef VO_PRW_LG
#define VO_PRW_LG 1
#endif
  constexpr int LG = VO_PRW_LG;               // last tap: row tiles per block (see conv)
#ifndef VO_PRW_XT
#define VO_PRW_XT 0
#endif
  constexpr int XT = K > 2 ? VO_PRW_XT : 0;   // P2 tap whose first plane also adds the residual (see p2_extra)
#ifndef VO_PRW_AP2
#define VO_PRW_AP2 1
#endif
  // ACC == 2: the MRF accumulator rows (HBM misses, unlike the residual rows the window staging just
  // brought into L2) requested over P2 taps 0 .. ANT - 1 and added at tap XA (AP2).  Requested with the
  // residual in P1's last two taps, the in-order vmcnt drained them at the next tap's weight wait:
  // those two taps ran 3,996 + 6,240 cycles for 2 x 1,168 (stamps, C = 64 k = 11); in P2 over four taps
  // a tile takes 38.4k cycles against 42.8k (C = 64 k = 11), 61.6k against 64.5k (C = 128 k = 11)
  constexpr bool AP2 = VO_PRW_AP2 != 0 && ACC == 2;
#ifndef VO_PRW_ANT
#define VO_PRW_ANT 4
#endif
  constexpr int ANT = VO_PRW_ANT, ARPT = NJ / ANT;  // taps carrying the requests, row tiles per tap
  constexpr int XA = AP2 ? (ANT + 1 < K - 1 ? ANT + 1 : K - 1) : XT;
  // (XT = 1 moved the identity MFMAs' cost to tap 1 unchanged: it is their issue, not a dependency stall)
  constexpr int NB = 10, DB = 8;              // B-fragment ring / prefetch distance (steps); 12 / 14 measured no faster
  // ACC: 0 = no MRF accumulator; 1 = y = acc_out * out_scale + acc_in (epilogue add); 2 = acc_in / out_scale
  // enters the accumulators through an identity MFMA (1 / out_scale exact in bf16, e.g. 3)
  static_assert(SPT * (K - 2) >= NWV && SP2 >= 2 && RPS % 8 == 0, "window staging");
  static_assert(NJ % LG == 0 && (4 * LG) % (LG * NP) == 0, "last-tap blocks");

  const int T = a.T, dil = a.dil;
  const int h1 = dil * H2;
  const float slope = a.slope;

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* win = reinterpret_cast<bf16_t*>(smem_raw);  // [NP][WP][32]
  bf16_t* t1 = win + NP * WP * 32;                     // [NP][TP][32]
  float* sbias = reinterpret_cast<float*>(t1 + NP * TP * 32);  // [b1 | b2]

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pw = w % NP, row0 = (w / NP) * 256;  // the wave's output plane and first row of the tile
  const int lr = lane & 15, lg = lane >> 4;
  // ST (diagnostic builds): s_memtime at fixed points of the first RW_NSTT tiles of workgroups
  // 0 .. RW_NSTW-1, written by lane 0 of each wave to a buffer nothing else reads
  int st_tile = 0;
  auto stamp = [&](int idx) {
    if constexpr (ST) {
      if (blockIdx.x < RW_NSTW && st_tile < RW_NSTT && lane == 0)
        a.stamps[((blockIdx.x * 4 + w) * RW_NSTT + st_tile) * RW_NPT + idx] = __builtin_amdgcn_s_memtime();
    }
  };

  // contiguous tile run of this workgroup (uniform per workgroup: the early exit is safe)
  const int G = gridDim.x;
  int tile = (int)(((int64_t)blockIdx.x * a.ntiles) / G);
  const int tile_end = (int)(((int64_t)(blockIdx.x + 1) * a.ntiles) / G);
  if (tile >= tile_end) return;

  for (int i = tid; i < 2 * C; i += 256) sbias[i] = i < C ? a.b1[i] : a.b2[i - C];

  // ---- A fragments: lane l holds W[tap][co][ci] for co = 32pw + 8(lr>>2) + 4t + (lr&3) (co tile t:
  // accumulator register i of lane l is then channel 32pw + 8lg + 4t + i) and ci = 32s + 8lg .. +7
  // loads through buffer resources: 32-bit lane offsets (a 64-bit address per load kept 2 VGPRs live
  // each and spilled), rows outside an utterance read as 0 (the convs' zero padding) with no clamp
  const int aoff = ((32 * pw + 8 * (lr >> 2) + (lr & 3)) * C + 8 * lg) * (int)sizeof(bf16_t);
  const int afr = pw * NAP * 1024 + lane * 16;  // FR: [tap][pw][s][t][lane][8]
  const __amdgpu_buffer_rsrc_t rw1 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w1, (short)0, K * C * C * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw2 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w2, (short)0, K * C * C * 2, 0x00020000);
  // 2-slot ring: tap u's fragments in slot u % 2; tap u + 1's are requested over the first 2 NAP steps of
  // tap u (2K is even, so a tile's last tap prefetches the next tile's first into slot 0)
  bf16x8 A[2][NP][2];
  auto loadA_piece = [&](int u, int i) {  // u: tap in the tile's 2K-tap sequence (mod 2K); i = 2s + t
    const int uu = u % (2 * K);
    const int tap_off = (uu < K ? uu : uu - K) * (C * C * 2);
    const int s = i >> 1, t = i & 1;
    // FR: fragment-ordered pack (vo_pack_frag): each piece one contiguous KiB -- the [K][Co][Ci] pack's
    // pieces touch 16 rows of 64 B each, and their occasional stalls held up whole waves (7 % per tile)
    const int lo = FR ? afr + i * 1024 : aoff + t * 4 * C * 2 + s * 64;
    A[uu & 1][s][t] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(uu < K ? rw1 : rw2,
                                             lo, tap_off, 0));
  };
  auto utt = [&](const bf16_t* p, int b) {  // one utterance of a (B, T, C) tensor
    return __builtin_amdgcn_make_buffer_rsrc((void*)(p + (int64_t)b * T * C), (short)0, T * C * 2, 0x00020000);
  };

  // ---- window staging: vector v = tid + 256 * slot = (row xr + RPS slot, 16-byte column xc)
  const int xr = tid / VPR, xc = tid % VPR;
  const int xl = (xc >> 2) * WP * 32 + rw_off(xr, xc & 3);  // + slot * RPS rows (swizzle unchanged)
  u32x4 xw[NWV];
  // window rows c1 reads: R1 + (K - 1) dil of the R1 + 64 staged (the rest are never read: their loads
  // are sent out of the buffer's range, which returns 0 without touching memory -- at d = 1 they were
  // 17 % of the window's HBM reads)
  const int wneed = R1 + (K - 1) * a.dil;
  auto load_win1 = [&](int tl, int sl) {
    const int b = tl / a.tiles_per_b;
    const int R0 = (tl - b * a.tiles_per_b) * BT - H2 - h1;
    // rows before 0 / past T are out of the utterance's range and read 0 (the conv's zero padding)
    const int off = xr + RPS * sl < wneed ? ((R0 + xr + RPS * sl) * C + xc * 8) * 2 : 0x7ffffff0;
    xw[sl] = __builtin_amdgcn_raw_buffer_load_b128(utt(a.x, b), off, 0, 0);
  };
  auto store_win1 = [&](int sl) { *reinterpret_cast<u32x4*>(win + xl + sl * RPS * 32) = lrelu8(xw[sl], slope); };

#pragma unroll
  for (int i = 0; i < NAP; ++i) loadA_piece(0, i);
#pragma unroll
  for (int sl = 0; sl < NWV; ++sl) load_win1(tile, sl);
#pragma unroll
  for (int sl = 0; sl < NWV; ++sl) store_win1(sl);

  f32x4 acc[2][NJ];
  bf16x8 Bq[NB];
  // identity A fragments (co tile t): lane (m = lr, lg) holds 1 at k = 4t + (m & 3) of its 8 when m / 4 == lg
  bf16x8 aid[2], ais[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool one = (lr >> 2) == lg && e == 4 * t + (lr & 3);
      aid[t][e] = (__bf16)(one ? 1.0f : 0.0f);
      ais[t][e] = (__bf16)(one ? 1.0f / a.out_scale : 0.0f);  // ACC == 2: exact by the launcher's check
    }

  // One conv over the tile: K taps x 4 input planes x 16 row tiles, steps j-major inside a tap.  PH = 0:
  // c1 over the window (row step dil, taps u = k); PH = 1: c2 over T1 (row step 1, taps u = K + k).
  // Every step is one B-fragment read (DB steps ahead) and two MFMAs; the other work is spread one piece
  // per step, so that it issues in the MFMAs' free issue cycles instead of stalling the matrix pipe:
  // the next tap's A fragments (steps 0, 2, .., 14), hook(k, jj) (window staging, residual loads), and
  // in the last tap the epilogue of row tile j in four parts during row tile j + 1's four steps (its
  // accumulators are final after its own four steps).
  auto conv = [&](auto ph, auto hook, auto post, auto cinit, auto extra) {
    constexpr int PH = decltype(ph)::value;
    const bf16_t* src = PH ? t1 : win;
    constexpr int PL = (PH ? TP : WP) * 32;  // plane stride (elements)
    const int step = PH ? 1 : dil;
    // the lane's row / chunk, opaque per tile: the per-tap B addresses are recomputed where they are
    // used (hoisted out of the tile loop, 2 x 2K of them were live throughout and spilled)
    int lro = lr, lgo = lg;
    asm volatile("" : "+v"(lro), "+v"(lgo));
    // step jj of tap k -> (row tile, plane): plane-major (16 row tiles, then the next plane: no two MFMAs
    // of a row tile back to back -- j-major ran c1's taps 9 % slower, 2,480 vs 2,260 cycles), except in
    // the last tap, which runs blocks of LG row tiles, plane-major inside the block, so that a block's
    // accumulators are final after its LG NP steps and its epilogue runs under the next block's MFMAs.
    // LG = 1 (j-major) measured best: the last tap's excess (4,100 cycles for 1,024 of MFMAs at C = 64)
    // is the epilogue's vector issue, not MFMA dependencies -- LG = 2 / 4 ran tiles 2 % slower
    auto rt = [&](int k, int jj) { return k < K - 1 ? jj % NJ : (jj / (LG * NP)) * LG + jj % LG; };
    auto pl = [&](int k, int jj) { return k < K - 1 ? jj / NJ : (jj % (LG * NP)) / LG; };
    auto readB = [&](int q) {  // q: step index over the conv (tap q / NST, row tile, plane)
      const int k = q / NST, j = rt(k, q % NST), s = pl(k, q % NST);
      // planes 0-1 and 2-3 from two bases: the ds_read offset field holds 16 bits
      const bf16_t* base = src + (s >> 1) * 2 * PL + rw_off(k * step + row0 + lro, lgo);
      Bq[q % NB] = *reinterpret_cast<const bf16x8*>(base + (s & 1) * PL + j * 512);
    };
#pragma unroll
    for (int q = 0; q < DB; ++q) readB(q);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int u = PH * K + k;
      stamp(2 + PH * (K + 2) + k);
      const bf16x8(&Ak)[NP][2] = A[u & 1];
#pragma unroll
      for (int jj = 0; jj < NST; ++jj) {
        const int q = k * NST + jj;
        const int j = rt(k, jj), s = pl(k, jj);
        if (q + DB < K * NST) readB(q + DB);
        if (jj < 2 * NAP && jj % 2 == 0) loadA_piece(u + 1, jj / 2);
        hook(k, jj);
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8 b = Bq[q % NB];
        if (k == 0 && s == 0) {
          acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ak[s][0], b, cinit(j, 0), 0, 0, 0);
          acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ak[s][1], b, cinit(j, 1), 0, 0, 0);
        } else {
          acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ak[s][0], b, acc[0][j], 0, 0, 0);
          acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ak[s][1], b, acc[1][j], 0, 0, 0);
        }
        extra(k, j, s);
        if (k == K - 1 && jj >= LG * NP) {  // the previous block's epilogue: 4 / NP of its 4 LG parts per step
          const int r = jj % (LG * NP), j0 = (jj / (LG * NP) - 1) * LG;
#pragma unroll
          for (int q = r * 4 / NP; q < (r + 1) * 4 / NP; ++q) post(j0 + q / 4, q % 4);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int q = 0; q < 4 * LG; ++q) post(NJ - LG + q / 4, q % 4);
  };

  for (; tile < tile_end; ++tile) {
    const int b = tile / a.tiles_per_b;
    const int t0 = (tile - b * a.tiles_per_b) * BT;
    const int ntile = tile + 1 < tile_end ? tile + 1 : tile;  // next window (unconditional loads)

    stamp(0);
    lds_barrier();  // window staged; the previous P2's T1 reads are done
    stamp(1);

    // ---- P1: T1 = lrelu(c1(window) + b1), rows outside [0, T) = 0 (c2's zero padding).  During its last
    // two taps this tile's residual rows x are requested in the accumulator layout: they enter P2 as the
    // C operand of its first MFMAs (acc = b2 + x + c2), a whole tap and the B1 barrier after the request
    const bool interior = t0 - H2 >= 0 && t0 - H2 + R1 <= T;
    const int cofs = 32 * pw + 8 * lg;
    const __amdgpu_buffer_rsrc_t rsx = utt(a.x, b);
    u32x4 xres[NJ], ares[NJ];
    const __amdgpu_buffer_rsrc_t rsa = utt(ACC ? a.acc : a.x, b);
    // requested after each tap's A pieces (steps 16, 22, .., 58 of taps K-2 and K-1): vmcnt retires in
    // issue order, so a residual load issued before an A piece would hold up the MFMAs that wait for it
    // (spread over the last K-2 taps, a few row tiles each, they measured slower: 2.5 % per tile)
#ifndef VO_PRW_NRT
#define VO_PRW_NRT 2
#endif
    constexpr int NRT = VO_PRW_NRT, RPT = NJ / NRT, RT0 = K - NRT, RSP = (NST - 2 * NAP) / RPT;
    auto p1_hook = [&](int k, int jj) {
      if (k < RT0 || jj < 2 * NAP || (jj - 2 * NAP) % RSP != 0) return;  // after the tap's A pieces
      const int i = (jj - 2 * NAP) / RSP;
      const int j = (k - RT0) * RPT + i;
      if (i >= RPT || j >= NJ) return;
      {
        const int off = ((t0 + row0 + 16 * j + lr) * C + cofs) * 2;  // rows past T: read 0
        xres[j] = __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0);
        if constexpr (ACC == 2 && !AP2) ares[j] = __builtin_amdgcn_raw_buffer_load_b128(rsa, off, 0, 0);
      }
    };
    const f32x4* bias1 = reinterpret_cast<const f32x4*>(sbias + cofs);
    const f32x4 b1z0 = bias1[0], b1z1 = bias1[1];
    auto p1_cinit = [&](int, int t) { return t ? b1z1 : b1z0; };
    uint32_t pv[4];
    auto p1_post = [&](int j, int p) {  // part p: channels 2p, 2p + 1 of the lane's 8; part 3 stores
      const int t = p >> 1, e = 2 * (p & 1);
      // scalar multiplies: the packed v_pk_mul_f32 form ran the last tap ~3 % slower (stamps, C = 64 / 128)
      pv[p] = pk_bf16(lrelu_max(acc[t][j][e], slope), lrelu_max(acc[t][j][e + 1], slope));
      if (p == 3) {
        const int r = row0 + 16 * j + lr;
        const int pos = t0 - H2 + r;
        u32x4 v = u32x4{pv[0], pv[1], pv[2], pv[3]};
        if (!interior) v &= (pos >= 0 && pos < T) ? 0xffffffffu : 0u;
        *reinterpret_cast<u32x4*>(t1 + pw * TP * 32 + rw_off(r, lg)) = v;
      }
    };
    conv(std::integral_constant<int, 0>{}, p1_hook, p1_post, p1_cinit, [&](int, int, int) {});
    stamp(2 + K);
    lds_barrier();  // T1 complete; every wave is past its window reads
    stamp(3 + K);

    // ---- P2: y = (b2 + x + c2(T1)) * out_scale (+ acc); the next window is staged meanwhile:
    // SPT slots loaded per tap in taps 0 .. K-3 and written (lrelu'd) two taps later
    const int valid = min(BT, T - t0);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.y + ((int64_t)b * T + t0) * C), (short)0, valid * C * (int)sizeof(bf16_t), 0x00020000);
    auto p2_hook = [&](int k, int jj) {
      if (jj >= 2 * NAP && (jj - 2 * NAP) % SP2 == 0) {
        const int i = (jj - 2 * NAP) / SP2, sl = k * SPT + i;
        if (i < SPT && k <= K - 3 && sl < NWV) load_win1(ntile, sl);
      }
      if (jj >= 2 * NAP + SP2 / 2 && (jj - 2 * NAP - SP2 / 2) % SP2 == 0) {
        const int i = (jj - 2 * NAP - SP2 / 2) / SP2, sl = (k - 2) * SPT + i;
        if (i < SPT && k >= 2 && sl < NWV) store_win1(sl);
      }
      if constexpr (AP2) {  // ARPT row tiles' accumulator rows per tap in taps 0 .. ANT - 1
        constexpr int ASP = (NST - 2 * NAP) / ARPT;
        if (k < ANT && jj >= 2 * NAP && (jj - 2 * NAP) % ASP == 0 && (jj - 2 * NAP) / ASP < ARPT) {
          const int j = ARPT * k + (jj - 2 * NAP) / ASP;
          ares[j] = __builtin_amdgcn_raw_buffer_load_b128(rsa, ((t0 + row0 + 16 * j + lr) * C + cofs) * 2, 0, 0);
        }
      }
      if constexpr (ACC == 1) {  // the MRF accumulator rows, RD steps before each row tile's epilogue
        // row tile j's epilogue starts at step (j + LG) NP of the last tap
        const int g = k * NST + jj, g0 = (K - 1) * NST + LG * NP - RD;
        if (g >= g0 && g < g0 + NST && (g - g0) % NP == 0) {
          const int j = (g - g0) / NP;
          ares[j] = __builtin_amdgcn_raw_buffer_load_b128(rsa, ((t0 + row0 + 16 * j + lr) * C + cofs) * 2, 0, 0);
        }
      }
    };
    const f32x4* bias2 = reinterpret_cast<const f32x4*>(sbias + C + cofs);
    const f32x4 b2z0 = bias2[0], b2z1 = bias2[1];
    auto p2_cinit = [&](int, int t) { return t ? b2z1 : b2z0; };
    // the residual x (and acc_in / out_scale) added by identity MFMAs in c2's tap XT: the lane's x
    // vector of row tile j IS the B fragment of input plane w, and A = I maps its 8 channels onto the
    // accumulator rows that hold them (exact: products of 1 and bf16, fp32 accumulation)
    auto p2_extra = [&](int k, int j, int s) {
      if (s != 0) return;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (k == XT)
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aid[t], __builtin_bit_cast(bf16x8, xres[j]), acc[t][j], 0, 0, 0);
        if constexpr (ACC == 2)
          if (k == XA)
            acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ais[t], __builtin_bit_cast(bf16x8, ares[j]), acc[t][j], 0, 0, 0);
      }
    };
    const float osc = a.out_scale;
    auto p2_post = [&](int j, int p) {  // part p: channels 2p, 2p + 1 of the lane's 8; part 3 stores
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
      if (p == 3)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{pv[0], pv[1], pv[2], pv[3]}, yrs,
                                               ((row0 + 16 * j + lr) * C + cofs) * (int)sizeof(bf16_t), 0, 0);
    };
    conv(std::integral_constant<int, 1>{}, p2_hook, p2_post, p2_cinit, p2_extra);
    stamp(4 + 2 * K);
    ++st_tile;
  }
}

template <int C, int K, int ACC, bool FR>
static int prw_launch(PrwArgs a, int B, hipStream_t st) {
  constexpr int BT = rw_r1(C) - 2 * ((K - 1) / 2);
  a.tiles_per_b = (a.T + BT - 1) / BT;
  a.ntiles = a.tiles_per_b * B;
  auto kern = mrf_prw_kernel<C, K, ACC, FR>;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  const int grid = (int)std::min<int64_t>((int64_t)cus, a.ntiles);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), rw_lds(C), st, a);
  VO_RETURN_LAUNCH();
}

}  // namespace vo

using namespace vo;

// Entry from vo_resblock_pair (resblock.hip): *handled = 1 when this kernel covers the shape
// (C = 64 / 128, K = 7 / 11, (K - 1) * dil <= 64).  pair_cfg 93 / 99 (C = 128) and 111 (C = 64) select the
// earlier LDS-tile kernels for A/B runs.  Measured at B = 32 (tools/mrf_bench.py, with the MRF accumulator):
// C = 64 k = 11 355 us vs 426, k = 7 275 vs 286 (mean over d = 1 / 3 / 5).
int vo_pair_rw_try(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                   const void* acc, int B, int T, int C, int K, int dil, float slope, float out_scale, int cfg,
                   hipStream_t st, int* handled, int frag) {
  *handled = 0;
  // (C = 32 instantiates too, but measured 4-9 % slower than the LDS-tile kernel at B = 32: 210-258 us vs
  // 197-242 for k = 7 / 11, tools/mrf_bench.py --stages 3 -- one 32-channel plane per wave leaves 16
  // steps per tap for the same per-tap A pieces, staging and epilogue work; not dispatched)
  if (!((C == 128 || C == 64) && (K == 7 || K == 11) && dil >= 1 && dil * (K - 1) <= 64)) return VO_OK;
  if (!frag && (cfg == 93 || cfg == 99)) return VO_OK;  // 93: the LDS-tile kernels (A/B)
  if (!frag && C == 64 && cfg == 111) return VO_OK;
  PrwArgs a;
  a.x = (const bf16_t*)x; a.w1 = (const bf16_t*)w1; a.b1 = b1; a.w2 = (const bf16_t*)w2; a.b2 = b2;
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)acc;
  a.T = T; a.dil = dil; a.slope = slope; a.out_scale = out_scale;
  a.tiles_per_b = a.ntiles = 0;
  a.stamps = nullptr;
  *handled = 1;
  // acc_in / out_scale through the identity MFMA when 1 / out_scale is a bf16 value (the MRF's 1/3 -> 3)
  int accm = 0;
  if (acc) {
    const float inv = 1.0f / out_scale;
    const float invb = __bfloat162float(__float2bfloat16(inv));
    accm = (invb == inv && std::isfinite(inv) && inv * out_scale == 1.0f) ? 2 : 1;
  }
#define VO_PRW_DISPATCH(CC, KK, FF) \
  return accm == 2 ? prw_launch<CC, KK, 2, FF>(a, B, st) : accm == 1 ? prw_launch<CC, KK, 1, FF>(a, B, st) \
                                                        : prw_launch<CC, KK, 0, FF>(a, B, st)
  if (C == 64) {
    if (frag) {
      if (K == 7) VO_PRW_DISPATCH(64, 7, true);
      VO_PRW_DISPATCH(64, 11, true);
    }
    if (K == 7) VO_PRW_DISPATCH(64, 7, false);
    VO_PRW_DISPATCH(64, 11, false);
  }
  if (frag) {
    if (K == 7) VO_PRW_DISPATCH(128, 7, true);
    VO_PRW_DISPATCH(128, 11, true);
  }
  if (K == 7) VO_PRW_DISPATCH(128, 7, false);
  VO_PRW_DISPATCH(128, 11, false);
#undef VO_PRW_DISPATCH
}

// [K][C][C] bf16 conv pack -> the fragment order the pair kernel streams (NP = C / 32 planes):
// dst[k][p][s][t][lane][e] = src[k][32p + 8(l >> 2) + 4t + (l & 3)][32s + 8(lane >> 4) + e], l = lane & 15
__global__ void pack_frag_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst, int C, int K) {
  const int v = blockIdx.x * 256 + threadIdx.x;  // one 16-byte vector per thread
  const int np = C / 32;
  if (v >= K * C * C / 8) return;
  const int lane = v & 63, t = (v >> 6) & 1, s = (v >> 7) % np, p = ((v >> 7) / np) % np, k = (v >> 7) / (np * np);
  const int lr = lane & 15, lg = lane >> 4;
  const int co = 32 * p + 8 * (lr >> 2) + 4 * t + (lr & 3), ci = 32 * s + 8 * lg;
  *reinterpret_cast<uint4*>(dst + (int64_t)v * 8) =
      *reinterpret_cast<const uint4*>(src + ((int64_t)k * C + co) * C + ci);
}

extern "C" int vo_pack_frag(const void* src, void* dst, int C, int K, void* stream) {
  VO_CHECK_ARG(src && dst && src != dst, "pack_frag: bad pointers");
  VO_CHECK_ARG(C == 64 || C == 128, "pack_frag: C=%d (64 or 128)", C);
  VO_CHECK_ARG(K >= 1 && K <= 15, "pack_frag: K=%d", K);
  const int n = K * C * C / 8;
  hipLaunchKernelGGL(pack_frag_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), (const bf16_t*)src, (bf16_t*)dst, C, K);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_resblock_pair_frag(const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                                     void* y, const void* acc, int B, int T, int C, int K, int dil, float slope,
                                     float out_scale, void* stream) {
  VO_CHECK_ARG(x && w1 && b1 && w2 && b2 && y, "resblock_pair_frag: null pointer");
  VO_CHECK_ARG((C == 64 || C == 128) && (K == 7 || K == 11) && dil >= 1 && dil * (K - 1) <= 64,
               "resblock_pair_frag: C=%d K=%d dil=%d unsupported (C = 64 / 128, K = 7 / 11, (K-1)*dil <= 64)", C, K,
               dil);
  VO_CHECK_ARG(slope >= 0.f && slope <= 1.f, "resblock_pair_frag: slope %g outside [0, 1]", slope);
  VO_CHECK_ARG(B > 0 && T > 0, "resblock_pair_frag: empty");
  VO_CHECK_ARG(y != x, "resblock_pair_frag: y must not alias x (neighbouring tiles re-read x)");
  VO_CHECK_ARG(acc == nullptr || acc == y || acc != x, "resblock_pair_frag: acc must not alias x");
  int handled = 0;
  return vo_pair_rw_try(x, w1, b1, w2, b2, y, acc, B, T, C, K, dil, slope, out_scale, 0,
                        reinterpret_cast<hipStream_t>(stream), &handled, 1);
}

#ifdef VO_PRW_STAMPS
// Diagnostic entry (tools/probes/prw_stamps.py builds its own library with -DVO_PRW_STAMPS): one stamped
// launch at the given shape (MRF accumulator on, out_scale 1/3); host_out receives RW_NSTW x 4 waves x
// RW_NSTT tiles x RW_NPT stamps.  v: bit 2 = fragment-ordered weights (else [K][Co][Ci]), bit 3 = C = 64, bit 4 = no accumulator.
extern "C" int vo_prw_stamps(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                             const void* acc, int B, int T, int K, int dil, int v, unsigned long long* host_out) {
  const size_t n = (size_t)RW_NSTW * 4 * RW_NSTT * RW_NPT;
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, n * 8) != hipSuccess) return -1;
  (void)hipMemset(d, 0, n * 8);
  PrwArgs a;
  a.x = (const bf16_t*)x; a.w1 = (const bf16_t*)w1; a.b1 = b1; a.w2 = (const bf16_t*)w2; a.b2 = b2;
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)acc;
  a.T = T; a.dil = dil; a.slope = 0.1f; a.out_scale = 1.f / 3; a.stamps = d;
  const int C = (v & 8) ? 64 : 128;
  const int BT = rw_r1(C) - 2 * ((K - 1) / 2);
  a.tiles_per_b = (T + BT - 1) / BT;
  a.ntiles = a.tiles_per_b * B;
  const int grid = std::min(256, a.ntiles);
  const size_t lds = rw_lds(C);
#define VO_PRW_STAMPED(CC, KK, FF)                                                                   \
  do {                                                                                               \
    if (v & 16) hipLaunchKernelGGL((mrf_prw_kernel<CC, KK, 0, FF, true>), dim3(grid), dim3(256), lds, 0, a); \
    else hipLaunchKernelGGL((mrf_prw_kernel<CC, KK, 2, FF, true>), dim3(grid), dim3(256), lds, 0, a);        \
  } while (0)
  const bool fr = (v & 4) != 0;
  if (C == 64) {
    if (K == 11) { if (fr) VO_PRW_STAMPED(64, 11, true); else VO_PRW_STAMPED(64, 11, false); }
    else { if (fr) VO_PRW_STAMPED(64, 7, true); else VO_PRW_STAMPED(64, 7, false); }
  } else {
    if (K == 11) { if (fr) VO_PRW_STAMPED(128, 11, true); else VO_PRW_STAMPED(128, 11, false); }
    else { if (fr) VO_PRW_STAMPED(128, 7, true); else VO_PRW_STAMPED(128, 7, false); }
  }
#undef VO_PRW_STAMPED
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(host_out, d, n * 8, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  return 0;
}
#endif
