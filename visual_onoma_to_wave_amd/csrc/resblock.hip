// Fused HiFi-GAN ResBlock1 pair for the narrow MRF stages (C = 32 / 64):
//   y = (x + c2(lrelu(c1_d(lrelu(x), slope), slope))) * out_scale (+ acc)
// (scripts/hifigan/models.py:96-103, one (c1, c2) iteration; the Generator's MRF sum and
// 1/num_kernels scale, models.py:155-160, ride in the epilogue).
//
// Persistent kernel: one workgroup per CU walks a contiguous run of time tiles.  A tile is
// R1 = WT*16*NJ c1-output rows = BT = R1 - (K-1) output positions:
//   P1: T1 = lrelu(c1(window) + b1) for positions [t0 - h2, t0 - h2 + R1) straight into LDS
//       (rows outside [0, T) forced to 0 = c2's zero padding); the lrelu'd input window
//       (R1 + (K-1)*dil rows, all channel planes) is staged once per tile;
//   P2: y = (c2(T1) + b2 + x) * out_scale (+ acc).
// Software pipeline (the C = 32 / 64 pair is HBM-bound, so loads must not wait behind the
// MFMAs): the NEXT tile's window is fetched into registers before this tile's P1 and written
// to LDS (lrelu applied) during P2; this tile's residual / MRF-accumulator rows are fetched
// in epilogue layout before P1 and consumed after P2.  Weights: RES = both convs resident in
// LDS for the whole kernel (no barrier inside a phase); otherwise TG-tap groups stream
// through a double buffer (one barrier per group), continuing across phases and tiles.
// Per position the pair moves x once (+ halo, L2-hot) in, x once more as the residual
// (L2-hot) and y once out: ~2 HBM activation passes against 5 for two conv launches.
// LDS rows are 64 B (32 bf16 of one channel plane) with the conflict-free XOR swizzle of
// conv1d.hip.

#include <algorithm>
#include <type_traits>

#include "mrf_common.h"

namespace vo {

struct PairArgs {
  const bf16_t* x; const bf16_t* w1; const float* b1; const bf16_t* w2; const float* b2;
  bf16_t* y; const bf16_t* acc;
  int T, K, dil, tiles_per_b, ntiles;
  float slope, out_scale;
};

// WC x WT waves: wave (wc, wt) owns channels [wc*C/WC, (wc+1)*C/WC) of rows [wt*16*NJ, ..+16*NJ)
// ABL (timing ablations only, garbage results; dispatched only with -DVO_ABLATIONS): 1 = no
// weight-group loads, 2 = no window /
// residual loads, 3 = neither; bit 4 = no weight LDS stores
// PRIO (A/B only; both within run-to-run noise on the C = 128 pair): 1 = s_setprio(1) around
// each MFMA cluster; 2 = static: the younger half of the waves runs at priority 1 (guide T5)
// SB: pin the software pipeline with sched_barrier: the fragment reads of step st + 1 are
// issued before, and kept above, the MFMAs of step st (hipcc otherwise sinks every
// ds_read down to its first use and waits lgkmcnt right before each MFMA pair, exposing
// the full LDS latency once per pair)
// IP: T1 overlays the window (the window is dead once P1's MFMAs end): LDS per tile drops
// from window + T1 to max(window, T1), so the C = 128 tile can grow to 256 rows and each
// streamed weight tap feeds twice the MFMAs.  Costs two barriers per tile and a window store
// after P2 instead of during it.
// VD (round 3, "VALU diet"): each conv's bias is the C operand of its first MFMAs (no accumulator
// zeroing, no bias adds), leaky ReLU in packed fp32, the T1 mask only in boundary tiles.
template <int C, int WC, int WT, int NJ, bool RES, int TG, int ABL = 0, int PRIO = 0, bool SB = false, bool GL = false,
          bool IP = false, bool HP = false, bool LATE = HP, bool VD = true>
__global__ void __launch_bounds__(WC * WT * 64, 2) mrf_pair_kernel(PairArgs a) {  // >= 2 waves per SIMD
  constexpr int NW = WC * WT;
  constexpr int NT = NW * 64;
  constexpr int NC = C / 32;              // 32-channel planes
  constexpr int NI = C / (16 * WC);       // co tiles per wave
  constexpr int R1 = WT * 16 * NJ;        // c1 rows per tile
  constexpr int SHW = NI >= 8 ? 5 : (NI == 4 ? 4 : 3);  // log2(4 * NI): weight-row swizzle
  constexpr int VPR = NC * 4;             // 16-byte vectors per activation row
  constexpr int MAXW = ((R1 + 64) * VPR + NT - 1) / NT;  // window vectors per thread, halo <= 64
  constexpr int TAPV = C * VPR;           // 16-byte vectors per weight tap (C co x C ci)
  constexpr int TAPE = NC * C * 32;       // LDS elements per weight tap
  constexpr int GV = (TG * TAPV + NT - 1) / NT;  // streamed weight vectors per thread per group
  constexpr int T1R = R1 + 16;            // P2 reads up to row R1 + K - 2 (feeds discarded rows only)
  constexpr int NH = NI / 2;              // 8-channel vectors per lane in epilogue layout

  const int K = a.K, dil = a.dil, T = a.T;
  const int h1 = dil * (K - 1) / 2, h2 = (K - 1) / 2;
  const int win_rows = R1 + 2 * h1;
  const int BT = R1 - 2 * h2;
  const float slope = a.slope;

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* win = reinterpret_cast<bf16_t*>(smem_raw);  // [NC][win_rows][32]
  bf16_t* t1 = IP ? win : win + NC * win_rows * 32;   // [NC][T1R][32]
  bf16_t* wls = IP ? win + NC * max(win_rows, T1R) * 32 : t1 + NC * T1R * 32;  // RES: [2][K] taps; else [2 bufs][TG] taps
  static_assert(!HP || (GL && TG == 1 && !RES && NC % 2 == 0), "half-tap groups: LDS-DMA streaming, one tap");
  static_assert(!(RES && IP) || LATE, "resident weights in place: the next window is fetched after P2");
  constexpr int GE = HP ? TAPE / 2 : TG * TAPE;  // LDS elements per streamed group buffer
  float* sbias = reinterpret_cast<float*>(wls + (RES ? 2 * K * TAPE : 2 * GE));  // [b1 | b2]
  bf16_t* spare = reinterpret_cast<bf16_t*>(sbias + 2 * C);  // 16 B sink for idle staging slots

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  const int wc = wave % WC, wt = wave / WC;
  const int cw0 = wc * (C / WC);    // the wave's first channel
  const int n0 = cw0 + NI * 4 * lq;  // epilogue: this lane's 4*NI contiguous output channels

  // contiguous tile run of this workgroup (uniform per workgroup: the early exit is safe)
  const int G = gridDim.x;
  int tile = (int)(((int64_t)blockIdx.x * a.ntiles) / G);
  const int tile_end = (int)(((int64_t)(blockIdx.x + 1) * a.ntiles) / G);
  if (tile >= tile_end) return;

  // ---- weights
  const int NG = HP ? 2 * K : (K + TG - 1) / TG;  // streamed groups per phase (HP: half taps)
  int wg_g[GV], wg_l[GV], wg_t[GV];
#pragma unroll
  for (int s = 0; s < GV; ++s) {
    const int v = tid + s * NT;
    // plane-major (tap, plane, co, q): 8 consecutive lanes fill 128 contiguous LDS bytes
    // (row-major order put two planes 4 KB+ apart in one 8-lane store group: 2-way conflicts)
    const int t = v / TAPV, vv = v - t * TAPV;
    const int pl = vv / (C * 4), rem = vv - pl * C * 4;
    const int co = rem >> 2, q = rem & 3;
    wg_t[s] = v < TG * TAPV ? t : TG;  // TG marks an idle slot (loads tap 0.., never stored)
    wg_g[s] = co * C + pl * 32 + q * 8;
    wg_l[s] = t * TAPE + pl * C * 32 + rb_off(co, q, SHW);
  }
  u32x4 wr[GV];
  // GL: the group is copied HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
  // instruction, lane-linear in LDS): no VGPR staging and no ds_write (the ablation without
  // weight stores ran 25-30 % faster).  The XOR swizzle moves to the source address: LDS
  // slot p of a group holds (tap t, plane pl, row co, chunk q' = q ^ swz(co)).
  constexpr int GVEC = HP ? TAPV / 2 : TG * TAPV;     // 16-byte vectors per streamed group
  constexpr int GLN = GL ? GVEC / (64 * NW) : 1;  // DMA instructions per wave per group
  static_assert(!GL || GVEC % (64 * NW) == 0, "glds: group must split into whole wave-KiB");
  // per-lane source: tap within the group (gl_t) and 32-bit element offset within a tap (gl_off);
  // the group's tap base is wave-uniform (SGPRs), the LDS destination too (m0 from an SGPR)
  int gl_t[GLN], gl_off[GLN];
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  if constexpr (GL) {
#pragma unroll
    for (int s = 0; s < GLN; ++s) {
      const int p = (s * NW + wave) * 64 + lane;
      const int t = HP ? 0 : p / TAPV, vv = p - t * TAPV;
      const int pl = vv / (C * 4), rem = vv - pl * C * 4;  // HP: plane within the half tap
      const int co = rem >> 2, q = (rem & 3) ^ ((co >> (SHW - 1)) & 2);
      gl_t[s] = t;
      gl_off[s] = co * C + pl * 32 + q * 8;
    }
  }
  auto load_group = [&](int gi, int buf) {  // gi in [0, 2*NG): conv gi / NG, taps (gi % NG) * TG + t
    const int ph = gi >= NG;
    const int k0 = (gi - ph * NG) * TG;
    const bf16_t* W = ph ? a.w2 : a.w1;
    if constexpr (GL) {
      if constexpr ((ABL & 1) != 0) return;
      typedef __attribute__((address_space(3))) void lds_void;
      typedef const __attribute__((address_space(1))) void g_void;
      // HP: group gi is half (gi & 1) of tap gi / 2 -- planes [half * NC/2, (half + 1) * NC/2)
      const bf16_t* Wk = HP ? W + ((gi - ph * NG) >> 1) * (C * C) + ((gi - ph * NG) & 1) * (NC / 2) * 32
                            : W + k0 * (C * C);  // uniform
#pragma unroll
      for (int s = 0; s < GLN; ++s) {
        // taps past K (last group, K % TG != 0) re-read tap K - 1; their MFMAs are skipped
        const int dt = TG == 1 ? 0 : min(gl_t[s], K - 1 - k0);
        const bf16_t* src = Wk + (dt * (C * C) + gl_off[s]);
        bf16_t* dst = wls + buf * GE + (s * NW + wave_u) * 64 * 8;
        __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)dst, 16, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int s = 0; s < GV; ++s) {
      const int k = k0 + (wg_t[s] < TG ? wg_t[s] : 0);
      if constexpr (ABL & 1)
        wr[s] = u32x4{(unsigned)k, 0u, 0u, 0u};
      else
        wr[s] = *reinterpret_cast<const u32x4*>(W + (int64_t)min(k, K - 1) * C * C + wg_g[s]);  // taps >= K unused
    }
  };
  auto store_group = [&](int buf) {
    if constexpr ((ABL & 4) != 0 || GL) return;
#pragma unroll
    for (int s = 0; s < GV; ++s)
      if (GV * NT == TG * TAPV || wg_t[s] < TG) *reinterpret_cast<u32x4*>(wls + buf * TG * TAPE + wg_l[s]) = wr[s];
  };

  for (int i = tid; i < 2 * C; i += NT) sbias[i] = i < C ? a.b1[i] : a.b2[i - C];
  if constexpr (RES) {
    // both convs, all taps, once per kernel: batches of 8 independent loads
    const int total = 2 * K * TAPV;
    for (int v0 = 0; v0 < total; v0 += 8 * NT) {
      u32x4 buf[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int v = v0 + u * NT + tid;
        const int ck = v / TAPV, vv = v - ck * TAPV;  // ck = conv * K + tap
        const bf16_t* W = ck >= K ? a.w2 + (int64_t)(ck - K) * C * C : a.w1 + (int64_t)ck * C * C;
        buf[u] = v < total ? *reinterpret_cast<const u32x4*>(W + vv * 8) : u32x4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int v = v0 + u * NT + tid;
        if (v < total) {
          const int ck = v / TAPV, vv = v - ck * TAPV;
          const int co = vv / VPR, rem = vv - co * VPR;
          *reinterpret_cast<u32x4*>(wls + ck * TAPE + (rem >> 2) * C * 32 + rb_off(co, rem & 3, SHW)) = buf[u];
        }
      }
    }
  } else {
    load_group(0, 0);
    store_group(0);
  }

  // ---- input window staging geometry (row-major vectors: consecutive lanes, consecutive 16 B).
  // NT is a multiple of VPR, so slot s of a thread is row r0 + s * RSTEP, same 16-byte column:
  // one base row / column / LDS offset per thread, the slots are compile-time offsets (adding
  // RSTEP rows keeps the XOR swizzle bit: RSTEP is a multiple of 8)
  static_assert(NT % VPR == 0 && (NT / VPR) % 8 == 0, "window slot stride must keep the swizzle");
  constexpr int RSTEP = NT / VPR;
  const int xr0 = tid / VPR, xrem = tid - xr0 * VPR;
  const int xg0 = xrem * 8;
  const int xl0 = (xrem >> 2) * win_rows * 32 + rb_off(xr0, xrem & 3, 2);
  // Global loads are unconditional (clamped rows, zeroed when written to LDS): a load under a
  // divergent branch gets an immediate vmcnt(0) from the compiler and the prefetch is lost.
  u32x4 xw[MAXW];
  bool xw_ok[MAXW];
  auto load_win = [&](int tl) {
    const int b = tl / a.tiles_per_b;
    const int R0 = (tl - b * a.tiles_per_b) * BT - h2 - h1;
    const bf16_t* base = a.x + (int64_t)b * T * C;
#pragma unroll
    for (int s = 0; s < MAXW; ++s) {
      const int t = R0 + xr0 + s * RSTEP;
      xw_ok[s] = t >= 0 && t < T && xr0 + s * RSTEP < win_rows;
      if constexpr ((ABL & 2) != 0)
        xw[s] = u32x4{(unsigned)t, 0u, 0u, 0u};
      else
        xw[s] = *reinterpret_cast<const u32x4*>(base + (int64_t)min(max(t, 0), T - 1) * C + xg0);
    }
  };
  auto store_win = [&]() {
#pragma unroll
    for (int s = 0; s < MAXW; ++s) {
      const u32x4 v = lrelu8(xw[s], slope);
      // idle slots (rows past the window) write the spare row after the bias table
      *reinterpret_cast<u32x4*>(xr0 + s * RSTEP < win_rows ? win + xl0 + s * RSTEP * 32 : spare) =
          xw_ok[s] ? v : u32x4{0u, 0u, 0u, 0u};
    }
  };

  int a_off[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) a_off[i] = rb_off(cw0 + NI * 4 * (lr >> 2) + 4 * i + (lr & 3), lq, SHW);
  const int brow0 = wt * 16 * NJ + lr;

  if constexpr (PRIO == 2)
    if (__builtin_amdgcn_readfirstlane(tid) >= NT / 2) __builtin_amdgcn_s_setprio(1);
  load_win(tile);
  store_win();
  if constexpr (GL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();

  f32x4 acc[NI][NJ];
  int gcount = 0;  // streamed groups consumed so far (selects the double buffer)

  // one tap of one plane: NI x NJ MFMAs; bias_row >= 0 (VD, a conv's first step): that conv's bias
  // is the C operand
  auto tap = [&](const bf16_t* wt, const bf16_t* src, int row, int bias_row = -1) {
    Frag<bf16_t> af[NI], bfr[NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i) af[i].load(wt + a_off[i]);
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
  };

  for (; tile < tile_end; ++tile) {
    const int b = tile / a.tiles_per_b;
    const int t0 = (tile - b * a.tiles_per_b) * BT;
    const bool has_next = tile + 1 < tile_end;

    // residual / accumulator rows of this tile (epilogue layout), consumed after P2
    u32x4 xres[NJ][NH], ares[NJ][NH];
    auto load_res = [&]() {
      const bf16_t* accp = a.acc ? a.acc : a.x;  // loaded either way (no branch), added only with acc
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int pos = min(t0 + wt * 16 * NJ + 16 * j + lr, T - 1);  // rows past the tile are not stored
        const int64_t off = ((int64_t)b * T + pos) * C + n0;
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          if constexpr ((ABL & 2) != 0) {
            xres[j][h] = ares[j][h] = u32x4{(unsigned)pos, 0u, 0u, 0u};
          } else {
            xres[j][h] = *reinterpret_cast<const u32x4*>(a.x + off + 8 * h);
            if constexpr (!IP) ares[j][h] = *reinterpret_cast<const u32x4*>(accp + off + 8 * h);
          }
        }
      }
    };
    // IP keeps the window prefetch live through P2, so its residual rows are fetched one
    // group (a tap: >= 1k MFMA cycles) before the epilogue instead of a whole tile ahead
    if constexpr (!IP) load_res();  // IP: one group before the epilogue; HP: in the epilogue
    if constexpr (!IP) {
      load_win(has_next ? tile + 1 : tile);  // unconditional (see load_win)
    }

    if constexpr (!VD) {
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // P1 epilogue: T1 = lrelu(acc + b1), zero outside [0, T) (c2's zero padding); clears acc
    // the lane's 8*NH bias values, read (as float4) before the epilogue's LDS stores: read
    // one by one between the T1 stores they were serialised behind them (possible aliasing)
    auto lane_bias = [&](int which, float (&bz)[8 * NH]) {
      const float4* bp = reinterpret_cast<const float4*>(sbias + which * C + n0);
#pragma unroll
      for (int u = 0; u < 2 * NH; ++u) {
        const float4 v = bp[u];
        bz[4 * u] = v.x; bz[4 * u + 1] = v.y; bz[4 * u + 2] = v.z; bz[4 * u + 3] = v.w;
      }
    };
    auto p1_epilogue = [&]() {
      if constexpr (VD) {  // the bias is in the accumulators
        const bool interior = t0 - h2 >= 0 && t0 - h2 + R1 <= T;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int r = wt * 16 * NJ + 16 * j + lr;
          const int pos = t0 - h2 + r;
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
            *reinterpret_cast<u32x4*>(t1 + (ch >> 5) * T1R * 32 + rb_off(r, (ch & 31) >> 3, 2)) = u32x4{w[0], w[1], w[2], w[3]};
          }
        }
        return;
      }
      float bz[8 * NH];
      lane_bias(0, bz);
      // rows outside [0, T) exist only in the first / last tile of an utterance
      const bool interior = t0 - h2 >= 0 && t0 - h2 + R1 <= T;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = wt * 16 * NJ + 16 * j + lr;
        const int pos = t0 - h2 + r;
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
          *reinterpret_cast<u32x4*>(t1 + (ch >> 5) * T1R * 32 + rb_off(r, (ch & 31) >> 3, 2)) = u32x4{w[0], w[1], w[2], w[3]};
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    };

    if constexpr (RES) {
      tap(wls, win, brow0, VD ? 0 : -1);  // c = 0, k = 0: the conv's first step
      for (int c = 0; c < NC; ++c)
        for (int k = c == 0 ? 1 : 0; k < K; ++k) tap(wls + k * TAPE + c * C * 32, win + c * win_rows * 32, brow0 + k * dil);
      if constexpr (IP) {  // T1 overwrites the window: every wave must be past its P1 reads
        lds_barrier();
        p1_epilogue();
        lds_barrier();
      } else {
        p1_epilogue();
        lds_barrier();
        if (has_next) store_win();
      }
      const bf16_t* wb = wls + K * TAPE;
      tap(wb, t1, brow0, VD ? 1 : -1);
      for (int c = 0; c < NC; ++c)
        for (int k = c == 0 ? 1 : 0; k < K; ++k) tap(wb + k * TAPE + c * C * 32, t1 + c * T1R * 32, brow0 + k);
    } else {
      // peeled per phase so the P1 epilogue / window store sit on straight-line paths
      auto group = [&](int ph, int g, bool p1_last, bool p2_first) {
        const int gi = ph * NG + g;
        const bool more = has_next || gi + 1 < 2 * NG;
        if constexpr (IP) {  // next window: fetched at P2 start, stored after P2 (registers
          if (!LATE && gi == NG) load_win(has_next ? tile + 1 : tile);  // are not live during P1;
                                                                        // LATE: fetched after P2)
          if (!LATE && gi + 1 == 2 * NG) load_res();
        }
        load_group(gi + 1 == 2 * NG ? 0 : gi + 1, (gcount + 1) & 1);  // unconditional; stored only if needed
        const bf16_t* wb = wls + (gcount & 1) * GE;
        const bf16_t* src = ph ? t1 : win;
        const int plane = ph ? T1R * 32 : win_rows * 32;
        const int step = ph ? 1 : dil;
        // software-pipelined over the group's TG x NC (tap, plane) steps: the fragments of step
        // st + 1 are read from LDS before the MFMAs of step st (two named register sets)
        constexpr int S = HP ? NC / 2 : TG * NC;
        if constexpr (!SB) {  // plain steps: hipcc schedules the reads (fewer live fragments)
#pragma unroll
          for (int st = 0; st < S; ++st) {
            const int brow_first = VD && g == 0 && st == 0 ? ph : -1;  // a conv's first step: bias as C
            if constexpr (HP) {  // half tap g & 1 of tap g >> 1: planes (g & 1) * S + st
              const int c = (g & 1) * S + st;
              tap(wb + st * C * 32, src + c * plane, brow0 + (g >> 1) * step, brow_first);
            } else if (TG == 1 || g * TG + st / NC < K) {
              const int t = st / NC, c = st - t * NC;
              tap(wb + t * TAPE + c * C * 32, src + c * plane, brow0 + (g * TG + t) * step, brow_first);
            }
          }
        }
        Frag<bf16_t> af[2][NI], bq[2][NJ];
        auto ld = [&](int st, int set) {
          const int t = st / NC, c = st - t * NC;
          const bf16_t* wt = wb + t * TAPE + c * C * 32;
#pragma unroll
          for (int i = 0; i < NI; ++i) af[set][i].load(wt + a_off[i]);
          const int boff = c * plane + rb_off(brow0 + (g * TG + t) * step, lq, 2);
#pragma unroll
          for (int j = 0; j < NJ; ++j) bq[set][j].load(src + boff + 16 * j * 32);
        };
        // SB (round 3 form): the next step's reads go out right after the step's first MFMA, so the
        // wait before that MFMA covers only reads issued a whole step earlier (two sets of 8 reads in
        // flight exceed the 4-bit lgkmcnt: hipcc then waited for the just-issued ones as well)
        static_assert(!SB || !HP, "SB: whole-tap groups");
        f32x4 bz4[NI];
        if (SB && VD && g == 0) {
#pragma unroll
          for (int i = 0; i < NI; ++i) bz4[i] = *reinterpret_cast<const f32x4*>(sbias + ph * C + n0 + 4 * i);
        }
        if constexpr (SB) ld(0, 0);
#pragma unroll
        for (int st = 0; st < (SB ? S : 0); ++st) {
          const bool valid = TG == 1 || g * TG + st / NC < K;
          const bool first = VD && g == 0 && st == 0;  // the conv's first step: its bias is the C operand
#pragma unroll
          for (int q = 0; q < NI * NJ; ++q) {
            const int i = q / NJ, j = q - i * NJ;
            if (valid) acc[i][j] = mfma(af[st & 1][i], bq[st & 1][j], first ? bz4[i] : acc[i][j]);
            if (q == 0) {
              __builtin_amdgcn_sched_barrier(0);
              if (st + 1 < S) ld(st + 1, (st + 1) & 1);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        if (!IP && p1_last) p1_epilogue();
        if (!IP && p2_first && has_next) store_win();  // P1 reads of the window ended at the last barrier
        if (more) store_group((gcount + 1) & 1);
        if constexpr (GL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA landed
        lds_barrier();
        ++gcount;
        if (IP && p1_last) {  // every wave is past its window reads: T1 may overwrite them
          p1_epilogue();
          lds_barrier();
        }
      };
      group(0, 0, NG == 1, false);  // peeled: the conv's first step is known statically
      for (int g = 1; g < NG - 1; ++g) group(0, g, false, false);
      if (NG > 1) group(0, NG - 1, true, false);
      group(1, 0, false, true);
      for (int g = 1; g < NG; ++g) group(1, g, false, false);
    }

    // P2 epilogue: y = (c2 + b2 + x) * out_scale (+ acc)
    if constexpr (LATE) {
      // the residual and accumulator rows; the next tile's window is requested before the y
      // stores (vmcnt retires in issue order: the window store no longer waits for them)
      const bf16_t* accp = a.acc ? a.acc : a.x;  // loaded either way (no branch), added only with acc
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int pos = min(t0 + wt * 16 * NJ + 16 * j + lr, T - 1);
        const int64_t off = ((int64_t)b * T + pos) * C + n0;
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          if constexpr ((ABL & 2) != 0) {
            xres[j][h] = ares[j][h] = u32x4{(unsigned)pos, 0u, 0u, 0u};
          } else {
            xres[j][h] = *reinterpret_cast<const u32x4*>(a.x + off + 8 * h);
            ares[j][h] = *reinterpret_cast<const u32x4*>(accp + off + 8 * h);
          }
        }
      }
    } else if constexpr (IP) {  // IP: the MRF accumulator rows are read here (registers are short)
      if (a.acc) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int pos = min(t0 + wt * 16 * NJ + 16 * j + lr, T - 1);
          const int64_t off = ((int64_t)b * T + pos) * C + n0;
#pragma unroll
          for (int h = 0; h < NH; ++h) ares[j][h] = *reinterpret_cast<const u32x4*>(a.acc + off + 8 * h);
        }
      }
    }
    float b2z[8 * NH];
    if constexpr (VD) {
#pragma unroll
      for (int u = 0; u < 8 * NH; ++u) b2z[u] = 0.f;  // the bias is in the accumulators
    } else {
      lane_bias(1, b2z);
    }
    // y rows through a buffer resource covering exactly this tile's valid rows: the rows past
    // it (r >= BT, or past T) fall outside the resource and their stores are dropped by the
    // hardware -- no per-lane branch, and a fixed number of stores per wave
    const int valid = min(BT, T - t0);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.y + ((int64_t)b * T + t0) * C), (short)0, valid * C * (int)sizeof(bf16_t), 0x00020000);
    u32x4 yv[NJ][NH];
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
              q[u] = (acc[2 * h + e / 4][j][e & 3] + b2z[8 * h + e] + xf[e]) * a.out_scale;
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
    // the next window's registers are taken once the y values are packed: with the accumulators,
    // residual and window live at once the C = 128 kernel spilled and the C = 32 kernel lost its
    // fourth wave per SIMD (146 VGPRs; s3 +12 %)
    if constexpr (LATE && IP) load_win(has_next ? tile + 1 : tile);  // unconditional (see load_win)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int r = wt * 16 * NJ + 16 * j + lr;
#pragma unroll
      for (int h = 0; h < NH; ++h)
        __builtin_amdgcn_raw_buffer_store_b128(yv[j][h], yrs, (r * C + n0 + 8 * h) * (int)sizeof(bf16_t), 0, 0);
    }
    if constexpr (RES) lds_barrier();
    if constexpr (IP) {  // P2's T1 reads ended at the last group barrier
      if (has_next) store_win();
      lds_barrier();
    }
  }
}

template <int C, int WC, int WT, int NJ, bool RES, int TG, int ABL = 0, int PRIO = 0, bool SB = false, bool GL = false,
          bool IP = false, bool HP = false, bool LATE = HP, bool VD = true>
static int pair_launch(PairArgs a, int B, hipStream_t st) {
  constexpr int NW = WC * WT;
  constexpr int R1 = WT * 16 * NJ;
  const int h1 = a.dil * (a.K - 1) / 2, h2 = (a.K - 1) / 2;
  const int BT = R1 - 2 * h2;
  a.tiles_per_b = (a.T + BT - 1) / BT;
  a.ntiles = a.tiles_per_b * B;
  const size_t wtaps = RES ? 2 * (size_t)a.K : (HP ? 1 : 2 * (size_t)TG);  // HP: two half-tap buffers
  const size_t act_rows = IP ? std::max<size_t>(R1 + 2 * h1, R1 + 16) : (size_t)(R1 + 2 * h1) + (R1 + 16);
  const size_t lds = (act_rows + wtaps * C) * (C / 32) * 32 * sizeof(bf16_t) +
                     2 * C * sizeof(float) + 16;
  if (lds > 160 * 1024) {
    vo_set_error("resblock_pair: LDS %zu B exceeds 160 KiB", lds);
    return VO_ERR_INVALID;
  }
  auto kern = mrf_pair_kernel<C, WC, WT, NJ, RES, TG, ABL, PRIO, SB, GL, IP, HP, LATE, VD>;
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

int vo_pair2_try(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                 const void* acc, int B, int T, int C, int K, int dil, float slope, float out_scale, int cfg,
                 hipStream_t st, int* handled);  // resblock2.hip
int vo_pair3_try(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                 const void* acc, int B, int T, int C, int K, int dil, float slope, float out_scale, int cfg,
                 hipStream_t st, int* handled);  // resblock4.hip
int vo_pair_pc_try(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                   const void* acc, int B, int T, int C, int K, int dil, float slope, float out_scale,
                   hipStream_t st, int* handled);  // resblock_pc.hip
int vo_pair_rs_try(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                   const void* acc, int B, int T, int C, int K, int dil, float slope, float out_scale, int cfg,
                   hipStream_t st, int* handled);  // resblock_rs.hip
int vo_pair_rr_try(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                   const void* acc, int B, int T, int C, int K, int dil, float slope, float out_scale, int cfg,
                   hipStream_t st, int* handled);  // resblock_rr.hip
int vo_pair_rw_try(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                   const void* acc, int B, int T, int C, int K, int dil, float slope, float out_scale, int cfg,
                   hipStream_t st, int* handled, int frag);  // resblock_rw.hip
int vo_pair_wave_try(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                     const void* acc, int B, int T, int C, int K, int dil, float slope, float out_scale, int cfg,
                     hipStream_t st, int* handled);  // resblock5.hip

extern "C" int vo_resblock_pair(const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                                void* y, const void* acc, int B, int T, int C, int K, int dil, float slope,
                                float out_scale, void* stream) {
  VO_CHECK_ARG(x && w1 && b1 && w2 && b2 && y, "resblock_pair: null pointer");
  VO_CHECK_ARG(C == 32 || C == 64 || C == 128, "resblock_pair: C=%d unsupported (32, 64 or 128)", C);
  VO_CHECK_ARG(K % 2 == 1 && K >= 1 && K <= 15 && dil >= 1 && dil * (K - 1) <= 64,
               "resblock_pair: K=%d dil=%d unsupported (odd K <= 15, (K-1)*dil <= 64)", K, dil);
  VO_CHECK_ARG(slope >= 0.f && slope <= 1.f, "resblock_pair: slope %g outside [0, 1]", slope);
  VO_CHECK_ARG(B > 0 && T > 0, "resblock_pair: empty");
  VO_CHECK_ARG(y != x, "resblock_pair: y must not alias x (neighbouring tiles re-read x)");
  VO_CHECK_ARG(acc == nullptr || acc == y || acc != x, "resblock_pair: acc must not alias x");
  PairArgs a;
  a.x = (const bf16_t*)x; a.w1 = (const bf16_t*)w1; a.b1 = b1; a.w2 = (const bf16_t*)w2; a.b2 = b2;
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)acc;
  a.T = T; a.K = K; a.dil = dil; a.slope = slope; a.out_scale = out_scale;
  a.tiles_per_b = a.ntiles = 0;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // measured on MI355X, B=32 MRF shapes (tools/ab_pair.py, tools/ab_sb.py): C=32 K<=7 ->
  // 256-row tiles (3 workgroups/CU), K=11 -> 512-row tiles.  pair_cfg selects the
  // alternatives for A/B runs.
  const int cfg = vo_tune_get("pair_cfg");
  {  // round 5: C = 64 / 128 k = 7 / 11 with wave-owned output planes (resblock_rw.hip); pair_cfg 93 = LDS tiles
    int handled = 0;
    const int rc = vo_pair_rw_try(x, w1, b1, w2, b2, y, acc, B, T, C, K, dil, slope, out_scale, cfg, st, &handled, 0);
    if (handled) return rc;
  }
  {  // round 4: register-resident frames (resblock_rr.hip) for C = 64 k = 7; pair_cfg 90-99 (A/B)
    int handled = 0;
    const int rc = vo_pair_rr_try(x, w1, b1, w2, b2, y, acc, B, T, C, K, dil, slope, out_scale, cfg, st, &handled);
    if (handled) return rc;
  }
#ifdef VO_ABLATIONS  // measured-and-dropped variants (A/B builds only: make abl)
  // round-4 C = 128 candidates (k = 7 / 11): pair_cfg 71 = producer roles (resblock_pc.hip),
  // 72 = register-streamed weights, one wave per SIMD (resblock_rs.hip; rs_cfg 2: two per SIMD)
  if (C == 128 && cfg == 71) {
    int handled = 0;
    const int rc = vo_pair_pc_try(x, w1, b1, w2, b2, y, acc, B, T, C, K, dil, slope, out_scale, st, &handled);
    if (handled) return rc;
  }
  if (C == 128 && cfg == 72) {
    int handled = 0;
    const int rc = vo_pair_rs_try(x, w1, b1, w2, b2, y, acc, B, T, C, K, dil, slope, out_scale,
                                  vo_tune_get("rs_cfg"), st, &handled);
    if (handled) return rc;
  }
  if (cfg == 50) {  // round 3: C = 32 with wave-private frames (resblock5.hip)
    int handled = 0;
    const int rc = vo_pair_wave_try(x, w1, b1, w2, b2, y, acc, B, T, C, K, dil, slope, out_scale, cfg, st, &handled);
    if (handled) return rc;
  }
  if (cfg == 40 || cfg == 41) {  // round 3: two 4-wave workgroups per CU, LDS-DMA windows (resblock4.hip)
    int handled = 0;
    const int rc = vo_pair3_try(x, w1, b1, w2, b2, y, acc, B, T, C, K, dil, slope, out_scale, cfg, st, &handled);
    if (handled) return rc;
  }
  if (cfg == 30 || cfg == 31) {  // the version-2 kernel at C = 128 (resblock2.hip): -1 % at k = 7, +5 % at k = 11
    int handled = 0;
    const int rc = vo_pair2_try(x, w1, b1, w2, b2, y, acc, B, T, C, K, dil, slope, out_scale, cfg, st, &handled);
    if (handled) return rc;
  }
  // VALU diet (VD): C = 128 -2..4 % (0.682 -> 0.668 ms at k = 11, 0.505 -> 0.485 at k = 7); C = 32
  // +2..3 % (0.201 -> 0.205, 0.234 -> 0.240): C = 32 ships without it (tools/mrf_bench.py --tune
  // pair_cfg=8,0, round 3).  cfg 8 swaps the C = 32 / 128 epilogues, for A/B
  if (cfg == 8) {
    if (C == 32) return pair_launch<32, 1, 8, 4, true, 1, 0, 0, false, false, true, false, true, true>(a, B, st);
    if (C == 128 && K <= 3) return pair_launch<128, 2, 4, 4, false, 1, 0, 0, false, true, true, true, true, false>(a, B, st);
    if (C == 128) return pair_launch<128, 2, 4, 4, false, 1, 0, 0, false, true, true, false, true, false>(a, B, st);
  }
  if (C == 32) {
    if (cfg == 3) return pair_launch<32, 1, 4, 8, true, 1>(a, B, st);
    if (cfg == 4) return pair_launch<32, 1, 8, 8, true, 1, 0, 0, false, false, true, false, true>(a, B, st);
    if (cfg == 6) return pair_launch<32, 1, 8, 6, true, 1, 0, 0, false, false, true, false, true>(a, B, st);
    if (cfg == 1 || cfg == 2 || cfg == 9) {  // the previous tilings (9: k <= 7 -> 256 rows, else 512)
      const bool small = cfg == 9 ? K <= 7 : cfg == 1;
      return small ? pair_launch<32, 1, 8, 2, true, 1>(a, B, st) : pair_launch<32, 1, 8, 4, true, 1>(a, B, st);
    }
  }
  if (C == 128) {
    // 2 x 4 waves of 64 channels (2 waves/SIMD), weights by LDS-DMA.  pair_cfg 1 = the register-staged
    // 128-row kernel, 13 = its no-global-load timing ablation.
    if (cfg == 1) return pair_launch<128, 2, 4, 2, false, 1>(a, B, st);
    if (cfg == 13) return pair_launch<128, 2, 4, 2, false, 1, 3>(a, B, st);
    if (cfg == 16) return pair_launch<128, 2, 4, 4, false, 1, 2, 0, false, true, true, true>(a, B, st);
    if (cfg == 17) return pair_launch<128, 2, 4, 4, false, 1, 2, 0, false, true, true, false, true>(a, B, st);
    if (cfg == 25) return pair_launch<128, 2, 4, 4, false, 1, 1, 0, false, true, true, false, true>(a, B, st);
    if (cfg == 2) return pair_launch<128, 2, 4, 2, false, 1, 0, 0, false, true>(a, B, st);
    if (cfg == 3) return pair_launch<128, 2, 4, 3, false, 1, 0, 0, false, true, true>(a, B, st);
    // two 4-wave workgroups per CU (79 KB LDS each: 128-row in-place tiles, half-tap weight
    // buffers), 64 x 64-row wave tiles: one workgroup's epilogue overlaps the other's MFMAs
    if (cfg == 4) return pair_launch<128, 2, 2, 4, false, 1, 0, 0, false, true, true, true>(a, B, st);
    // one 8-wave workgroup per CU with half-tap buffers: 256- / 384-row in-place tiles halve the
    // weight stream per MFMA of the 192-row kernel (384 rows spill)
    if (cfg == 6) return pair_launch<128, 2, 4, 4, false, 1, 0, 0, false, true, true, true>(a, B, st);
    if (cfg == 7) return pair_launch<128, 2, 4, 4, false, 1, 0, 0, false, true, true, false, true>(a, B, st);
    if (cfg == 60) return pair_launch<128, 2, 4, 4, false, 1, 0, 0, true, true, true, false, true>(a, B, st);
    if (cfg == 9) {  // the round-2 defaults
      if (K <= 3) return pair_launch<128, 2, 4, 2, false, 1, 0, 0, false, true>(a, B, st);
      return pair_launch<128, 2, 4, 3, false, 1, 0, 0, false, true, true>(a, B, st);
    }
    if (cfg == 61 && K > 3) return pair_launch<128, 2, 4, 4, false, 1, 0, 0, false, true, true, false, true>(a, B, st);
  }
  if (C == 64) {
    // pair_cfg 3 / 4 / 5: 512-row IP + LDS-DMA / 384-row IP + LDS-DMA / 512-row IP
    // pair_cfg 1 = LDS-DMA weights + pinned fragment pipeline: 7 % faster alone (tools/ab_sb.py)
    // but 15 % slower inside the bench step with the MRF accumulator (tools/bench_ab.sh)
    if (cfg == 3) return pair_launch<64, 1, 8, 4, false, 2, 0, 0, false, true, true, false, true>(a, B, st);
    if (cfg == 4) return pair_launch<64, 1, 8, 3, false, 2, 0, 0, false, true, true, false, true>(a, B, st);
    if (cfg == 5) return pair_launch<64, 1, 8, 4, false, 2, 0, 0, false, false, true, false, true>(a, B, st);
    if (cfg == 1) return pair_launch<64, 1, 8, 3, false, 2, 0, 0, true, true>(a, B, st);
    if (cfg == 9) return pair_launch<64, 1, 8, 3, false, 2>(a, B, st);  // the round-2 default
    if (cfg == 2 && K <= 3) return pair_launch<64, 1, 8, 4, false, 2, 0, 0, false, false, true, false, true>(a, B, st);
  }
#endif
  // C = 64, k >= 7: the version-2 kernel (resblock2.hip: compile-time K, next window fetched during
  // P2): 0.453 -> 0.408 ms at k = 11, 0.359 -> 0.326 at k = 7, bit-identical (tools/ab_pair2.py).
  if (C == 64) {
    int handled = 0;
    const int rc = vo_pair2_try(x, w1, b1, w2, b2, y, acc, B, T, C, K, dil, slope, out_scale, cfg, st, &handled);
    if (handled) return rc;
  }
  if (C == 32) {
    // 512-row in-place tiles, window / residual fetched after P2: k = 11 -13 %, k = 7 -3 %
    // (k = 3 is HBM-bound at ~5 TB/s either way; tools/ab_sb.py pair32 9 5); without the VALU diet
    return pair_launch<32, 1, 8, 4, true, 1, 0, 0, false, false, true, false, true, false>(a, B, st);
  }
  if (C == 128) {
    // 256-row in-place tiles, window / residual fetched after P2 (no window registers live in the
    // MFMA loop): k = 3 with half-tap buffers (-10 %), k >= 7 with whole taps and the software-
    // pipelined steps (SB: the next (tap, plane) step's fragments read right after the current step's
    // first MFMA, -1..2 %).  Measured and dropped (tools/ab_sb.py, tools/mrf_bench.py, DESIGN.md
    // section 3): one wave per SIMD with 128 x 64-row wave tiles (20-45 % slower), three waves per SIMD
    // (15 % slower), the next window staged through registers during P2 (+20 %), 320 / 384-row tiles
    // (spill), an L2 / MALL prefetch of the epilogue's bytes by LDS-DMA pieces (+7..18 %), the weights
    // out of LDS (A fragments from global one tap ahead: +20 %).  Timing ablations (VO_ABLATIONS
    // builds): no window / residual loads 0.70 -> 0.58 ms at k = 11; no weight DMA 0.70 -> 0.63.
    if (K <= 3) return pair_launch<128, 2, 4, 4, false, 1, 0, 0, false, true, true, true>(a, B, st);
    return pair_launch<128, 2, 4, 4, false, 1, 0, 0, true, true, true, false, true>(a, B, st);
  }
  // C = 64: k = 3 -> both convs resident in LDS; other k (the version-2 kernel covers 7 / 11) ->
  // 512-row in-place tiles, window / residual fetched after P2 (-5 % against the 384-row kernel)
  if (K <= 3) return pair_launch<64, 1, 8, 2, true, 1>(a, B, st);
  return pair_launch<64, 1, 8, 4, false, 2, 0, 0, false, false, true, false, true>(a, B, st);
}
