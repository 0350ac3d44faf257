// HiFi-GAN ResBlock1 pair for the C = 128 MRF stage, register-streamed weights (round 4):
//   y = (x + c2(lrelu(c1_d(lrelu(x), slope), slope))) * out_scale (+ acc)
// (scripts/hifigan/models.py:96-103, one (c1, c2) iteration; the MRF sum and 1/num_kernels
// scale of models.py:155-160 ride in the epilogue).
//
// What bounds the LDS-streamed pair kernels (resblock.hip, resblock_pc.hip) is their per-group
// barrier: every 4 weight slices (2048 MFMA cycles per SIMD) all 8 waves meet so the next 32 KiB
// of weights can land in the shared LDS buffer, and s_memtime stamps (tools/probes/pc_stamps.py)
// put a group at ~2900 cycles even with no memory traffic at all.  Here the weights never touch
// LDS:
//  * one wave per SIMD (4 waves, up to 512 VGPRs each), wave (wc, wt) owns 64 output channels x
//    RW = 16 JW rows, so a tile is 128 channels x 2 RW c1 rows;
//  * each wave loads its own A fragments (the 64-channel half of a weight slice = 4 KiB: input
//    plane c, tap k) from L2 straight into a register ring, PF slices ahead -- the two waves of a
//    channel half read the same bytes (L1 hits); no barrier is needed for weights at all;
//  * activations (window / T1) stay in LDS, read into a small fragment ring D rows ahead;
//  * plane-major slice order as in resblock_pc.hip: the next tile's window plane c is loaded into
//    registers once every wave is past the dead T1 plane c (a barrier per plane in P2) and written
//    (leaky ReLU, zero padding) two slices later; the last plane during the next P1, which reads it
//    last.  Every load is an ordinary global load the compiler counts (no LDS-DMA, no hand-counted
//    waits): 7 barriers per tile instead of 2 NG + 4;
//  * the residual rows are requested two slices before P1 ends and added in P2's accumulator init
//    (acc = b2 + x), the MRF accumulator rows two slices before P2 ends and added in the y
//    epilogue: y = acc * out_scale + acc_in.

#ifdef VO_ABLATIONS  // round-4 C = 128 candidate (register-streamed weights): measured slower, A/B builds only
#include <type_traits>

#include "mrf_common.h"  // visual_onoma_to_wave_amd/csrc (make abl adds it to the include path)

namespace vo {

struct RsArgs {
  const bf16_t* x; const bf16_t* w1; const float* b1; const bf16_t* w2; const float* b2;
  bf16_t* y; const bf16_t* acc;
  int B, T, dil, tiles_per_b, ntiles;
  float slope, out_scale, inv_scale;
};

#ifdef VO_ABLATIONS
// diagnostic stamps (rs_cfg 9, ablation library only): s_memtime at each slice start of wave 0 of
// workgroups 0-7, tiles 1-2: [wg][tile][phase][slice]
__device__ unsigned long long g_rs_stamp[8 * 2 * 2 * 64];
extern "C" int vo_rs_stamps(unsigned long long* host, int n) {
  const int cap = (int)(sizeof(g_rs_stamp) / sizeof(g_rs_stamp[0]));
  if (n > cap) n = cap;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rs_stamp), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
#endif

template <int JW, int NWV> struct RsGeom {  // NWV waves: 2 channel halves x NWV / 2 row blocks
  static constexpr int RW = JW * 16, R1 = NWV / 2 * RW;
  static constexpr int PQ = 16 * NWV;  // plane rows: a multiple of PQ (whole window vectors per thread)
  static constexpr int PSR = ((R1 + 64 + PQ - 1) / PQ) * PQ;  // window <= R1 + 64 rows, T1 R1 + 16
  static constexpr int PLANE_E = PSR * 32;
  static constexpr size_t LDS = (size_t)4 * PLANE_E * 2 + 2 * 128 * 4;
};

// JW row fragments per wave, PF: A slices prefetched ahead (ring of 4 sets), D: B rows ahead
// (ring of 6)
template <int K, bool HAS_ACC, int JW, int PF, int D, int NWV, bool STAMP = false>
__global__ void __launch_bounds__(NWV * 64, NWV / 4) mrf_pair_rs_kernel(RsArgs a) {
  constexpr int C = 128, NC = 4, NI = 4, NT = NWV * 64;
  using Gm = RsGeom<JW, NWV>;
  constexpr int RW = Gm::RW, R1 = Gm::R1, PSR = Gm::PSR, PLANE_E = Gm::PLANE_E;
  constexpr int NS = NC * K;           // slices per conv (plane-major: s = c K + k)
  constexpr int h2 = (K - 1) / 2;
  constexpr int BT = R1 - 2 * h2;
  constexpr int NH = 2;
  constexpr int WV = PSR * 4 / NT;     // 16-byte window vectors per thread per plane
  constexpr int RB = 6;                // B-fragment ring
  constexpr int RA = PF == 1 ? 2 : 4;  // A-set ring
  static_assert(NS % 4 == 0, "slices in groups of 4");
  static_assert(PF >= 1 && PF <= 3 && D >= 1 && D < RB && (JW % RB) == 0, "rings");
  static_assert((PSR * 4) % NT == 0, "window vectors");

  const int T = a.T, dil = a.dil;
  const int h1 = dil * (K - 1) / 2;
  const float slope = a.slope;

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* act = reinterpret_cast<bf16_t*>(smem_raw);  // [NC][PSR][32]: window, then T1
  float* sbias = reinterpret_cast<float*>(act + NC * PLANE_E);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lq = lane >> 4;
  const int wc = wave & 1, wt = wave >> 1;
  const int cw0 = wc * 64;

  const int G = gridDim.x;
  int tile = (int)(((int64_t)blockIdx.x * a.ntiles) / G);
  const int tile_end = (int)(((int64_t)(blockIdx.x + 1) * a.ntiles) / G);
  if (tile >= tile_end) return;

  for (int i = tid; i < 2 * C; i += NT) sbias[i] = i < C ? a.b1[i] : a.b2[i - C];

  // ---- A stream: slices of (c1, c2) in order, continuous across phases and tiles.  The lane's
  // fragment i of a slice: W[k][co][32 c + 8 lq .. + 8], co = cw0 + 16 (lr >> 2) + 4 i + (lr & 3)
  // (the accumulator of MFMA i then holds channels n0 + 4 i .. + 3 of its rows)
  // every global load goes through a buffer resource (uniform base in SGPRs, 32-bit per-lane byte
  // offsets): 64-bit per-lane pointers, hoisted for every slice, were spilled to scratch
  const __amdgpu_buffer_rsrc_t wrs1 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w1, (short)0, K * C * C * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs2 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w2, (short)0, K * C * C * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.B * T * C * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc((void*)(a.acc ? a.acc : a.x), (short)0,
                                                                       a.B * T * C * 2, 0x00020000);
  int a_off[NI];  // bytes
#pragma unroll
  for (int i = 0; i < NI; ++i) a_off[i] = 2 * ((cw0 + 16 * (lr >> 2) + 4 * i + (lr & 3)) * C + 8 * lq);
  Frag<bf16_t> aq[RA][NI];               // ring of A sets (set = slice % RA)
  auto a_load = [&](int gs, Frag<bf16_t> (&dst)[NI]) {  // gs: slice index over (P1, P2) = [0, 2 NS)
    const int ph = gs >= NS;
    const int s = gs - ph * NS;
    const int c = s / K, k = s - c * K;
    const int so = 2 * (k * (C * C) + c * 32);
#pragma unroll
    for (int i = 0; i < NI; ++i)
      dst[i].v = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ph ? wrs2 : wrs1, a_off[i], so, 0));
  };

  // ---- window of a tile, plane c, through registers: vector v = tid + NT u -> row v / 4, chunk v & 3
  u32x4 wreg[WV];
  auto win_load = [&](int tv, int c, int b, int R0) {
#pragma unroll
    for (int u = 0; u < WV; ++u) {
      const int v = tv + NT * u;
      const int t = min(max(R0 + (v >> 2), 0), T - 1);
      wreg[u] = __builtin_amdgcn_raw_buffer_load_b128(xrs, 2 * ((b * T + t) * C + 8 * (v & 3)), 64 * c, 0);
    }
  };
  auto win_store = [&](int tv, int c, int R0) {  // leaky ReLU, rows outside [0, T) -> 0 (c1's padding)
#pragma unroll
    for (int u = 0; u < WV; ++u) {
      const int v = tv + NT * u;
      const int t = R0 + (v >> 2);
      const u32x4 q = lrelu8_pk(wreg[u], slope);
      *reinterpret_cast<u32x4*>(act + c * PLANE_E + rb_off(v >> 2, v & 3, 2)) =
          (t >= 0 && t < T) ? q : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto tile_geo = [&](int tl, int& b, int& t0) {
    b = tl / a.tiles_per_b;
    t0 = (tl - b * a.tiles_per_b) * BT;
  };

  // prologue: the first tile's window, the first A sets
  {
    int b, t0;
    tile_geo(tile, b, t0);
    const int R0 = t0 - h2 - h1;
#pragma unroll
    for (int c = 0; c < NC - 1; ++c) {
      win_load(tid, c, b, R0);
      win_store(tid, c, R0);
    }
    win_load(tid, NC - 1, b, R0);  // stored at the first P1's slice 2, as in every later tile
  }
#pragma unroll
  for (int p = 0; p < PF; ++p) a_load(p, aq[p % RA]);
  __syncthreads();

  int titer = 0;
  f32x4 acc[NI][JW];
  // residual rows in the lane's epilogue layout: x (requested two slices before P1 ends, added in
  // P2's accumulator init), then the MRF accumulator (requested two slices before P2 ends, added in
  // the y epilogue) -- both where the accumulators pass through VALU anyway (a separate pass over
  // the AGPR-resident accumulators cost ~1300 cycles per 4-row chunk)
  u32x4 rx[JW][NH];

  for (; tile < tile_end; ++tile) {
    // the lane's indices, re-derived each tile from an opaque copy of the thread id: hoisted out of
    // the tile loop, the per-lane addresses of the epilogues, window and residual rows (dozens of
    // them) were spilled to scratch
    int tv = tid;
    asm volatile("" : "+v"(tv));
    const int lr = tv & 15, lq = (tv & 63) >> 4;
    const int n0 = cw0 + 16 * lq;
    const int brow0 = wt * RW + lr;
    int b, t0;
    tile_geo(tile, b, t0);
    const int R0 = t0 - h2 - h1;
    int nb, nt0;
    tile_geo(min(tile + 1, a.ntiles - 1), nb, nt0);  // next window (a valid dummy after the run)
    const int nR0 = nt0 - h2 - h1;

#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + n0 + 4 * i);
#pragma unroll
      for (int j = 0; j < JW; ++j) acc[i][j] = bv;
    }

    auto res_load = [&](const __amdgpu_buffer_rsrc_t& rs) {
#pragma unroll
      for (int j = 0; j < JW; ++j) {
        const int pos = min(t0 + wt * RW + 16 * j + lr, T - 1);
        const int off = 2 * ((b * T + pos) * C + n0);
#pragma unroll
        for (int h = 0; h < NH; ++h) rx[j][h] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 16 * h, 0);
      }
    };
    // one phase: NS slices in groups of 4 (A set = slice & 3 static), B rows streamed D ahead
    // through a ring of RB fragments (slot = row % RB; JW % RB == 0 keeps slices aligned)
    auto phase = [&](const int ph) {
      const int step = ph ? 1 : dil;
      auto boff = [&](int s) {
        const int c = s / K, k = s - c * K;
        return c * PLANE_E + rb_off(brow0 + k * step, lq, 2);
      };
      Frag<bf16_t> bq[RB];
      {
        const int o = boff(0);
#pragma unroll
        for (int r = 0; r < D; ++r) bq[r].load(act + o + 16 * r * 32);
      }
      // the group holding the residual loads (P1's last) and the one holding the accumulator rows
      // (P2's first) are peeled out of the loop: a value a loop iteration may define is live around
      // the whole loop, and 96 registers of residual rows through a phase spilled
      auto group = [&](const int g4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int s = g4 * 4 + u;
#ifdef VO_ABLATIONS
          if constexpr (STAMP) {
            if (blockIdx.x < 8 && titer >= 1 && titer <= 2 && wave == 0 && lane == 0)
              g_rs_stamp[((blockIdx.x * 2 + titer - 1) * 2 + ph) * 64 + s] = __builtin_amdgcn_s_memtime();
          }
#endif
          // A set of slice s + PF (the stream runs on into the next phase / tile), requested BEFORE
          // this slice's window / residual loads: vmcnt retires in order, so the wait for an A set
          // would otherwise also wait for every HBM load issued ahead of it
          {
            const int gs = ph * NS + s + PF;
            a_load(gs >= 2 * NS ? gs - 2 * NS : gs, aq[(u + PF) % RA]);
          }
          // events at slice boundaries (uniform branches)
          if (ph == 0) {
            if (s == 2) win_store(tv, NC - 1, R0);  // the late plane of this tile's window
            // plane NC - 1 written by every wave: before slice 3K - 1, whose B stream already reads
            // slice 3K's first rows
            if (s == (NC - 1) * K - 1) __syncthreads();
          } else {
#pragma unroll
            for (int c = 0; c < NC - 1; ++c) {
              if (s == (c + 1) * K) {  // every wave is past T1 plane c: load the next window's plane c
                __syncthreads();
                win_load(tv, c, nb, nR0);
              }
              if (s == (c + 1) * K + 2) win_store(tv, c, nR0);
            }
            if (HAS_ACC && s == NS - 2) res_load(ars);
          }
          if (ph == 0 && s == NS - 2) res_load(xrs);
          const int o_cur = boff(s);
          const int o_nxt = s + 1 < NS ? boff(s + 1) : o_cur;
          // the schedule is pinned (sched_barrier): hipcc otherwise sinks each fragment read to its
          // first use and waits for it there -- with one wave per SIMD nothing hides that latency
#pragma unroll
          for (int j = 0; j < JW; ++j) {
            const int jr = j + D;  // the row fragment D ahead: this slice's or the next one's
            __builtin_amdgcn_sched_barrier(0);
            if (jr < JW) bq[jr % RB].load(act + o_cur + 16 * jr * 32);
            else if (s + 1 < NS) bq[jr % RB].load(act + o_nxt + 16 * (jr - JW) * 32);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < NI; ++i) acc[i][j] = mfma(aq[u % RA][i], bq[j % RB], acc[i][j]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      // the last group (residual loads) is peeled out of the loop: a value a loop iteration may
      // define is live around the whole loop
      for (int g4 = 0; g4 < NS / 4 - 1; ++g4) group(g4);
      group(NS / 4 - 1);
    };

    phase(0);
    __syncthreads();  // every wave is past its window reads
    // P1 epilogue: T1 = lrelu(acc) over the window, zero outside [0, T) (c2's padding)
    {
      const bool interior = t0 - h2 >= 0 && t0 - h2 + R1 <= T;
#pragma unroll
      for (int j = 0; j < JW; ++j) {
        const int r = wt * RW + 16 * j + lr;
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
          const int ch = n0 + 8 * h;
          *reinterpret_cast<u32x4*>(act + (ch >> 5) * PLANE_E + rb_off(r, (ch & 31) >> 3, 2)) = u32x4{w[0], w[1], w[2], w[3]};
        }
      }
    }
    // P2 accumulators start at b2 + x
#pragma unroll
    for (int j = 0; j < JW; ++j)
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        float xf[8];
        unpack8(rx[j][h], xf);
#pragma unroll
        for (int e8 = 0; e8 < 8; ++e8) {
          const int i = 2 * h + e8 / 4, e = e8 & 3;
          acc[i][j][e] = sbias[C + n0 + 4 * i + e] + xf[e8];
        }
      }
    __syncthreads();  // T1 complete

    phase(1);
    __syncthreads();  // every wave is past T1: the last plane's next window may be loaded
    win_load(tv, NC - 1, nb, nR0);  // written at the next P1's slice 2 (P1 reads plane NC - 1 last)

    // y = acc * out_scale; rows past the tile / past T fall outside the buffer resource (dropped)
    const int valid = min(BT, T - t0);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.y + ((int64_t)b * T + t0) * C), (short)0, valid * C * (int)sizeof(bf16_t), 0x00020000);
#pragma unroll
    for (int j = 0; j < JW; ++j) {
      const int r = wt * RW + 16 * j + lr;
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        uint32_t w[4];
        float af8[8];
        if constexpr (HAS_ACC) unpack8(rx[j][h], af8);
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          const int e = 2 * e2;
          float q0 = acc[2 * h + e / 4][j][e & 3] * a.out_scale, q1 = acc[2 * h + (e + 1) / 4][j][(e + 1) & 3] * a.out_scale;
          if constexpr (HAS_ACC) {
            q0 += af8[e];
            q1 += af8[e + 1];
          }
          w[e2] = pk_bf16(q0, q1);
        }
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{w[0], w[1], w[2], w[3]}, yrs,
                                               (r * C + n0 + 8 * h) * (int)sizeof(bf16_t), 0, 0);
      }
    }
#ifdef VO_ABLATIONS
    if constexpr (STAMP) {  // slot 63 of phase 1: tile end
      if (blockIdx.x < 8 && titer >= 1 && titer <= 2 && wave == 0 && lane == 0)
        g_rs_stamp[((blockIdx.x * 2 + titer - 1) * 2 + 1) * 64 + 63] = __builtin_amdgcn_s_memtime();
    }
#endif
    ++titer;
  }
}

template <int K, bool HAS_ACC, int JW, int PF, int D, int NWV = 4, bool STAMP = false>
static int rs_launch(RsArgs a, int B, hipStream_t st) {
  using Gm = RsGeom<JW, NWV>;
  constexpr int h2 = (K - 1) / 2;
  constexpr int BT = Gm::R1 - 2 * h2;
  a.tiles_per_b = (a.T + BT - 1) / BT;
  a.ntiles = a.tiles_per_b * B;
  auto kern = mrf_pair_rs_kernel<K, HAS_ACC, JW, PF, D, NWV, STAMP>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)Gm::LDS);
    attr = true;
  }
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  const int grid = (int)std::min<int64_t>((int64_t)cus, a.ntiles);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NWV * 64), Gm::LDS, st, a);
  VO_RETURN_LAUNCH();
}

}  // namespace vo

using namespace vo;

// C = 128, K in {7, 11}, dil * (K - 1) <= 64, out_scale > 0.  *handled = 0 when not covered.
int vo_pair_rs_try(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                   const void* acc, int B, int T, int C, int K, int dil, float slope, float out_scale, int cfg,
                   hipStream_t st, int* handled) {
  *handled = 0;
  if (C != 128 || (K != 7 && K != 11) || dil < 1 || dil * (K - 1) > 64 || !(out_scale > 0.f) ||
      (int64_t)B * T * C * 2 >= ((int64_t)1 << 31))  // 32-bit buffer offsets
    return VO_OK;
  *handled = 1;
  RsArgs a;
  a.B = B;
  a.x = (const bf16_t*)x; a.w1 = (const bf16_t*)w1; a.b1 = b1; a.w2 = (const bf16_t*)w2; a.b2 = b2;
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)acc;
  a.T = T; a.dil = dil; a.slope = slope; a.out_scale = out_scale; a.inv_scale = 1.f / out_scale;
  a.tiles_per_b = a.ntiles = 0;
#ifdef VO_ABLATIONS
  if (cfg == 9) return K == 7 ? rs_launch<7, true, 12, 1, 5, 4, true>(a, B, st) : rs_launch<11, true, 12, 1, 5, 4, true>(a, B, st);
  if (cfg == 10) return K == 7 ? rs_launch<7, true, 6, 1, 5, 8, true>(a, B, st) : rs_launch<11, true, 6, 1, 5, 8, true>(a, B, st);
  if (cfg == 1) {  // B rows 3 ahead (default 5)
    if (K == 7) return acc ? rs_launch<7, true, 12, 1, 3>(a, B, st) : rs_launch<7, false, 12, 1, 3>(a, B, st);
    return acc ? rs_launch<11, true, 12, 1, 3>(a, B, st) : rs_launch<11, false, 12, 1, 3>(a, B, st);
  }
#endif
  if (cfg == 2) {  // two waves per SIMD: 8 waves of 64 channels x 96 rows
    if (K == 7) return acc ? rs_launch<7, true, 6, 1, 5, 8>(a, B, st) : rs_launch<7, false, 6, 1, 5, 8>(a, B, st);
    return acc ? rs_launch<11, true, 6, 1, 5, 8>(a, B, st) : rs_launch<11, false, 6, 1, 5, 8>(a, B, st);
  }
  if (K == 7) return acc ? rs_launch<7, true, 12, 1, 5>(a, B, st) : rs_launch<7, false, 12, 1, 5>(a, B, st);
  return acc ? rs_launch<11, true, 12, 1, 5>(a, B, st) : rs_launch<11, false, 12, 1, 5>(a, B, st);
}

#endif  // VO_ABLATIONS
