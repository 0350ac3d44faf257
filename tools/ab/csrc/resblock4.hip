// Fused HiFi-GAN ResBlock1 pair, version 3 (round 3): narrow MRF stages (C = 32 / 64, k = 7 / 11)
//   y = (x + c2(lrelu(c1_d(lrelu(x), slope), slope))) * out_scale (+ acc)
// (scripts/hifigan/models.py:96-103, one (c1, c2) iteration; the Generator's MRF sum and
// 1/num_kernels scale, models.py:155-160, in the epilogue).
//
// Why a third version: the v1 / v2 pairs run ONE 8-wave workgroup per CU, so every exposed
// global round trip -- the next tile's window, the residual and MRF-accumulator rows of the
// epilogue -- stalls the whole CU, and the synchronous epilogues never overlap MFMA work.  At
// C = 32 / 64 the pairs ran at 2.6-3.8 TB/s and 0.23-0.39 of the MFMA peak, bound by neither.
// Here two 4-wave workgroups share a CU (LDS <= 80 KiB each, 2 waves per SIMD) and drift apart:
// while one waits for its window or its epilogue rows the other runs MFMAs.  Per workgroup:
//  * the tile's input window lands in LDS by LDS-DMA (global_load_lds_dwordx4, no VGPR
//    staging; the row swizzle on the source address), issued for the NEXT tile right after a
//    tile's last barrier -- before its y stores, so the wait for it leaves the stores in flight;
//  * the residual x rows are read from the raw window in LDS (no second global read), then the
//    window is lrelu'd in place (rows outside [0, T) zeroed: c1's zero padding);
//  * T1 = lrelu(c1 + b1) overwrites the dead window (in place), c2 reads it;
//  * weights: all 2K taps resident in LDS (C = 32) or streamed one group of TG taps at a time
//    through a double buffer by LDS-DMA (C = 64);
//  * the MRF accumulator rows are requested in the last c2 group and consumed by the epilogue.
// Each wave owns all C output channels of 16 NJ consecutive rows (NI = C / 16 co tiles).

// Measured-and-dropped (round 3): compiled only into the A/B library (make abl, -DVO_ABLATIONS).
#ifdef VO_ABLATIONS
#include <algorithm>
#include <type_traits>

#include "mrf_common.h"  // visual_onoma_to_wave_amd/csrc (make abl adds it to the include path)

namespace vo {

struct Pair3Args {
  const bf16_t* x; const bf16_t* w1; const float* b1; const bf16_t* w2; const float* b2;
  bf16_t* y; const bf16_t* acc;
  int T, dil, tiles_per_b, ntiles;
  float slope, out_scale;
};

constexpr int PAIR3_DMAX = 5;

typedef __attribute__((address_space(3))) void p3_lds_void;
typedef const __attribute__((address_space(1))) void p3_g_void;

template <int C, int NJ, int K, bool RESW, int TG>
__global__ void __launch_bounds__(256, 2) mrf_pair3_kernel(Pair3Args a) {
  constexpr int NW = 4;                  // waves per workgroup (two workgroups per CU)
  constexpr int NT = NW * 64;
  constexpr int NC = C / 32;             // 32-channel planes
  constexpr int NI = C / 16;             // co tiles per wave (all channels)
  constexpr int R1 = NW * 16 * NJ;       // c1 rows per tile
  constexpr int SHW = NI >= 8 ? 5 : (NI == 4 ? 4 : 3);  // log2(4 * NI): weight-row swizzle
  constexpr int H2 = (K - 1) / 2;
  constexpr int WRMAX = R1 + 2 * PAIR3_DMAX * H2;       // window rows at the largest dilation
  constexpr int WR = ((WRMAX > R1 + 16 ? WRMAX : R1 + 16) + 63) / 64 * 64;  // region rows / plane
  constexpr int TAPV = C * NC * 4;       // 16-byte vectors per weight tap
  constexpr int TAPE = NC * C * 32;      // LDS elements per weight tap
  constexpr int NG = RESW ? 1 : (K + TG - 1) / TG;  // streamed weight groups per conv
  constexpr int GE = TG * TAPE;          // LDS elements per group buffer
  constexpr int GLN = RESW ? 1 : TG * TAPV / NT;    // weight DMA instructions per wave per group
  static_assert(RESW || (TG * TAPV) % NT == 0, "weight groups split into whole wave-KiB DMA pieces");
  constexpr int WPC = NC * WR / 16;      // window DMA pieces (16 rows x one plane, 1 KiB)
  static_assert(WPC % NW == 0, "window pieces split evenly over the waves");
  constexpr int WPW = WPC / NW;          // window pieces per wave
  constexpr int NH = NI / 2;             // 8-channel vectors per lane in epilogue layout
  constexpr int NST = NJ * NH;           // y stores per wave per tile
  constexpr bool XL = RESW;              // residual from the raw window in LDS (C = 32), else from global
  constexpr int NACC = (XL ? 1 : 2) * NJ * NH;  // epilogue row loads per wave per tile
  constexpr int BT = R1 - 2 * H2;        // output rows per tile
  constexpr int LV = NC * WR * 4 / NT;   // lrelu-pass vectors per thread
  static_assert((NC * WR * 4) % NT == 0, "lrelu pass splits evenly");

  const int dil = a.dil, T = a.T;
  const int h1 = dil * H2;
  const int win_rows = R1 + 2 * h1;
  const float slope = a.slope;

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* reg = reinterpret_cast<bf16_t*>(smem_raw);    // [NC][WR][32]: raw window -> lrelu'd -> T1
  bf16_t* wls = reg + NC * WR * 32;                      // RESW: [2K] taps; else [2][GE]
  float* sbias = reinterpret_cast<float*>(wls + (RESW ? 2 * K * TAPE : 2 * GE));  // [b1 | b2]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int lr = lane & 15, lq = lane >> 4;
  const int n0 = NI * 4 * lq;            // epilogue: this lane's 4*NI contiguous output channels

  const int G = gridDim.x;
  int tile = (int)(((int64_t)blockIdx.x * a.ntiles) / G);
  const int tile_end = (int)(((int64_t)(blockIdx.x + 1) * a.ntiles) / G);
  if (tile >= tile_end) return;          // uniform per workgroup

  for (int i = tid; i < 2 * C; i += NT) sbias[i] = i < C ? a.b1[i] : a.b2[i - C];

  // ---- weights: LDS slot p of a tap holds (plane pl, row co, chunk q' = q ^ swz(co)); the
  // swizzle moves to the DMA source address (global_load_lds writes lane-linear LDS)
  int gl_off[GLN];
#pragma unroll
  for (int s = 0; s < GLN; ++s) {
    const int p = (s * NW + wave) * 64 + lane;
    const int t = p / TAPV, vv = p - t * TAPV;
    const int pl = vv / (C * 4), rem = vv - pl * C * 4;
    const int co = rem >> 2, q = (rem & 3) ^ ((co >> (SHW - 1)) & 2);
    gl_off[s] = t * (C * C) + co * C + pl * 32 + q * 8;
  }
  auto load_group = [&](int q, int buf) {  // streamed group q in [0, 2 NG): conv q / NG, taps (q % NG) * TG + t
    const int ph = q >= NG;
    const int k0 = (q - ph * NG) * TG;
    const bf16_t* W = (ph ? a.w2 : a.w1) + k0 * (C * C);
#pragma unroll
    for (int s = 0; s < GLN; ++s) {
      // taps past K (last group, K % TG != 0) re-read in-range taps: their MFMAs are skipped
      const int off = min(gl_off[s], (K - 1 - k0) * (C * C) + (gl_off[s] % (C * C)));
      __builtin_amdgcn_global_load_lds((p3_g_void*)(W + off), (p3_lds_void*)(wls + buf * GE + (s * NW + wave_u) * 512),
                                       16, 0, 0);
    }
  };
  if constexpr (RESW) {  // both convs, all taps, once per kernel (register staged, swizzled)
    const int total = 2 * K * TAPV;
    for (int v = tid; v < total; v += NT) {
      const int ck = v / TAPV, vv = v - ck * TAPV;  // ck = conv * K + tap
      const bf16_t* W = ck >= K ? a.w2 + (int64_t)(ck - K) * C * C : a.w1 + (int64_t)ck * C * C;
      const int co = vv / (NC * 4), rem = vv - co * NC * 4;
      *reinterpret_cast<u32x4*>(wls + ck * TAPE + (rem >> 2) * C * 32 + rb_off(co, rem & 3, SHW)) =
          *reinterpret_cast<const u32x4*>(W + vv * 8);
    }
  } else {
    load_group(0, 0);
  }

  // ---- window by LDS-DMA: piece pc = rows [16 rb, 16 rb + 16) of plane pl; lane l writes LDS row
  // 16 rb + l / 4, slot l % 4, which holds chunk (l % 4) ^ swz(row) of that row (rb_off's swizzle)
  const int wrow = lane >> 2, wq = (lane & 3) ^ ((wrow >> 1) & 2);  // swz(16 rb + wrow) = swz(wrow)
  auto issue_window = [&](int tl) {
    const int b = tl / a.tiles_per_b;
    const int R0 = (tl - b * a.tiles_per_b) * BT - H2 - h1;
    const bf16_t* xb = a.x + (int64_t)b * T * C + wq * 8;
#pragma unroll
    for (int s = 0; s < WPW; ++s) {
      const int pc = s * NW + wave_u;            // wave-uniform piece
      const int pl = pc / (WR / 16), rb = pc - pl * (WR / 16);
      const int t = min(max(R0 + rb * 16 + wrow, 0), T - 1);  // clamped; zeroed by the lrelu pass
      __builtin_amdgcn_global_load_lds((p3_g_void*)(xb + (int64_t)t * C + pl * 32),
                                       (p3_lds_void*)(reg + pl * WR * 32 + rb * 512), 16, 0, 0);
    }
  };

  int a_off[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) a_off[i] = rb_off(NI * 4 * (lr >> 2) + 4 * i + (lr & 3), lq, SHW);
  const int brow0_ = wave * 16 * NJ + lr;

  issue_window(tile);
  f32x4 acc[NI][NJ];
  int gc = 0;  // streamed groups consumed (double-buffer parity)

  auto lane_bias = [&](int which, float (&bz)[8 * NH]) {
    const float4* bp = reinterpret_cast<const float4*>(sbias + which * C + n0);
#pragma unroll
    for (int u = 0; u < 2 * NH; ++u) {
      const float4 v = bp[u];
      bz[4 * u] = v.x; bz[4 * u + 1] = v.y; bz[4 * u + 2] = v.z; bz[4 * u + 3] = v.w;
    }
  };
  auto tap = [&](const bf16_t* wt_, const bf16_t* src, int row) {
    Frag<bf16_t> af[NI], bfr[NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i) af[i].load(wt_ + a_off[i]);
    const int boff = rb_off(row, lq, 2);
#pragma unroll
    for (int j = 0; j < NJ; ++j) bfr[j].load(src + boff + 16 * j * 32);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma(af[i], bfr[j], acc[i][j]);
    __builtin_amdgcn_sched_barrier(0);
  };

  // first tile: the window (and the first weight group / resident weights) before anything reads it
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (; tile < tile_end; ++tile) {
    const int b = tile / a.tiles_per_b;
    const int t0 = (tile - b * a.tiles_per_b) * BT;
    const bool has_next = tile + 1 < tile_end;
    int brow0 = brow0_;
    asm volatile("" : "+v"(brow0));

    // ---- residual rows (raw x at window row r + H2 + h1) into registers, epilogue layout: from the
    // raw window in LDS (C = 32), or -- where registers are short (C = 64) -- from global with the
    // accumulator rows in the last c2 group (L2 hits: this tile's window brought them in)
    u32x4 xres[NJ][NH];
    if constexpr (XL) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = wave * 16 * NJ + 16 * j + lr + H2 + h1;
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          const int ch = n0 + 8 * h;
          xres[j][h] = *reinterpret_cast<const u32x4*>(reg + (ch >> 5) * WR * 32 + rb_off(r, (ch & 31) >> 3, 2));
        }
      }
      lds_barrier();  // every residual read done before the window is rewritten in place
    }
    // ---- lrelu the window in place; rows outside [0, T) -> 0 (c1's zero padding)
    {
      const int R0 = t0 - H2 - h1;
#pragma unroll
      for (int s = 0; s < LV; ++s) {
        const int v = tid + s * NT;
        const int pl = v / (WR * 4), rem = v - pl * WR * 4;
        const int r = rem >> 2;
        bf16_t* p = reg + pl * WR * 32 + rem * 8;  // lane-linear slot: the swizzle is a permutation within the row
        const int t = R0 + r;
        const u32x4 u = lrelu8(*reinterpret_cast<const u32x4*>(p), slope);
        *reinterpret_cast<u32x4*>(p) = (t >= 0 && t < T && r < win_rows) ? u : u32x4{0u, 0u, 0u, 0u};
      }
    }
    lds_barrier();

#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // ---- P1: c1 over the lrelu'd window
    if constexpr (RESW) {
#pragma unroll 1
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int c = 0; c < NC; ++c) tap(wls + k * TAPE + c * C * 32, reg + c * WR * 32, brow0 + k * dil);
      lds_barrier();  // every wave past its window reads: T1 overwrites them
    } else {
#pragma unroll 1
      for (int g = 0; g < NG; ++g) {
        load_group(g + 1, (gc + 1) & 1);  // g = NG - 1: P2's first group
        const bf16_t* wb = wls + (gc & 1) * GE;
#pragma unroll
        for (int t = 0; t < TG; ++t) {
          if (g * TG + t >= K) continue;
#pragma unroll
          for (int c = 0; c < NC; ++c) tap(wb + t * TAPE + c * C * 32, reg + c * WR * 32, brow0 + (g * TG + t) * dil);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next group's DMA landed (this wave's part)
        lds_barrier();
        ++gc;
      }
    }

    // ---- P1 epilogue: T1 = lrelu(acc + b1) over the dead window; rows outside [0, T) -> 0
    {
      float bz[8 * NH];
      lane_bias(0, bz);
      const bool interior = t0 - H2 >= 0 && t0 - H2 + R1 <= T;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = wave * 16 * NJ + 16 * j + lr;
        const int pos = t0 - H2 + r;
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

    // ---- P2: c2 over T1; the accumulator rows are requested with the last group
    u32x4 ares[NJ][NH];
    const bf16_t* accp = a.acc ? a.acc : a.x;  // loaded either way (no branch), added only with acc
    auto load_acc = [&]() {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int pos = min(t0 + wave * 16 * NJ + 16 * j + lr, T - 1);
        const int64_t off = ((int64_t)b * T + pos) * C + n0;
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          if constexpr (!XL) xres[j][h] = *reinterpret_cast<const u32x4*>(a.x + off + 8 * h);
          ares[j][h] = *reinterpret_cast<const u32x4*>(accp + off + 8 * h);
        }
      }
    };
    if constexpr (RESW) {
      load_acc();
      const bf16_t* wb = wls + K * TAPE;
#pragma unroll 1
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int c = 0; c < NC; ++c) tap(wb + k * TAPE + c * C * 32, reg + c * WR * 32, brow0 + k);
      lds_barrier();  // T1 reads done: the region takes the next window
    } else {
#pragma unroll 1
      for (int g = 0; g < NG - 1; ++g) {
        load_group(NG + g + 1, (gc + 1) & 1);
        const bf16_t* wb = wls + (gc & 1) * GE;
#pragma unroll
        for (int t = 0; t < TG; ++t) {
          if (g * TG + t >= K) continue;
#pragma unroll
          for (int c = 0; c < NC; ++c) tap(wb + t * TAPE + c * C * 32, reg + c * WR * 32, brow0 + g * TG + t);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        ++gc;
      }
      {  // last group: the next tile's first weight group, then the accumulator rows
        constexpr int g = NG - 1;
        load_group(0, (gc + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
        load_acc();
        __builtin_amdgcn_sched_barrier(0);
        const bf16_t* wb = wls + (gc & 1) * GE;
#pragma unroll
        for (int t = 0; t < TG; ++t) {
          if (g * TG + t >= K) continue;
#pragma unroll
          for (int c = 0; c < NC; ++c) tap(wb + t * TAPE + c * C * 32, reg + c * WR * 32, brow0 + g * TG + t);
        }
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NACC) : "memory");  // the weight DMA landed; acc may fly
        lds_barrier();
        ++gc;
      }
    }

    // ---- epilogue: y = (c2 + b2 + x) * out_scale (+ acc).  The loaded rows are consumed first
    // (empty asm uses: hipcc waits for them here), THEN the next window's DMA is issued -- an
    // ordinary load used after a global_load_lds would make hipcc drain the DMA at that use --
    // and the y stores go out after it (vmcnt retires in order: the wait for the window at the
    // tile's end leaves the stores in flight)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        asm volatile("" ::"v"(ares[j][h]));
        if constexpr (!XL) asm volatile("" ::"v"(xres[j][h]));
      }
    if (has_next) issue_window(tile + 1);  // uniform; the region's T1 reads ended at the last barrier
    float b2z[8 * NH];
    lane_bias(1, b2z);
    const int valid = min(BT, T - t0);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.y + ((int64_t)b * T + t0) * C), (short)0, valid * C * (int)sizeof(bf16_t), 0x00020000);
    auto epilogue = [&](auto with_acc) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = wave * 16 * NJ + 16 * j + lr;
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
    if (has_next) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");  // this wave's window pieces landed
      lds_barrier();
    }
  }
}

template <int C, int NJ, int K, bool RESW, int TG>
static int pair3_launch(Pair3Args a, int B, hipStream_t st) {
  constexpr int R1 = 4 * 16 * NJ;
  constexpr int H2 = (K - 1) / 2;
  constexpr int WRMAX = R1 + 2 * PAIR3_DMAX * H2;
  constexpr int WR = ((WRMAX > R1 + 16 ? WRMAX : R1 + 16) + 63) / 64 * 64;
  constexpr int BT = R1 - 2 * H2;
  a.tiles_per_b = (a.T + BT - 1) / BT;
  a.ntiles = a.tiles_per_b * B;
  const size_t wel = RESW ? 2 * (size_t)K * C * C : 2 * (size_t)TG * C * C;
  const size_t lds = ((size_t)WR * C + wel) * sizeof(bf16_t) + 2 * C * sizeof(float);
  if (lds > 80 * 1024) {
    vo_set_error("resblock_pair (v3): LDS %zu B exceeds 80 KiB (two workgroups per CU)", lds);
    return VO_ERR_INVALID;
  }
  auto kern = mrf_pair3_kernel<C, NJ, K, RESW, TG>;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, lds) != hipSuccess || per_cu < 1) per_cu = 1;
  const int grid = (int)std::min<int64_t>((int64_t)cus * per_cu, a.ntiles);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), lds, st, a);
  VO_RETURN_LAUNCH();
}

}  // namespace vo

using namespace vo;

// Entry from vo_resblock_pair (resblock.hip): *handled = 1 when this kernel covers the shape
// (C = 32 / 64, K = 7 / 11, dilation <= 5) for the selected pair_cfg.
int vo_pair3_try(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y,
                 const void* acc, int B, int T, int C, int K, int dil, float slope, float out_scale, int cfg,
                 hipStream_t st, int* handled) {
  *handled = 0;
  if (!((C == 64 || C == 32) && (K == 7 || K == 11) && dil >= 1 && dil <= PAIR3_DMAX)) return VO_OK;
  Pair3Args a;
  a.x = (const bf16_t*)x; a.w1 = (const bf16_t*)w1; a.b1 = b1; a.w2 = (const bf16_t*)w2; a.b2 = b2;
  a.y = (bf16_t*)y; a.acc = (const bf16_t*)acc;
  a.T = T; a.dil = dil; a.slope = slope; a.out_scale = out_scale;
  a.tiles_per_b = a.ntiles = 0;
  *handled = 1;
  if (C == 64) {  // 256-row tiles, one-tap weight groups streamed by LDS-DMA (cfg 41: two-tap groups)
    if (cfg == 41) {
      if (K == 7) return pair3_launch<64, 4, 7, false, 2>(a, B, st);
      return pair3_launch<64, 4, 11, false, 2>(a, B, st);
    }
    if (K == 7) return pair3_launch<64, 4, 7, false, 1>(a, B, st);
    return pair3_launch<64, 4, 11, false, 1>(a, B, st);
  }
  // C = 32: both convs resident; 448-row tiles (k = 11: 76 KiB), 512-row tiles at k = 7
  if (K == 7) return pair3_launch<32, 8, 7, true, 1>(a, B, st);
  return pair3_launch<32, 7, 11, true, 1>(a, B, st);
}
#endif  // VO_ABLATIONS
