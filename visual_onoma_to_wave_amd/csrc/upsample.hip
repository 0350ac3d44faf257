// Polyphase ConvTranspose1d for the narrow HiFi-GAN upsamplers (ups2: 128 -> 64, ups3: 64 -> 32,
// kernel 4, stride 2; scripts/hifigan/models.py:139-141,153-154 with the lrelu(0.1) in front).
//
// In polyphase form (conv1d.hip header) the upsampler is a K = 2, pad = 1 conv producing
// s * C_out phase columns per input step m:  P[m][n] = sum_ci W[0][n][ci] x[m-1][ci] +
// W[1][n][ci] x[m][ci], column n = r * C_out + co landing at output time m * s + r - p.
// The reduction is only 2 * Ci = 128 / 256 deep, so the generic tiled conv spends a tile's
// life on its prologue (window + weight staging, one HBM round trip, then a handful of
// MFMAs) with one or two workgroups per CU: 225 / 182 us for 537 MB each (ups2 / ups3 at
// B = 32 x 512 frames), 2.4 / 2.9 TB/s.  This kernel: 146 / 125 us, 3.7 / 4.3 TB/s.
//
// This kernel is persistent and streams: the packed weights (16 / 64 KB) are copied to LDS
// once per workgroup, then every wave walks a contiguous run of units of 16 * NJ input steps.
// The x operand never touches LDS: the MFMA B fragment of lane (lq, lr) is the 16 bytes
// x[m0 + lr - 1 + tap][32 ks + 8 lq ..], i.e. 16 consecutive rows read as 64-byte row
// segments straight into registers; only the tap-1 rows are loaded, the tap-0 fragment is a
// DPP lane rotate of them (ups_kernel).  HBM traffic is x once + y once.  The next unit's
// fragments are in flight while the current unit's MFMAs and stores run.  The accumulation order
// (32-channel chunk outer, tap inner) and the f32 -> bf16 roundings (lrelu before the MFMA,
// bias add after) are those of conv1d_kernel, so the result is bit-identical to it.
//
// A row index lr of i-tile i is channel 4 NI (lr >> 2) + 4 i + (lr & 3): after the MFMA, lane
// (g, lr) holds the 4 NI consecutive columns [4 NI g, 4 NI g + 4 NI) of step m0 + lr, all in
// one phase (4 NI divides C_out), written as one contiguous run of the output row.
#include "mrf_common.h"

namespace vo {

constexpr int ups_log2(int v) { return v <= 1 ? 0 : 1 + ups_log2(v / 2); }

struct UpsArgs {
  const bf16_t* x;
  const bf16_t* w;     // [2][NC][CI]
  const float* bias;   // [C_out] or null
  bf16_t* y;           // (B, up_tout, C_out)
  int64_t xbs, ybs;
  int T_in, up_tout, up_stride, up_pad, cout;
  int nblk, units;
  float slope;         // pre-lrelu slope (1 = none)
};

// DPP row rotate by one lane (row_ror:1): lane lr of each 16-lane row receives lane
// (lr - 1) mod 16 of the same row
__device__ __forceinline__ u32x4 ror1(u32x4 v) {
  return u32x4{(uint32_t)__builtin_amdgcn_mov_dpp((int)v.x, 0x121, 0xf, 0xf, false),
               (uint32_t)__builtin_amdgcn_mov_dpp((int)v.y, 0x121, 0xf, 0xf, false),
               (uint32_t)__builtin_amdgcn_mov_dpp((int)v.z, 0x121, 0xf, 0xf, false),
               (uint32_t)__builtin_amdgcn_mov_dpp((int)v.w, 0x121, 0xf, 0xf, false)};
}

// Each wave walks a contiguous run of units (16 NJ steps of one utterance), so only the tap-1
// rows x[m0 .. m0 + 16 NJ) are loaded: the tap-0 fragment (rows shifted by one) is the tap-1
// fragment rotated one lane down each 16-lane row, lane 0 taking the last row of the previous
// 16-row group -- of the previous unit for j = 0 (zero at an utterance start; one halo load
// for the first unit of a run).  The loop body is a compiler barrier away from the weight
// reads, so the loop-invariant LDS fragments are re-read per unit instead of being hoisted
// into registers (256 VGPRs and one wave per SIMD for CI = 128).
template <int CI, int NC, int NJ>
__global__ void __launch_bounds__(256) ups_kernel(UpsArgs a) {
  constexpr int NI = NC / 16;        // 16-column i-tiles
  constexpr int KS = CI / 32;        // 32-deep k-steps per tap
  constexpr int CPR = CI / 8;        // 16-byte chunks per weight row
  constexpr int SH = ups_log2(4 * NI);
  constexpr int MB = 16 * NJ;        // input steps per unit
  __shared__ __attribute__((aligned(16))) bf16_t wl[2 * NC * CI];
  __shared__ __attribute__((aligned(16))) float bl[NC];

  // weights -> LDS, chunk q of row n stored at chunk q ^ key(n): key spreads the 8 rows a
  // quarter-wave reads (lr = 0..7: (lr >> 2) picks the 4NI-row block, lr & 3 the row in it)
  // over 8 distinct chunks
  auto key = [](int n) { return (n & 3) | (((n >> SH) & 1) << 2); };
  for (int v = threadIdx.x; v < 2 * NC * CPR; v += 256) {
    const int row = v / CPR, q = v % CPR;  // row = tap * NC + n
    const int n = row % NC;
    const u32x4 u = *reinterpret_cast<const u32x4*>(a.w + (int64_t)v * 8);
    *reinterpret_cast<u32x4*>(wl + row * CI + 8 * (q ^ key(n))) = u;
  }
  for (int v = threadIdx.x; v < a.cout; v += 256) bl[v] = a.bias ? a.bias[v] : 0.f;

  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lq = lane >> 4;
  int a_off[NI];  // A fragment (row n(i, lr), chunk lq of k-step 0), tap 0
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int n = NI * 4 * (lr >> 2) + 4 * i + (lr & 3);
    a_off[i] = n * CI;
  }
  const int kq = key(NI * 4 * (lr >> 2) + (lr & 3));  // key(n) is the same for every i (4 i < 4 NI)

  // epilogue geometry: lane g = lq holds columns [4 NI lq, 4 NI lq + 4 NI)
  const int n0 = 4 * NI * lq;
  const int phase = n0 / a.cout;
  const int col = n0 - phase * a.cout;
  __syncthreads();

  const int wave_id = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * 4;
  const int per = (a.units + nwaves - 1) / nwaves;
  const int u_begin = wave_id * per;
  const int u_end = min(u_begin + per, a.units);
  if (u_begin >= u_end) return;

  auto unit_pos = [&](int u, int& b, int& m0) {
    b = u / a.nblk;
    m0 = (u - b * a.nblk) * MB;
  };
  auto load_unit = [&](int u, u32x4 (&dst)[NJ][KS]) {
    int b, m0;
    unit_pos(min(u, u_end - 1), b, m0);  // past the run: re-read its last unit (unused)
    const bf16_t* X = a.x + (int64_t)b * a.xbs;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int rc = min(m0 + 16 * j + lr, a.T_in - 1);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        dst[j][ks] = *reinterpret_cast<const u32x4*>(X + (int64_t)rc * CI + 32 * ks + 8 * lq);
    }
  };

  u32x4 xf[NJ][KS], xn[NJ][KS], prev[KS];
  {  // halo of the run's first unit: row m0 - 1 (lane 15 is what the rotate hands to lane 0)
    int b, m0;
    unit_pos(u_begin, b, m0);
    const bf16_t* X = a.x + (int64_t)b * a.xbs + (int64_t)max(m0 - 1, 0) * CI;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const u32x4 v = lrelu8(*reinterpret_cast<const u32x4*>(X + 32 * ks + 8 * lq), a.slope);
      prev[ks] = m0 > 0 ? v : u32x4{0u, 0u, 0u, 0u};
    }
  }
  load_unit(u_begin, xf);
  for (int u = u_begin; u < u_end; ++u) {
    asm volatile("" ::: "memory");
    load_unit(u + 1, xn);
    int b, m0;
    unit_pos(u, b, m0);
    if (m0 == 0) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) prev[ks] = u32x4{0u, 0u, 0u, 0u};
    }

    // pre-activation; rows at or past T_in are the conv's zero padding
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const bool ok = m0 + 16 * j + lr < a.T_in;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const u32x4 v = lrelu8(xf[j][ks], a.slope);
        xf[j][ks] = ok ? v : u32x4{0u, 0u, 0u, 0u};
      }
    }

    f32x4 acc[NI][NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 bt[2][NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const u32x4 own = ror1(xf[j][ks]);
        const u32x4 up = ror1(j == 0 ? prev[ks] : xf[j - 1][ks]);
        bt[0][j] = __builtin_bit_cast(bf16x8, lr == 0 ? up : own);
        bt[1][j] = __builtin_bit_cast(bf16x8, xf[j][ks]);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int ch = 8 * ((4 * ks + lq) ^ kq);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(wl + t * NC * CI + a_off[i] + ch);
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bt[t][j], acc[i][j], 0, 0, 0);
        }
      }
    }

    bf16_t* Y = a.y + (int64_t)b * a.ybs;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int m = m0 + 16 * j + lr;
      const int trow = m * a.up_stride + phase - a.up_pad;
      if (m > a.T_in || trow < 0 || trow >= a.up_tout) continue;
      bf16_t* dst = Y + (int64_t)trow * a.cout + col;
#pragma unroll
      for (int h = 0; h < NI / 2; ++h) {
        const float4 b0 = *reinterpret_cast<const float4*>(bl + col + 8 * h);
        const float4 b1 = *reinterpret_cast<const float4*>(bl + col + 8 * h + 4);
        const f32x4 p = acc[2 * h][j], q = acc[2 * h + 1][j];
        *reinterpret_cast<u32x4*>(dst + 8 * h) =
            u32x4{pack_bf16x2(p[0] + b0.x, p[1] + b0.y), pack_bf16x2(p[2] + b0.z, p[3] + b0.w),
                  pack_bf16x2(q[0] + b1.x, q[1] + b1.y), pack_bf16x2(q[2] + b1.z, q[3] + b1.w)};
      }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      prev[ks] = xf[NJ - 1][ks];
#pragma unroll
      for (int j = 0; j < NJ; ++j) xf[j][ks] = xn[j][ks];
    }
  }
}

// Wide upsamplers (ups1: 256 -> 128, k16 s8: s * C_out = 1024 phase columns) do not fit one
// LDS weight copy (1 MB).  upsw_kernel gives each persistent
// workgroup one NCB-column block (128 KB of weights in LDS) and a contiguous run of input
// steps; its 8 waves split that run.  Blocks are assigned so that the 8 column blocks of one
// run of steps sit on the same XCD (workgroup id w -> XCD w % 8): the x rows they all read
// stay in that XCD's L2.  Fragment layout, tap shift, order of accumulation and roundings
// are ups_kernel's (bit-identical to the generic tiled conv).
struct UpswArgs {
  UpsArgs u;
  int nc;       // total phase columns (s * C_out)
  int ncb_n;    // column blocks = nc / NCB
  int rgroups;  // run groups (grid = ncb_n * rgroups)
};

template <int CI, int NCB, int NJ, int NW>
__global__ void __launch_bounds__(NW * 64) upsw_kernel(UpswArgs w) {
  const UpsArgs& a = w.u;
  constexpr int NI = NCB / 16;
  constexpr int KS = CI / 32;
  constexpr int CPR = CI / 8;
  constexpr int SH = ups_log2(4 * NI);
  constexpr int MB = 16 * NJ;
  extern __shared__ __attribute__((aligned(16))) char upsw_smem[];
  bf16_t* wl = reinterpret_cast<bf16_t*>(upsw_smem);            // [2][NCB][CI]
  float* bl = reinterpret_cast<float*>(upsw_smem + 2 * NCB * CI * sizeof(bf16_t));  // [NCB]

  // workgroup -> (column block, run group): ids g, g + 8, g + 16, ... share an XCD
  const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
  const int cblk = slot % w.ncb_n;
  const int rgrp = (slot / w.ncb_n) * 8 + xcd;
  if (rgrp >= w.rgroups) return;
  const int cb = cblk * NCB;

  auto key = [](int n) { return (n & 3) | (((n >> SH) & 1) << 2); };
  for (int v = threadIdx.x; v < 2 * NCB * CPR; v += NW * 64) {
    const int row = v / CPR, q = v % CPR;  // row = tap * NCB + n (block-local)
    const int t = row / NCB, n = row % NCB;
    const u32x4 u = *reinterpret_cast<const u32x4*>(a.w + ((int64_t)t * w.nc + cb + n) * CI + 8 * q);
    *reinterpret_cast<u32x4*>(wl + row * CI + 8 * (q ^ key(n))) = u;
  }
  for (int v = threadIdx.x; v < NCB; v += NW * 64) {
    const int n = cb + v;
    bl[v] = a.bias ? a.bias[n % a.cout] : 0.f;
  }

  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lq = lane >> 4;
  int a_off[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) a_off[i] = (NI * 4 * (lr >> 2) + 4 * i + (lr & 3)) * CI;
  const int kq = key(NI * 4 * (lr >> 2) + (lr & 3));
  const int nl0 = 4 * NI * lq;                 // block-local first column of this lane
  const int phase = (cb + nl0) / a.cout;
  const int col = cb + nl0 - phase * a.cout;
  __syncthreads();

  // this wave's contiguous run of units
  const int workers = w.rgroups * NW;
  const int wid = rgrp * NW + (threadIdx.x >> 6);
  const int per = (a.units + workers - 1) / workers;
  const int u_begin = wid * per;
  const int u_end = min(u_begin + per, a.units);
  if (u_begin >= u_end) return;

  auto unit_pos = [&](int u, int& b, int& m0) {
    b = u / a.nblk;
    m0 = (u - b * a.nblk) * MB;
  };
  auto load_unit = [&](int u, u32x4 (&dst)[NJ][KS]) {
    int b, m0;
    unit_pos(min(u, u_end - 1), b, m0);
    const bf16_t* X = a.x + (int64_t)b * a.xbs;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int rc = min(m0 + 16 * j + lr, a.T_in - 1);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        dst[j][ks] = *reinterpret_cast<const u32x4*>(X + (int64_t)rc * CI + 32 * ks + 8 * lq);
    }
  };

  u32x4 xf[NJ][KS], xn[NJ][KS], prev[KS];
  {
    int b, m0;
    unit_pos(u_begin, b, m0);
    const bf16_t* X = a.x + (int64_t)b * a.xbs + (int64_t)max(m0 - 1, 0) * CI;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const u32x4 v = lrelu8(*reinterpret_cast<const u32x4*>(X + 32 * ks + 8 * lq), a.slope);
      prev[ks] = m0 > 0 ? v : u32x4{0u, 0u, 0u, 0u};
    }
  }
  load_unit(u_begin, xf);
  for (int u = u_begin; u < u_end; ++u) {
    asm volatile("" ::: "memory");
    load_unit(u + 1, xn);
    int b, m0;
    unit_pos(u, b, m0);
    if (m0 == 0) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) prev[ks] = u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const bool ok = m0 + 16 * j + lr < a.T_in;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const u32x4 v = lrelu8(xf[j][ks], a.slope);
        xf[j][ks] = ok ? v : u32x4{0u, 0u, 0u, 0u};
      }
    }
    f32x4 acc[NI][NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 bt[2][NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const u32x4 own = ror1(xf[j][ks]);
        const u32x4 up = ror1(j == 0 ? prev[ks] : xf[j - 1][ks]);
        bt[0][j] = __builtin_bit_cast(bf16x8, lr == 0 ? up : own);
        bt[1][j] = __builtin_bit_cast(bf16x8, xf[j][ks]);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int ch = 8 * ((4 * ks + lq) ^ kq);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(wl + t * NCB * CI + a_off[i] + ch);
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bt[t][j], acc[i][j], 0, 0, 0);
        }
      }
    }
    bf16_t* Y = a.y + (int64_t)b * a.ybs;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int m = m0 + 16 * j + lr;
      const int trow = m * a.up_stride + phase - a.up_pad;
      if (m > a.T_in || trow < 0 || trow >= a.up_tout) continue;
      bf16_t* dst = Y + (int64_t)trow * a.cout + col;
#pragma unroll
      for (int h = 0; h < NI / 2; ++h) {
        const float4 b0 = *reinterpret_cast<const float4*>(bl + nl0 + 8 * h);
        const float4 b1 = *reinterpret_cast<const float4*>(bl + nl0 + 8 * h + 4);
        const f32x4 p = acc[2 * h][j], q = acc[2 * h + 1][j];
        *reinterpret_cast<u32x4*>(dst + 8 * h) =
            u32x4{pack_bf16x2(p[0] + b0.x, p[1] + b0.y), pack_bf16x2(p[2] + b0.z, p[3] + b0.w),
                  pack_bf16x2(q[0] + b1.x, q[1] + b1.y), pack_bf16x2(q[2] + b1.z, q[3] + b1.w)};
      }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      prev[ks] = xf[NJ - 1][ks];
#pragma unroll
      for (int j = 0; j < NJ; ++j) xf[j][ks] = xn[j][ks];
    }
  }
}

template <int CI, int NCB, int NJ, int NW = 8>
static int launch_upsw(const vo_conv1d_desc* d, hipStream_t st) {
  UpswArgs w;
  UpsArgs& a = w.u;
  a.x = reinterpret_cast<const bf16_t*>(d->x);
  a.w = reinterpret_cast<const bf16_t*>(d->w);
  a.bias = d->bias;
  a.y = reinterpret_cast<bf16_t*>(d->y);
  a.xbs = d->x_bstride; a.ybs = d->y_bstride;
  a.T_in = d->T_in; a.up_tout = d->up_tout; a.up_stride = d->up_stride; a.up_pad = d->up_pad;
  a.cout = d->up_cout;
  a.nblk = (d->T_in + 1 + 16 * NJ - 1) / (16 * NJ);
  a.units = a.nblk * d->B;
  a.slope = d->pre_act == VO_ACT_LRELU ? d->pre_slope : (d->pre_act == VO_ACT_RELU ? 0.f : 1.f);
  w.nc = d->Co;
  w.ncb_n = d->Co / NCB;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  // resident workgroups only (persistent); run groups in multiples of 8 (one per XCD slot)
  const size_t lds_b = 2 * (size_t)NCB * CI * sizeof(bf16_t) + NCB * sizeof(float);
  int per_cu = 0;  // LDS- and register-limited resident workgroups per CU
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, upsw_kernel<CI, NCB, NJ, NW>, NW * 64, lds_b) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  const int slots = std::max(1, cus * per_cu / 8);         // workgroup slots per XCD
  const int rg_per_xcd = std::max(1, slots / w.ncb_n);
  const int need = (a.units + 8 * NW - 1) / (8 * NW);      // >= 8 units per wave
  w.rgroups = std::min(8 * rg_per_xcd, std::max(1, need));
  const int grid = 8 * w.ncb_n * ((w.rgroups + 7) / 8);
  const size_t lds = 2 * (size_t)NCB * CI * sizeof(bf16_t) + NCB * sizeof(float);
  hipLaunchKernelGGL((upsw_kernel<CI, NCB, NJ, NW>), dim3((unsigned)grid), dim3(NW * 64), lds, st, w);
  VO_RETURN_LAUNCH();
}

template <int CI, int NC, int NJ>
static int launch_ups(const vo_conv1d_desc* d, hipStream_t st) {
  UpsArgs a;
  a.x = reinterpret_cast<const bf16_t*>(d->x);
  a.w = reinterpret_cast<const bf16_t*>(d->w);
  a.bias = d->bias;
  a.y = reinterpret_cast<bf16_t*>(d->y);
  a.xbs = d->x_bstride; a.ybs = d->y_bstride;
  a.T_in = d->T_in; a.up_tout = d->up_tout; a.up_stride = d->up_stride; a.up_pad = d->up_pad;
  a.cout = d->up_cout;
  a.nblk = (d->T_in + 1 + 16 * NJ - 1) / (16 * NJ);
  a.units = a.nblk * d->B;
  a.slope = d->pre_act == VO_ACT_LRELU ? d->pre_slope : (d->pre_act == VO_ACT_RELU ? 0.f : 1.f);
  auto kern = ups_kernel<CI, NC, NJ>;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0) != hipSuccess || per_cu < 1) per_cu = 1;
  const int grid = (int)std::min<int64_t>((int64_t)cus * per_cu, (a.units + 3) / 4);  // a wave per run
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), 0, st, a);
  VO_RETURN_LAUNCH();
}

}  // namespace vo

// Called by vo_conv1d for a polyphase ConvTranspose1d (already validated there).  *handled = 0
// when the descriptor is not one of the streaming kernel's shapes: the caller then runs the
// generic tiled conv.  vo_tune("ups_cfg", 1) forces the generic path (A/B).
int vo_ups_try(const vo_conv1d_desc* d, hipStream_t st, int* handled) {
  using namespace vo;
  *handled = 0;
  if (vo_tune_get("ups_cfg") == 1) return VO_OK;
  if (!d->transposed || d->compute_dtype != VO_BF16 || d->x_dtype != VO_BF16 || d->y_dtype != VO_BF16) return VO_OK;
  if (d->res1 || d->res2 || d->post_act != VO_ACT_NONE || d->out_scale != 1.f) return VO_OK;
  if (d->ldx != d->Ci || d->ldy != d->up_cout || d->T_out != d->T_in + 1 || d->T_in < 1) return VO_OK;
  if (d->x_bstride % 8 || d->y_bstride % 8 || (d->stride > 1) || (d->groups > 1)) return VO_OK;
  // unit length (tools/probes/ups_probe.py, B = 32 x 512 frames): CI = 128 NJ 1 / 2 / 4 =
  // 169 / 166 / 146 us (generic tiled conv 225); CI = 64 NJ 2 / 4 / 8 = 127 / 125 / 131 us
  // (generic 182).  ups_cfg 2 / 3 select the other two.
  const int cfg = vo_tune_get("ups_cfg");
  if (d->Ci == 128 && d->Co == 128 && d->up_cout % 32 == 0) {
    *handled = 1;
    if (cfg == 2) return launch_ups<128, 128, 2>(d, st);
    if (cfg == 3) return launch_ups<128, 128, 1>(d, st);
    return launch_ups<128, 128, 4>(d, st);
  }
  // wide upsamplers: ups_cfg 4 forces the generic path for these alone
  if (cfg != 4 && d->Ci == 256 && d->Co % 128 == 0 && d->up_cout % 32 == 0 && d->Co >= 256) {
    *handled = 1;
    if (cfg == 5) return launch_upsw<256, 64, 2>(d, st);
    return launch_upsw<256, 128, 1>(d, st);
  }
  // ups0 (512 -> 256, k16 s8) as 64-column blocks on 4-wave workgroups (one wave per SIMD; its
  // 16 x-fragment k-steps spill at 8 waves) took 230 us against 145 on the tiled conv
  // (profiles/r01l/ups_probe_ups0.txt): ups0 stays on the tiled conv.
  if (d->Ci == 64 && d->Co == 64 && d->up_cout % 16 == 0) {
    *handled = 1;
    if (cfg == 2) return launch_ups<64, 64, 2>(d, st);
    if (cfg == 3) return launch_ups<64, 64, 8>(d, st);
    return launch_ups<64, 64, 4>(d, st);
  }
  return VO_OK;
}
