// Weight / bias gradients of the channels-last Conv1d and polyphase ConvTranspose1d on MFMA
// (training paths C4 / C5): replaces the MIOpen ``convolution_backward`` weight pass that
// SURVEY.md 8(b) allowed as the initial fallback.
//
//   dW[m, n, k] = sum_{b, t < T_A} A[b, t, m] * B[b, t * S + k * dil - pad, n]
// (the per-split partial tiles are tap-major (K, M, N): a wave's stores cover runs of 16
// consecutive floats; round 1's fp32 atomics in the weight's (m, n, k) order hit one cache line
// per lane and took 70-85 % of the time)
//
// (rows of B outside [0, T_B) are zero; optional leaky-ReLU applied to either operand as it is
// staged).  Conv1d (Co, Ci, K):      A = dY (rows T_out, M = Co), B = pre(x) (rows T_in, N = Ci),
//                                    S = stride, dil, pad of the conv.
// ConvTranspose1d (Ci, Co, K = 2s):  A = pre(x) (rows T_in, M = Ci), B = dY (rows T_up, N = Co),
//                                    S = s, dil = 1, pad = p.
// GEMM view per tap: M x N output, reduction over the B*T_A rows.  Grid: (row splits, M/64 x
// N/64 tiles, taps); each workgroup stages 64-row chunks of both operands into LDS in their
// natural channels-last layout and reads the MFMA fragments transposed -- ds_read_b64_tr_b16
// (gfx950) delivers 4 rows of one channel per lane, so the reduction dimension (rows) lands
// on the fragment's k without a transpose pass.  Every row split stores its partial tile into a
// caller-owned workspace; a second kernel adds the splits in order and writes dW in the conv
// weight's own (M, N, K) order -- deterministic (bit-identical run to run, so a graph replay can
// be checked bit for bit against eager steps), no zero fill, no permute copy.  fp32 parity mode:
// the same tiles with 16x16x4 f32 MFMAs.

#include <algorithm>
#include <type_traits>

#include "vo_common.h"

namespace vo {

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

constexpr int WG_R = 64;   // rows per staged chunk (two 32-deep MFMA k-steps)
constexpr int WG_T = 64;   // output tile (M and N)

struct WgradArgs {
  const void* a; int lda; int T_A;
  const void* bsrc; int ldb; int T_B;
  int M, N, K, S, dil, pad, Bn;
  int pre_a, pre_b; float slope;
  int rows_per_split;
  float* part;  // [split][groups][K][M][N] partial tiles, then [split][groups][M] bias partials
  int64_t n_w;  // groups * K * M * N
  int64_t n_tot;  // n_w + groups * M (with bias) or n_w: floats per split
  bool bias;  // bias gradient (column sums of A) fused into the tap-0 / n-tile-0 workgroups
  int abl;  // timing ablation (wgrad_cfg 11): 2 = no loads
  int gpt;  // groups per tile (grouped convs with narrow groups, per-tap kernel): see wgrad_gpt
  float* dwf;  // per-tap kernel with one row split: dW (and db) written in their final layout, no reduce
  float* dbf;
};
// groups > 1 (grouped conv): grid z = group * K + tap; group g reads A columns [g M, (g+1) M)
// and B columns [g N, (g+1) N) and writes block g of the (groups, K, M, N) result

typedef short v4s __attribute__((ext_vector_type(4)));

template <typename T> struct WgTile;
template <> struct WgTile<bf16_t> { static constexpr int PITCH = 72; };  // 144-B rows: tr reads of 4 rows hit distinct banks
template <> struct WgTile<float> { static constexpr int PITCH = 68; };
// VO_F32X3: fp32 operands split into a hi and a lo bf16 plane of the bf16 tile's geometry (the two
// planes of 64 x 72 bf16 fill the 64 x 72 four-byte elements the tile declares)
template <> struct WgTile<bx3_t> { static constexpr int PITCH = 72; };

__device__ __forceinline__ uint32_t lrelu_pack(uint32_t w, float s) {
  const float lo = __uint_as_float(w << 16), hi = __uint_as_float(w & 0xffff0000u);
  return pk_bf16(lrelu_max(lo, s), lrelu_max(hi, s));
}

// 4 waves as 2 x 2, each a 32 x 32 sub-tile = 2 x 2 MFMA tiles
template <typename TC>
__global__ void __launch_bounds__(256) wgrad_kernel(WgradArgs p) {
  constexpr int P = WgTile<TC>::PITCH;
  __shared__ __attribute__((aligned(16))) TC sa[WG_R * P];
  __shared__ __attribute__((aligned(16))) TC sb[WG_R * P];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave & 1) * 32, wn = (wave >> 1) * 32;
  // gpt > 1: gpt consecutive groups share one tile -- their A columns (gpt M) and B columns (gpt N)
  // are contiguous, the tile computes the whole gpt M x gpt N product and keeps its diagonal blocks
  const int Mv = p.M * p.gpt, Nv = p.N * p.gpt;
  const int tiles_n = (Nv + WG_T - 1) / WG_T;
  const int m0 = (blockIdx.y / tiles_n) * WG_T, n0 = (blockIdx.y % tiles_n) * WG_T;
  const int k = blockIdx.z % p.K, grp = (blockIdx.z / p.K) * p.gpt;
  const int64_t rows = (int64_t)p.Bn * p.T_A;
  const int64_t r_begin = (int64_t)blockIdx.x * p.rows_per_split;
  const int64_t r_end = min(rows, r_begin + p.rows_per_split);
  const TC* A = reinterpret_cast<const TC*>(p.a) + (int64_t)grp * p.M;
  const TC* Bs = reinterpret_cast<const TC*>(p.bsrc) + (int64_t)grp * p.N;
  float* dw = p.part + (int64_t)blockIdx.x * p.n_tot;
  constexpr int EV = 16 / sizeof(TC);       // elements per 16-byte vector
  constexpr int VPR = WG_T / EV;            // vectors per staged row
  constexpr int NV = WG_R * VPR / 256;      // vectors per thread per operand

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fused bias gradient: the workgroups of tap 0 and the first N tile see every A row of their M
  // tile exactly once -> column sums of the staged A chunks (thread: column tid & 63, rows 16 x
  // (tid >> 6) ..), one LDS reduction and one partial per column at the end
  const bool do_bias = p.bias && k == 0 && n0 == 0;  // workgroup-uniform
  float bsum = 0.f;

  // ---- stage 64 rows of A (rows r0..) and of B (gathered rows of the same utterances); the next chunk's
  // loads are issued before this chunk's MFMAs (the serial chain of a split is otherwise one load round
  // trip per chunk: the encoder's 384-row wgrads walk 6 chunks)
  u32x4_t va[NV], vb[NV];
  auto load_chunk = [&](int64_t r0) {
#pragma unroll
    for (int s = 0; s < NV; ++s) {
      const int v = tid + s * 256;
      const int r = v / VPR, c = (v % VPR) * EV;
      const int64_t q = r0 + r;
      const bool qok = q < r_end;
      const int64_t qq = qok ? q : r_begin;
      const int b = (int)(qq / p.T_A), t = (int)(qq - (int64_t)b * p.T_A);
      const int tb = t * p.S + k * p.dil - p.pad;
      const bool bok = qok && tb >= 0 && tb < p.T_B;
      const int ma = min(m0 + c, Mv - EV), nb = min(n0 + c, Nv - EV);
      if (p.abl & 2) {
        va[s] = vb[s] = u32x4_t{(unsigned)tb, (unsigned)ma, 1u, 1u};
      } else {
        va[s] = *reinterpret_cast<const u32x4_t*>(A + ((int64_t)b * p.T_A + t) * p.lda + ma);
        vb[s] = *reinterpret_cast<const u32x4_t*>(Bs + ((int64_t)b * p.T_B + min(max(tb, 0), p.T_B - 1)) * p.ldb + nb);
      }
      if (!qok || m0 + c >= Mv) va[s] = u32x4_t{0u, 0u, 0u, 0u};
      if (!bok || n0 + c >= Nv) vb[s] = u32x4_t{0u, 0u, 0u, 0u};
    }
  };
  if (r_begin < r_end) load_chunk(r_begin);
  for (int64_t r0 = r_begin; r0 < r_end; r0 += WG_R) {
    __syncthreads();  // previous chunk's fragment reads are done
#pragma unroll
    for (int s = 0; s < NV; ++s) {
      const int v = tid + s * 256;
      const int r = v / VPR, c = (v % VPR) * EV;
      u32x4_t x = va[s], y = vb[s];
      if constexpr (std::is_same<TC, bx3_t>::value) {
        float f[8] = {__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z), __uint_as_float(x.w),
                      __uint_as_float(y.x), __uint_as_float(y.y), __uint_as_float(y.z), __uint_as_float(y.w)};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (p.pre_a) f[e] = fmaxf(f[e], f[e] * p.slope);
          if (p.pre_b) f[4 + e] = fmaxf(f[4 + e], f[4 + e] * p.slope);
        }
        uint4 hi, lo;  // (x.xy, x.zw, y.xy, y.zw) as bf16 pairs
        split8(f, hi, lo);
        bf16_t* ha = reinterpret_cast<bf16_t*>(sa);
        bf16_t* hb = reinterpret_cast<bf16_t*>(sb);
        *reinterpret_cast<uint2*>(ha + r * P + c) = make_uint2(hi.x, hi.y);
        *reinterpret_cast<uint2*>(ha + (WG_R + r) * P + c) = make_uint2(lo.x, lo.y);
        *reinterpret_cast<uint2*>(hb + r * P + c) = make_uint2(hi.z, hi.w);
        *reinterpret_cast<uint2*>(hb + (WG_R + r) * P + c) = make_uint2(lo.z, lo.w);
        continue;
      } else if constexpr (sizeof(TC) == 2) {
        if (p.pre_a) x = u32x4_t{lrelu_pack(x.x, p.slope), lrelu_pack(x.y, p.slope), lrelu_pack(x.z, p.slope), lrelu_pack(x.w, p.slope)};
        if (p.pre_b) y = u32x4_t{lrelu_pack(y.x, p.slope), lrelu_pack(y.y, p.slope), lrelu_pack(y.z, p.slope), lrelu_pack(y.w, p.slope)};
      } else {
        if (p.pre_a) {
          float f[4] = {__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z), __uint_as_float(x.w)};
          x = u32x4_t{__float_as_uint(fmaxf(f[0], f[0] * p.slope)), __float_as_uint(fmaxf(f[1], f[1] * p.slope)),
                      __float_as_uint(fmaxf(f[2], f[2] * p.slope)), __float_as_uint(fmaxf(f[3], f[3] * p.slope))};
        }
        if (p.pre_b) {
          float f[4] = {__uint_as_float(y.x), __uint_as_float(y.y), __uint_as_float(y.z), __uint_as_float(y.w)};
          y = u32x4_t{__float_as_uint(fmaxf(f[0], f[0] * p.slope)), __float_as_uint(fmaxf(f[1], f[1] * p.slope)),
                      __float_as_uint(fmaxf(f[2], f[2] * p.slope)), __float_as_uint(fmaxf(f[3], f[3] * p.slope))};
        }
      }
      *reinterpret_cast<u32x4_t*>(sa + r * P + c) = x;
      *reinterpret_cast<u32x4_t*>(sb + r * P + c) = y;
    }
    __syncthreads();
    if (r0 + WG_R < r_end) load_chunk(r0 + WG_R);
    if (do_bias) {
      const int col = tid & 63, r16 = (tid >> 6) * 16;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if constexpr (std::is_same<TC, bx3_t>::value) {  // hi + lo: within 2^-18 of the fp32 value
          const bf16_t* ha = reinterpret_cast<const bf16_t*>(sa);
          bsum += to_f32(ha[(r16 + i) * P + col]) + to_f32(ha[(WG_R + r16 + i) * P + col]);
        } else {
          bsum += to_f32(sa[(r16 + i) * P + col]);
        }
      }
    }

    // ---- two 32-row k-steps
#pragma unroll
    for (int ks = 0; ks < WG_R / 32; ++ks) {
      const int kr = ks * 32;
      if constexpr (sizeof(TC) == 2 || std::is_same<TC, bx3_t>::value) {
        // fragment of 16 channels (c0..c0+15) x 8 rows (kr + 8g ..): two transposed 4-row reads
        const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
        auto frag = [&](const bf16_t* tile, int c0) {
          const bf16_t* base = tile + (kr + 8 * g + q) * P + c0 + 4 * pp;
          typedef __attribute__((address_space(3))) v4s lds_v4s;
          const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)base);
          const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(base + 4 * P));
          // whole-vector bit cast: per-element __bf16 inserts were mis-lowered by hipcc (only the
          // low dword of each read survived)
          typedef short v8s __attribute__((ext_vector_type(8)));
          const v8s all = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          Frag<bf16_t> f;
          f.v = __builtin_bit_cast(bf16x8, all);
          return f;
        };
        const bf16_t* ta = reinterpret_cast<const bf16_t*>(sa);
        const bf16_t* tb = reinterpret_cast<const bf16_t*>(sb);
        Frag<bf16_t> fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) fa[i] = frag(ta, wm + 16 * i);
#pragma unroll
        for (int j = 0; j < 2; ++j) fb[j] = frag(tb, wn + 16 * j);
        if constexpr (std::is_same<TC, bx3_t>::value) {  // lo planes: the small terms first
          Frag<bf16_t> la[2], lb[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) la[i] = frag(ta + WG_R * P, wm + 16 * i);
#pragma unroll
          for (int j = 0; j < 2; ++j) lb[j] = frag(tb + WG_R * P, wn + 16 * j);
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              acc[i][j] = mfma(la[i], fb[j], acc[i][j]);
              acc[i][j] = mfma(fa[i], lb[j], acc[i][j]);
            }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma(fa[i], fb[j], acc[i][j]);
      } else {
        // f32: element j of lane l = row kr + 8 (l >> 4) + j, channel l & 15 (scalar LDS reads)
        const int g = lane >> 4, li = lane & 15;
        Frag<float> fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            fa[i].v[e] = sa[(kr + 8 * g + e) * P + wm + 16 * i + li];
          }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e) fb[j].v[e] = sb[(kr + 8 * g + e) * P + wn + 16 * j + li];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma(fa[i], fb[j], acc[i][j]);
      }
    }
  }

  if (do_bias) {
    __shared__ float bred[4][64];
    bred[tid >> 6][tid & 63] = bsum;
    __syncthreads();
    if (tid < 64 && m0 + tid < Mv) {
      const float v = bred[0][tid] + bred[1][tid] + bred[2][tid] + bred[3][tid];
      if (p.dbf)
        p.dbf[(int64_t)grp * p.M + m0 + tid] = v;
      else
        p.part[(int64_t)blockIdx.x * p.n_tot + p.n_w + (int64_t)grp * p.M + m0 + tid] = v;
    }
  }

  // ---- epilogue: D[m][n] (row = m: 4 (lane >> 4) + e, col = n: lane & 15) -> dW[k][m][n]
  const int li = lane & 15, g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm + 16 * i + 4 * g + e, n = n0 + wn + 16 * j + li;
        const int gm = m / p.M;  // group of the row (0 unless gpt > 1); keep the diagonal blocks
        if (m < Mv && n < Nv && gm == n / p.N) {
          if (p.dwf)  // final (groups, M, N, K) order
            p.dwf[(((int64_t)(grp + gm) * p.M + (m - gm * p.M)) * p.N + (n - gm * p.N)) * p.K + k] = acc[i][j][e];
          else
            dw[(((int64_t)(grp + gm) * p.K + k) * p.M + (m - gm * p.M)) * p.N + (n - gm * p.N)] = acc[i][j][e];
        }
      }
}

// K = 1 weight gradient (round 6; bf16, stride 1, no padding, ungrouped, no prologue activation): the
// Linear layers of the C4 decoder (q/k/v 256 -> 768, fc, FFN w_2 1024 -> 256, mel_linear) at 16 k rows,
// dW (M x N) = A^T B over the rows.  On the per-tap kernel's 64 x 64 tiles these ran at ~0.05 of the
// bf16 peak (19 launches, ~1 ms of the C4 step): 8 MFMAs per wave per staged 16 KB and a load round trip
// per 64-row chunk.  Here a workgroup owns a 128 x 128 tile (4 waves of 64 x 64 = 16 MFMA tiles: 16
// MFMAs per 32-row k-step for 8 fragment pairs), both operands double-buffered in LDS with the next
// chunk's loads in registers over the current chunk's MFMAs, bare barriers.  LDS rows are 256 B with
// the 16-byte chunk q of row r at q ^ 2 ((r & 3) | ((r >> 3 & 1) << 2)): the transposed reads
// (ds_read_b64_tr_b16: rows kr + 8g + q, two 8-byte column quads) hit 32 distinct bank pairs per half
// wave, the staging stores 8 distinct chunks per 8 lanes.  Bias gradient (column sums of A) fused into
// the n-tile-0 workgroups from the staged registers.  Partials / reduce / determinism as the per-tap
// kernel (tap-major partials with K = 1 are (M, N): an unsplit launch writes dW directly).
constexpr int K1_T = 128;  // output tile (M and N)
constexpr int K1_R = 64;   // rows per chunk
__device__ __forceinline__ int k1_swz(int r, int q) { return q ^ (((r & 3) | (((r >> 3) & 1) << 2)) << 1); }

__global__ void __launch_bounds__(256, 2) wgrad_k1_kernel(WgradArgs p) {
  __shared__ __attribute__((aligned(16))) bf16_t sa[2][K1_R * K1_T];
  __shared__ __attribute__((aligned(16))) bf16_t sb[2][K1_R * K1_T];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave & 1) * 64, wn = (wave >> 1) * 64;
  const int tiles_n = (p.N + K1_T - 1) / K1_T;
  const int m0 = (blockIdx.y / tiles_n) * K1_T, n0 = (blockIdx.y % tiles_n) * K1_T;
  const int64_t rows = (int64_t)p.Bn * p.T_A;
  const int64_t r_begin = (int64_t)blockIdx.x * p.rows_per_split;
  const int64_t r_end = min(rows, r_begin + p.rows_per_split);
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.a);
  const bf16_t* Bs = reinterpret_cast<const bf16_t*>(p.bsrc);
  const bool do_bias = p.bias && n0 == 0;  // workgroup-uniform

  // staging slot s of thread t: row r = (t + 256 s) >> 4, 16-byte chunk c = t & 15 (8 columns)
  const int sc = tid & 15, sr0 = tid >> 4;
  const int ma = min(m0 + 8 * sc, p.M - 8), nb = min(n0 + 8 * sc, p.N - 8);
  const bool mok = m0 + 8 * sc < p.M, nok = n0 + 8 * sc < p.N;
  uint4 ra[4], rb[4];
  auto load = [&](int64_t r0) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int64_t q = r0 + sr0 + 16 * s;
      const bool ok = q < r_end;
      const int64_t qq = ok ? q : r_begin;
      ra[s] = *reinterpret_cast<const uint4*>(A + qq * p.lda + ma);
      rb[s] = *reinterpret_cast<const uint4*>(Bs + qq * p.ldb + nb);
      if (!ok || !mok) ra[s] = make_uint4(0u, 0u, 0u, 0u);
      if (!ok || !nok) rb[s] = make_uint4(0u, 0u, 0u, 0u);
    }
  };
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto store = [&](int buf) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int r = sr0 + 16 * s;
      *reinterpret_cast<uint4*>(&sa[buf][r * K1_T + k1_swz(r, sc) * 8]) = ra[s];
      *reinterpret_cast<uint4*>(&sb[buf][r * K1_T + k1_swz(r, sc) * 8]) = rb[s];
      if (do_bias) {
        const uint32_t w[4] = {ra[s].x, ra[s].y, ra[s].z, ra[s].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bsum[2 * e] += __uint_as_float(w[e] << 16);
          bsum[2 * e + 1] += __uint_as_float(w[e] & 0xffff0000u);
        }
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fragment of 16 channels (c0..c0+15) x 8 rows (kr + 8g ..): two transposed 4-row reads (lane li:
  // row kr + 8g + (li >> 2), the 8-byte column quad c0 + 4 (li & 3))
  const int g = lane >> 4, li = lane & 15, fq = li >> 2, fp = li & 3;
  auto frag = [&](const bf16_t* tile, int kr, int c0) {
    const int r = kr + 8 * g + fq, col = c0 + 4 * fp;
    typedef __attribute__((address_space(3))) v4s lds_v4s;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(tile + r * K1_T + k1_swz(r, col >> 3) * 8 + (col & 7)));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_v4s*)(tile + (r + 4) * K1_T + k1_swz(r + 4, col >> 3) * 8 + (col & 7)));
    typedef short v8s __attribute__((ext_vector_type(8)));
    const v8s all = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    Frag<bf16_t> f;
    f.v = __builtin_bit_cast(bf16x8, all);
    return f;
  };

  const int nchunks = (int)((r_end - r_begin + K1_R - 1) / K1_R);
  load(r_begin);
  store(0);
  if (nchunks > 1) load(r_begin + K1_R);
  lds_barrier();
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
#pragma unroll
    for (int ks = 0; ks < K1_R / 32; ++ks) {
      Frag<bf16_t> fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag(sa[buf], 32 * ks, wm + 16 * i);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag(sb[buf], 32 * ks, wn + 16 * j);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma(fa[i], fb[j], acc[i][j]);
    }
    if (c + 1 < nchunks) {
      store(buf ^ 1);  // chunk c + 1 (its buffer was read in chunk c - 1, before the last barrier)
      if (c + 2 < nchunks) load(r_begin + (int64_t)(c + 2) * K1_R);
    }
    lds_barrier();
  }

  if (do_bias) {  // 16 row-threads per 8-column chunk: one LDS reduction in thread order (deterministic)
    float* red = reinterpret_cast<float*>(&sa[0][0]);  // [16 row-threads][128 columns], after the last barrier
#pragma unroll
    for (int e = 0; e < 8; ++e) red[sr0 * K1_T + 8 * sc + e] = bsum[e];
    __syncthreads();
    if (tid < K1_T && m0 + tid < p.M) {
      float v = 0.f;
      for (int q = 0; q < 16; ++q) v += red[q * K1_T + tid];
      if (p.dbf)
        p.dbf[m0 + tid] = v;
      else
        p.part[(int64_t)blockIdx.x * p.n_tot + p.n_w + m0 + tid] = v;
    }
  }
  float* dw = p.dwf ? p.dwf : p.part + (int64_t)blockIdx.x * p.n_tot;  // K = 1: (M, N) either way
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm + 16 * i + 4 * g + e, n = n0 + wn + 16 * j + li;
        if (m < p.M && n < p.N) dw[(int64_t)m * p.N + n] = acc[i][j][e];
      }
}

// Multi-tap weight gradient (round 3; stride-1 convs, bf16): the per-tap kernel above restages
// both operands for every tap -- a K = 11 conv reads dY and x eleven times and feeds 8 MFMAs per
// wave per staged 16 KB (C5's MRF weight gradients ran at 0.05-0.18 PF/s).  Here a workgroup owns
// a TM x TM tile for a run of up to KG taps: per 64-row chunk it stages A (64 rows) and the B WINDOW
// (64 + (nk - 1) dil rows) once, and every tap reads its B fragments at a row offset k * dil of that
// window (the transposed LDS reads name their row per lane, so a shift costs nothing) -- nk x the
// MFMAs per staged byte.  Chunks never cross an utterance (64-row chunks per utterance, the last one
// zero-padded), so the window of a chunk is one contiguous run of B rows.  The next chunk is loaded
// into registers during the current chunk's MFMAs.  Partials, their order and the reduce are the
// per-tap kernel's (tap-major [split][group][k][M][N]; the tap run only changes which workgroup
// computes a tap), so the result is deterministic run to run; per element the sum over a split's
// rows runs in the same chunk / k-step order as the per-tap kernel.
constexpr int WM_R = 64;       // rows per chunk
constexpr int WM_MAXW = 128;   // window rows: 64 + (nk - 1) * dil <= 128

// Round 6: strided convs (the MSD's grouped stride-2 / 4 layers, k = 41: on the per-tap kernel each tap
// restaged both operands -- a 147-chunk serial chain of 8 MFMAs per 12 KB staged): SW > 1 sizes the window
// for stride S <= SW, 64 SW + 64 rows; A row r of a chunk meets window row r S + kk dil for tap kk (the
// transposed reads name their row per lane, so the stride costs nothing in the reads).
template <int TM, int KG, int SW = 1>
__global__ void __launch_bounds__(256, 2) wgrad_mt_kernel(WgradArgs p, int chunks_per_b, int chunks_per_split,
                                                         int ntg) {
  constexpr int WMW = SW == 1 ? WM_MAXW : 64 * SW + 64;  // window capacity (rows)
  constexpr int P = TM == 64 ? 72 : 48;  // pitch (elements): the 4 rows of a transposed read on distinct banks
  constexpr int WT = TM / 2;             // wave sub-tile (2 x 2 waves)
  constexpr int MI = WT / 16;            // MFMA tiles per wave and dimension
  constexpr int VPR = TM / 8;            // 16-byte vectors per staged row
  constexpr int NVA = WM_R * VPR / 256;  // A vectors per thread
  constexpr int NVB = (WMW * VPR + 255) / 256;  // B window vectors per thread (upper bound)
  // strided windows at TM = 32 (96-byte rows): the rows a half-wave's transposed reads name are (r + 8g + q) S +
  // kk -- at S = 2 the two 16-lane groups (rows 16 apart) hit the same banks, at S = 4 also q and q + 2 (2.2
  // conflicts per LDS instruction measured).  Row R is placed at R P + ROFF(R): 32 B more per 16 rows (S = 2),
  // 64 B per 8 rows + 32 B per 32 rows (S = 4) -- monotonic (no two rows overlap), and the lanes' 32-byte slots
  // of a half-wave land on 8 distinct bank slots
  constexpr bool SWZ = SW > 1 && TM == 32;
  auto roff = [&](int R) -> int {
    if constexpr (!SWZ) return R * P;
    if constexpr (SW == 2) return R * P + 16 * (R >> 4);
    return R * P + 32 * (R >> 3) + 16 * (R >> 5);
  };
  constexpr int SB_EXTRA = SWZ ? 32 * (WMW / 8 + 1) + 16 * (WMW / 32 + 1) : 0;
  __shared__ __attribute__((aligned(16))) bf16_t sa[WM_R * P];
  __shared__ __attribute__((aligned(16))) bf16_t sb[WMW * P + SB_EXTRA];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave & 1) * WT, wn = (wave >> 1) * WT;
  const int tiles_n = (p.N + TM - 1) / TM;
  const int m0 = (blockIdx.y / tiles_n) * TM, n0 = (blockIdx.y % tiles_n) * TM;
  const int tg = blockIdx.z % ntg, grp = blockIdx.z / ntg;
  const int k0 = tg * KG, nk = min(KG, p.K - k0);
  const int WR = (WM_R - 1) * p.S + 1 + (nk - 1) * p.dil;  // window rows of this tap run
  const int c_begin = blockIdx.x * chunks_per_split;
  const int c_end = min(p.Bn * chunks_per_b, c_begin + chunks_per_split);
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.a) + (int64_t)grp * p.M;
  const bf16_t* Bs = reinterpret_cast<const bf16_t*>(p.bsrc) + (int64_t)grp * p.N;
  float* dw = p.part + (int64_t)blockIdx.x * p.n_tot;

  f32x4 acc[KG][MI][MI];
#pragma unroll
  for (int kk = 0; kk < KG; ++kk)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < MI; ++j) acc[kk][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = p.bias && tg == 0 && n0 == 0;  // workgroup-uniform
  float bsum = 0.f;

  // two register sets, alternated by the 2x-unrolled chunk loop: a chunk's loads are issued two
  // chunks of MFMAs before its LDS store (one chunk was too short to cover the load latency)
  u32x4_t va0[NVA], vb0[NVB], va1[NVA], vb1[NVB];
  auto load = [&](int c, u32x4_t (&va)[NVA], u32x4_t (&vb)[NVB]) {  // chunk c -> registers (unconditional
                                                                   // loads, clamped; zeroed when stored)
    const int b = c / chunks_per_b, t0 = (c - b * chunks_per_b) * WM_R;
#pragma unroll
    for (int s = 0; s < NVA; ++s) {
      const int v = tid + s * 256, r = v / VPR, col = (v % VPR) * 8;
      const int t = min(t0 + r, p.T_A - 1);
      va[s] = *reinterpret_cast<const u32x4_t*>(A + ((int64_t)b * p.T_A + t) * p.lda + min(m0 + col, p.M - 8));
    }
    const int tb0 = t0 * p.S - p.pad + k0 * p.dil;
#pragma unroll
    for (int s = 0; s < NVB; ++s) {
      const int v = tid + s * 256, w = min(v / VPR, WMW - 1), col = (v % VPR) * 8;
      const int tb = min(max(tb0 + w, 0), p.T_B - 1);
      vb[s] = *reinterpret_cast<const u32x4_t*>(Bs + ((int64_t)b * p.T_B + tb) * p.ldb + min(n0 + col, p.N - 8));
    }
  };
  auto store = [&](int c, const u32x4_t (&va)[NVA], const u32x4_t (&vb)[NVB]) {
    const int b = c / chunks_per_b, t0 = (c - b * chunks_per_b) * WM_R;
    (void)b;
#pragma unroll
    for (int s = 0; s < NVA; ++s) {
      const int v = tid + s * 256, r = v / VPR, col = (v % VPR) * 8;
      u32x4_t x = va[s];
      if (t0 + r >= p.T_A || m0 + col >= p.M) x = u32x4_t{0u, 0u, 0u, 0u};
      if (p.pre_a) x = u32x4_t{lrelu_pack(x.x, p.slope), lrelu_pack(x.y, p.slope), lrelu_pack(x.z, p.slope), lrelu_pack(x.w, p.slope)};
      *reinterpret_cast<u32x4_t*>(sa + r * P + col) = x;
    }
    const int tb0 = t0 * p.S - p.pad + k0 * p.dil;
#pragma unroll
    for (int s = 0; s < NVB; ++s) {
      const int v = tid + s * 256, w = v / VPR, col = (v % VPR) * 8;
      if (w < WR) {  // uniform per 8-lane row group; rows past the window are never read
        u32x4_t y = vb[s];
        const int tb = tb0 + w;
        if (tb < 0 || tb >= p.T_B || n0 + col >= p.N) y = u32x4_t{0u, 0u, 0u, 0u};
        if (p.pre_b) y = u32x4_t{lrelu_pack(y.x, p.slope), lrelu_pack(y.y, p.slope), lrelu_pack(y.z, p.slope), lrelu_pack(y.w, p.slope)};
        *reinterpret_cast<u32x4_t*>(sb + roff(w) + col) = y;
      }
    }
  };

  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  typedef __attribute__((address_space(3))) v4s lds_v4s;
  typedef short v8s __attribute__((ext_vector_type(8)));
  // fragment of 16 channels (c0 + li) x 8 rows (row0 + 8 g ..): two transposed 4-row reads
  auto frag = [&](const bf16_t* tile, int row0, int c0) {
    const bf16_t* base = tile + (row0 + 8 * g + q) * P + c0 + 4 * pp;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)base);
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(base + 4 * P));
    Frag<bf16_t> f;
    f.v = __builtin_bit_cast(bf16x8, (v8s)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    return f;
  };
  // B fragment of A rows arow0 + 8 g .. (+ 8) for tap kk: window rows (A row) S + kk dil
  auto frag_b = [&](int arow0, int kk, int c0) {
    if constexpr (SW == 1) return frag(sb, arow0 + kk * p.dil, c0);
    const int r = arow0 + 8 * g + q;
    const bf16_t* lo_p = sb + roff(r * p.S + kk * p.dil) + c0 + 4 * pp;
    const bf16_t* hi_p = sb + roff((r + 4) * p.S + kk * p.dil) + c0 + 4 * pp;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)lo_p);
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)hi_p);
    Frag<bf16_t> f;
    f.v = __builtin_bit_cast(bf16x8, (v8s)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    return f;
  };

  auto compute = [&]() {
    if (do_bias) {
      const int col = tid & 63, r16 = (tid >> 6) * 16;
      if (col < TM) {
#pragma unroll
        for (int i = 0; i < 16; ++i) bsum += to_f32(sa[(r16 + i) * P + col]);
      }
    }
#pragma unroll
    for (int ks = 0; ks < WM_R / 32; ++ks) {
      Frag<bf16_t> fa[MI];
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = frag(sa, ks * 32, wm + 16 * i);
#pragma unroll
      for (int kk = 0; kk < KG; ++kk) {
        if (kk < nk) {  // uniform
          Frag<bf16_t> fb[MI];
#pragma unroll
          for (int j = 0; j < MI; ++j) fb[j] = frag_b(ks * 32, kk, wn + 16 * j);
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < MI; ++j) acc[kk][i][j] = mfma(fa[i], fb[j], acc[kk][i][j]);
        }
      }
    }
  };
  if (c_begin < c_end) {
    load(c_begin, va0, vb0);
    store(c_begin, va0, vb0);
  }
  __syncthreads();
  if (c_begin + 1 < c_end) load(c_begin + 1, va0, vb0);
  for (int c = c_begin; c < c_end; c += 2) {
    // LDS holds chunk c; set 0 holds chunk c + 1 (in flight)
    if (c + 2 < c_end) load(c + 2, va1, vb1);
    compute();
    __syncthreads();  // every wave is past this chunk's fragment reads
    if (c + 1 >= c_end) break;
    store(c + 1, va0, vb0);
    __syncthreads();
    if (c + 3 < c_end) load(c + 3, va0, vb0);
    compute();
    __syncthreads();
    if (c + 2 < c_end) {
      store(c + 2, va1, vb1);
      __syncthreads();
    }
  }

  if (do_bias) {
    __shared__ float bred[4][64];
    bred[tid >> 6][tid & 63] = bsum;
    __syncthreads();
    if (tid < TM && m0 + tid < p.M)
      dw[p.n_w + (int64_t)grp * p.M + m0 + tid] = bred[0][tid] + bred[1][tid] + bred[2][tid] + bred[3][tid];
  }
  // D[m][n] (row = m: 4 g + e, col = n: li) -> part[split][grp][k][m][n]
#pragma unroll
  for (int kk = 0; kk < KG; ++kk) {
    if (kk < nk) {
      float* dk = dw + ((int64_t)grp * p.K + k0 + kk) * p.M * p.N;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MI; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int m = m0 + wm + 16 * i + 4 * g + e, n = n0 + wn + 16 * j + li;
            if (m < p.M && n < p.N) dk[(int64_t)m * p.N + n] = acc[kk][i][j][e];
          }
    }
  }
}

// dW[((g M + m) N + n) K + k] = sum over splits of part[s][g][k][m][n]; db likewise.
// A block holds G groups of 64 consecutive outputs (lane = output: coalesced) and W waves per
// group: wave w of a group adds splits w, w + W, .. in order, then the W wave sums are added in
// wave order -- a fixed order (deterministic run to run).  Many splits (small M x N tiles: ~340 at
// M = N = 32, K = 3) take W = 16, 16 x the memory parallelism of one thread walking every split
// (which took most of such a wgrad call); few splits over many outputs take W = 1, G = 4.
template <int W, int G>
__global__ void __launch_bounds__(64 * W * G) wgrad_reduce_kernel(const float* __restrict__ part, int splits,
                                                                  int64_t n_w, int64_t n_tot, int M, int N, int K,
                                                                  float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float red[W > 1 ? W * G : 1][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int w = wave % W, grp = wave / W;
  const int64_t i = ((int64_t)blockIdx.x * G + grp) * 64 + lane;
  float s = 0.f;
  if (i < n_tot)
    for (int q = w; q < splits; q += W) s += part[(int64_t)q * n_tot + i];
  if constexpr (W > 1) {
    red[wave][lane] = s;
    __syncthreads();
    if (w != 0) return;
    s = red[grp * W][lane];
#pragma unroll
    for (int q = 1; q < W; ++q) s += red[grp * W + q][lane];
  }
  if (i >= n_tot) return;
  if (i < n_w) {
    const int n = (int)(i % N);
    const int64_t r = i / N;
    const int m = (int)(r % M);
    const int64_t gk = r / M;
    const int k = (int)(gk % K), g = (int)(gk / K);
    dw[(((int64_t)g * M + m) * N + n) * K + k] = s;
  } else {
    db[i - n_w] = s;
  }
}

static void wgrad_reduce_launch(const float* part, int splits, int64_t n_w, int64_t n_tot, int M, int N, int K,
                                float* dw, float* db, hipStream_t st) {
  if (splits >= 32)
    hipLaunchKernelGGL((wgrad_reduce_kernel<16, 1>), dim3((unsigned)((n_tot + 63) / 64)), dim3(1024), 0, st, part,
                       splits, n_w, n_tot, M, N, K, dw, db);
  else
    hipLaunchKernelGGL((wgrad_reduce_kernel<1, 4>), dim3((unsigned)((n_tot + 255) / 256)), dim3(256), 0, st, part,
                       splits, n_w, n_tot, M, N, K, dw, db);
}

// column sums of a (rows x C) channels-last tensor -> out[C] (written): per-block partials in a
// workspace, added in block order by wgrad_reduce_kernel's bias path (deterministic).
// Thread t owns the 8-channel vector t % (C / 8) of rows t / (C / 8) + k * (256 / (C / 8)):
// coalesced 16-byte loads, register accumulation, one LDS reduction and C partials per block.
template <typename T>
__global__ void __launch_bounds__(256) colsum_kernel(const T* __restrict__ x, int64_t rows, int C, int ld,
                                                     int rows_per_block, float* __restrict__ out) {
  __shared__ float red[256 * 8];
  const int nv = C / 8;                       // 8-channel vectors per row (C % 8 == 0, nv <= 256)
  const int per = 256 / nv;                   // row lanes per block
  const int tid = threadIdx.x, cv = tid % nv, ro = tid / nv;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (ro < per)
    for (int64_t r = r0 + ro; r < r1; r += per) {
      float v[8];
      load8(x + r * ld + cv * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[tid * 8 + e] = acc[e];
  __syncthreads();
  for (int c = tid; c < C; c += 256) {  // channel c = vector c / 8, element c % 8
    float s = 0.f;
    for (int q = 0; q < per; ++q) s += red[(q * nv + c / 8) * 8 + (c % 8)];
    out[(int64_t)blockIdx.x * C + c] = s;
  }
}

}  // namespace vo

using namespace vo;

// row-split plan shared by the workspace query and the launch: enough workgroups to fill 256
// CUs ~4 deep, at least 4 chunks of 64 rows each, serial row chains of at most 64 chunks (a small
// tile x tap grid -- the MSD's 32 x 16 groups -- otherwise leaves one workgroup walking every row)
// groups per tile of the per-tap kernel: narrow groups (the MSD's 16 x 8 .. 64 x 32 per group) are
// packed side by side up to the 64 x 64 tile (one launch computed a 16 x 8 group in a 64 x 64 tile:
// 1/32 of its MFMA work useful)
static int wgrad_gpt(int M, int N, int groups) {
  if (groups <= 1 || vo_tune_get("wgrad_cfg") == 12) return 1;  // 12: one group per tile (A/B)
  int gpt = 1;
  for (int d = 2; d <= groups; ++d)
    if (groups % d == 0 && d * M <= WG_T && d * N <= WG_T) gpt = d;
  return gpt;
}

static void wgrad_plan(int B, int T_A, int M, int N, int K, int groups, int64_t* splits_out, int* rps_out) {
  const int gpt = wgrad_gpt(M, N, groups);
  const int64_t zk = (int64_t)K * (groups / gpt);
  const int64_t rows = (int64_t)B * T_A;
  const int tiles = ((M * gpt + WG_T - 1) / WG_T) * ((N * gpt + WG_T - 1) / WG_T);
  const int wc = vo_tune_get("wgrad_cfg");
  const int64_t target = wc == 1 ? 4096 : wc == 2 ? 8192 : wc == 3 ? 16384 : 1024;
  int64_t splits = std::max<int64_t>(1, (target + (int64_t)tiles * zk - 1) / ((int64_t)tiles * zk));
  // short sequences (<= 4096 rows: the encoder's 384, split-bf16 / fp32): one chunk per split is allowed --
  // their 6-chunk serial chains were a load round trip each (31.6 us per launch); wgrad_cfg 17 keeps >= 4
  const int min_chunks = (rows <= 4096 && wc != 17) ? 1 : 4;
  splits = std::min<int64_t>(splits, std::max<int64_t>(1, rows / (min_chunks * WG_R)));
  const int64_t max_rows = wc == 4 ? 2048 : wc == 5 ? 8192 : wc == 6 ? (int64_t)1 << 40 : 4096;
  splits = std::max<int64_t>(splits, (rows + max_rows - 1) / max_rows);
  const int rps = (int)(((rows + splits - 1) / splits + WG_R - 1) / WG_R * WG_R);
  *splits_out = (rows + rps - 1) / rps;
  *rps_out = rps;
}

// multi-tap plan (wgrad_mt_kernel): the partials of a split cover the whole (K, M, N) output, so
// splits are capped by their traffic (at most max(operand bytes, 16 MB) of partials); the taps are
// then cut into runs (ntg per workgroup column) only as far as needed to give ~256 workgroups, the
// rest of the parallelism comes from splits.  dil bounds a run's window (64 + (KG - 1) dil <= 128
// rows); the splits never grow with dil, so the plan at dil = 1 sizes the workspace.
struct MtPlan { int tm, kg, ntg, chunks_per_b, cps, splits; };
static void wgrad_mt_plan(int B, int T_A, int M, int N, int K, int groups, int dil, MtPlan* pl, int S = 1) {
  pl->tm = (M <= 32 && N <= 32) ? 32 : 64;
  const int64_t tiles = (int64_t)((M + pl->tm - 1) / pl->tm) * ((N + pl->tm - 1) / pl->tm) * groups;
  pl->chunks_per_b = (T_A + WM_R - 1) / WM_R;
  const int64_t total = (int64_t)B * pl->chunks_per_b;
  const int64_t rows = (int64_t)B * T_A;
  const int64_t operand = rows * ((int64_t)M + N) * groups * 2;
  const int64_t per_split = ((int64_t)groups * K * M * N + (int64_t)groups * M) * 4;
  const int64_t smax = std::max<int64_t>(1, std::min<int64_t>(total, std::max<int64_t>(operand, 16 << 20) / per_split));
  // TM 64 x 9+ taps spill (strided: 5, the larger window's staging registers); the window (stride S: 64 S + 64
  // rows) bounds a run to 1 + 64 / dil taps either way
  const int kgmax = std::min(pl->tm == 64 ? (S > 1 ? 5 : 8) : 11, 1 + 64 / std::max(dil, 1));
  const int forced = vo_tune_get("wgrad_kg");  // A/B: taps per run
  int ntg = (int)std::max<int64_t>(1, (256 + tiles * smax - 1) / (tiles * smax));
  int kg = forced > 0 ? forced : (K + ntg - 1) / ntg;
  kg = std::max(1, std::min(kg, std::min(kgmax, K)));
  ntg = (K + kg - 1) / kg;
  if (forced <= 0) kg = (K + ntg - 1) / ntg;  // balanced runs (K = 9 at 8 taps max: 5 + 4, not 8 + 1)
  pl->kg = kg;
  pl->ntg = ntg;
  const int wc = vo_tune_get("wgrad_cfg");  // A/B: 19 / 20 = ~2048 / ~1024 workgroups
  const int64_t wtarget = wc == 19 ? 2048 : wc == 20 ? 1024 : 512;
  const int64_t want = std::max<int64_t>(1, (wtarget + tiles * ntg - 1) / (tiles * ntg));
  const int64_t splits = std::min(smax, want);
  pl->cps = (int)((total + splits - 1) / splits);
  pl->splits = (int)((total + pl->cps - 1) / pl->cps);
}

// K = 1 plan (wgrad_k1_kernel): ~512 workgroups (two per CU; wgrad_cfg 15 = 256, 16 = 1024), at least 4
// chunks of 64 rows per split
static void k1_plan(int B, int T_A, int M, int N, int64_t* splits_out, int* rps_out) {
  const int64_t tiles = (int64_t)((M + K1_T - 1) / K1_T) * ((N + K1_T - 1) / K1_T);
  const int64_t rows = (int64_t)B * T_A;
  const int wc = vo_tune_get("wgrad_cfg");
  const int64_t target = wc == 15 ? 256 : wc == 16 ? 1024 : 512;
  int64_t splits = (target + tiles - 1) / tiles;
  splits = std::max<int64_t>(1, std::min<int64_t>(splits, rows / (4 * K1_R)));
  const int rps = (int)(((rows + splits - 1) / splits + K1_R - 1) / K1_R * K1_R);
  *splits_out = (rows + rps - 1) / rps;
  *rps_out = rps;
}

extern "C" int64_t vo_conv1d_wgrad_workspace_size(int B, int T_A, int M, int N, int K, int groups) {
  if (B <= 0 || T_A <= 0 || M <= 0 || N <= 0 || K <= 0 || groups <= 0) return 0;
  int64_t splits;
  int rps;
  wgrad_plan(B, T_A, M, N, K, groups, &splits, &rps);
  MtPlan mt;
  wgrad_mt_plan(B, T_A, M, N, K, groups, 1, &mt);
  splits = std::max<int64_t>(splits, mt.splits);
  if (K == 1 && groups == 1) {
    int64_t k1s;
    int k1r;
    k1_plan(B, T_A, M, N, &k1s, &k1r);
    splits = std::max<int64_t>(splits, k1s);
  }
  return splits * ((int64_t)groups * K * M * N + (int64_t)groups * M) * (int64_t)sizeof(float);
}

template <int TM, int KG, int SW>
static void wgrad_mt_launch(const WgradArgs& p, const MtPlan& pl, int groups, hipStream_t st) {
  const int tiles = ((p.M + TM - 1) / TM) * ((p.N + TM - 1) / TM);
  hipLaunchKernelGGL((wgrad_mt_kernel<TM, KG, SW>), dim3((unsigned)pl.splits, (unsigned)tiles,
                     (unsigned)(pl.ntg * groups)), dim3(256), 0, st, p, pl.chunks_per_b, pl.cps, pl.ntg);
}
template <int TM, int SW>
static void wgrad_mt_dispatch(const WgradArgs& p, const MtPlan& pl, int groups, hipStream_t st) {
  switch (pl.kg) {
    case 1: return wgrad_mt_launch<TM, 1, SW>(p, pl, groups, st);
    case 2: return wgrad_mt_launch<TM, 2, SW>(p, pl, groups, st);
    case 3: return wgrad_mt_launch<TM, 3, SW>(p, pl, groups, st);
    case 4: return wgrad_mt_launch<TM, 4, SW>(p, pl, groups, st);
    case 5: return wgrad_mt_launch<TM, 5, SW>(p, pl, groups, st);
  }
  if constexpr (TM == 32 || SW == 1) {  // TM 64 runs at most 8 taps, 5 when strided (wgrad_mt_plan)
    switch (pl.kg) {
      case 6: return wgrad_mt_launch<TM, 6, SW>(p, pl, groups, st);
      case 7: return wgrad_mt_launch<TM, 7, SW>(p, pl, groups, st);
      case 8: return wgrad_mt_launch<TM, 8, SW>(p, pl, groups, st);
    }
  }
  if constexpr (TM == 32) {
    switch (pl.kg) {
      case 9: return wgrad_mt_launch<32, 9, SW>(p, pl, groups, st);
      case 10: return wgrad_mt_launch<32, 10, SW>(p, pl, groups, st);
      default: return wgrad_mt_launch<32, 11, SW>(p, pl, groups, st);
    }
  }
}

extern "C" int vo_conv1d_wgrad_bias(const void* a, int lda, int T_A, const void* b, int ldb, int T_B, int B, int M,
                                    int N, int K, int S, int dil, int pad, int groups, int pre_a, int pre_b,
                                    float slope, int dtype, float* dw, float* db, float* workspace, void* stream) {
  VO_CHECK_ARG(a && b && dw && workspace, "conv1d_wgrad: null pointer");
  VO_CHECK_ARG(!db || !pre_a, "conv1d_wgrad: the fused bias gradient sums A as stored (pre_a must be off)");
  VO_CHECK_ARG(B > 0 && T_A > 0 && T_B > 0 && K >= 1 && S >= 1 && dil >= 1 && groups >= 1, "conv1d_wgrad: bad sizes");
  VO_CHECK_ARG(dtype == VO_BF16 || dtype == VO_F32 || (dtype == VO_F32X3 && S == 1 && groups == 1),
               "conv1d_wgrad: dtype %d (VO_F32X3: stride 1, ungrouped)", dtype);
  const int ev = dtype == VO_BF16 ? 8 : 4;
  VO_CHECK_ARG(M % ev == 0 && N % ev == 0 && lda % ev == 0 && ldb % ev == 0 && lda >= (int64_t)groups * M &&
                   ldb >= (int64_t)groups * N,
               "conv1d_wgrad: M=%d N=%d (per group, and leading dims) must be multiples of %d", M, N, ev);
  WgradArgs p;
  p.a = a; p.lda = lda; p.T_A = T_A; p.bsrc = b; p.ldb = ldb; p.T_B = T_B;
  p.M = M; p.N = N; p.K = K; p.S = S; p.dil = dil; p.pad = pad; p.Bn = B;
  p.pre_a = pre_a; p.pre_b = pre_b; p.slope = slope;
  p.part = workspace;
  p.bias = db != nullptr;
  p.n_w = (int64_t)groups * K * M * N;
  p.n_tot = p.n_w + (db ? (int64_t)groups * M : 0);
  p.abl = vo_tune_get("wgrad_cfg") == 11 ? 2 : 0;  // 11: no loads (timing)
  p.gpt = 1;
  p.dwf = p.dbf = nullptr;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // K = 1 (Linear layers, bf16): the 128 x 128 tile kernel (wgrad_cfg 14 = the per-tap kernel, A/B)
  if (dtype == VO_BF16 && K == 1 && S == 1 && pad == 0 && groups == 1 && !pre_a && !pre_b && T_A == T_B &&
      vo_tune_get("wgrad_cfg") != 14 && p.abl == 0) {
    int64_t splits;
    k1_plan(B, T_A, M, N, &splits, &p.rows_per_split);
    const int tiles = ((M + K1_T - 1) / K1_T) * ((N + K1_T - 1) / K1_T);
    VO_CHECK_ARG(splits < (1 << 30) && tiles < 65536, "conv1d_wgrad: grid too large");
    const bool direct = splits == 1;
    if (direct) {
      p.dwf = dw;
      p.dbf = db;
    }
    hipLaunchKernelGGL(wgrad_k1_kernel, dim3((unsigned)splits, (unsigned)tiles), dim3(256), 0, st, p);
    if (!direct) wgrad_reduce_launch(workspace, (int)splits, p.n_w, p.n_tot, M, N, K, dw, db, st);
    VO_RETURN_LAUNCH();
  }
  // stride-1 bf16 convs: the multi-tap kernel (wgrad_mt 1 = the per-tap kernel, A/B)
  // (K >= 2 and utterances of >= 8 whole chunks' worth: the per-utterance chunks of short sequences --
  // the MPD's period columns, T_A = 10-34 -- are mostly padding: 207 us per call against the per-tap
  // kernel's flattened rows)
  const int64_t padded = (int64_t)((T_A + WM_R - 1) / WM_R) * WM_R;
  // (K = 1 on the multi-tap kernel measured 4-13 % slower at the C4 decoder's 1x1 shapes)
  // (many-tap convs -- the MSD's k = 41 layers at T_A = 65..257 -- also with up to half the chunk rows padding:
  // the per-tap kernel restages both operands per tap, 41 times; wgrad_mt 3 = the 1/8 rule only)
  const bool mt_ok = K >= 2 && (8 * (padded - T_A) <= T_A ||
                                (K >= 16 && padded <= 2 * (int64_t)T_A && vo_tune_get("wgrad_mt") != 3));
  // strided convs (S <= 4: the MSD's grouped layers) on the multi-tap kernel's wider windows (wgrad_mt 2 = off)
  const bool mt_stride = S == 1 || (S <= 4 && vo_tune_get("wgrad_mt") != 2);
  if (dtype == VO_BF16 && mt_stride && mt_ok && vo_tune_get("wgrad_mt") != 1 && p.abl == 0) {
    MtPlan pl;
    wgrad_mt_plan(B, T_A, M, N, K, groups, dil, &pl, S);
    VO_CHECK_ARG(pl.splits < (1 << 30) && pl.ntg * groups < 65536, "conv1d_wgrad: grid too large");
    if (S == 1)
      pl.tm == 32 ? wgrad_mt_dispatch<32, 1>(p, pl, groups, st) : wgrad_mt_dispatch<64, 1>(p, pl, groups, st);
    else if (S == 2)
      pl.tm == 32 ? wgrad_mt_dispatch<32, 2>(p, pl, groups, st) : wgrad_mt_dispatch<64, 2>(p, pl, groups, st);
    else
      pl.tm == 32 ? wgrad_mt_dispatch<32, 4>(p, pl, groups, st) : wgrad_mt_dispatch<64, 4>(p, pl, groups, st);
    wgrad_reduce_launch(workspace, pl.splits, p.n_w, p.n_tot, M, N, K, dw, db, st);
    VO_RETURN_LAUNCH();
  }
  p.gpt = wgrad_gpt(M, N, groups);
  const int64_t zk = (int64_t)K * (groups / p.gpt);
  const int tiles = ((M * p.gpt + WG_T - 1) / WG_T) * ((N * p.gpt + WG_T - 1) / WG_T);
  int64_t splits;
  wgrad_plan(B, T_A, M, N, K, groups, &splits, &p.rows_per_split);
  VO_CHECK_ARG(splits < (1 << 30) && tiles < 65536 && zk < 65536, "conv1d_wgrad: grid too large");
  dim3 grid((unsigned)splits, (unsigned)tiles, (unsigned)zk);
  // one row split (short sequences: the encoder's 384 rows): the workgroups write dW / db in their final
  // layout -- the reduce pass would only permute (K, M, N) -> (M, N, K); wgrad_cfg 13 keeps it (A/B)
  const bool direct = splits == 1 && vo_tune_get("wgrad_cfg") != 13;
  if (direct) {
    p.dwf = dw;
    p.dbf = db;
  }
  if (dtype == VO_BF16)
    hipLaunchKernelGGL(wgrad_kernel<bf16_t>, grid, dim3(256), 0, st, p);
  else if (dtype == VO_F32X3)
    hipLaunchKernelGGL(wgrad_kernel<bx3_t>, grid, dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL(wgrad_kernel<float>, grid, dim3(256), 0, st, p);
  if (!direct) wgrad_reduce_launch(workspace, (int)splits, p.n_w, p.n_tot, M, N, K, dw, db, st);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_conv1d_wgrad_grouped(const void* a, int lda, int T_A, const void* b, int ldb, int T_B, int B, int M,
                                       int N, int K, int S, int dil, int pad, int groups, int pre_a, int pre_b,
                                       float slope, int dtype, float* dw, float* workspace, void* stream) {
  return vo_conv1d_wgrad_bias(a, lda, T_A, b, ldb, T_B, B, M, N, K, S, dil, pad, groups, pre_a, pre_b, slope, dtype,
                              dw, nullptr, workspace, stream);
}

extern "C" int vo_conv1d_wgrad(const void* a, int lda, int T_A, const void* b, int ldb, int T_B, int B, int M, int N,
                               int K, int S, int dil, int pad, int pre_a, int pre_b, float slope, int dtype, float* dw,
                               float* workspace, void* stream) {
  return vo_conv1d_wgrad_grouped(a, lda, T_A, b, ldb, T_B, B, M, N, K, S, dil, pad, 1, pre_a, pre_b, slope, dtype, dw,
                                 workspace, stream);
}

static int colsum_blocks(int64_t rows, int C, int* rpb) {
  // ~1024 blocks of >= 8 row passes each: enough parallelism for 256 CUs
  const int per = 256 / (C / 8 > 0 ? C / 8 : 1);
  *rpb = (int)std::max<int64_t>(8 * std::max(per, 1), (rows + 1023) / 1024);
  return (int)((rows + *rpb - 1) / *rpb);
}

extern "C" int64_t vo_colsum_workspace_size(int64_t rows, int C) {
  if (rows <= 0 || C <= 0) return 0;
  int rpb;
  return (int64_t)colsum_blocks(rows, C, &rpb) * C * (int64_t)sizeof(float);
}

extern "C" int vo_colsum(const void* x, int64_t rows, int C, int ld, int dtype, float* out, float* workspace,
                         void* stream) {
  VO_CHECK_ARG(x && out && workspace && rows > 0 && C > 0 && ld >= C && C % 8 == 0 && ld % 8 == 0 && C <= 2048,
               "colsum: bad arguments (C %% 8 == 0, C <= 2048)");
  int rpb;
  const int g = colsum_blocks(rows, C, &rpb);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == VO_BF16)
    hipLaunchKernelGGL(colsum_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)x, rows, C, ld, rpb, workspace);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)x, rows, C, ld, rpb, workspace);
  // the block partials [g][C] added in block order: the reduce kernel's bias path (n_w = 0)
  wgrad_reduce_launch(workspace, g, 0, C, 1, 1, 1, nullptr, out, st);
  VO_RETURN_LAUNCH();
}
