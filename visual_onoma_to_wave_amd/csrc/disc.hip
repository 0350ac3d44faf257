// HiFi-GAN training (config C5) glue around the discriminator convs: weight packing for
// grouped convs, the MPD period fold, the MSD average pool, the (B, T) -> (B, T, 8)
// channels-last input, and the GAN / feature-matching / L1 reductions with their gradients.
//
// The reference ships only the HiFi-GAN generator and its training hyper-parameters
// (scripts/hifigan/models.py, scripts/hifigan/config.json:1-31); the discriminators and
// losses follow the HiFi-GAN V1 recipe the config belongs to:
//   MPD  : periods 2, 3, 5, 7, 11; wav reflect-padded to a multiple of p, viewed (T/p, p);
//          Conv2d (k, 1) / (s, 1) = Conv1d along T/p per period column (conv1d stride);
//   MSD  : raw wav, AvgPool1d(4, 2, padding 2) x1, x2; grouped strided Conv1d (conv1d groups);
//   loss : D = sum mean((1 - D(y))^2) + mean(D(G(x))^2); G = sum mean((1 - D(G(x)))^2)
//          + 2 * sum_layers mean|f(y) - f(G(x))| + 45 * L1(mel(y), mel(G(x))).

#include <algorithm>

#include "vo_common.h"

namespace vo {

// dense [K][Co][Ci_pad] from (Co, Ci / groups, K): block-diagonal, zero outside the groups and
// past Ci (Ci_pad >= Ci rounds the 1-channel input layers up to the 8-channel minimum)
template <typename TD>
__global__ void __launch_bounds__(256) pack_grouped_kernel(const float* __restrict__ src, int Co, int Ci, int K,
                                                           int groups, int Ci_pad, TD* __restrict__ dst) {
  const int cig = Ci / groups, cog = Co / groups;
  const int64_t n = (int64_t)K * Co * Ci_pad;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int ci = (int)(i % Ci_pad);
    const int64_t r = i / Ci_pad;
    const int co = (int)(r % Co), k = (int)(r / Co);
    float v = 0.f;
    if (ci < Ci && ci / cig == co / cog) v = src[((int64_t)co * cig + (ci - (co / cog) * cig)) * K + k];
    dst[i] = from_f32<TD>(v);
  }
}

// The diagonal blocks only (dst's other entries are left as they are: a persistent packed
// buffer is zeroed once and then updated in place after each optimizer step -- the dense
// kernel above wrote groups x more, mostly zeros, on every repack).  One thread per source
// element, consecutive threads on consecutive input channels of one (tap, output row): the
// stores of a block row are contiguous.
template <typename TD>
__global__ void __launch_bounds__(256) pack_grouped_blocks_kernel(const float* __restrict__ src, int Co, int cig,
                                                                  int cog, int K, int Ci_pad, TD* __restrict__ dst) {
  const int64_t n = (int64_t)K * Co * cig;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % cig);
    const int64_t r = i / cig;  // k * Co + co
    const int co = (int)(r % Co), k = (int)(r / Co);
    dst[r * Ci_pad + (co / cog) * cig + c] = from_f32<TD>(src[((int64_t)co * cig + c) * K + k]);
  }
}

// Input-gradient weights of one stride phase of a strided / grouped conv (hifigan/gan_ops._dgrad):
// from w (Co, cig, K) fp32 straight to the packed [J][Ci_out][Co_in] layout of the stride-1 grouped
// conv over dY -- tap t <- k_r + S (J - 1 - t) (the phase's taps reversed), channel roles swapped
// per group -- replacing a transpose copy, a zero-row concat, a flip and the grouped pack.
// BLOCKS: write only the diagonal blocks (a persistent buffer zeroed once); else every entry.
template <typename TD, bool BLOCKS>
__global__ void __launch_bounds__(256) pack_dgrad_phase_kernel(const float* __restrict__ w, int Co, int cig, int K,
                                                               int groups, int S, int k_r, int J, int ci_out,
                                                               int co_in, TD* __restrict__ dst) {
  const int Ci = cig * groups, cog = Co / groups;
  const int64_t n = BLOCKS ? (int64_t)J * Ci * cog : (int64_t)J * ci_out * co_in;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    int t, ci, cc;
    if constexpr (BLOCKS) {
      const int c = (int)(i % cog);
      const int64_t r = i / cog;
      ci = (int)(r % Ci); t = (int)(r / Ci);
      cc = (ci / cig) * cog + c;
    } else {
      cc = (int)(i % co_in);
      const int64_t r = i / co_in;
      ci = (int)(r % ci_out); t = (int)(r / ci_out);
    }
    float v = 0.f;
    if (BLOCKS || (ci < Ci && cc < Co && cc / cog == ci / cig))
      v = w[((int64_t)cc * cig + (ci - (ci / cig) * cig)) * K + k_r + S * (J - 1 - t)];
    dst[((int64_t)t * ci_out + ci) * co_in + cc] = from_f32<TD>(v);
  }
}

// Every pack above (and vocoder_glue's plain / input-gradient / ConvTranspose1d packs) as one job of
// a batch: the C5 step re-packs ~270 weights after each optimizer step, 146 + 125 launches of 4-27 us
// (2.6 ms per step) that move ~0.7 GB in all.  A job writes, for rows r < rows and columns
// c = cbase(r) + j (j < width, cbase(r) = (r / rpg) * cpg: the diagonal block of a grouped layout),
// dst[(t * dst_rows + r) * ld + c] for t < T, from src (src_rows, cig, K) fp32:
//   GATHER, swap 0 (forward packs):        src[r][j][tap0 + tstep t]
//   GATHER, swap 1 (input-gradient packs): src[cbase(r) + j][r mod rpg][tap0 + tstep t]
//   CONVT (ConvTranspose1d (Ci, Co = cig, 2s), tap0 = s): src[j][r mod cig][r / cig + s (1 - t)]
// Entries a job does not name are left as they are (persistent buffers zeroed once).
// Each (r, j) reads a run of taps that is contiguous in src; a wave takes 64 such runs (64
// consecutive j of one row, or for narrow rows several whole rows), stages them in its own LDS
// region with coalesced loads (swap 0: the 64 runs are one contiguous block), and then writes tap
// after tap, each a contiguous stretch of dst per row.  (One thread per (r, 4 columns) looping over
// the taps with direct loads ran latency-bound: C5 +0.8 ms against the per-layer kernels.)
constexpr int PJ_MAX = 32;
constexpr int PJ_KMAX = 48;  // tap range staged per run
struct PackBatchArgs {
  VoPackJob j[PJ_MAX];
  int blk0[PJ_MAX + 1];  // first workgroup of each job; blk0[n] = grid size
  int n;
  int kp;                // LDS floats per staged run (max over the launch's jobs; dynamic LDS)
};

__host__ __device__ inline int pj_wpow(int width) {  // lanes per row: the power of two >= width, <= 64
  int w = 1;
  while (w < width && w < 64) w <<= 1;
  return w;
}

template <typename TD>
__global__ void __launch_bounds__(256) pack_batch_kernel(PackBatchArgs a) {
  extern __shared__ float lds[];  // 4 waves x (64 runs x a.kp floats), then 4 x 64 run offsets
  const int b = blockIdx.x;
  const int li = table_find(a.blk0, a.n, b);  // uniform per workgroup
  // the job by value: its fields are read from the kernel arguments once (through a reference
  // the compiler re-read them around every load: a scalar-memory round trip per element)
  const VoPackJob J = a.j[li];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wpow = pj_wpow(J.width), rpw = 64 / wpow;  // rows per wave (narrow rows)
  const int jchunks = (J.width + 63) / 64;              // 64-column chunks per row (wide rows)
  const int unit = (b - a.blk0[li]) * 4 + wv;
  const int r0 = (unit / jchunks) * rpw, j0 = (unit % jchunks) * 64;
  // staged tap range [k0, k0 + L)
  int k0, L;
  if (J.mode == VO_PJ_CONVT) {
    k0 = 0; L = J.K;
  } else {
    const int last = J.tap0 + J.tstep * (J.T - 1);
    k0 = min(J.tap0, last); L = abs(last - J.tap0) + 1;
  }
  const int Kp = L | 1;  // odd LDS row stride: the per-tap reads below hit 64 distinct banks
  float* my = lds + wv * 64 * a.kp;
  int* tab = reinterpret_cast<int*>(lds + 4 * 64 * a.kp) + wv * 64;
  // this lane's run: (r, j) and the source offset of its tap k0 (-1: no such run)
  const int r = r0 + lane / wpow, j = j0 + lane % wpow;
  int base = -1;
  if (r < J.rows && j < J.width) {
    if (J.mode == VO_PJ_CONVT) base = (j * J.cig + r % J.cig) * J.K + k0;
    else if (J.swap) base = (((r / J.rpg) * J.cpg + j) * J.cig + r % J.rpg) * J.K + k0;
    else base = (r * J.cig + j) * J.K + k0;
  }
  tab[lane] = base;
  __syncthreads();
  // stage the 64 runs: element e = q L + k of the wave's block, 64 consecutive e per load
  // (swap 0 and wide rows: one contiguous stretch of src)
  constexpr int NL = 16;  // loads in flight per lane
  const int n = 64 * L, dq = 64 / L, dk = 64 - dq * L;
  int q = lane / L, k = lane - q * L;
  for (int e0 = 0; e0 < n; e0 += NL * 64) {
    float v[NL];
    int at[NL];
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const bool in = e0 + u * 64 + lane < n;
      const int o = in ? tab[q] : -1;
      v[u] = o >= 0 ? J.src[o + k] : 0.f;
      at[u] = in ? q * Kp + k : -1;
      q += dq;
      k += dk;
      if (k >= L) { k -= L; ++q; }
    }
#pragma unroll
    for (int u = 0; u < NL; ++u)
      if (at[u] >= 0) my[at[u]] = v[u];
  }
  __syncthreads();
  if (base < 0) return;
  TD* dst = reinterpret_cast<TD*>(J.dst) + (int64_t)r * J.ld + (r / J.rpg) * J.cpg + j;
  const int64_t plane = (int64_t)J.dst_rows * J.ld;
  const float* row = my + lane * Kp;
  const int tb = J.mode == VO_PJ_CONVT ? r / J.cig + J.tap0 : J.tap0 - k0;
  const int ts = J.mode == VO_PJ_CONVT ? -J.tap0 : J.tstep;
  for (int t = 0; t < J.T; ++t) dst[plane * t] = from_f32<TD>(row[tb + ts * t]);
}

// Row remap between the joined and the per-sequence layouts of the short discriminator sequences
// (hifigan/gan_ops._conv_joined): dst row r = (n, t) with n = r / Td, t = r mod Td receives src row
// n Ss + t + shift when lo <= t < hi, zeros otherwise -- the join (sequences laid end to end with
// their zero padding), the split (valid output slots back to (N, T_out)) and both adjoints, each one
// streaming pass of 16-byte units (F.pad / slice / contiguous ran it as 4-5 fill and copy kernels).
template <typename U>  // U: the copy unit (16, 8 or 4 bytes, the largest that divides a row)
__global__ void __launch_bounds__(256) seq_remap_kernel(const U* __restrict__ src, U* __restrict__ dst, int64_t dst_rows,
                                                        int uv, int Td, int64_t Ss, int lo, int hi, int shift) {
  const int64_t n_units = dst_rows * uv;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_units; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / uv;
    const int c = (int)(i - r * uv);
    const int64_t n = r / Td;
    const int t = (int)(r - n * Td);
    U v = {};
    if (t >= lo && t < hi) v = src[(n * Ss + t + shift) * uv + c];
    dst[i] = v;
  }
}

// Two remaps in one launch (grid y = job), and a job may add a second gathered source (same
// row map, its own sequence stride / shift) in the tensor's dtype: where one joined conv feeds the
// next (gan_ops.RejoinFn) the forward writes the split output and the next joined input from one
// read of the joined output, and the backward adds the two gradients as it gathers them (bit for
// bit autograd's bf16 / fp32 add of the split and join adjoints, which were 2-3 launches).
struct RemapJob {
  const void* src; const void* src2; void* dst;
  int64_t dst_rows, Ss, Ss2;
  int Td, lo, hi, shift, shift2;
};
struct RemapArgs { RemapJob j[2]; int uv; };

template <int DT>  // 16 bytes of bf16 (DT 1) or fp32 (DT 2) added, rounded as the dtype's add
__device__ __forceinline__ uint4 add16(uint4 a, uint4 b) {
  if constexpr (DT == 1) {
    const uint32_t x[4] = {a.x, a.y, a.z, a.w}, y[4] = {b.x, b.y, b.z, b.w};
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      o[i] = pk_bf16(__uint_as_float(x[i] << 16) + __uint_as_float(y[i] << 16),
                     __uint_as_float(x[i] & 0xffff0000u) + __uint_as_float(y[i] & 0xffff0000u));
    return make_uint4(o[0], o[1], o[2], o[3]);
  } else {
    return make_uint4(__float_as_uint(__uint_as_float(a.x) + __uint_as_float(b.x)),
                      __float_as_uint(__uint_as_float(a.y) + __uint_as_float(b.y)),
                      __float_as_uint(__uint_as_float(a.z) + __uint_as_float(b.z)),
                      __float_as_uint(__uint_as_float(a.w) + __uint_as_float(b.w)));
  }
}

template <int DT>
__global__ void __launch_bounds__(256) seq_remap2_kernel(RemapArgs a) {
  const RemapJob& J = a.j[blockIdx.y];
  const uint4* __restrict__ src = reinterpret_cast<const uint4*>(J.src);
  const uint4* __restrict__ src2 = reinterpret_cast<const uint4*>(J.src2);
  uint4* __restrict__ dst = reinterpret_cast<uint4*>(J.dst);
  const int uv = a.uv;
  const int64_t n_units = J.dst_rows * uv;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_units; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / uv;
    const int c = (int)(i - r * uv);
    const int64_t n = r / J.Td;
    const int t = (int)(r - n * J.Td);
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (t >= J.lo && t < J.hi) {
      v = src[(n * J.Ss + t + J.shift) * uv + c];
      if (src2) v = add16<DT>(v, src2[(n * J.Ss2 + t + J.shift2) * uv + c]);
    }
    dst[i] = v;
  }
}

// wav (B, T) fp32 -> (B * P, H, 8) channels-last, H = ceil(T / P): row h of column c holds the
// reflect-padded sample h * P + c in channel 0 (channels 1..7 zero)
template <typename TD>
__global__ void __launch_bounds__(256) period_fold_kernel(const float* __restrict__ wav, int T, int P, int H,
                                                          TD* __restrict__ out) {
  const int b = blockIdx.y;
  const int64_t n = (int64_t)P * H;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i / H), h = (int)(i % H);
    int t = h * P + c;
    if (t >= T) t = 2 * (T - 1) - t;  // F.pad(..., "reflect") on the right
    float v[8] = {wav[(int64_t)b * T + t], 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    store8(out + (((int64_t)b * P + c) * H + h) * 8, v);
  }
}

// (B, T) fp32 -> (B, T, 8) channels-last (channel 0)
template <typename TD>
__global__ void __launch_bounds__(256) wav_cl8_kernel(const float* __restrict__ wav, int64_t n, TD* __restrict__ out) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float v[8] = {wav[i], 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    store8(out + i * 8, v);
  }
}

// AvgPool1d(4, stride 2, padding 2, count_include_pad): y[o] = sum_{i<4} x[2o + i - 2] / 4
__global__ void __launch_bounds__(256) avgpool_kernel(const float* __restrict__ x, int T, int T_out,
                                                      float* __restrict__ y) {
  const int b = blockIdx.y;
  const float* xb = x + (int64_t)b * T;
  for (int o = blockIdx.x * 256 + threadIdx.x; o < T_out; o += gridDim.x * 256) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = 2 * o + i - 2;
      s += (t >= 0 && t < T) ? xb[t] : 0.f;
    }
    y[(int64_t)b * T_out + o] = 0.25f * s;
  }
}

// reductions over a (rows x width) view with leading dimensions lda / ldb:
//   0: sum |a - b|     1: sum (1 - a)^2     2: sum a^2
template <typename TA>
__global__ void __launch_bounds__(256) gan_reduce_kernel(int kind, const TA* __restrict__ a, int lda,
                                                         const TA* __restrict__ b, int ldb, int64_t rows, int width,
                                                         float* __restrict__ part) {
  __shared__ float red[4];
  const int64_t n = rows * width;
  float s = 0.f;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / width;
    const int c = (int)(i - r * width);
    const float x = to_f32(a[r * lda + c]);
    if (kind == 0) {
      s += fabsf(x - to_f32(b[r * ldb + c]));
    } else if (kind == 1) {
      s += (1.f - x) * (1.f - x);
    } else {
      s += x * x;
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// *out += the block partials added in block order (one wave: lanes stride the blocks, a fixed tree)
__global__ void __launch_bounds__(64) gan_reduce_final_kernel(const float* __restrict__ part, int n,
                                                              float* __restrict__ out) {
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 64) s += part[i];
  s = wave_sum(s);
  if (threadIdx.x == 0) out[0] += s;
}

// gradient of scale * reduction wrt a (b held constant), written in a's layout
template <typename TA>
__global__ void __launch_bounds__(256) gan_reduce_grad_kernel(int kind, const TA* __restrict__ a, int lda,
                                                              const TA* __restrict__ b, int ldb, int64_t rows,
                                                              int width, const float* __restrict__ scale,
                                                              TA* __restrict__ ga, int ldg) {
  const int64_t n = rows * width;
  const float s = *scale;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / width;
    const int c = (int)(i - r * width);
    const float x = to_f32(a[r * lda + c]);
    float g;
    if (kind == 0) {
      const float d = x - to_f32(b[r * ldb + c]);
      g = d > 0.f ? s : (d < 0.f ? -s : 0.f);
    } else if (kind == 1) {
      g = -2.f * (1.f - x) * s;
    } else {
      g = 2.f * x * s;
    }
    ga[r * ldg + c] = from_f32<TA>(g);
  }
}

static int grid_for(int64_t n) { return (int)std::min<int64_t>((n + 255) / 256, 4096); }

// 8-element vector forms of the three kernels above (width and leading dimensions multiples of 8,
// 16-byte aligned bases): one 16 / 32-byte load per operand per 8 elements, and the row / column
// split of the flat index (a 64-bit division per ELEMENT in the scalar kernels, which made them
// 10-30 us calls) per vector, or none at all when every operand is contiguous (FLAT)
struct RowMap {
  int64_t wv;  // vectors per row
  __device__ __forceinline__ void at(int64_t v, int64_t* r, int* c) const {
    *r = v / wv;
    *c = (int)(v - *r * wv) * 8;
  }
};

template <typename TA, bool FLAT>
__global__ void __launch_bounds__(256) gan_reduce_v8_kernel(int kind, const TA* __restrict__ a, int lda,
                                                            const TA* __restrict__ b, int ldb, int64_t rows,
                                                            int width, float* __restrict__ part) {
  __shared__ float red[4];
  const RowMap rm{width / 8};
  const int64_t nv = rows * rm.wv;
  float s = 0.f;
  for (int64_t v = blockIdx.x * 256 + threadIdx.x; v < nv; v += (int64_t)gridDim.x * 256) {
    int64_t oa = v * 8, ob = v * 8;
    if constexpr (!FLAT) {
      int64_t r;
      int c;
      rm.at(v, &r, &c);
      oa = r * lda + c;
      ob = r * ldb + c;
    }
    float x[8];
    load8(a + oa, x);
    if (kind == 0) {
      float y[8];
      load8(b + ob, y);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += fabsf(x[e] - y[e]);
    } else if (kind == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) s += (1.f - x[e]) * (1.f - x[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) s += x[e] * x[e];
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

template <typename TA, bool FLAT>
__global__ void __launch_bounds__(256) gan_reduce_grad_v8_kernel(int kind, const TA* __restrict__ a, int lda,
                                                                 const TA* __restrict__ b, int ldb, int64_t rows,
                                                                 int width, const float* __restrict__ scale,
                                                                 TA* __restrict__ ga, int ldg) {
  const RowMap rm{width / 8};
  const int64_t nv = rows * rm.wv;
  const float sc = *scale;
  for (int64_t v = blockIdx.x * 256 + threadIdx.x; v < nv; v += (int64_t)gridDim.x * 256) {
    int64_t oa = v * 8, ob = v * 8, og = v * 8;
    if constexpr (!FLAT) {
      int64_t r;
      int c;
      rm.at(v, &r, &c);
      oa = r * lda + c;
      ob = r * ldb + c;
      og = r * ldg + c;
    }
    float x[8], g[8];
    load8(a + oa, x);
    if (kind == 0) {
      float y[8];
      load8(b + ob, y);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = x[e] - y[e];
        g[e] = d > 0.f ? sc : (d < 0.f ? -sc : 0.f);
      }
    } else if (kind == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = -2.f * (1.f - x[e]) * sc;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = 2.f * x[e] * sc;
    }
    store8(ga + og, g);
  }
}

// ADD 1: out = round(masked) + add[r, c] (then rounded): a residual's gradient summed in the same
// pass -- bit for bit the masked tensor followed by autograd's add of the two gradients.
// ADD 2: out = mask(round(g + add)): two gradients of the activation's output (the next conv's and a
// feature-matching loss's) summed as autograd sums them, then masked
template <typename TG, typename TR, bool FLAT, int ADD = 0>
__global__ void __launch_bounds__(256) lrelu_mask_v8_kernel(const TG* __restrict__ g, int ldg,
                                                            const TR* __restrict__ ref, int ldr, int64_t rows,
                                                            int width, float slope, TG* __restrict__ out, int ldo,
                                                            const TG* __restrict__ add = nullptr, int lda = 0) {
  const RowMap rm{width / 8};
  const int64_t nv = rows * rm.wv;
  for (int64_t v = blockIdx.x * 256 + threadIdx.x; v < nv; v += (int64_t)gridDim.x * 256) {
    int64_t og = v * 8, orf = v * 8, oo = v * 8, oa = v * 8;
    if constexpr (!FLAT) {
      int64_t r;
      int c;
      rm.at(v, &r, &c);
      og = r * ldg + c;
      orf = r * ldr + c;
      oo = r * ldo + c;
      oa = r * lda + c;
    }
    float x[8], q[8];
    load8(g + og, x);
    load8(ref + orf, q);
    if constexpr (ADD == 2) {
      float a[8];
      load8(add + oa, a);
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = to_f32(from_f32<TG>(x[e] + a[e]));
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = q[e] > 0.f ? x[e] : x[e] * slope;
    if constexpr (ADD == 1) {
      float a[8];
      load8(add + oa, a);
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = to_f32(from_f32<TG>(x[e])) + a[e];
    }
    store8(out + oo, x);
  }
}

// Many loss terms per launch (the C5 G step's 54 feature-matching L1 terms and 8 adversarial ones,
// the D step's 16 halves): term i's blocks are blk0[i] .. blk0[i + 1] - 1 of one grid, each doing what
// block b of the single-term kernel's g_i-block grid does (same elements per thread, same sums), so
// the partials, and the per-term sums of them added by one wave each, are those of vo_gan_reduce bit
// for bit; the sums are written times the term's scale.  The gradient kernel likewise covers every
// term's elements in one launch.  (Each term was a reduction, a final sum, and backward a gradient
// launch: ~230 launches of 3-6 us per C5 step.)
constexpr int GT_MAX = 32;
struct GanTerm {
  const void* a; const void* b; void* ga;
  int64_t rows;
  int kind, width, lda, ldb, ldg, v8, g;
};
struct GanArgs {
  GanTerm t[GT_MAX];
  int blk0[GT_MAX + 1];
  int n;
};

template <typename TA>
__global__ void __launch_bounds__(256) gan_multi_reduce_kernel(GanArgs A, float* __restrict__ part) {
  __shared__ float red[4];
  const int li = table_find(A.blk0, A.n, blockIdx.x);
  const GanTerm& T = A.t[li];
  const int64_t bi = blockIdx.x - A.blk0[li], gs = (int64_t)T.g * 256;
  const TA* a = reinterpret_cast<const TA*>(T.a);
  const TA* b = reinterpret_cast<const TA*>(T.b);
  float s = 0.f;
  if (T.v8) {
    const RowMap rm{T.width / 8};
    const int64_t nv = T.rows * rm.wv;
    const bool flat = T.lda == T.width && (!b || T.ldb == T.width);
    for (int64_t v = bi * 256 + threadIdx.x; v < nv; v += gs) {
      int64_t oa = v * 8, ob = v * 8;
      if (!flat) {
        int64_t r;
        int c;
        rm.at(v, &r, &c);
        oa = r * T.lda + c;
        ob = r * T.ldb + c;
      }
      float x[8];
      load8(a + oa, x);
      if (T.kind == 0) {
        float y[8];
        load8(b + ob, y);
#pragma unroll
        for (int e = 0; e < 8; ++e) s += fabsf(x[e] - y[e]);
      } else if (T.kind == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) s += (1.f - x[e]) * (1.f - x[e]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) s += x[e] * x[e];
      }
    }
  } else {
    const int64_t n = T.rows * T.width;
    for (int64_t i = bi * 256 + threadIdx.x; i < n; i += gs) {
      const int64_t r = i / T.width;
      const int c = (int)(i - r * T.width);
      const float x = to_f32(a[r * T.lda + c]);
      if (T.kind == 0) {
        s += fabsf(x - to_f32(b[r * T.ldb + c]));
      } else if (T.kind == 1) {
        s += (1.f - x) * (1.f - x);
      } else {
        s += x * x;
      }
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// one wave per term: its partials added as gan_reduce_final_kernel adds them, times the term's scale
__global__ void __launch_bounds__(64) gan_multi_final_kernel(GanArgs A, const float* __restrict__ part,
                                                             const float* __restrict__ scale, float* __restrict__ out) {
  const int li = blockIdx.x;
  const int p0 = A.blk0[li], n = A.blk0[li + 1] - p0;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 64) s += part[p0 + i];
  s = wave_sum(s);
  if (threadIdx.x == 0) out[li] = (0.f + s) * (scale ? scale[li] : 1.f);
}

template <typename TA>
__global__ void __launch_bounds__(256) gan_multi_grad_kernel(GanArgs A, const float* __restrict__ scale) {
  const int li = table_find(A.blk0, A.n, blockIdx.x);
  const GanTerm& T = A.t[li];
  const int64_t bi = blockIdx.x - A.blk0[li], gs = (int64_t)(A.blk0[li + 1] - A.blk0[li]) * 256;
  const TA* a = reinterpret_cast<const TA*>(T.a);
  const TA* b = reinterpret_cast<const TA*>(T.b);
  TA* ga = reinterpret_cast<TA*>(T.ga);
  const float sc = scale[li];
  if (T.v8) {
    const RowMap rm{T.width / 8};
    const int64_t nv = T.rows * rm.wv;
    for (int64_t v = bi * 256 + threadIdx.x; v < nv; v += gs) {
      int64_t r;
      int c;
      rm.at(v, &r, &c);
      float x[8], g[8];
      load8(a + r * T.lda + c, x);
      if (T.kind == 0) {
        float y[8];
        load8(b + r * T.ldb + c, y);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = x[e] - y[e];
          g[e] = d > 0.f ? sc : (d < 0.f ? -sc : 0.f);
        }
      } else if (T.kind == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = -2.f * (1.f - x[e]) * sc;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = 2.f * x[e] * sc;
      }
      store8(ga + r * T.ldg + c, g);
    }
  } else {
    const int64_t n = T.rows * T.width;
    for (int64_t i = bi * 256 + threadIdx.x; i < n; i += gs) {
      const int64_t r = i / T.width;
      const int c = (int)(i - r * T.width);
      const float x = to_f32(a[r * T.lda + c]);
      float g;
      if (T.kind == 0) {
        const float d = x - to_f32(b[r * T.ldb + c]);
        g = d > 0.f ? sc : (d < 0.f ? -sc : 0.f);
      } else if (T.kind == 1) {
        g = -2.f * (1.f - x) * sc;
      } else {
        g = 2.f * x * sc;
      }
      ga[r * T.ldg + c] = from_f32<TA>(g);
    }
  }
}

static bool v8_ok(const void* p, int64_t ld) { return p == nullptr || (((uintptr_t)p & 15) == 0 && ld % 8 == 0); }


// leaky-ReLU backward mask: out = g * (ref > 0 ? 1 : slope) over a (rows x width) view with
// leading dimensions (out may alias g).  ref = the activation's input or its output (same sign
// for slope > 0).  One launch instead of PyTorch's compare / where / cast / mul chain.
template <typename TG, typename TR>
__global__ void __launch_bounds__(256) lrelu_mask_kernel(const TG* __restrict__ g, int ldg, const TR* __restrict__ ref,
                                                         int ldr, int64_t rows, int width, float slope,
                                                         TG* __restrict__ out, int ldo) {
  const int64_t n = rows * width;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / width;
    const int c = (int)(i - r * width);
    const float v = to_f32(g[r * ldg + c]);
    out[r * ldo + c] = from_f32<TG>(to_f32(ref[r * ldr + c]) > 0.f ? v : v * slope);
  }
}

// adjoints of the three input transforms above (dL/dwav, fp32):
//  period fold: sample t gets row t / P of column t % P, plus the right-pad row that mirrored it
template <typename TG>
__global__ void __launch_bounds__(256) period_fold_bwd_kernel(const TG* __restrict__ g, int T, int P, int H,
                                                              float* __restrict__ gw) {
  const int b = blockIdx.y;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < T; t += gridDim.x * 256) {
    float s = to_f32(g[(((int64_t)b * P + t % P) * H + t / P) * 8]);
    const int tm = 2 * (T - 1) - t;  // the padded position that copied sample t, if it exists
    if (tm >= T && tm < H * P) s += to_f32(g[(((int64_t)b * P + tm % P) * H + tm / P) * 8]);
    gw[(int64_t)b * T + t] = s;
  }
}

template <typename TG>
__global__ void __launch_bounds__(256) wav_cl8_bwd_kernel(const TG* __restrict__ g, int64_t n, float* __restrict__ gw) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) gw[i] = to_f32(g[i * 8]);
}

//  average pool: x[t] feeds outputs o with 2o - 2 <= t <= 2o + 1, each with weight 1/4
__global__ void __launch_bounds__(256) avgpool_bwd_kernel(const float* __restrict__ g, int T, int T_out,
                                                          float* __restrict__ gx) {
  const int b = blockIdx.y;
  const float* gb = g + (int64_t)b * T_out;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < T; t += gridDim.x * 256) {
    const int o0 = t / 2;  // outputs o0 (taps 2, 3) and o0 + 1 (taps 0, 1)
    float s = 0.f;
    if (o0 < T_out) s += gb[o0];
    if (o0 + 1 < T_out) s += gb[o0 + 1];
    gx[(int64_t)b * T + t] = 0.25f * s;
  }
}

}  // namespace vo

using namespace vo;

extern "C" int vo_pack_grouped(const float* src, int Co, int Ci, int K, int groups, int Ci_pad, void* dst,
                               int dst_dtype, void* stream) {
  VO_CHECK_ARG(src && dst, "pack_grouped: null pointer");
  VO_CHECK_ARG(groups >= 1 && Co % groups == 0 && Ci % groups == 0 && Ci_pad >= Ci && K >= 1,
               "pack_grouped: bad sizes Co=%d Ci=%d groups=%d Ci_pad=%d", Co, Ci, groups, Ci_pad);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int g = grid_for((int64_t)K * Co * Ci_pad);
  if (dst_dtype == VO_BF16)
    hipLaunchKernelGGL(pack_grouped_kernel<bf16_t>, dim3(g), dim3(256), 0, st, src, Co, Ci, K, groups, Ci_pad,
                       (bf16_t*)dst);
  else
    hipLaunchKernelGGL(pack_grouped_kernel<float>, dim3(g), dim3(256), 0, st, src, Co, Ci, K, groups, Ci_pad,
                       (float*)dst);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_pack_grouped_blocks(const float* src, int Co, int Ci, int K, int groups, int Ci_pad, void* dst,
                                      int dst_dtype, void* stream) {
  VO_CHECK_ARG(src && dst, "pack_grouped_blocks: null pointer");
  VO_CHECK_ARG(groups >= 1 && Co % groups == 0 && Ci % groups == 0 && Ci_pad >= Ci && K >= 1,
               "pack_grouped_blocks: bad sizes Co=%d Ci=%d groups=%d Ci_pad=%d", Co, Ci, groups, Ci_pad);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int cig = Ci / groups, cog = Co / groups;
  const int g = grid_for((int64_t)K * Co * cig);
  if (dst_dtype == VO_BF16)
    hipLaunchKernelGGL(pack_grouped_blocks_kernel<bf16_t>, dim3(g), dim3(256), 0, st, src, Co, cig, cog, K, Ci_pad,
                       (bf16_t*)dst);
  else
    hipLaunchKernelGGL(pack_grouped_blocks_kernel<float>, dim3(g), dim3(256), 0, st, src, Co, cig, cog, K, Ci_pad,
                       (float*)dst);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_pack_dgrad_phase(const float* w, int Co, int cig, int K, int groups, int S, int k_r, int J,
                                   int ci_out, int co_in, int blocks_only, void* dst, int dst_dtype, void* stream) {
  VO_CHECK_ARG(w && dst, "pack_dgrad_phase: null pointer");
  VO_CHECK_ARG(groups >= 1 && Co % groups == 0 && cig >= 1 && K >= 1 && S >= 1 && k_r >= 0 && J >= 1 &&
                   k_r + S * (J - 1) < K && ci_out >= cig * groups && co_in >= Co,
               "pack_dgrad_phase: bad sizes Co=%d cig=%d K=%d groups=%d S=%d k_r=%d J=%d ci_out=%d co_in=%d", Co, cig,
               K, groups, S, k_r, J, ci_out, co_in);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = blocks_only ? (int64_t)J * cig * groups * (Co / groups) : (int64_t)J * ci_out * co_in;
  const int g = grid_for(n);
#define VO_PDP(TD, B)                                                                                          \
  hipLaunchKernelGGL((pack_dgrad_phase_kernel<TD, B>), dim3(g), dim3(256), 0, st, w, Co, cig, K, groups, S, k_r, \
                     J, ci_out, co_in, (TD*)dst)
  if (dst_dtype == VO_BF16) {
    if (blocks_only) VO_PDP(bf16_t, true); else VO_PDP(bf16_t, false);
  } else {
    if (blocks_only) VO_PDP(float, true); else VO_PDP(float, false);
  }
#undef VO_PDP
  VO_RETURN_LAUNCH();
}

extern "C" int vo_pack_batch(int n, const VoPackJob* jobs, int dst_dtype, void* stream) {
  VO_CHECK_ARG(n >= 0 && (n == 0 || jobs), "pack_batch: null job table");
  VO_CHECK_ARG(dst_dtype == VO_BF16 || dst_dtype == VO_F32, "pack_batch: dst dtype %d", dst_dtype);
  for (int i = 0; i < n; ++i) {
    const VoPackJob& J = jobs[i];
    VO_CHECK_ARG(J.src && J.dst, "pack_batch: job %d: null pointer", i);
    VO_CHECK_ARG(J.mode == VO_PJ_GATHER || J.mode == VO_PJ_CONVT, "pack_batch: job %d: mode %d", i, J.mode);
    VO_CHECK_ARG(J.T >= 1 && J.rows >= 1 && J.width >= 1 && J.rpg >= 1 && J.cpg >= 0 && J.cig >= 1 && J.K >= 1 &&
                     J.src_rows >= 1 && J.dst_rows >= J.rows,
                 "pack_batch: job %d: bad sizes", i);
    VO_CHECK_ARG(J.mode == VO_PJ_CONVT ? J.K <= PJ_KMAX : std::abs(J.tstep) * (J.T - 1) + 1 <= PJ_KMAX,
                 "pack_batch: job %d: tap range over %d", i, PJ_KMAX);
    VO_CHECK_ARG((int64_t)((J.rows - 1) / J.rpg) * J.cpg + J.width <= J.ld, "pack_batch: job %d: row exceeds ld", i);
    VO_CHECK_ARG((int64_t)J.src_rows * J.cig * J.K < (1LL << 31) && (int64_t)J.rows * J.width < (1LL << 30),
                 "pack_batch: job %d too large", i);
    if (J.mode == VO_PJ_CONVT) {
      VO_CHECK_ARG(J.T == 2 && J.K == 2 * J.tap0 && J.rows == J.tap0 * J.cig && J.width <= J.src_rows,
                   "pack_batch: job %d: ConvTranspose1d job needs T = 2, K = 2 s, rows = s Co", i);
    } else {
      const int last = J.tap0 + J.tstep * (J.T - 1);
      VO_CHECK_ARG(J.tap0 >= 0 && J.tap0 < J.K && last >= 0 && last < J.K, "pack_batch: job %d: taps outside [0, K)",
                   i);
      if (J.swap)
        VO_CHECK_ARG(J.rpg <= J.cig && ((J.rows - 1) / J.rpg) * J.cpg + J.width <= J.src_rows,
                     "pack_batch: job %d: source row / channel out of range", i);
      else
        VO_CHECK_ARG(J.rows <= J.src_rows && J.width <= J.cig, "pack_batch: job %d: source row / channel out of range",
                     i);
    }
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int i0 = 0; i0 < n; i0 += PJ_MAX) {
    PackBatchArgs a;
    a.n = std::min(PJ_MAX, n - i0);
    int64_t blocks = 0;
    a.kp = 1;
    for (int i = 0; i < a.n; ++i) {
      a.j[i] = jobs[i0 + i];
      a.blk0[i] = (int)blocks;
      const VoPackJob& J = a.j[i];
      const int rpw = 64 / pj_wpow(J.width);
      const int64_t units = (int64_t)((J.rows + rpw - 1) / rpw) * ((J.width + 63) / 64);  // one wave each
      blocks += (units + 3) / 4;
      const int L = J.mode == VO_PJ_CONVT ? J.K : std::abs(J.tstep) * (J.T - 1) + 1;
      a.kp = std::max(a.kp, L | 1);
    }
    VO_CHECK_ARG(blocks < (1LL << 31), "pack_batch: grid too large");
    const size_t lds = (size_t)4 * 64 * (a.kp + 1) * sizeof(float);
    a.blk0[a.n] = (int)blocks;
    if (dst_dtype == VO_BF16)
      hipLaunchKernelGGL(pack_batch_kernel<bf16_t>, dim3((unsigned)blocks), dim3(256), lds, st, a);
    else
      hipLaunchKernelGGL(pack_batch_kernel<float>, dim3((unsigned)blocks), dim3(256), lds, st, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      vo_set_error("pack_batch: launch failed: %s", hipGetErrorString(e));
      return (int)e;
    }
  }
  return VO_OK;
}

extern "C" int vo_seq_remap(const void* src, int64_t src_rows, void* dst, int64_t dst_rows, int row_bytes, int Td,
                            int64_t Ss, int lo, int hi, int shift, void* stream) {
  VO_CHECK_ARG(src && dst && src != dst, "seq_remap: null or aliased pointers");
  const int unit = row_bytes % 16 == 0 ? 16 : row_bytes % 8 == 0 ? 8 : 4;
  VO_CHECK_ARG(row_bytes > 0 && row_bytes % 4 == 0 && (reinterpret_cast<uintptr_t>(src) % unit) == 0 &&
                   (reinterpret_cast<uintptr_t>(dst) % unit) == 0,
               "seq_remap: rows of %d bytes / pointers not 4-byte multiples", row_bytes);
  VO_CHECK_ARG(dst_rows >= 0 && Td >= 1 && Ss >= 0 && 0 <= lo && lo <= hi && hi <= Td, "seq_remap: bad layout");
  if (dst_rows == 0) return VO_OK;
  if (lo < hi) {  // every row read lies in src
    const int64_t n_last = (dst_rows - 1) / Td;
    const int t_hi = (int)std::min<int64_t>(hi, n_last == 0 ? dst_rows : Td) - 1;
    VO_CHECK_ARG(lo + shift >= 0 && n_last * Ss + t_hi + shift < src_rows,
                 "seq_remap: reads outside the %lld source rows", (long long)src_rows);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int uv = row_bytes / unit;
  const dim3 g(grid_for(dst_rows * uv));
  if (unit == 16)
    hipLaunchKernelGGL(seq_remap_kernel<uint4>, g, dim3(256), 0, st, (const uint4*)src, (uint4*)dst, dst_rows, uv, Td,
                       Ss, lo, hi, shift);
  else if (unit == 8)
    hipLaunchKernelGGL(seq_remap_kernel<uint2>, g, dim3(256), 0, st, (const uint2*)src, (uint2*)dst, dst_rows, uv, Td,
                       Ss, lo, hi, shift);
  else
    hipLaunchKernelGGL(seq_remap_kernel<uint32_t>, g, dim3(256), 0, st, (const uint32_t*)src, (uint32_t*)dst,
                       dst_rows, uv, Td, Ss, lo, hi, shift);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_seq_remap2(int n, const VoRemapJob* jobs, int row_bytes, int dtype, void* stream) {
  VO_CHECK_ARG(n >= 1 && n <= 2 && jobs, "seq_remap2: 1 or 2 jobs");
  VO_CHECK_ARG(row_bytes > 0 && row_bytes % 16 == 0 && (dtype == VO_BF16 || dtype == VO_F32),
               "seq_remap2: rows of whole 16-byte units (got %d bytes), bf16 or fp32", row_bytes);
  RemapArgs a;
  a.uv = row_bytes / 16;
  int64_t units = 0;
  for (int i = 0; i < n; ++i) {
    const VoRemapJob& s = jobs[i];
    VO_CHECK_ARG(s.src && s.dst && s.src != s.dst && s.src2 != s.dst, "seq_remap2: job %d: null or aliased pointers", i);
    VO_CHECK_ARG(((reinterpret_cast<uintptr_t>(s.src) | reinterpret_cast<uintptr_t>(s.dst) |
                   reinterpret_cast<uintptr_t>(s.src2)) & 15) == 0, "seq_remap2: job %d: pointers not 16-byte aligned", i);
    VO_CHECK_ARG(s.dst_rows >= 0 && s.Td >= 1 && s.Ss >= 0 && s.Ss2 >= 0 && 0 <= s.lo && s.lo <= s.hi && s.hi <= s.Td,
                 "seq_remap2: job %d: bad layout", i);
    if (s.dst_rows > 0 && s.lo < s.hi) {  // every row read lies in its source
      const int64_t n_last = (s.dst_rows - 1) / s.Td;
      const int t_hi = (int)std::min<int64_t>(s.hi, n_last == 0 ? s.dst_rows : s.Td) - 1;
      VO_CHECK_ARG(s.lo + s.shift >= 0 && n_last * s.Ss + t_hi + s.shift < s.src_rows,
                   "seq_remap2: job %d: reads outside the %lld source rows", i, (long long)s.src_rows);
      VO_CHECK_ARG(!s.src2 || (s.lo + s.shift2 >= 0 && n_last * s.Ss2 + t_hi + s.shift2 < s.src2_rows),
                   "seq_remap2: job %d: reads outside the %lld rows of the second source", i, (long long)s.src2_rows);
    }
    a.j[i] = RemapJob{s.src, s.src2, s.dst, s.dst_rows, s.Ss, s.Ss2, s.Td, s.lo, s.hi, s.shift, s.shift2};
    units = std::max<int64_t>(units, s.dst_rows * a.uv);
  }
  if (n == 1) a.j[1] = a.j[0];
  if (units == 0) return VO_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 g((unsigned)grid_for(units), (unsigned)n);
  if (dtype == VO_BF16)
    hipLaunchKernelGGL(seq_remap2_kernel<1>, g, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(seq_remap2_kernel<2>, g, dim3(256), 0, st, a);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_period_fold(const float* wav, int B, int T, int P, void* out, int dtype, void* stream) {
  VO_CHECK_ARG(wav && out, "period_fold: null pointer");
  VO_CHECK_ARG(B > 0 && P >= 1 && T > P, "period_fold: need T > P (B=%d T=%d P=%d)", B, T, P);
  const int H = (T + P - 1) / P;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(grid_for((int64_t)P * H), B);
  if (dtype == VO_BF16)
    hipLaunchKernelGGL(period_fold_kernel<bf16_t>, grid, dim3(256), 0, st, wav, T, P, H, (bf16_t*)out);
  else
    hipLaunchKernelGGL(period_fold_kernel<float>, grid, dim3(256), 0, st, wav, T, P, H, (float*)out);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_wav_cl8(const float* wav, int64_t n, void* out, int dtype, void* stream) {
  VO_CHECK_ARG(wav && out && n > 0, "wav_cl8: bad arguments");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == VO_BF16)
    hipLaunchKernelGGL(wav_cl8_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, wav, n, (bf16_t*)out);
  else
    hipLaunchKernelGGL(wav_cl8_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, wav, n, (float*)out);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_avgpool_wav(const float* x, int B, int T, float* y, void* stream) {
  VO_CHECK_ARG(x && y && B > 0 && T > 0, "avgpool_wav: bad arguments");
  const int T_out = T / 2 + 1;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(avgpool_kernel, dim3(grid_for(T_out), B), dim3(256), 0, st, x, T, T_out, y);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_gan_reduce(int kind, const void* a, int lda, const void* b, int ldb, int64_t rows, int width,
                             int dtype, float* out, float* workspace, void* stream) {
  VO_CHECK_ARG(a && out && workspace && kind >= 0 && kind <= 2 && (kind != 0 || b), "gan_reduce: bad arguments");
  VO_CHECK_ARG(rows > 0 && width > 0 && lda >= width && (kind != 0 || ldb >= width), "gan_reduce: bad shape");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // at most 512 block partials (workspace: 512 floats), added in order by one wave (deterministic;
  // the grid-stride loop keeps the loads coalesced)
  int g = std::min(grid_for(rows * width), 512);
  if (width % 8 == 0 && v8_ok(a, lda) && v8_ok(b, ldb)) {
    g = std::min(grid_for(rows * (width / 8)), 512);
    const bool flat = lda == width && (!b || ldb == width);
#define VO_GR(TA, F)                                                                                     \
  hipLaunchKernelGGL((gan_reduce_v8_kernel<TA, F>), dim3(g), dim3(256), 0, st, kind, (const TA*)a, lda, \
                     (const TA*)b, ldb, rows, width, workspace)
    if (dtype == VO_BF16) {
      if (flat) VO_GR(bf16_t, true); else VO_GR(bf16_t, false);
    } else {
      if (flat) VO_GR(float, true); else VO_GR(float, false);
    }
#undef VO_GR
  } else if (dtype == VO_BF16) {
    hipLaunchKernelGGL(gan_reduce_kernel<bf16_t>, dim3(g), dim3(256), 0, st, kind, (const bf16_t*)a, lda,
                       (const bf16_t*)b, ldb, rows, width, workspace);
  } else {
    hipLaunchKernelGGL(gan_reduce_kernel<float>, dim3(g), dim3(256), 0, st, kind, (const float*)a, lda,
                       (const float*)b, ldb, rows, width, workspace);
  }
  hipLaunchKernelGGL(gan_reduce_final_kernel, dim3(1), dim3(64), 0, st, workspace, g, out);
  VO_RETURN_LAUNCH();
}

// the term table of one launch: the block grid of each term as the single-term entry points size it
static int gan_multi_args(const VoGanTerm* terms, int n, bool grad, GanArgs* A, int* blocks) {
  int total = 0;
  for (int i = 0; i < n; ++i) {
    const VoGanTerm& s = terms[i];
    VO_CHECK_ARG(s.a && s.kind >= 0 && s.kind <= 2 && (s.kind != 0 || s.b) && (!grad || s.ga),
                 "gan_reduce_multi: term %d: bad arguments", i);
    VO_CHECK_ARG(s.rows > 0 && s.width > 0 && s.lda >= s.width && (s.kind != 0 || s.ldb >= s.width) &&
                     (!grad || s.ldg >= s.width),
                 "gan_reduce_multi: term %d: bad shape", i);
    GanTerm& t = A->t[i];
    t.a = s.a; t.b = s.b; t.ga = s.ga; t.rows = s.rows;
    t.kind = s.kind; t.width = s.width; t.lda = s.lda; t.ldb = s.ldb; t.ldg = s.ldg;
    t.v8 = s.width % 8 == 0 && v8_ok(s.a, s.lda) && v8_ok(s.b, s.ldb) && (!grad || v8_ok(s.ga, s.ldg));
    const int64_t units = t.v8 ? s.rows * (s.width / 8) : s.rows * s.width;
    t.g = grad ? grid_for(units) : std::min(grid_for(units), 512);
    A->blk0[i] = total;
    total += t.g;
  }
  A->blk0[n] = total;
  A->n = n;
  *blocks = total;
  return VO_OK;
}

extern "C" int64_t vo_gan_reduce_multi_workspace_size(int n) {
  return n <= 0 ? 0 : (int64_t)std::min(n, GT_MAX) * 512 * (int64_t)sizeof(float);
}

extern "C" int vo_gan_reduce_multi(int n, const VoGanTerm* terms, int dtype, const float* scale, float* out,
                                   float* workspace, void* stream) {
  VO_CHECK_ARG(n >= 0 && (n == 0 || (terms && out && workspace)) && (dtype == VO_BF16 || dtype == VO_F32),
               "gan_reduce_multi: bad arguments");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int i0 = 0; i0 < n; i0 += GT_MAX) {
    GanArgs A;
    int blocks;
    const int m = std::min(GT_MAX, n - i0);
    const int rc = gan_multi_args(terms + i0, m, false, &A, &blocks);
    if (rc != VO_OK) return rc;
    if (dtype == VO_BF16)
      hipLaunchKernelGGL(gan_multi_reduce_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, A, workspace);
    else
      hipLaunchKernelGGL(gan_multi_reduce_kernel<float>, dim3(blocks), dim3(256), 0, st, A, workspace);
    hipLaunchKernelGGL(gan_multi_final_kernel, dim3(m), dim3(64), 0, st, A, workspace, scale ? scale + i0 : nullptr,
                       out + i0);
  }
  VO_RETURN_LAUNCH();
}

extern "C" int vo_gan_reduce_grad_multi(int n, const VoGanTerm* terms, int dtype, const float* scale, void* stream) {
  VO_CHECK_ARG(n >= 0 && (n == 0 || (terms && scale)) && (dtype == VO_BF16 || dtype == VO_F32),
               "gan_reduce_grad_multi: bad arguments");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int i0 = 0; i0 < n; i0 += GT_MAX) {
    GanArgs A;
    int blocks;
    const int m = std::min(GT_MAX, n - i0);
    const int rc = gan_multi_args(terms + i0, m, true, &A, &blocks);
    if (rc != VO_OK) return rc;
    if (dtype == VO_BF16)
      hipLaunchKernelGGL(gan_multi_grad_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, A, scale + i0);
    else
      hipLaunchKernelGGL(gan_multi_grad_kernel<float>, dim3(blocks), dim3(256), 0, st, A, scale + i0);
  }
  VO_RETURN_LAUNCH();
}

extern "C" int vo_gan_reduce_grad(int kind, const void* a, int lda, const void* b, int ldb, int64_t rows, int width,
                                  int dtype, const float* scale, void* ga, int ldg, void* stream) {
  VO_CHECK_ARG(a && ga && scale && kind >= 0 && kind <= 2 && (kind != 0 || b), "gan_reduce_grad: bad arguments");
  VO_CHECK_ARG(rows > 0 && width > 0 && lda >= width && ldg >= width, "gan_reduce_grad: bad shape");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (width % 8 == 0 && v8_ok(a, lda) && v8_ok(b, ldb) && v8_ok(ga, ldg)) {
    const int gv = grid_for(rows * (width / 8));
    const bool flat = lda == width && (!b || ldb == width) && ldg == width;
#define VO_GG(TA, F)                                                                                           \
  hipLaunchKernelGGL((gan_reduce_grad_v8_kernel<TA, F>), dim3(gv), dim3(256), 0, st, kind, (const TA*)a, lda, \
                     (const TA*)b, ldb, rows, width, scale, (TA*)ga, ldg)
    if (dtype == VO_BF16) {
      if (flat) VO_GG(bf16_t, true); else VO_GG(bf16_t, false);
    } else {
      if (flat) VO_GG(float, true); else VO_GG(float, false);
    }
#undef VO_GG
    VO_RETURN_LAUNCH();
  }
  const int g = grid_for(rows * width);
  if (dtype == VO_BF16)
    hipLaunchKernelGGL(gan_reduce_grad_kernel<bf16_t>, dim3(g), dim3(256), 0, st, kind, (const bf16_t*)a, lda,
                       (const bf16_t*)b, ldb, rows, width, scale, (bf16_t*)ga, ldg);
  else
    hipLaunchKernelGGL(gan_reduce_grad_kernel<float>, dim3(g), dim3(256), 0, st, kind, (const float*)a, lda,
                       (const float*)b, ldb, rows, width, scale, (float*)ga, ldg);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_lrelu_mask(const void* g, int ldg, int g_dtype, const void* ref, int ldr, int ref_dtype,
                             int64_t rows, int width, float slope, void* out, int ldo, void* stream) {
  VO_CHECK_ARG(g && ref && out, "lrelu_mask: null pointer");
  VO_CHECK_ARG(rows > 0 && width > 0 && ldg >= width && ldr >= width && ldo >= width, "lrelu_mask: bad shape");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (width % 8 == 0 && v8_ok(g, ldg) && v8_ok(ref, ldr) && v8_ok(out, ldo)) {
    const int gv = grid_for(rows * (width / 8));
    const bool flat = ldg == width && ldr == width && ldo == width;
#define VO_LM8(TG, TR)                                                                                             \
  do {                                                                                                             \
    if (flat)                                                                                                      \
      hipLaunchKernelGGL((lrelu_mask_v8_kernel<TG, TR, true>), dim3(gv), dim3(256), 0, st, (const TG*)g, ldg,      \
                         (const TR*)ref, ldr, rows, width, slope, (TG*)out, ldo);                                  \
    else                                                                                                           \
      hipLaunchKernelGGL((lrelu_mask_v8_kernel<TG, TR, false>), dim3(gv), dim3(256), 0, st, (const TG*)g, ldg,     \
                         (const TR*)ref, ldr, rows, width, slope, (TG*)out, ldo);                                  \
  } while (0)
    if (g_dtype == VO_BF16 && ref_dtype == VO_BF16) VO_LM8(bf16_t, bf16_t);
    else if (g_dtype == VO_F32 && ref_dtype == VO_F32) VO_LM8(float, float);
    else if (g_dtype == VO_BF16 && ref_dtype == VO_F32) VO_LM8(bf16_t, float);
    else if (g_dtype == VO_F32 && ref_dtype == VO_BF16) VO_LM8(float, bf16_t);
    else {
      vo_set_error("lrelu_mask: bad dtypes");
      return VO_ERR_INVALID;
    }
#undef VO_LM8
    VO_RETURN_LAUNCH();
  }
  const int gr = grid_for(rows * width);
#define VO_LM(TG, TR)                                                                                          \
  hipLaunchKernelGGL((lrelu_mask_kernel<TG, TR>), dim3(gr), dim3(256), 0, st, (const TG*)g, ldg, (const TR*)ref, \
                     ldr, rows, width, slope, (TG*)out, ldo)
  if (g_dtype == VO_BF16 && ref_dtype == VO_BF16) VO_LM(bf16_t, bf16_t);
  else if (g_dtype == VO_F32 && ref_dtype == VO_F32) VO_LM(float, float);
  else if (g_dtype == VO_BF16 && ref_dtype == VO_F32) VO_LM(bf16_t, float);
  else if (g_dtype == VO_F32 && ref_dtype == VO_BF16) VO_LM(float, bf16_t);
  else {
    vo_set_error("lrelu_mask: bad dtypes");
    return VO_ERR_INVALID;
  }
#undef VO_LM
  VO_RETURN_LAUNCH();
}

static int lrelu_mask_add_run(const void* g, int ldg, int g_dtype, const void* ref, int ldr, int ref_dtype,
                              const void* add, int lda, int64_t rows, int width, float slope, void* out, int ldo,
                              bool presum, void* stream) {
  VO_CHECK_ARG(g && ref && add && out, "lrelu_mask_add: null pointer");
  VO_CHECK_ARG(rows > 0 && width > 0 && ldg >= width && ldr >= width && ldo >= width && lda >= width,
               "lrelu_mask_add: bad shape");
  VO_CHECK_ARG(width % 8 == 0 && v8_ok(g, ldg) && v8_ok(ref, ldr) && v8_ok(out, ldo) && v8_ok(add, lda),
               "lrelu_mask_add: rows must be 8-element vectors, 16-byte aligned");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int gv = grid_for(rows * (width / 8));
#define VO_LMA(TG, TR)                                                                                                 \
  if (presum)                                                                                                          \
    hipLaunchKernelGGL((lrelu_mask_v8_kernel<TG, TR, false, 2>), dim3(gv), dim3(256), 0, st, (const TG*)g, ldg,         \
                       (const TR*)ref, ldr, rows, width, slope, (TG*)out, ldo, (const TG*)add, lda);                   \
  else                                                                                                                 \
    hipLaunchKernelGGL((lrelu_mask_v8_kernel<TG, TR, false, 1>), dim3(gv), dim3(256), 0, st, (const TG*)g, ldg,         \
                       (const TR*)ref, ldr, rows, width, slope, (TG*)out, ldo, (const TG*)add, lda)
  if (g_dtype == VO_BF16 && ref_dtype == VO_BF16) VO_LMA(bf16_t, bf16_t);
  else if (g_dtype == VO_F32 && ref_dtype == VO_F32) VO_LMA(float, float);
  else if (g_dtype == VO_BF16 && ref_dtype == VO_F32) VO_LMA(bf16_t, float);
  else if (g_dtype == VO_F32 && ref_dtype == VO_BF16) VO_LMA(float, bf16_t);
  else {
    vo_set_error("lrelu_mask_add: bad dtypes");
    return VO_ERR_INVALID;
  }
#undef VO_LMA
  VO_RETURN_LAUNCH();
}

extern "C" int vo_lrelu_mask_add(const void* g, int ldg, int g_dtype, const void* ref, int ldr, int ref_dtype,
                                 const void* add, int lda, int64_t rows, int width, float slope, void* out, int ldo,
                                 void* stream) {
  return lrelu_mask_add_run(g, ldg, g_dtype, ref, ldr, ref_dtype, add, lda, rows, width, slope, out, ldo, false, stream);
}

extern "C" int vo_lrelu_mask_sum(const void* g, int ldg, int g_dtype, const void* ref, int ldr, int ref_dtype,
                                 const void* add, int lda, int64_t rows, int width, float slope, void* out, int ldo,
                                 void* stream) {
  return lrelu_mask_add_run(g, ldg, g_dtype, ref, ldr, ref_dtype, add, lda, rows, width, slope, out, ldo, true, stream);
}

extern "C" int vo_period_fold_bwd(const void* g, int dtype, int B, int T, int P, float* gwav, void* stream) {
  VO_CHECK_ARG(g && gwav && B > 0 && P >= 1 && T > P, "period_fold_bwd: bad arguments");
  const int H = (T + P - 1) / P;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == VO_BF16)
    hipLaunchKernelGGL(period_fold_bwd_kernel<bf16_t>, dim3(grid_for(T), B), dim3(256), 0, st, (const bf16_t*)g, T, P,
                       H, gwav);
  else
    hipLaunchKernelGGL(period_fold_bwd_kernel<float>, dim3(grid_for(T), B), dim3(256), 0, st, (const float*)g, T, P, H,
                       gwav);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_wav_cl8_bwd(const void* g, int dtype, int64_t n, float* gwav, void* stream) {
  VO_CHECK_ARG(g && gwav && n > 0, "wav_cl8_bwd: bad arguments");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == VO_BF16)
    hipLaunchKernelGGL(wav_cl8_bwd_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, (const bf16_t*)g, n, gwav);
  else
    hipLaunchKernelGGL(wav_cl8_bwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, (const float*)g, n, gwav);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_avgpool_wav_bwd(const float* g, int B, int T, float* gx, void* stream) {
  VO_CHECK_ARG(g && gx && B > 0 && T > 0, "avgpool_wav_bwd: bad arguments");
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for(T), B), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), g,
                     T, T / 2 + 1, gx);
  VO_RETURN_LAUNCH();
}
