// Channels-last implicit-GEMM Conv1d on gfx950 MFMA.
//
// GEMM view of one launch:  C[co][pos] = sum_{tap k, ci} W[k][co][ci] * X[pos + k*dil - pad][ci]
//   M = output channels (A operand = packed weights, rows read from LDS),
//   N = output positions of one batch element (B operand = the input window in LDS),
//   reduction = (input-channel chunk of 32) x (tap).
// One workgroup owns a BCO x BT output tile.  For every 32-channel chunk it stages the
// input WINDOW (BT + (K-1)*dil rows) once and reuses it for all K taps by shifting the
// row index -- a dilated conv costs no extra HBM/L2 traffic over a 1x1 conv.  The weight
// tile of the next (chunk, tap) step and the next chunk's window are fetched into
// registers before the current step's MFMAs and written to the other LDS buffer after
// them (issue-early / write-late), so there is one barrier per step.
//
// Accumulator -> output mapping: MFMA row m of co-tile i is channel NI*4*(m>>2) + 4*i +
// (m&3), so lane (g = lane>>4, n = lane&15) ends up holding 4*NI CONTIGUOUS channels of
// ONE position -> vector stores of whole channel runs (channels-last).
//
// The lrelu/relu prologue is applied while staging (replaces F.leaky_relu before every
// HiFi-GAN conv), and the epilogue fuses bias, post-activation (relu/tanh), residual add,
// scale and MRF accumulate (y = (post(acc + b) + res1) * scale + res2).
//
// References: PositionwiseFeedForward (scripts/transformer/SubLayers.py:85-93), PostNet
// (scripts/transformer/Layers.py:129-137), VariancePredictor.Conv (scripts/model/
// modules.py:216-259), ResBlock (scripts/hifigan/models.py:96-103), Generator conv_pre /
// ups (models.py:149-160).

#include <string.h>

#include <algorithm>
#include <type_traits>

#include "vo_common.h"

namespace vo {

constexpr int KC = 32;        // reduction chunk = one bf16 MFMA k-depth
constexpr int HALO_MAX = 64;  // (K-1)*dil supported by the register staging arrays

struct ConvArgs {
  const void* x; int64_t xbs; int ldx;
  const void* w; const float* bias;
  void* y; int64_t ybs; int ldy;
  const void* res1; const void* res2;
  int T_in, T_out, Ci, Co, K, dil, pad;
  int pre_act; float pre_slope; int post_act; float post_slope; float out_scale;
  int transposed, up_stride, up_pad, up_cout, up_tout;
  int tiles_per_b, co_tiles, B;
  int cig, cog;  // channels per group (in / out): grouped conv = block-diagonal packed weights
  float* partial;  // split reduction: fp32 partials [splits][B][T_out][Co] (null = off)
  int kcs;         // 32-channel chunks per split (grid z = split)
  const void* ymask;  // outputs stored as round(round(v) * (ymask > 0 ? 1 : ymask_slope)) (y's layout)
  float ymask_slope;
};

template <typename T> struct Raw8;  // 8 elements of T held in registers
template <> struct Raw8<bf16_t> {
  uint4 u;
  __device__ __forceinline__ void load(const bf16_t* p) { u = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void zero() { u = make_uint4(0, 0, 0, 0); }
  __device__ __forceinline__ void to_f32(float (&v)[8]) const {
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
};
template <> struct Raw8<float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const float4*>(p);
    b = *reinterpret_cast<const float4*>(p + 4);
  }
  __device__ __forceinline__ void zero() { a = b = make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ __forceinline__ void to_f32(float (&v)[8]) const {
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
};

// VO_F32X3: the packed weights are fp32 ([K][Co][Ci], the VO_F32 packing), staged as fp32 and split
// into hi / lo bf16 on their way into LDS (store8 / lds_put below)
template <> struct Raw8<bx3_t> : Raw8<float> {
  __device__ __forceinline__ void load(const bx3_t* p) { Raw8<float>::load(reinterpret_cast<const float*>(p)); }
};

// ---------------------------------------------------------------- LDS tile layout
// bf16: 32 elements (64 B) per row; 16-byte chunk q of row r lives at chunk
//   q ^ ((r >> (SH - 1)) & 2).  With SH = 2 the B-fragment reads (16 consecutive rows from
//   ANY starting row -- taps shift the window by k*dil -- x 4 chunks) are free of
//   ds_read_b128 bank conflicts; with SH = log2(4*NI) so are the A-fragment reads of the
//   weight rows NI*4*(m>>2) + 4*i + (m&3) (checked exhaustively against the gfx950 lane
//   groups; the first version's unswizzled 80-byte pitch was 2-way (B) / 4-way (A)).
//   Adding 16*j rows never changes the swizzle bit, so one offset serves all NJ tiles.
// f32 (parity mode): 40-float padded rows, no swizzle.
template <typename TC> struct Lds;
template <> struct Lds<bf16_t> {
  static constexpr int PITCH = 32;
  template <int SH> __device__ static __forceinline__ int off(int r, int q) {
    return r * 32 + 8 * (q ^ ((r >> (SH - 1)) & 2));
  }
};
template <> struct Lds<float> {
  static constexpr int PITCH = 40;
  template <int SH> __device__ static __forceinline__ int off(int r, int q) { return r * 40 + 8 * q; }
};
// split-bf16 (VO_F32X3): the fp32 tile's geometry, each 32-byte vector slot holding [hi x 8 | lo x 8]
template <> struct Lds<bx3_t> {
  static constexpr int PITCH = 40;
  template <int SH> __device__ static __forceinline__ int off(int r, int q) { return r * 40 + 8 * q; }
};

__device__ __forceinline__ void lds_put(bf16_t* p, const Raw8<bf16_t>& v) { *reinterpret_cast<uint4*>(p) = v.u; }
__device__ __forceinline__ void lds_put(float* p, const Raw8<float>& v) {
  *reinterpret_cast<float4*>(p) = v.a;
  *reinterpret_cast<float4*>(p + 4) = v.b;
}
__device__ __forceinline__ void lds_put(bx3_t* p, const Raw8<bx3_t>& v) {
  float f[8];
  v.to_f32(f);
  store8(p, f);
}

constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v / 2); }

// epilogue: lane (g = lane>>4, lr = lane&15) holds channels [n0, n0 + 4*NI) of position
// pos for each of its NJ position tiles
// bf16 output, plain conv, whole 8-channel runs (vec_ok: ldy / y_bstride multiples of 8):
// every residual / accumulator row of JG positions is requested before any is used (one memory
// round trip per JG positions instead of one per position: the scalar form waited for each row's
// load before its store, 8 times per 128-row wave tile), 16-byte loads and stores; the same
// arithmetic in the same order as the scalar form (bit-identical)
template <int NI, int NJ, int EJ = 2>
__device__ __forceinline__ void conv_epilogue_vec(const ConvArgs& a, f32x4 (&acc)[NI][NJ], int b, int t0, int n0,
                                                  int wave_t0, int lr) {
  static_assert(NI % 2 == 0, "8-channel runs");
  constexpr int NH = NI / 2;
  constexpr int JG = NJ < EJ ? NJ : EJ;  // position tiles whose rows are requested together
  bf16_t* Y = reinterpret_cast<bf16_t*>(a.y) + (int64_t)b * a.ybs;
  const bf16_t* R1 = reinterpret_cast<const bf16_t*>(a.res1 ? a.res1 : a.y) + (int64_t)b * a.ybs;
  const bf16_t* R2 = reinterpret_cast<const bf16_t*>(a.res2 ? a.res2 : a.y) + (int64_t)b * a.ybs;
  const bool r1 = a.res1 != nullptr, r2 = a.res2 != nullptr, om = a.ymask != nullptr;
  const bf16_t* YM = reinterpret_cast<const bf16_t*>(om ? a.ymask : a.y) + (int64_t)b * a.ybs;
  float bias[4 * NI];
#pragma unroll
  for (int e = 0; e < 4 * NI; ++e) bias[e] = a.bias ? a.bias[n0 + e] : 0.f;
  const float ps = a.post_act == VO_ACT_RELU ? 0.f : (a.post_act == VO_ACT_LRELU ? a.post_slope : 1.f);
  const bool tanh_act = a.post_act == VO_ACT_TANH;
#pragma unroll
  for (int j0 = 0; j0 < NJ; j0 += JG) {
    uint4 rv1[JG][NH], rv2[JG][NH], rvm[JG][NH];
#pragma unroll
    for (int jj = 0; jj < JG; ++jj) {  // rows past T_out re-read the last row (not stored)
      const int pos = min(t0 + wave_t0 + 16 * (j0 + jj) + lr, a.T_out - 1);
      const int64_t off = (int64_t)pos * a.ldy + n0;
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        if (r1) rv1[jj][h] = *reinterpret_cast<const uint4*>(R1 + off + 8 * h);
        if (r2) rv2[jj][h] = *reinterpret_cast<const uint4*>(R2 + off + 8 * h);
        if (om) rvm[jj][h] = *reinterpret_cast<const uint4*>(YM + off + 8 * h);
      }
    }
#pragma unroll
    for (int jj = 0; jj < JG; ++jj) {
      const int j = j0 + jj;
      const int pos = t0 + wave_t0 + 16 * j + lr;
      const int64_t off = (int64_t)min(pos, a.T_out - 1) * a.ldy + n0;
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        float q[8], x1[8], x2[8];
        if (r1) {
          const uint32_t w[4] = {rv1[jj][h].x, rv1[jj][h].y, rv1[jj][h].z, rv1[jj][h].w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            x1[2 * u] = __uint_as_float(w[u] << 16);
            x1[2 * u + 1] = __uint_as_float(w[u] & 0xffff0000u);
          }
        }
        if (r2) {
          const uint32_t w[4] = {rv2[jj][h].x, rv2[jj][h].y, rv2[jj][h].z, rv2[jj][h].w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            x2[2 * u] = __uint_as_float(w[u] << 16);
            x2[2 * u + 1] = __uint_as_float(w[u] & 0xffff0000u);
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int i = 2 * h + e / 4, r = e & 3;
          float v = acc[i][j][r] + bias[8 * h + e];
          v = tanh_act ? tanhf(v) : lrelu_max(v, ps);  // ps in [0, 1]
          if (r1) v += x1[e];
          v *= a.out_scale;
          if (r2) v += x2[e];
          q[e] = v;
        }
        if (om) {  // the leaky-ReLU backward of the layer whose output ymask is, on the stored value
          const uint32_t w[4] = {rvm[jj][h].x, rvm[jj][h].y, rvm[jj][h].z, rvm[jj][h].w};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float m = __uint_as_float((e & 1) ? (w[e >> 1] & 0xffff0000u) : (w[e >> 1] << 16));
            const float r = to_f32(from_f32<bf16_t>(q[e]));
            q[e] = m > 0.f ? r : r * a.ymask_slope;
          }
        }
        if (pos < a.T_out) store8(Y + off + 8 * h, q);
      }
    }
  }
}

template <typename TOUT, int NI, int NJ, int EJ = 2>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, f32x4 (&acc)[NI][NJ], int b, int t0, int co_blk,
                                              int wave_co0, int wave_t0, int lane) {
  const int lr = lane & 15;
  const int g = lane >> 4;
  const int n0 = co_blk + wave_co0 + NI * 4 * g;
  if (n0 >= a.Co) return;
  if constexpr (std::is_same<TOUT, bf16_t>::value && NI % 2 == 0) {
    // uniform per launch: plain conv, 8-element aligned rows, the lane's whole run inside Co
    if (!a.transposed && (a.ldy & 7) == 0 && (a.ybs & 7) == 0 && a.Co % (4 * NI) == 0) {
      conv_epilogue_vec<NI, NJ, EJ>(a, acc, b, t0, n0, wave_t0, lr);
      return;
    }
  }
  TOUT* Y = reinterpret_cast<TOUT*>(a.y) + (int64_t)b * a.ybs;
  const TOUT* R1 = a.res1 ? reinterpret_cast<const TOUT*>(a.res1) + (int64_t)b * a.ybs : nullptr;
  const TOUT* R2 = a.res2 ? reinterpret_cast<const TOUT*>(a.res2) + (int64_t)b * a.ybs : nullptr;

  int col = n0, trow_shift = 0;
  if (a.transposed) {
    const int phase = n0 / a.up_cout;
    col = n0 - phase * a.up_cout;
    trow_shift = phase - a.up_pad;
  }
  float bias[4 * NI];
#pragma unroll
  for (int e = 0; e < 4 * NI; ++e) bias[e] = a.bias ? a.bias[(a.transposed ? col : n0) + e] : 0.f;

#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int pos = t0 + wave_t0 + 16 * j + lr;
    if (pos >= a.T_out) continue;
    int trow = pos;
    if (a.transposed) {
      trow = pos * a.up_stride + trow_shift;
      if (trow < 0 || trow >= a.up_tout) continue;
    }
    const int64_t off = (int64_t)trow * a.ldy + col;
    float v[4 * NI];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[4 * i + r] = acc[i][j][r] + bias[4 * i + r];
    if (a.post_act == VO_ACT_TANH) {
#pragma unroll
      for (int e = 0; e < 4 * NI; ++e) v[e] = tanhf(v[e]);
    } else {
      const float ps = a.post_act == VO_ACT_RELU ? 0.f : (a.post_act == VO_ACT_LRELU ? a.post_slope : 1.f);
#pragma unroll
      for (int e = 0; e < 4 * NI; ++e) v[e] = lrelu_max(v[e], ps);  // ps in [0, 1]
    }
#pragma unroll
    for (int h = 0; h < NI; ++h) {
      if (n0 + 4 * h >= a.Co) break;  // Co % (4 * NI) != 0: the lane's run crosses the end
      float q[4] = {v[4 * h], v[4 * h + 1], v[4 * h + 2], v[4 * h + 3]};
      if (R1) {
        float rr[4];
        load4(R1 + off + 4 * h, rr);
#pragma unroll
        for (int e = 0; e < 4; ++e) q[e] += rr[e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) q[e] *= a.out_scale;
      if (R2) {
        float rr[4];
        load4(R2 + off + 4 * h, rr);
#pragma unroll
        for (int e = 0; e < 4; ++e) q[e] += rr[e];
      }
      if (a.ymask) {
        float mm[4];
        load4(reinterpret_cast<const TOUT*>(a.ymask) + (int64_t)b * a.ybs + off + 4 * h, mm);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float r = to_f32(from_f32<TOUT>(q[e]));
          q[e] = mm[e] > 0.f ? r : r * a.ymask_slope;
        }
      }
      store4(Y + off + 4 * h, q);
    }
  }
}

// split reduction, first pass: raw fp32 accumulators of this split's chunks (lane layout of
// conv_epilogue: channels [n0, n0 + 4 NI) of each of its NJ positions)
template <int NI, int NJ>
__device__ __forceinline__ void conv_partial_store(const ConvArgs& a, f32x4 (&acc)[NI][NJ], int b, int t0,
                                                   int co_blk, int wave_co0, int wave_t0, int lane) {
  const int lr = lane & 15;
  const int n0 = co_blk + wave_co0 + NI * 4 * (lane >> 4);
  if (n0 >= a.Co) return;
  float* P = a.partial + ((int64_t)blockIdx.z * a.B + b) * (int64_t)a.T_out * a.Co;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int pos = t0 + wave_t0 + 16 * j + lr;
    if (pos >= a.T_out) continue;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (n0 + 4 * i >= a.Co) break;
      *reinterpret_cast<float4*>(P + (int64_t)pos * a.Co + n0 + 4 * i) =
          make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
  }
}

// ROLE only names the instantiation (0 = generic, 1..4 = HiFi-GAN MRF stage 0..3), so a
// profiler attributes the vocoder's stages to distinct kernels; the code is identical.
// TPS = taps per pipeline step: the weight tiles of TPS taps are staged together so one
// barrier covers TPS x NI x NJ MFMAs per wave.  NICE = (Ci % 32 == 0 && Co % BCO == 0):
// no channel bounds checks in the staging loops.
// Instruction budget: every staging / fragment address is precomputed once per thread;
// the loop body is LDS reads + MFMAs + a few global loads / LDS stores per step (the
// first version spent ~15 VALU+SALU instructions per MFMA on address math).
// PRIO: s_setprio(1) around each MFMA cluster (keeps hipcc from moving the cluster across
// the barriers; guide T5) -- A/B via conv_cfg.  ABL (timing ablation, garbage results):
// 1 = no global loads in the main loop.
// GL (bf16, NICE, stride 1): the weight taps are copied HBM / L2 -> LDS by LDS-DMA
// (global_load_lds_dwordx4, 1 KiB per wave instruction, the XOR swizzle moved to the source
// address as in the fused ResBlock kernels): no staging VGPRs and no ds_write for them.  The
// next chunk's window is then fetched after the first step's DMA (so a step's vmcnt wait does not
// drain it), which leaves it two steps instead of a whole chunk to arrive.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N <= 8, "wait_vmcnt: 0..8");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  if constexpr (N == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
}

// RS (with GL): the waves split the staging by role -- the first half issue every weight DMA piece,
// the second half load and store every window chunk.  vmcnt is per wave and retires in issue order,
// so a wave that waits for its weight DMA each step no longer drains the next chunk's window loads
// (issued one chunk ahead, they got one step to land); and the step barriers are bare s_barrier
// (LDS writes drained by lgkmcnt): __syncthreads' workgroup release fence waits vmcnt(0) too.
// SEG (4-byte TC, stride 1, T_out <= 16): utterance-segment tiles -- each 16-row position tile j of a
// wave is one whole utterance (b0 + its index), staged as its own window of 16 + (K-1) dil rows (rows
// outside [0, T_in) zeroed), so the BT / 16 utterances of a workgroup share every staged weight tap.
// The short-sequence convs (glyph encoder, variance predictors: T ~ 12) otherwise ran one utterance
// per workgroup and re-read the whole weight once per utterance (FFN w_1 at B = 32: 302 MB of L2
// reads for 9.4 MB of weights).  Halo <= SEG_HALO.
constexpr int SEG_HALO = 8;
template <typename TIN, typename TC, typename TOUT, int NI, int NJ, int WCO, int WT, int TPS, bool NICE, int ROLE,
          int PRIO = 0, int ABL = 0, int S = 1, bool GL = false, bool RS = false, int EJ = 2, bool SEG = false>
__global__ void __launch_bounds__(WCO * WT * 64)
conv1d_kernel(ConvArgs a) {
  static_assert(!SEG || (sizeof(TC) == 4 && S == 1 && !GL), "conv1d SEG: 4-byte compute, stride 1");
  constexpr int NT = WCO * WT * 64;
  constexpr int BCO = 16 * NI * WCO;
  constexpr int BT = 16 * NJ * WT;
  constexpr int P = Lds<TC>::PITCH;
  constexpr int VPR = KC / 8;                 // 8-element vectors per row (4)
  constexpr bool DMA = GL && NICE && S == 1 && sizeof(TC) == 2 && sizeof(TIN) == 2 && ABL == 0;
  constexpr bool SPLIT = RS && DMA && (NT / 64) % 2 == 0;
  constexpr int MAXV = SPLIT ? 1 : SEG ? ((BT / 16) * (16 + SEG_HALO) * VPR + NT - 1) / NT
                                      : (((BT - 1) * S + 1 + HALO_MAX) * VPR + NT - 1) / NT;
  // SPLIT: the window waves copy each chunk's window by LDS-DMA (XPW 1-KiB pieces per wave,
  // lane-linear) into a raw staging area; at the chunk's end each lane applies the prologue
  // activation to the 16 bytes it fetched and stores them into the swizzled window buffer
  constexpr int XPW = SPLIT ? (((BT - 1) * S + 1 + HALO_MAX) * VPR + 64 * (NT / 128) - 1) / (64 * (NT / 128)) : 1;
  constexpr int WV = (TPS * BCO * VPR + NT - 1) / NT;
  constexpr int SHW = ilog2(4 * NI);

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  TC* smem = reinterpret_cast<TC*>(smem_raw);

  const int seg_rows = 16 + (a.K - 1) * a.dil;  // SEG: window rows per utterance
  const int win_rows = SEG ? (BT / 16) * seg_rows : (BT - 1) * S + 1 + (a.K - 1) * a.dil;  // S: conv stride
  TC* const win0 = smem;
  TC* const wt0 = smem + 2 * win_rows * P;
  const int win_stride = win_rows * P;      // elements between the two window buffers
  constexpr int WSTRIDE = TPS * BCO * P;    // elements between the two weight buffers
  TC* const dummy = wt0 + 2 * WSTRIDE;      // one row that absorbs the stores of idle staging slots

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_co0 = (wave % WCO) * 16 * NI;
  const int wave_t0 = (wave / WCO) * 16 * NJ;

  const int b = SEG ? blockIdx.x * (BT / 16) : blockIdx.x / a.tiles_per_b;  // SEG: the tile's first utterance
  const int t0 = SEG ? 0 : (blockIdx.x - b * a.tiles_per_b) * BT;
  const int co_blk = blockIdx.y * BCO;

  const TIN* __restrict__ X = reinterpret_cast<const TIN*>(a.x) + (int64_t)b * a.xbs;
  const TC* __restrict__ Wp = reinterpret_cast<const TC*>(a.w);
  // grouped conv: this block's output channels [co_blk, co_blk + BCO) read only input
  // channels [ci_lo, ci_hi) of their groups (32-aligned; the packed weights are
  // block-diagonal, so the extra channels of a partial chunk multiply zeros)
  const int co_last = min(co_blk + BCO, a.Co) - 1;
  int ci_lo = (co_blk / a.cog) * a.cig / KC * KC;
  const int ci_hi = min(a.Ci, (co_last / a.cog + 1) * a.cig);
  int n_chunks = (ci_hi - ci_lo + KC - 1) / KC;
  if (a.partial) {  // split reduction: this workgroup's run of chunks
    const int z0 = blockIdx.z * a.kcs;
    ci_lo += z0 * KC;
    n_chunks = min(a.kcs, n_chunks - z0);
  }
  const int tsteps = (a.K + TPS - 1) / TPS;
  const bool raw_window = std::is_same<TIN, TC>::value && a.pre_act == VO_ACT_NONE;
  // prologue activation as one select: none -> slope 1, relu -> 0, lrelu -> slope
  const float pre_s = a.pre_act == VO_ACT_RELU ? 0.f : (a.pre_act == VO_ACT_LRELU ? a.pre_slope : 1.f);
  const int64_t tap_stride = (int64_t)a.Co * a.Ci;

  // ---- per-thread staging geometry, computed once
  // Every global load below is UNCONDITIONAL (addresses clamped into the tensor) and the
  // out-of-range vectors are zeroed when they are written to LDS: a load under a divergent
  // branch gets an immediate s_waitcnt vmcnt(0) from the compiler, which serialised the
  // prefetch against HBM latency (seen in the ISA of the first version).
  constexpr int MAXVA = MAXV;
  int xg[MAXVA], xl[MAXVA], xr[MAXVA], xc[MAXVA];  // xr: row-in-range flag
#pragma unroll
  for (int s = 0; s < MAXVA; ++s) {
    const int v = tid + s * NT;
    const int r = v / VPR, q = v % VPR;
    xc[s] = q * 8;
    if constexpr (SEG) {
      const int seg = r / seg_rows, row = r - seg * seg_rows - a.pad;
      xr[s] = r < win_rows && b + seg < a.B && row >= 0 && row < a.T_in;
      xg[s] = (int)(min(seg, a.B - 1 - b) * a.xbs) + min(max(row, 0), a.T_in - 1) * a.ldx + q * 8;
    } else {
      const int row = t0 * S - a.pad + r;
      xr[s] = r < win_rows && row >= 0 && row < a.T_in;  // row in range
      xg[s] = min(max(row, 0), a.T_in - 1) * a.ldx + q * 8;
    }
    xl[s] = r < win_rows ? Lds<TC>::template off<2>(r, q) : -1;
  }
  int wg[WV], wl[WV], wk[WV], wq[WV];
  bool wok[WV];
#pragma unroll
  for (int s = 0; s < WV; ++s) {
    const int v = tid + s * NT;
    const int r = v / VPR, q = v % VPR;   // r = tap_in_step * BCO + co_local
    const int t = r / BCO, col = r - t * BCO;
    wk[s] = t;
    wq[s] = q * 8;
    wok[s] = r < TPS * BCO && (NICE || co_blk + col < a.Co);
    wg[s] = min(co_blk + col, a.Co - 1) * a.Ci + q * 8;
    wl[s] = t * BCO * P + Lds<TC>::template off<SHW>(col, q);
  }

  Raw8<TIN> win_r[MAXV];
  // SEG: second register sets -- weights fetched two steps ahead, and (one-tap convs) windows two chunks ahead
  Raw8<TIN> win_r2[SEG ? MAXV : 1];
  bool win_ok2[SEG ? MAXV : 1];
  Raw8<TC> w_r2[SEG ? WV : 1];
  bool w_ok2[SEG ? WV : 1];
  constexpr int NW = NT / 64;
  constexpr int NWW = SPLIT ? NW / 2 : NW;  // waves issuing the weight DMA
  constexpr int GLN = DMA ? (TPS * BCO * VPR) / (64 * NWW) : 1;  // DMA instructions per wave per step
  static_assert(!DMA || (TPS * BCO * VPR) % (64 * NWW) == 0, "conv1d GL: a step's weights must split into whole wave-KiB");
  Raw8<TC> w_r[DMA ? 1 : WV];
  bool win_ok[MAXVA], w_ok[DMA ? 1 : WV];
  constexpr int GLNA = SPLIT ? 1 : GLN;
  int gl_t[GLNA], gl_src[GLNA];
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int wave_w = wave_u % NWW;
  // wave roles (uniform): SPLIT -> waves [0, NW/2) weights, [NW/2, NW) window; else every wave both
  const bool wwave = !SPLIT || wave_u < NWW, xwave = !SPLIT || wave_u >= NWW;
  const int wave_x = wave_u - NWW;  // SPLIT: window wave index
  TC* const xraw = dummy + P;       // SPLIT: raw window pieces [NW - NWW][XPW][64 lanes][8]
  if constexpr (DMA && !SPLIT) {
#pragma unroll
    for (int s = 0; s < GLN; ++s) {
      const int p = (s * NWW + wave_w) * 64 + lane;  // LDS slot (16 B): tap t, row col, chunk q'
      const int t = p / (BCO * VPR), rem = p - t * BCO * VPR;
      const int col = rem / VPR, qs = rem - col * VPR;
      const int q = qs ^ ((col >> (SHW - 1)) & 2);  // the swizzle of Lds<bf16_t>::off, on the source
      gl_t[s] = t;
      gl_src[s] = (co_blk + col) * a.Ci + q * 8;
    }
  }
  auto load_w_dma = [&](int c, int k0, int buf) {
    if constexpr (DMA) {
      typedef __attribute__((address_space(3))) void lds_void;
      typedef const __attribute__((address_space(1))) void g_void;
      const int c0 = ci_lo + c * KC;
      if constexpr (SPLIT) {
        // piece s = tap s / PPT, rows (s % PPT) * CSTEP + (wave_w * 64 + lane) / VPR; its swizzle
        // bit does not depend on s, so one per-lane offset (opaque: not hoisted as GLN 64-bit
        // addresses, which spilled) plus a scalar offset per piece
        constexpr int PPT = BCO * VPR / (64 * NWW), CSTEP = 64 * NWW / VPR;
        static_assert(GLN % PPT == 0 && CSTEP % (1 << SHW) == 0, "conv1d RS: whole taps per step, swizzle kept");
        const int p0 = wave_w * 64 + lane, col0 = p0 / VPR;
        int lane_off = (co_blk + col0) * a.Ci + ((p0 % VPR) ^ ((col0 >> (SHW - 1)) & 2)) * 8;
        asm volatile("" : "+v"(lane_off));
#pragma unroll
        for (int s = 0; s < GLN; ++s) {
          const int k = min(k0 + s / PPT, a.K - 1);  // taps >= K are skipped by the MFMA loop
          const TC* src = Wp + (k * tap_stride + (s % PPT) * CSTEP * a.Ci + c0) + lane_off;
          TC* dst = wt0 + buf * WSTRIDE + (s * NWW + wave_w) * 64 * 8;
          __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)dst, 16, 0, 0);
        }
        return;
      }
#pragma unroll
      for (int s = 0; s < GLN; ++s) {
        int gt, gsrc;
        {
          gt = gl_t[s];
          gsrc = gl_src[s];
        }
        const int k = min(k0 + gt, a.K - 1);  // taps >= K are skipped by the MFMA loop
        const TC* src = Wp + k * tap_stride + gsrc + c0;
        TC* dst = wt0 + buf * WSTRIDE + (s * NWW + wave_w) * 64 * 8;
        __builtin_amdgcn_global_load_lds((g_void*)src, (lds_void*)dst, 16, 0, 0);
      }
    }
  };

  // SPLIT: two raw areas -- chunk c + 2's window is fetched while chunk c computes and chunk c + 1's
  // lands; the pass at chunk c's end waits only for chunk c + 1 (vmcnt(XPW): the younger pieces of
  // chunk c + 2 stay in flight), so each window DMA has a whole chunk or more to land
  constexpr int XRAW = (NT / 128) * XPW * 64 * 8;  // elements per raw area
  static_assert(!SPLIT || XPW <= 8, "conv1d RS: wait_vmcnt<XPW>");
  auto load_window_to = [&](auto& wr, auto& wo, int c) {
    const int c0 = ci_lo + c * KC;
#pragma unroll
    for (int s = 0; s < MAXVA; ++s) {
      wo[s] = xr[s] && (NICE || c0 + xc[s] < a.Ci);
      if constexpr (ABL == 1) {
        if (c > 0) { wr[s].zero(); continue; }
      }
      wr[s].load(X + xg[s] + (NICE ? c0 : min(c0, a.Ci - 8 - xc[s])));
    }
  };
  auto load_window = [&](int c, int rb = 0) {
    const int c0 = ci_lo + c * KC;
    if constexpr (SPLIT) {  // NICE: no channel bounds; rows clamped (zeroed by the LDS pass)
      typedef __attribute__((address_space(3))) void lds_void;
      typedef const __attribute__((address_space(1))) void g_void;
      int lrow = lane / VPR;  // opaque per call (see load_w_dma)
      asm volatile("" : "+v"(lrow));
      const TIN* xq = X + (lane % VPR) * 8 + c0;
#pragma unroll
      for (int s = 0; s < XPW; ++s) {
        const int row = min(max(t0 * S - a.pad + (wave_x * XPW + s) * (64 / VPR) + lrow, 0), a.T_in - 1);
        __builtin_amdgcn_global_load_lds((g_void*)(xq + (int64_t)row * a.ldx),
                                         (lds_void*)(xraw + rb * XRAW + (wave_x * XPW + s) * 64 * 8), 16, 0, 0);
      }
      return;
    }
    load_window_to(win_r, win_ok, c);
  };
  auto store_window_from = [&](auto& wr, auto& wo, int buf) {
    TC* base = win0 + buf * win_stride;
#pragma unroll
    for (int s = 0; s < MAXV; ++s) {  // branch-free: idle slots store to the dummy row
      TC* dst;
      {
        dst = xl[s] >= 0 ? base + xl[s] : dummy;
        if (!wo[s]) wr[s].zero();
      }
      if constexpr (std::is_same<TIN, TC>::value) {
        if (raw_window) {
          lds_put(dst, wr[s]);
          continue;
        }
      }
      float f[8];
      wr[s].to_f32(f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = lrelu_max(f[e], pre_s);  // pre_s in [0, 1]
      store8(dst, f);
    }
  };
  auto store_window = [&](int buf, int rb = 0, bool young = false) {
    TC* base = win0 + buf * win_stride;
    if constexpr (SPLIT) {  // this wave's own DMA pieces (same lanes): no barrier needed first
      if (young)
        wait_vmcnt<XPW>();  // the next chunk's pieces (issued after these) may stay in flight
      else
        wait_vmcnt<0>();
#pragma unroll
      for (int s = 0; s < XPW; ++s) {
        const int v = (wave_x * XPW + s) * 64 + lane, r = v / VPR, row = t0 * S - a.pad + r;
        Raw8<TIN> u;
        u.load(reinterpret_cast<const TIN*>(xraw + rb * XRAW + v * 8));
        if (!(row >= 0 && row < a.T_in)) u.zero();
        float f[8];
        u.to_f32(f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = lrelu_max(f[e], pre_s);  // pre_s in [0, 1]
        store8(r < win_rows ? base + Lds<TC>::template off<2>(r, v % VPR) : dummy, f);
      }
      return;
    }
    store_window_from(win_r, win_ok, buf);
  };
  auto load_w_to = [&](auto& wr, auto& wo, int c, int k0) {
    if constexpr (DMA) return;
    const int c0 = ci_lo + c * KC;
#pragma unroll
    for (int s = 0; s < WV; ++s) {
      const int k = min(k0 + wk[s], a.K - 1);  // taps >= K are skipped by the MFMA loop
      wo[s] = wok[s] && (NICE || c0 + wq[s] < a.Ci);
      if constexpr (ABL == 1) {
        if (c > 0 || k0 > 0) { wr[s].zero(); continue; }
      }
      wr[s].load(Wp + k * tap_stride + wg[s] + (NICE ? c0 : min(c0, a.Ci - 8 - wq[s])));
    }
  };
  auto store_w_from = [&](auto& wr, auto& wo, int buf) {
    if constexpr (DMA) return;
    TC* base = wt0 + buf * WSTRIDE;
#pragma unroll
    for (int s = 0; s < WV; ++s) {
      if (!wo[s]) wr[s].zero();
      lds_put((tid + s * NT) / VPR < TPS * BCO ? base + wl[s] : dummy, wr[s]);
    }
  };
  auto load_w = [&](int c, int k0) { load_w_to(w_r, w_ok, c, k0); };
  auto store_w = [&](int buf) { store_w_from(w_r, w_ok, buf); };

  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (elements)
  const int lr = lane & 15;
  const int lq = lane >> 4;
  int a_off[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i)
    a_off[i] = Lds<TC>::template off<SHW>(wave_co0 + NI * 4 * (lr >> 2) + 4 * i + (lr & 3), lq);
  const int brow0 = SEG ? (wave_t0 / 16) * seg_rows + lr : wave_t0 + lr;
  const int jst = SEG ? seg_rows * P : 16 * S * P;  // rows between position tiles j (SEG: one utterance window)

  // prologue
  if (xwave) load_window(0);
  load_w(0, 0);
  if (wwave) load_w_dma(0, 0, 0);
  if (xwave) store_window(0);
  store_w(0);
  if constexpr (DMA) wait_vmcnt<0>();
  __syncthreads();

  // One pipeline step = TPS taps of one 32-channel chunk c (weights in buffer s & 1).  The
  // next chunk's window is fetched when a chunk starts and written to LDS in its last step.
  // Loads are issued on every path (re-fetching the last chunk instead of branching): a
  // conditional load makes the compiler's wait counts conservative on every path.
  auto mfma_step = [&](int c, int tg, int s) {
    const TC* xb = win0 + (c & 1) * win_stride;
    const TC* wb = wt0 + (s & 1) * WSTRIDE;
    const int k0 = tg * TPS;
#pragma unroll
    for (int t = 0; t < TPS; ++t) {
      if (k0 + t < a.K) {
        Frag<TC> af[NI], bfr[NJ];
#pragma unroll
        for (int i = 0; i < NI; ++i) af[i].load(wb + t * BCO * P + a_off[i]);
        const int br = brow0 * S + (k0 + t) * a.dil;
        const int boff = Lds<TC>::template off<2>(br, lq);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[j].load(xb + boff + (SEG ? j * jst : 16 * S * j * P));  // +16S rows keeps the swizzle
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = mfma(af[i], bfr[j], acc[i][j]);
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      }
    }
  };

  if constexpr (SEG) {
    // Short chains (9..72 steps of 2..8 MFMAs per wave): every step of the generic loop below waited a
    // whole load round trip (its weights are fetched at the step's start, and __syncthreads drains
    // vmcnt).  Here step q's weights are fetched two steps ahead (register sets A / B alternate),
    // written to LDS one step ahead, and the barriers are bare (lds_barrier): loads stay in flight
    // across them.  One-tap convs (a step per chunk) fetch windows two chunks ahead the same way.
    // Step q = chunk q / tsteps, tap group q % tsteps: the generic loop's order (bit-identical).
    const int nq = n_chunks * tsteps;
    auto wload = [&](auto& wr, auto& wo, int q) {
      q = min(q, nq - 1);  // clamped re-fetch past the end: loads stay unconditional
      const int c = q / tsteps;
      load_w_to(wr, wo, c, (q - c * tsteps) * TPS);
    };
    if (tsteps == 1) {
      load_window_to(win_r, win_ok, min(1, n_chunks - 1));
      wload(w_r, w_ok, 1);
      auto body1 = [&](int c, auto& cw, auto& cwo, auto& cx, auto& cxo, auto& nw, auto& nwo, auto& nx, auto& nxo) {
        load_window_to(nx, nxo, min(c + 2, n_chunks - 1));
        wload(nw, nwo, c + 2);
        mfma_step(c, 0, c);
        if (c + 1 < n_chunks) {
          store_window_from(cx, cxo, (c + 1) & 1);
          store_w_from(cw, cwo, (c + 1) & 1);
        }
        lds_barrier();
      };
      for (int c = 0; c < n_chunks; c += 2) {
        body1(c, w_r, w_ok, win_r, win_ok, w_r2, w_ok2, win_r2, win_ok2);
        if (c + 1 < n_chunks) body1(c + 1, w_r2, w_ok2, win_r2, win_ok2, w_r, w_ok, win_r, win_ok);
      }
    } else {
      wload(w_r, w_ok, 1);
      auto body = [&](int q, auto& cw, auto& cwo, auto& nw, auto& nwo) {
        const int c = q / tsteps, tg = q - c * tsteps;
        if (tg == 0) load_window(min(c + 1, n_chunks - 1));
        wload(nw, nwo, q + 2);
        mfma_step(c, tg, q);
        store_w_from(cw, cwo, (q + 1) & 1);  // past the last step: a buffer no step reads
        if (tg == tsteps - 1 && c + 1 < n_chunks) store_window((c + 1) & 1);
        lds_barrier();
      };
      for (int q = 0; q < nq; q += 2) {
        body(q, w_r, w_ok, w_r2, w_ok2);
        if (q + 1 < nq) body(q + 1, w_r2, w_ok2, w_r, w_ok);
      }
    }
    wait_vmcnt<0>();  // the clamped re-fetches land before the registers are reused by the epilogue
  }
  int s = 0;
  if constexpr (SPLIT) {
    for (int c = 0; c < n_chunks; ++c) {
      const bool more_chunks = c + 1 < n_chunks;
      if (xwave) {  // chunk c's raw area was consumed at chunk c - 1's end
        if (c == 0) load_window(min(1, n_chunks - 1), 1);
        load_window(min(c + 2, n_chunks - 1), c & 1);
      }
      for (int tg = 0; tg < tsteps - 1; ++tg, ++s) {
        if (wwave) load_w_dma(c, (tg + 1) * TPS, (s + 1) & 1);
        mfma_step(c, tg, s);
        if (wwave) wait_vmcnt<0>();  // this wave's DMA pieces landed
        lds_barrier();
      }
      if (wwave) load_w_dma(min(c + 1, n_chunks - 1), 0, (s + 1) & 1);
      mfma_step(c, tsteps - 1, s);
      if (xwave && more_chunks) store_window((c + 1) & 1, (c + 1) & 1, true);
      if (wwave) wait_vmcnt<0>();
      lds_barrier();
      ++s;
    }
    if (xwave) wait_vmcnt<0>();  // the clamped re-fetches of the last chunks land before the epilogue
  }
  for (int c = 0; c < (SPLIT || SEG ? 0 : n_chunks); ++c) {
    const bool more_chunks = c + 1 < n_chunks;
    if constexpr (!DMA) load_window(min(c + 1, n_chunks - 1));  // a whole chunk of MFMAs ahead of its use
    for (int tg = 0; tg < tsteps - 1; ++tg, ++s) {
      load_w(c, (tg + 1) * TPS);
      if constexpr (DMA) {
        load_w_dma(c, (tg + 1) * TPS, (s + 1) & 1);
        if (tg == 0) load_window(min(c + 1, n_chunks - 1));  // issued after the DMA: in-order vmcnt
      }
      mfma_step(c, tg, s);
      store_w((s + 1) & 1);
      if constexpr (DMA) {  // this wave's DMA pieces landed (the window loads after them may not)
        if (tg == 0)
          wait_vmcnt<MAXV>();
        else
          wait_vmcnt<0>();
      }
      __syncthreads();
    }
    load_w(min(c + 1, n_chunks - 1), 0);
    if constexpr (DMA) {
      load_w_dma(min(c + 1, n_chunks - 1), 0, (s + 1) & 1);
      if (tsteps == 1) load_window(min(c + 1, n_chunks - 1));
    }
    mfma_step(c, tsteps - 1, s);
    if (more_chunks) {
      store_w((s + 1) & 1);
      store_window((c + 1) & 1);
    }
    if constexpr (DMA) wait_vmcnt<0>();
    __syncthreads();
    ++s;
  }
  if constexpr (SEG) {  // position tile j = utterance b + wave_t0 / 16 + j, positions 0..15
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int bj = b + wave_t0 / 16 + j;
      if (bj >= a.B) continue;
      f32x4 a1[NI][1];
#pragma unroll
      for (int i = 0; i < NI; ++i) a1[i][0] = acc[i][j];
      if (a.partial)
        conv_partial_store<NI, 1>(a, a1, bj, 0, co_blk, wave_co0, 0, lane);
      else
        conv_epilogue<TOUT, NI, 1, EJ>(a, a1, bj, 0, co_blk, wave_co0, 0, lane);
    }
    return;
  }
  if (a.partial) {
    conv_partial_store<NI, NJ>(a, acc, b, t0, co_blk, wave_co0, wave_t0, lane);
    return;
  }
  conv_epilogue<TOUT, NI, NJ, EJ>(a, acc, b, t0, co_blk, wave_co0, wave_t0, lane);
}

// split reduction, second pass: y = epilogue(sum_z partial[z] + bias) with the partials added
// in split order; the epilogue (activation, residual, scale, accumulate) is conv_epilogue's
template <typename TOUT>
__global__ void __launch_bounds__(256) conv_splitk_reduce_kernel(ConvArgs a, int splits) {
  const int cg = a.Co / 4;
  const int64_t rows = (int64_t)a.B * a.T_out;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * cg) return;
  const int64_t row = idx / cg;
  const int c = (int)(idx - row * cg) * 4;
  const int b = (int)(row / a.T_out), t = (int)(row - (int64_t)b * a.T_out);
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  for (int z = 0; z < splits; ++z) {
    const float4 p = *reinterpret_cast<const float4*>(a.partial + ((int64_t)z * rows + row) * a.Co + c);
    v[0] += p.x; v[1] += p.y; v[2] += p.z; v[3] += p.w;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] += a.bias ? a.bias[c + e] : 0.f;
  if (a.post_act == VO_ACT_TANH) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = tanhf(v[e]);
  } else {
    const float ps = a.post_act == VO_ACT_RELU ? 0.f : (a.post_act == VO_ACT_LRELU ? a.post_slope : 1.f);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = lrelu_max(v[e], ps);  // ps in [0, 1]
  }
  const int64_t off = (int64_t)b * a.ybs + (int64_t)t * a.ldy + c;
  if (a.res1) {
    float rr[4];
    load4(reinterpret_cast<const TOUT*>(a.res1) + off, rr);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] += rr[e];
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] *= a.out_scale;
  if (a.res2) {
    float rr[4];
    load4(reinterpret_cast<const TOUT*>(a.res2) + off, rr);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] += rr[e];
  }
  store4(reinterpret_cast<TOUT*>(a.y) + off, v);
}

// fp32 convs over short sequences (T_out <= 16 rows: glyph encoder, variance predictors at
// T_src ~ 12) are a serial chain of (Ci / 32) * K pipeline steps per workgroup, each bound by
// a load round trip (FFN w_1: 72 steps, 51 us for 1.8 GFLOP).  Split the chunks so a workgroup
// runs about 4 steps; the partials are added by conv_splitk_reduce_kernel.  splitk_cfg 1 = off.
// bf16 deep reductions into narrow outputs (the C4 decoder's FFN w_1 input gradient: 1024 -> 256, k = 9,
// 16 k rows: a 9216-deep reduction, 106 us on 64 x 128 tiles): the 256 x 256 tile with its chunks split
// over ~256 workgroups, the fp32 partials added in split order by conv_splitk_reduce_kernel.  Plain convs
// only (no bias, activation, residual, scale or mask).  splitk_cfg 3 = off (A/B).
static bool splitk_bf16_ok(const vo_conv1d_desc* d) {
  return d->compute_dtype == VO_BF16 && d->x_dtype == VO_BF16 && !d->transposed && d->stride <= 1 && d->groups <= 1 &&
         d->variant == 0 && !d->bias && !d->res1 && !d->res2 && !d->ymask && d->pre_act == VO_ACT_NONE &&
         d->post_act == VO_ACT_NONE && d->out_scale == 1.f && d->Co <= 256 && d->Co % 64 == 0 && d->Ci % KC == 0 &&
         (int64_t)(d->Ci / KC) * d->K >= 64 && (int64_t)d->B * d->T_out >= 8192 && d->ldy == d->Co &&
         vo_tune_get("splitk_cfg") != 3 && vo_tune_get("splitk_cfg") != 1 && vo_tune_get("gen_cfg") == 0;
}

static bool splitk_plan(const vo_conv1d_desc* d, int* splits, int* kcs) {
  *splits = 1;
  *kcs = 0;
  if (vo_tune_get("splitk_cfg") == 1 || vo_tune_get("gen_cfg") != 0) return false;
  if (d->compute_dtype == VO_BF16) {
    if (!splitk_bf16_ok(d)) return false;
    const int n_chunks = d->Ci / KC;
    const int64_t tiles = (int64_t)d->B * ((d->T_out + 255) / 256) * ((d->Co + 255) / 256);
    int s = (int)std::min<int64_t>(n_chunks / 4, std::max<int64_t>(2, (256 + tiles - 1) / tiles));
    if (s < 2) return false;
    const int k = (n_chunks + s - 1) / s;
    *splits = (n_chunks + k - 1) / k;
    *kcs = k;
    return *splits >= 2;
  }
  if ((d->compute_dtype != VO_F32 && d->compute_dtype != VO_F32X3) || d->x_dtype != VO_F32 || d->y_dtype != VO_F32)
    return false;
  if (d->transposed || d->stride > 1 || d->groups > 1 || d->variant != 0) return false;
  if (d->T_out > 16 || d->Co < 64 || d->Co % 4 || d->ldy % 4) return false;
  const int n_chunks = (d->Ci + KC - 1) / KC;
  if (n_chunks * d->K < 16) return false;
  // ~4 steps per split (bench step 13.78 ms vs 13.85 with ~8 and 13.93 unsplit,
  // tools/bench_splitk_ab.sh); splitk_cfg 2 = ~8, 4 = ~16
  const int target = vo_tune_get("splitk_cfg") == 2 ? 8 : vo_tune_get("splitk_cfg") == 4 ? 16 : 4;
  const int k = std::max(1, target / d->K);
  const int s = (n_chunks + k - 1) / k;
  if (s < 2) return false;
  *splits = s;
  *kcs = k;
  return true;
}

// ------------------------------------------------------------------ K = 1 convs (Linear layers)
// The transformer's fused q/k/v, fc and FFN w_2 are plain GEMMs over B*T = 16k rows with a
// 256..1024-deep reduction (SubLayers.py:39-54,85-93).  conv1d_kernel stages one 32-channel chunk
// per barrier with one chunk of prefetch; at 8..32 chunks that pipeline never fills (q/k/v: 21 us
// for 33 MB, 1.6 TB/s).  Here each wave reads its own A (weight rows) and B (input rows) fragments
// straight from L2 through a D-step register ring -- no LDS, no barriers; the waves of a workgroup
// that share weight rows or input rows meet in L1.  Every accumulator sees the same MFMA sequence
// as in conv1d_kernel (chunks in order, lane group q = channels 8q..8q+7, the same weight-row
// permutation) and the same epilogue, so the outputs are bit-identical to it.
// Measured and dropped (tools/probes/lin_probe.py, profiles/r05/lin_probe.txt): 1.3-2.2x SLOWER than
// conv1d_kernel at every tile (q/k/v 23.0 us -> 30.8 at 128 x 128, 41.3 at 128 co x 64 rows) -- the
// per-wave fragment loads (16 rows x 64 B per instruction) bind where the LDS tile shares them.
// A/B library only (make abl; lin_cfg 2 / 3 / 4 / 5).
#ifdef VO_ABLATIONS
template <typename TOUT, int NI, int NJ, int WCO, int WT, int D, int NC>
__global__ void __launch_bounds__(WCO * WT * 64) lin_kernel(ConvArgs a) {
  // NC = Ci / 32 chunks, fully unrolled: straight-line code, so the compiler's vmcnt waits count
  // exactly D - 1 chunks of loads in flight (a rolled loop got a near-drain wait at its back-edge)
  constexpr int BCO = 16 * NI * WCO;
  constexpr int BT = 16 * NJ * WT;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wave_co0 = (wave % WCO) * 16 * NI;
  const int wave_t0 = (wave / WCO) * 16 * NJ;
  const int b = blockIdx.x / a.tiles_per_b;
  const int t0 = (blockIdx.x - b * a.tiles_per_b) * BT;
  const int co_blk = blockIdx.y * BCO;
  const int lr = lane & 15, lq = lane >> 4;
  const bf16_t* W = reinterpret_cast<const bf16_t*>(a.w) + lq * 8;
  const bf16_t* X = reinterpret_cast<const bf16_t*>(a.x) + (int64_t)b * a.xbs + lq * 8;
  const bf16_t* ap[NI];
  const bf16_t* bp[NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i) ap[i] = W + (int64_t)(co_blk + wave_co0 + NI * 4 * (lr >> 2) + 4 * i + (lr & 3)) * (NC * KC);
#pragma unroll
  for (int j = 0; j < NJ; ++j) bp[j] = X + (int64_t)min(t0 + wave_t0 + 16 * j + lr, a.T_in - 1) * a.ldx;

  Frag<bf16_t> af[D][NI], bfr[D][NJ];
#pragma unroll
  for (int d = 0; d < D && d < NC; ++d) {
#pragma unroll
    for (int i = 0; i < NI; ++i) af[d][i].load(ap[i] + d * KC);
#pragma unroll
    for (int j = 0; j < NJ; ++j) bfr[d][j].load(bp[j] + d * KC);
  }
  // sched_barrier: keep every chunk's loads where they are written (hipcc otherwise sinks them next
  // to their MFMAs -- fewer registers, no loads in flight)
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int d = c % D;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma(af[d][i], bfr[d][j], acc[i][j]);
    if (c + D < NC) {  // chunk c + D into the freed slot
#pragma unroll
      for (int i = 0; i < NI; ++i) af[d][i].load(ap[i] + (c + D) * KC);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bfr[d][j].load(bp[j] + (c + D) * KC);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  conv_epilogue<TOUT, NI, NJ>(a, acc, b, t0, co_blk, wave_co0, wave_t0, lane);
}
#endif  // VO_ABLATIONS

// ------------------------------------------------------------------ host dispatch
static bool splitk_plan(const vo_conv1d_desc* d, int* splits, int* kcs);
template <typename TIN, typename TC, typename TOUT, int NI, int NJ, int WCO, int WT, int TPS_BF16, int ROLE = 0,
          int PRIO = 0, int ABL = 0, int S = 1, bool GL = false, bool RS = false, int EJ = 2, bool SEG = false>
static int launch_cfg_s(const vo_conv1d_desc* d, hipStream_t st) {
  constexpr int BCO = 16 * NI * WCO;
  constexpr int BT = 16 * NJ * WT;
  constexpr int TPS = sizeof(TC) == 2 ? TPS_BF16 : 1;
  ConvArgs a;
  a.x = d->x; a.xbs = d->x_bstride; a.ldx = d->ldx;
  a.w = d->w; a.bias = d->bias;
  a.y = d->y; a.ybs = d->y_bstride; a.ldy = d->ldy;
  a.res1 = d->res1; a.res2 = d->res2;
  a.T_in = d->T_in; a.T_out = d->T_out; a.Ci = d->Ci; a.Co = d->Co;
  a.K = d->K; a.dil = d->dil; a.pad = d->pad;
  a.pre_act = d->pre_act; a.pre_slope = d->pre_slope;
  a.post_act = d->post_act; a.post_slope = d->post_slope; a.out_scale = d->out_scale;
  a.transposed = d->transposed; a.up_stride = d->up_stride; a.up_pad = d->up_pad;
  a.up_cout = d->up_cout; a.up_tout = d->up_tout;
  a.tiles_per_b = SEG ? 1 : (d->T_out + BT - 1) / BT;
  a.co_tiles = (d->Co + BCO - 1) / BCO;
  a.B = d->B;
  a.ymask = d->ymask; a.ymask_slope = d->ymask_slope;
  const int groups = d->groups > 1 ? d->groups : 1;
  a.cig = d->Ci / groups;
  a.cog = d->Co / groups;
  const int win_rows = SEG ? (BT / 16) * (16 + (d->K - 1) * d->dil) : (BT - 1) * S + 1 + (d->K - 1) * d->dil;
  const bool nice = d->Ci % KC == 0 && d->Co % BCO == 0;
  // role-split kernels (RS): + the raw window staging area of conv1d_kernel (XPW pieces per window wave)
  constexpr bool SPL = RS && GL && S == 1 && sizeof(TC) == 2 && sizeof(TIN) == 2 && ABL == 0 && (WCO * WT) % 2 == 0;
  constexpr int NWX = WCO * WT / 2;
  constexpr size_t RAW = SPL ? 2 * (size_t)((((BT - 1) * S + 1 + HALO_MAX) * (KC / 8) + 64 * NWX - 1) / (64 * NWX)) * NWX * 1024 : 0;
  const size_t lds = (size_t)(2 * win_rows + 2 * TPS * BCO + 1) * Lds<TC>::PITCH * sizeof(TC) + (nice ? RAW : 0);
  if (lds > 160 * 1024) {
    vo_set_error("conv1d: LDS request %zu B exceeds 160 KiB", lds);
    return VO_ERR_INVALID;
  }
  auto kern = nice ? conv1d_kernel<TIN, TC, TOUT, NI, NJ, WCO, WT, TPS, true, ROLE, PRIO, ABL, S, GL, RS, EJ, SEG>
                   : conv1d_kernel<TIN, TC, TOUT, NI, NJ, WCO, WT, TPS, false, ROLE, PRIO, ABL, S, false, false, 2, SEG>;
  a.partial = nullptr;
  a.kcs = 0;
  int splits = 1;
  if constexpr (S == 1) {
    int kcs = 0;
    if (d->workspace && splitk_plan(d, &splits, &kcs) &&
        d->workspace_bytes >= (int64_t)splits * d->B * d->T_out * d->Co * (int64_t)sizeof(float)) {
      a.partial = reinterpret_cast<float*>(d->workspace);
      a.kcs = kcs;
    } else {
      splits = 1;
    }
  }
  const unsigned gx = SEG ? (unsigned)((d->B + BT / 16 - 1) / (BT / 16)) : (unsigned)(a.tiles_per_b * d->B);
  dim3 grid(gx, (unsigned)a.co_tiles, (unsigned)splits);
  hipLaunchKernelGGL(kern, grid, dim3(WCO * WT * 64), lds, st, a);
  if (a.partial) {
    const int64_t n = (int64_t)d->B * d->T_out * (d->Co / 4);
    hipLaunchKernelGGL(conv_splitk_reduce_kernel<TOUT>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, splits);
  }
  VO_RETURN_LAUNCH();
}

template <typename TIN, typename TC, typename TOUT, int NI, int NJ, int WCO, int WT, int TPS_BF16, int ROLE = 0,
          int PRIO = 0, int ABL = 0, bool GL = false, bool RS = false, int EJ = 2>
static int launch_cfg(const vo_conv1d_desc* d, hipStream_t st) {
  return launch_cfg_s<TIN, TC, TOUT, NI, NJ, WCO, WT, TPS_BF16, ROLE, PRIO, ABL, 1, GL, RS, EJ>(d, st);
}
template <typename TIN, typename TC, typename TOUT, int NI, int NJ, int WCO, int WT>
static int launch_seg(const vo_conv1d_desc* d, hipStream_t st) {
  return launch_cfg_s<TIN, TC, TOUT, NI, NJ, WCO, WT, 1, 0, 0, 0, 1, false, false, 2, true>(d, st);
}

#ifdef VO_ABLATIONS
// lin_kernel: K = 1, bf16 input and compute, Ci = 32 NC, Co % BCO == 0 (checked by the caller)
template <typename TOUT, int NI, int NJ, int WCO, int WT, int D, int NC>
static int launch_lin(const vo_conv1d_desc* d, hipStream_t st) {
  constexpr int BCO = 16 * NI * WCO;
  constexpr int BT = 16 * NJ * WT;
  ConvArgs a;
  memset(&a, 0, sizeof(a));
  a.x = d->x; a.xbs = d->x_bstride; a.ldx = d->ldx;
  a.w = d->w; a.bias = d->bias;
  a.y = d->y; a.ybs = d->y_bstride; a.ldy = d->ldy;
  a.res1 = d->res1; a.res2 = d->res2;
  a.T_in = d->T_in; a.T_out = d->T_out; a.Ci = d->Ci; a.Co = d->Co;
  a.K = 1; a.dil = 1; a.pad = 0;
  a.pre_act = VO_ACT_NONE;
  a.post_act = d->post_act; a.post_slope = d->post_slope; a.out_scale = d->out_scale;
  a.tiles_per_b = (d->T_out + BT - 1) / BT;
  a.co_tiles = d->Co / BCO;
  a.B = d->B;
  a.cig = d->Ci; a.cog = d->Co;
  a.ymask = d->ymask; a.ymask_slope = d->ymask_slope;
  auto kern = lin_kernel<TOUT, NI, NJ, WCO, WT, D, NC>;
  dim3 grid((unsigned)(a.tiles_per_b * d->B), (unsigned)a.co_tiles);
  hipLaunchKernelGGL(kern, grid, dim3(WCO * WT * 64), 0, st, a);
  VO_RETURN_LAUNCH();
}
#endif  // VO_ABLATIONS

// HiFi-GAN discriminator layers (strided and/or grouped, C5): 64-row tiles so that a stride-4
// window ((64 - 1) * 4 + 1 + 40 rows) still double-buffers in LDS; output-channel tiles no
// wider than a group where groups are narrow (block-diagonal weights: a tile spanning g
// groups reduces over g groups' input channels).
template <typename TIN, typename TC, typename TOUT, int S>
static int launch_disc_s(const vo_conv1d_desc* d, hipStream_t st) {
  const int groups = d->groups > 1 ? d->groups : 1;
  const int cog = d->Co / groups;
  if constexpr (S >= 8) return launch_cfg_s<TIN, TC, TOUT, 4, 1, 2, 2, 2, 0, 0, 0, S>(d, st);  // 128 x 32
  if (d->Co <= 32 || cog <= 32) return launch_cfg_s<TIN, TC, TOUT, 2, 1, 1, 4, 4, 0, 0, 0, S>(d, st);  // 32 x 64
  if (d->Co <= 64 || cog <= 64) return launch_cfg_s<TIN, TC, TOUT, 4, 1, 1, 4, 4, 0, 0, 0, S>(d, st);  // 64 x 64
  // 64 x 64 where 128 x 64 tiles would leave fewer than 256 workgroups (the MPD's stride-3 layers over joined
  // period columns): C5 23.63 -> 23.57 ms in one process (tile_cfg 4 = off)
  const int64_t t64 = (int64_t)d->B * ((d->T_out + 63) / 64) * ((d->Co + 127) / 128);
  if (vo_tune_get("tile_cfg") != 4 && t64 < 256) return launch_cfg_s<TIN, TC, TOUT, 4, 1, 1, 4, 4, 0, 0, 0, S>(d, st);
  return launch_cfg_s<TIN, TC, TOUT, 4, 2, 2, 2, 2, 0, 0, 0, S>(d, st);                                 // 128 x 64
}
template <typename TIN, typename TC, typename TOUT>
static int launch_disc(const vo_conv1d_desc* d, hipStream_t st) {
  switch (d->stride > 1 ? d->stride : 1) {
    case 1: return launch_disc_s<TIN, TC, TOUT, 1>(d, st);
    case 2: return launch_disc_s<TIN, TC, TOUT, 2>(d, st);
    case 3: return launch_disc_s<TIN, TC, TOUT, 3>(d, st);
    case 4: return launch_disc_s<TIN, TC, TOUT, 4>(d, st);
    case 8: return launch_disc_s<TIN, TC, TOUT, 8>(d, st);  // ConvTranspose1d(k 16, s 8) input gradient
    default: vo_set_error("conv1d: stride %d unsupported (1..4, 8)", d->stride); return VO_ERR_INVALID;
  }
}

#ifdef VO_ABLATIONS
// the lin_kernel tile for a launch; kLinSkip = Co fits no tile
constexpr int kLinSkip = -1000;
template <typename TOUT, int NC>
static int lin_tile(const vo_conv1d_desc* d, hipStream_t st, int lc) {
  if (lc == 2 && d->Co % 64 == 0) return launch_lin<TOUT, 2, 2, 2, 2, 4, NC>(d, st);
  if (lc == 3 && d->Co % 128 == 0) return launch_lin<TOUT, 4, 4, 2, 2, 3, NC>(d, st);
  if (lc == 4 && d->Co % 64 == 0) return launch_lin<TOUT, 2, 4, 2, 2, 4, NC>(d, st);
  if (lc == 5 && d->Co % 128 == 0) return launch_lin<TOUT, 4, 2, 2, 2, 4, NC>(d, st);
  return kLinSkip;
}
#endif  // VO_ABLATIONS

template <typename TIN, typename TC, typename TOUT>
static int launch_types(const vo_conv1d_desc* d, hipStream_t st) {
  const int64_t rows = (int64_t)d->B * d->T_out;
  // short sequences (the glyph encoder / phoneme-level predictors run at T_src ~ 12): one
  // 16- or 32-row time tile, waves spread over output channels
  if constexpr (sizeof(TC) == 4) {
    // fp32 / split-bf16 at T_out <= 16: utterance-segment tiles (SEG, see conv1d_kernel), 4 utterances
    // x 64 output channels (32 below Co = 512); seg_cfg 3 = 8 utterances, 4 = off (the tiles below)
    const int gc = vo_tune_get("seg_cfg");
    if (d->T_out <= 16 && !d->transposed && d->stride <= 1 && (d->K - 1) * d->dil <= SEG_HALO && d->Co >= 32 &&
        gc != 4 && (int64_t)d->B * d->x_bstride < ((int64_t)1 << 31)) {
      if (gc == 3) return d->Co >= 512 ? launch_seg<TIN, TC, TOUT, 2, 4, 2, 2>(d, st) : launch_seg<TIN, TC, TOUT, 1, 4, 2, 2>(d, st);
      return d->Co >= 512 ? launch_seg<TIN, TC, TOUT, 2, 2, 2, 2>(d, st) : launch_seg<TIN, TC, TOUT, 1, 2, 2, 2>(d, st);
    }
  }
  if (d->T_out <= 16 && d->Co >= 64) {
    // fp32 (glyph encoder, variance predictors at B = 32, T = 12): 32 x 16 tiles, 4x the
    // workgroups of 128 x 16: FFN w_1 66 -> 51 us, w_2 28 -> 20, predictor k3 20 -> 13
    // (tools/ab_sb.py genf32 5 3); gen_cfg 2 = 64 x 16, 5 = 128 x 16
    const int gc = vo_tune_get("gen_cfg");
    if (gc == 2) return launch_cfg<TIN, TC, TOUT, 1, 1, 4, 1, 4>(d, st);  // 64 x 16
    if (gc != 5 && sizeof(TC) == 4) return launch_cfg<TIN, TC, TOUT, 1, 1, 2, 1, 4>(d, st);  // 32 x 16
    return launch_cfg<TIN, TC, TOUT, 2, 1, 4, 1, 4>(d, st);  // 128 x 16
  }
  if (d->T_out <= 32 && d->Co >= 64) return launch_cfg<TIN, TC, TOUT, 2, 2, 4, 1, 4>(d, st);  // 128 x 32
  if (d->Co <= 32) return launch_cfg<TIN, TC, TOUT, 2, 4, 1, 4, 4>(d, st);   // 32 x 256
  if (d->Co <= 64 || d->Co == 80) {
    // Co = 80 (PostNet output conv, mel_linear at B*T = 16384 rows): 64 x 128 tiles, twice the
    // workgroups of 64 x 256 (512 -> 80 k5 36.7 -> 29.7 us; tools/probes/small_convs.py)
    const int gc = vo_tune_get("gen_cfg");
    if (gc == 6 || (d->Co == 80 && gc != 8)) return launch_cfg<TIN, TC, TOUT, 4, 2, 1, 4, 4>(d, st);  // 64 x 128
    if (gc == 7) return launch_cfg<TIN, TC, TOUT, 4, 1, 1, 4, 4>(d, st);  // 64 x 64
    return launch_cfg<TIN, TC, TOUT, 4, 4, 1, 4, 4>(d, st);  // 64 x 256
  }
  if (rows <= 2048) return launch_cfg<TIN, TC, TOUT, 2, 2, 2, 2, 2>(d, st);  // 64 x 64
#ifdef VO_ABLATIONS
  if constexpr (sizeof(TC) == 2 && sizeof(TIN) == 2) {
    // K = 1 (Linear layers), A/B only: the LDS-free register-ring kernel, lin_cfg 2 / 3 / 4 / 5 =
    // 64 x 64, 128 x 128, 64 co x 128 rows, 128 co x 64 rows (measured slower, see lin_kernel)
    const int lc = vo_tune_get("lin_cfg");
    if (lc >= 2 && d->K == 1 && d->pad == 0 && d->T_in == d->T_out && !d->transposed && d->variant == 0 &&
        d->pre_act == VO_ACT_NONE && d->Ci % KC == 0 && d->x_bstride % 8 == 0) {
      int rc = kLinSkip;
      if (d->Ci == 256) rc = lin_tile<TOUT, 8>(d, st, lc);
      if (d->Ci == 512) rc = lin_tile<TOUT, 16>(d, st, lc);
      if (d->Ci == 1024) rc = lin_tile<TOUT, 32>(d, st, lc);
      if (rc != kLinSkip) return rc;
    }
  }
#endif
#ifdef VO_ABLATIONS
  if constexpr (sizeof(TC) == 2) {  // K = 1 staging A/B: one tap per step (TPS 1), weights by LDS-DMA (GL), role split (RS)
    const int gq = vo_tune_get("gen_cfg");
    if (gq == 13 && d->Co % 256 == 0) return launch_cfg<TIN, TC, TOUT, 4, 8, 4, 2, 1, 0, 0, 0, true, false>(d, st);
    if (gq == 14 && d->Co % 256 == 0) return launch_cfg<TIN, TC, TOUT, 4, 8, 4, 2, 1, 0, 0, 0, true, true>(d, st);
    if (gq == 15 && d->Co % 128 == 0) return launch_cfg<TIN, TC, TOUT, 4, 4, 2, 2, 1, 0, 0, 0, true, false>(d, st);
    if (gq == 16 && d->Co % 256 == 0) return launch_cfg<TIN, TC, TOUT, 4, 8, 4, 2, 1>(d, st);
    if (gq == 17) return launch_cfg<TIN, TC, TOUT, 2, 4, 2, 2, 1>(d, st);  // 64 x 128, TPS 1
  }
#endif
  if constexpr (sizeof(TC) == 2) {
    if (d->workspace && splitk_bf16_ok(d)) return launch_cfg<TIN, TC, TOUT, 4, 8, 4, 2, 2>(d, st);  // split 256 x 256
  }
  if constexpr (sizeof(TC) == 2) {
    // decoder shapes at B*T = 16384 rows (tools/ab_sb.py gen): wide outputs (FFN w_1 k9 1024,
    // fused q/k/v 768) -> 256 x 256 tiles (-18 %); 1x1 convs to 256 channels -> 64 x 128
    // (twice the workgroups, -12 %).  gen_cfg 1 forces the 128 x 128 tile (A/B).
    if (vo_tune_get("gen_cfg") != 1) {
      // 256 x 256 for the wide convs.  In isolation (tools/probes/wide_convs.py,
      // profiles/r01j/wide_convs.txt) 256 co x 128 rows looked 11 % faster on FFN w_1, but in the
      // bench step its 12 decoder launches took 818 us against 584 (profiles/r01k/): kept out.
      // ups0 (polyphase 512 -> 8 x 256, K = 2) on the role-split staging was 11-20 % slower (its
      // one-step chunks: 8 weight-DMA pieces per weight wave per 2-tap step; tools/probes/ups0_probe.py)
      // (unless that leaves fewer than 128 workgroups: the MPD's joined period columns, ~4-5k rows x
      // 1024 channels, got 68-80 -- there the 128 x 128 tile below)
      const int64_t t256 = (int64_t)d->B * ((d->T_out + 255) / 256) * (d->Co / 256);
      // (utterances of >= 256 rows: at T_out = 128 -- the MSD's 1024-channel layers -- half of every 256-row
      // tile was padding: C5 23.68 -> 23.43 ms with them on the tiles below; tile_cfg 9 = the round-5 rule)
      const bool t_ok = d->T_out >= 256 || vo_tune_get("tile_cfg") == 9;
      if (vo_tune_get("gen_cfg") != 11 && t_ok && d->Co >= 768 && d->Co % 256 == 0 && t256 >= 128) return launch_cfg<TIN, TC, TOUT, 4, 8, 4, 2, 2>(d, st);  // 256 x 256
      if (vo_tune_get("gen_cfg") < 9 && d->K == 1 && d->Co <= 256) return launch_cfg<TIN, TC, TOUT, 2, 4, 2, 2, 2>(d, st);         // 64 x 128
      // Co <= 256 k > 1 with fewer than 512 128 x 128 tiles (the C4 decoder's FFN w_1 input gradient, 1024 ->
      // 256 k9 at 16384 rows: 125 -> 106 us, tools/probes/dgrad_tiles.py): 64 x 128, twice the workgroups
      const int64_t t128 = (int64_t)d->B * ((d->T_out + 127) / 128) * ((d->Co + 127) / 128);
      if (d->Co <= 256 && d->Co % 64 == 0 && t128 < 512) return launch_cfg<TIN, TC, TOUT, 2, 4, 2, 2, 2>(d, st);
      // wide convs with fewer than 256 128 x 128 tiles (C5's MPD over joined period columns, 1024 -> 1024
      // k = 5 at 2-5 k rows: 136-312 workgroups) on 64 x 128 tiles too: C5 24.07 -> 23.75 ms (tile_cfg 1 = off)
      if (vo_tune_get("tile_cfg") != 1 && d->Co % 64 == 0 && t128 < 256) return launch_cfg<TIN, TC, TOUT, 2, 4, 2, 2, 2>(d, st);
    }
    // mid-width convs (PostNet 512 -> 512 k5, conv_pre 80 -> 512 k7 at 16384 rows): 128 x 256
    // tiles (twice the rows per staged weight tap): 512 k5 67.9 -> 63.4 us, 80 k7 27.6 -> 27.0,
    // bit-identical (tools/probes/mid_convs.py); the Co = 128 polyphase upsampler is slower with
    // it (210 -> 234 us).  gen_cfg 9 forces it, gen_cfg 10 = 256 x 128 (no gain), gen_cfg 1 = 128 x 128.
    const int gc = vo_tune_get("gen_cfg");
    if (gc == 9 || (gc != 1 && gc != 10 && d->Co >= 512 && d->Co < 768 && d->Co % 128 == 0 && !d->transposed))
      return launch_cfg<TIN, TC, TOUT, 4, 4, 2, 4, 2>(d, st);  // 128 x 256
    if (gc == 10) return launch_cfg<TIN, TC, TOUT, 4, 4, 4, 2, 2>(d, st);  // 256 x 128
    if (gc == 11) return launch_cfg<TIN, TC, TOUT, 2, 4, 2, 2, 2>(d, st);  // 64 x 128 (A/B)
    if (gc == 12 && d->Co % 256 == 0) return launch_cfg<TIN, TC, TOUT, 4, 8, 4, 2, 2>(d, st);  // 256 x 256 (A/B)
  }
  if constexpr (sizeof(TC) == 2) {  // bf16: 64 x 128 in place of the 128 x 128 default (C5 23.68 -> 23.52 ms, C4 and
                                    // inference shapes unaffected); tile_cfg 9 = the round-5 rule
    if (vo_tune_get("tile_cfg") != 9) return launch_cfg<TIN, TC, TOUT, 2, 4, 2, 2, 2>(d, st);
  }
  return launch_cfg<TIN, TC, TOUT, 4, 4, 2, 2, 2>(d, st);                    // 128 x 128
}

}  // namespace vo

using namespace vo;

int vo_ups_try(const vo_conv1d_desc* d, hipStream_t st, int* handled);  // upsample.hip

extern "C" int64_t vo_conv1d_workspace_size(const vo_conv1d_desc* d) {
  int splits = 1, kcs = 0;
  if (!d || !splitk_plan(d, &splits, &kcs)) return 0;
  return (int64_t)splits * d->B * d->T_out * d->Co * (int64_t)sizeof(float);
}

extern "C" int vo_conv1d(const vo_conv1d_desc* d, void* stream) {
  VO_CHECK_ARG(d != nullptr, "conv1d: null descriptor");
  VO_CHECK_ARG(d->x && d->w && d->y, "conv1d: null tensor pointer");
  VO_CHECK_ARG((d->pre_act != VO_ACT_LRELU || (d->pre_slope >= 0.f && d->pre_slope <= 1.f)) &&
                   (d->post_act != VO_ACT_LRELU || (d->post_slope >= 0.f && d->post_slope <= 1.f)),
               "conv1d: leaky-ReLU slope outside [0, 1]");
  VO_CHECK_ARG(d->B > 0 && d->T_in > 0 && d->T_out > 0 && d->Ci > 0 && d->Co > 0 && d->K > 0,
               "conv1d: non-positive size (B=%d T_in=%d T_out=%d Ci=%d Co=%d K=%d)", d->B,
               d->T_in, d->T_out, d->Ci, d->Co, d->K);
  VO_CHECK_ARG(d->Ci % 8 == 0 && d->ldx % 8 == 0 && d->ldx >= d->Ci,
               "conv1d: Ci (%d) and ldx (%d) must be multiples of 8, ldx >= Ci", d->Ci, d->ldx);
  VO_CHECK_ARG(d->Co % 4 == 0 && d->ldy % 4 == 0, "conv1d: Co (%d) and ldy (%d) must be multiples of 4",
               d->Co, d->ldy);
  VO_CHECK_ARG(d->dil >= 1 && (d->K - 1) * d->dil <= HALO_MAX,
               "conv1d: (K-1)*dil = %d exceeds the supported halo %d", (d->K - 1) * d->dil, HALO_MAX);
  VO_CHECK_ARG(d->variant == 0 || (d->variant == 1 && d->Co >= 128) || (d->variant == 2 && d->Co >= 128) ||
                   (d->variant == 3 && d->Co <= 64 && d->Co % 16 == 0) || (d->variant == 4 && d->Co <= 32),
               "conv1d: variant %d does not fit Co=%d", d->variant, d->Co);
  if (d->transposed) {
    VO_CHECK_ARG(d->up_stride >= 1 && d->up_cout > 0 && d->Co == d->up_stride * d->up_cout &&
                     d->up_cout % 16 == 0 && d->K == 2 && d->pad == 1,
                 "conv1d: bad polyphase ConvTranspose1d descriptor");
  } else {
    VO_CHECK_ARG(d->Co % 16 == 0 || d->Co == 80 || d->Co <= 32, "conv1d: unsupported Co %d", d->Co);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(const_cast<void*>(stream));
  VO_CHECK_ARG(!d->ymask || (d->y_dtype == VO_BF16 && !d->transposed && !d->bias && !d->res1 && !d->res2 &&
                             d->post_act == VO_ACT_NONE && d->out_scale == 1.f && d->variant == 0 &&
                             d->ymask_slope >= 0.f && d->ymask_slope <= 1.f),
               "conv1d: ymask needs a bf16 output without bias, residuals, activation or scale, slope in [0, 1]");
  if (d->transposed) {  // narrow upsamplers: the persistent streaming kernel (upsample.hip)
    int handled = 0;
    const int rc = vo_ups_try(d, st, &handled);
    if (handled) return rc;
  }
  const int xi = d->x_dtype, yo = d->y_dtype;
  if (d->compute_dtype == VO_F32X3) {  // split-bf16 fp32 contractions (vonoma.h)
    VO_CHECK_ARG(xi == VO_F32 && yo == VO_F32 && d->stride <= 1 && d->groups <= 1 && d->variant == 0,
                 "conv1d: VO_F32X3 compute needs fp32 I/O, stride 1, no groups");
    return launch_types<float, bx3_t, float>(d, st);
  }
  if (d->stride > 1 || d->groups > 1) {  // discriminator layers
    const int g = d->groups > 1 ? d->groups : 1;
    VO_CHECK_ARG(!d->transposed && d->variant == 0, "conv1d: stride/groups exclude transposed and variants");
    VO_CHECK_ARG(d->Ci % g == 0 && d->Co % g == 0, "conv1d: Ci %d / Co %d not divisible by groups %d", d->Ci,
                 d->Co, g);
    if (d->compute_dtype == VO_F32) {
      VO_CHECK_ARG(xi == VO_F32 && yo == VO_F32, "conv1d: fp32 compute needs fp32 I/O");
      return launch_disc<float, float, float>(d, st);
    }
    VO_CHECK_ARG(d->compute_dtype == VO_BF16 && xi == VO_BF16, "conv1d: strided/grouped bf16 needs bf16 input");
    if (yo == VO_BF16) return launch_disc<bf16_t, bf16_t, bf16_t>(d, st);
    return launch_disc<bf16_t, bf16_t, float>(d, st);
  }
  if (d->compute_dtype == VO_F32) {
    VO_CHECK_ARG(xi == VO_F32 && yo == VO_F32, "conv1d: fp32 compute needs fp32 I/O");
    return launch_types<float, float, float>(d, st);
  }
  VO_CHECK_ARG(d->compute_dtype == VO_BF16, "conv1d: bad compute dtype");
  if (xi == VO_BF16 && yo == VO_BF16) {
    switch (d->variant) {  // HiFi-GAN MRF stages: own instantiations (same tiles as generic)
      case 1: {  // C = 256: 256 x 256 tile, 8 waves of 64 co x 128 rows (each weight tap feeds
                 // twice the rows of the 128 x 128 tile: 0.095/0.151/0.208 -> 0.077/0.125/0.172 ms
                 // for k = 3/7/11 at B = 32, bit-identical).  conv_cfg 1 = the 128 x 128 tile.
        // s_setprio(1) around each MFMA cluster: +1-3 % (0.1667 -> 0.1654 ms at k = 11); conv_cfg 2 = without
        // Round 2: weights by LDS-DMA (GL): 0.084 / 0.134 / 0.171 -> 0.083 / 0.126 / 0.163 ms for
        // k = 3 / 7 / 11 alone (tools/ab_conv_cfg.py, bit-identical), within noise in the bench step;
        // conv_cfg 3 = register-staged weights, 4 = GL with 3-tap steps (spills)
#ifdef VO_ABLATIONS  // measured-and-dropped tiles (A/B builds only: make abl)
        if (vo_tune_get("conv_cfg") == 1) return launch_cfg<bf16_t, bf16_t, bf16_t, 4, 4, 2, 2, 2, 1>(d, st);
        if (vo_tune_get("conv_cfg") == 2) return launch_cfg<bf16_t, bf16_t, bf16_t, 4, 8, 4, 2, 2, 1>(d, st);
        if (vo_tune_get("conv_cfg") == 3) return launch_cfg<bf16_t, bf16_t, bf16_t, 4, 8, 4, 2, 2, 1, 1>(d, st);
        if (vo_tune_get("conv_cfg") == 4) return launch_cfg<bf16_t, bf16_t, bf16_t, 4, 8, 4, 2, 3, 1, 1, 0, true>(d, st);
        // one tap per step (k = 3's second 2-tap step re-fetches tap 2 as its padding tap)
        if (vo_tune_get("conv_cfg") == 7) return launch_cfg<bf16_t, bf16_t, bf16_t, 4, 8, 4, 2, 1, 1, 1, 0, true>(d, st);
        if (vo_tune_get("conv_cfg") == 8) return launch_cfg<bf16_t, bf16_t, bf16_t, 4, 8, 4, 2, 1, 1, 1, 0, true, true>(d, st);
#endif
        // Round 2: role-split staging (RS: half the waves issue the weight DMA, half copy the window by
        // LDS-DMA two chunks ahead; bare step barriers): k = 7 / 11 0.137 / 0.175 -> 0.130 / 0.168 ms,
        // k = 3 0.084 -> 0.096 (two-step chunks: the weight waves' 8 DMA pieces per step, not the
        // window, bind) -- k >= 5 only; conv_cfg 5 forces it, 6 disables it (tools/probes/s0_probe.py,
        // bit-identical)
        const int cc = vo_tune_get("conv_cfg");
        // Round 3, measured and dropped (tools/mrf_bench.py --stages 0, conv pairs): 4-wave tiles, two
        // workgroups per CU (256 co x 128 rows, 1 tap per step, with and without RS; 128 co x 256 rows)
        // -- 27-45 % slower than the 8-wave 256 x 256 tile at k = 3 / 7 / 11
        // (EJ, the epilogue's position tiles whose residual / accumulator rows are requested
        // together: 4 measured within 1 % of 2, 8 spills and runs 10-20 % slower -- kept at 2)
        if (cc == 5 || (cc != 6 && d->K >= 5))
          return launch_cfg<bf16_t, bf16_t, bf16_t, 4, 8, 4, 2, 2, 1, 1, 0, true, true>(d, st);
        return launch_cfg<bf16_t, bf16_t, bf16_t, 4, 8, 4, 2, 2, 1, 1, 0, true>(d, st);
      }
      case 2: return launch_cfg<bf16_t, bf16_t, bf16_t, 4, 4, 2, 2, 2, 2>(d, st);
      case 3: return launch_cfg<bf16_t, bf16_t, bf16_t, 4, 4, 1, 4, 4, 3>(d, st);
      case 4: return launch_cfg<bf16_t, bf16_t, bf16_t, 2, 4, 1, 4, 4, 4>(d, st);
      default: return launch_types<bf16_t, bf16_t, bf16_t>(d, st);
    }
  }
  if (xi == VO_F32 && yo == VO_BF16) return launch_types<float, bf16_t, bf16_t>(d, st);
  if (xi == VO_BF16 && yo == VO_F32) return launch_types<bf16_t, bf16_t, float>(d, st);
  if (xi == VO_F32 && yo == VO_F32) return launch_types<float, bf16_t, float>(d, st);
  vo_set_error("conv1d: bad dtypes");
  return VO_ERR_INVALID;
}
