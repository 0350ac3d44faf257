// LengthRegulator as a device-side scan + gather (bit-exact indices).
//
// Reference: LengthRegulator.LR/expand (scripts/model/modules.py:132-159) repeats token
// j of batch b max(int(d[b, j]), 0) times (int() truncates toward zero), concatenates,
// and pads with zeros (scripts/utils/tools.py:669-687) to max_len -- or CROPS when the
// expansion is longer (F.pad with a negative amount).  mel_len[b] is the uncropped
// expansion length.  The reference issues one .item() device->host sync per token; here
// frame t of batch b reads token j = min{ j : cs[j] > t } (cs = inclusive cumsum).

#include "vo_common.h"

namespace vo {

__device__ __forceinline__ int reps_of(float d) {
  const float tr = truncf(d);
  return tr > 0.f ? (int)tr : 0;
}

__global__ void lr_lengths_kernel(const float* __restrict__ dur, int B, int T, int64_t* mel_len,
                                  int32_t* mel_len32) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int64_t s = 0;
  for (int j = 0; j < T; ++j) s += reps_of(dur[(int64_t)b * T + j]);
  if (mel_len) mel_len[b] = s;
  if (mel_len32) mel_len32[b] = (int32_t)s;
}

constexpr int LR_ROWS = 32;     // output frames per workgroup
constexpr int LR_TMAX = 2048;   // max tokens per utterance held in LDS

template <typename TX, typename TY>
__global__ void __launch_bounds__(256) lr_gather_kernel(const TX* __restrict__ x, const float* __restrict__ dur,
                                                        int T, int D, int max_len, TY* __restrict__ out,
                                                        int64_t* __restrict__ mel_len, int32_t* __restrict__ index) {
  __shared__ int cs[LR_TMAX];
  __shared__ int src[LR_ROWS];
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * LR_ROWS;
  const int tid = threadIdx.x;
  // inclusive cumsum of the truncated repeats (T is small: one wave scans in chunks of 64)
  if (tid < 64) {
    int carry = 0;
    for (int base = 0; base < T; base += 64) {
      const int j = base + tid;
      int v = (j < T) ? reps_of(dur[(int64_t)b * T + j]) : 0;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int n = __shfl_up(v, o, 64);
        if (tid >= o) v += n;
      }
      if (j < T) cs[j] = carry + v;
      carry += __shfl(v, 63, 64);
    }
  }
  __syncthreads();
  const int total = T > 0 ? cs[T - 1] : 0;
  if (blockIdx.x == 0 && tid == 0 && mel_len) mel_len[b] = total;
  if (tid < LR_ROWS) {
    const int t = t0 + tid;
    int j = -1;
    if (t < total && t < max_len) {
      int lo = 0, hi = T - 1;  // first j with cs[j] > t
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cs[mid] > t) hi = mid; else lo = mid + 1;
      }
      j = lo;
    }
    src[tid] = j;
    if (index && t < max_len) index[(int64_t)b * max_len + t] = j;
  }
  __syncthreads();
  const int vpr = D / 4;  // 4-element vectors per row
  for (int v = tid; v < LR_ROWS * vpr; v += 256) {
    const int r = v / vpr, c = (v - r * vpr) * 4;
    const int t = t0 + r;
    if (t >= max_len) continue;
    float q[4] = {0.f, 0.f, 0.f, 0.f};
    const int j = src[r];
    if (j >= 0) load4(x + ((int64_t)b * T + j) * D + c, q);
    store4(out + ((int64_t)b * max_len + t) * D + c, q);
  }
}

// Backward (training, C4): gx[b, j, :] = sum of go[b, t, :] over the frames token j was copied
// to, t in [cs[j-1], min(cs[j], max_len)) -- a segmented row sum (frames of one token are
// contiguous), added in frame order: deterministic, no atomics, no index tensor.  One workgroup
// per (token, utterance); 256 threads = 8 frame phases x 32 threads of 8 channels (D <= 256 per
// pass, looped for wider rows), the phases added in LDS in a fixed order.
// Replaces the autograd of the LR concat / pad (modules.py:132-159, tools.py:669-687).
template <typename TG, typename TX>
__global__ void __launch_bounds__(256) lr_bwd_kernel(const TG* __restrict__ go, const float* __restrict__ dur,
                                                     int T, int D, int max_len, TX* __restrict__ gx) {
  __shared__ float red[8][256];
  const int j = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, ph = tid >> 5, cl = (tid & 31) * 8;
  int start = 0;
  for (int i = 0; i < j; ++i) start += reps_of(dur[(int64_t)b * T + i]);
  const int end = min(start + reps_of(dur[(int64_t)b * T + j]), max_len);
  for (int c0 = 0; c0 < D; c0 += 256) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (c0 + cl < D)
      for (int t = start + ph; t < end; t += 8) {
        float v[8];
        load8(go + ((int64_t)b * max_len + t) * D + c0 + cl, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += v[e];
      }
#pragma unroll
    for (int e = 0; e < 8; ++e) red[ph][cl + e] = acc[e];
    __syncthreads();
    if (ph == 0 && c0 + cl < D) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) t += red[q][cl + e];
        o[e] = t;
      }
      store8(gx + ((int64_t)b * T + j) * D + c0 + cl, o);
    }
    __syncthreads();
  }
}

}  // namespace vo

using namespace vo;

extern "C" int vo_lr_lengths(const float* dur, int B, int T_src, int64_t* mel_len, int32_t* mel_len32,
                             void* stream) {
  VO_CHECK_ARG(dur && (mel_len || mel_len32), "lr_lengths: null pointer");
  VO_CHECK_ARG(B > 0 && T_src >= 0, "lr_lengths: bad sizes");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(lr_lengths_kernel, dim3((B + 255) / 256), dim3(256), 0, st, dur, B, T_src, mel_len,
                     mel_len32);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_length_regulate(const void* x, int x_dtype, const float* dur, int B, int T_src, int D,
                                  int max_len, void* out, int out_dtype, int64_t* mel_len, int32_t* index,
                                  void* stream) {
  VO_CHECK_ARG(x && dur && out, "length_regulate: null pointer");
  VO_CHECK_ARG(B > 0 && T_src > 0 && T_src <= LR_TMAX, "length_regulate: T_src=%d out of range (1..%d)",
               T_src, LR_TMAX);
  VO_CHECK_ARG(D % 4 == 0 && D > 0, "length_regulate: D=%d must be a multiple of 4", D);
  VO_CHECK_ARG(max_len >= 0, "length_regulate: negative max_len");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (max_len == 0) {
    if (mel_len) hipLaunchKernelGGL(lr_lengths_kernel, dim3((B + 255) / 256), dim3(256), 0, st, dur, B, T_src,
                                    mel_len, (int32_t*)nullptr);
    VO_RETURN_LAUNCH();
  }
  dim3 grid((unsigned)((max_len + LR_ROWS - 1) / LR_ROWS), (unsigned)B);
#define VO_LR(TX, TY)                                                                                     \
  hipLaunchKernelGGL((lr_gather_kernel<TX, TY>), grid, dim3(256), 0, st, (const TX*)x, dur, T_src, D, max_len, \
                     (TY*)out, mel_len, index)
  if (x_dtype == VO_BF16 && out_dtype == VO_BF16) VO_LR(bf16_t, bf16_t);
  else if (x_dtype == VO_F32 && out_dtype == VO_F32) VO_LR(float, float);
  else if (x_dtype == VO_F32 && out_dtype == VO_BF16) VO_LR(float, bf16_t);
  else if (x_dtype == VO_BF16 && out_dtype == VO_F32) VO_LR(bf16_t, float);
  else {
    vo_set_error("length_regulate: bad dtypes");
    return VO_ERR_INVALID;
  }
#undef VO_LR
  VO_RETURN_LAUNCH();
}

extern "C" int vo_length_regulate_bwd(const void* go, int go_dtype, const float* dur, int B, int T_src, int D,
                                      int max_len, void* gx, int gx_dtype, void* stream) {
  VO_CHECK_ARG(go && dur && gx, "length_regulate_bwd: null pointer");
  VO_CHECK_ARG(B > 0 && T_src > 0 && max_len >= 0, "length_regulate_bwd: bad sizes");
  VO_CHECK_ARG(D % 8 == 0 && D > 0, "length_regulate_bwd: D=%d must be a multiple of 8", D);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((unsigned)T_src, (unsigned)B);
#define VO_LRB(TG, TX)                                                                                        \
  hipLaunchKernelGGL((lr_bwd_kernel<TG, TX>), grid, dim3(256), 0, st, (const TG*)go, dur, T_src, D, max_len, \
                     (TX*)gx)
  if (go_dtype == VO_BF16 && gx_dtype == VO_F32) VO_LRB(bf16_t, float);
  else if (go_dtype == VO_F32 && gx_dtype == VO_F32) VO_LRB(float, float);
  else if (go_dtype == VO_BF16 && gx_dtype == VO_BF16) VO_LRB(bf16_t, bf16_t);
  else if (go_dtype == VO_F32 && gx_dtype == VO_BF16) VO_LRB(float, bf16_t);
  else {
    vo_set_error("length_regulate_bwd: bad dtypes");
    return VO_ERR_INVALID;
  }
#undef VO_LRB
  VO_RETURN_LAUNCH();
}
