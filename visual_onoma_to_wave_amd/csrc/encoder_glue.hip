// Encoder front: the visual feature extractor's per-glyph stencil stack, and the
// positional / class embedding adds.
//
// vfe_stencil replaces VisualFeatureExtractor.forward up to the bridge Linear
// (scripts/model/visual_feature_extractor.py:60-80): the Python loop that slices the
// strip into 102-px character columns becomes the grid (one workgroup per slice), and
// the three Conv2d(1->1, 3x3, pad 1) -> BatchNorm2d(eval) -> ReLU layers run in LDS on
// the 24 x 102 tile with a zero border.  Output is the flattened (h*W + w) row the
// bridge GEMM reads.

#include "vo_common.h"

namespace vo {

constexpr int VFE_MAXH = 32;
constexpr int VFE_MAXW = 128;

template <typename TY>
__global__ void __launch_bounds__(256) vfe_kernel(const float* __restrict__ img, int H, int W, int sw, int n_slices,
                                                  const float* __restrict__ conv, const float* __restrict__ bn,
                                                  int n_layers, TY* __restrict__ out) {
  __shared__ float buf[2][(VFE_MAXH + 2) * (VFE_MAXW + 2)];
  const int P = sw + 2;  // pitch with a 1-px zero border on each side
  const int slice = blockIdx.x;
  const int b = slice / n_slices, i = slice - b * n_slices;
  const float* src = img + (int64_t)b * H * W + (int64_t)i * sw;
  const int tid = threadIdx.x;
  for (int v = tid; v < (H + 2) * P; v += 256) {
    const int r = v / P, c = v - r * P;
    float val = 0.f;
    if (r >= 1 && r <= H && c >= 1 && c <= sw) val = src[(int64_t)(r - 1) * W + (c - 1)];
    buf[0][v] = val;
    buf[1][v] = 0.f;
  }
  __syncthreads();
  int cur = 0;
  for (int l = 0; l < n_layers; ++l) {
    const float* k = conv + l * 10;
    const float sc = bn[2 * l], sh = bn[2 * l + 1];
    for (int v = tid; v < H * sw; v += 256) {
      const int r = v / sw + 1, c = v - (r - 1) * sw + 1;
      const float* s = buf[cur];
      float acc = k[9];
#pragma unroll
      for (int dr = -1; dr <= 1; ++dr)
#pragma unroll
        for (int dc = -1; dc <= 1; ++dc) acc += k[(dr + 1) * 3 + (dc + 1)] * s[(r + dr) * P + (c + dc)];
      const float y = acc * sc + sh;
      buf[cur ^ 1][r * P + c] = y > 0.f ? y : 0.f;
    }
    __syncthreads();
    cur ^= 1;
  }
  TY* o = out + (int64_t)slice * H * sw;
  for (int v = tid; v < H * sw; v += 256) {
    const int r = v / sw, c = v - r * sw;
    o[v] = from_f32<TY>(buf[cur][(r + 1) * P + (c + 1)]);
  }
}

template <typename TX>
__global__ void add_pos_class_kernel(TX* __restrict__ x, const float* __restrict__ pe, const float* __restrict__ cls,
                                     const int64_t* __restrict__ cls_idx, int per_token, int B, int T, int D) {
  const int64_t n4 = (int64_t)B * T * D / 4;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n4; v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = v * 4;
    const int c = (int)(e % D);
    const int64_t bt = e / D;
    const int t = (int)(bt % T), b = (int)(bt / T);
    float q[4];
    load4(x + e, q);
    if (pe) {
      float p[4];
      load4(pe + (int64_t)t * D + c, p);
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] += p[k];
    }
    if (cls) {
      float p[4];
      load4(cls + cls_idx[per_token ? bt : b] * D + c, p);
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] += p[k];
    }
    store4(x + e, q);
  }
}

// mask[b, t] = t >= len[b] (True = padding), len given as int64, int32 or float
template <typename TL>
__global__ void mask_kernel(const TL* __restrict__ lens, int B, int L, bool* __restrict__ mask,
                            int32_t* __restrict__ lens32) {
  const int64_t n = (int64_t)B * L;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(v / L), t = (int)(v - (int64_t)b * L);
    if (mask) mask[v] = (double)t >= (double)lens[b];
    if (lens32 && t == 0) lens32[b] = (int32_t)lens[b];
  }
  if (L == 0 && lens32) {
    for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < B; b += gridDim.x * blockDim.x) lens32[b] = (int32_t)lens[b];
  }
}

}  // namespace vo

using namespace vo;

extern "C" int vo_mask_from_lengths(const void* lens, int lens_dtype, int B, int L, bool* mask, int32_t* lens32,
                                    void* stream) {
  VO_CHECK_ARG(lens && (mask || lens32), "mask_from_lengths: null pointer");
  if (B == 0) return VO_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = std::max<int64_t>((int64_t)B * L, B);
  dim3 grid((unsigned)std::min<int64_t>((n + 255) / 256, 1024));
  if (lens_dtype == 0)
    hipLaunchKernelGGL(mask_kernel<float>, grid, dim3(256), 0, st, (const float*)lens, B, L, mask, lens32);
  else if (lens_dtype == 2)
    hipLaunchKernelGGL(mask_kernel<int64_t>, grid, dim3(256), 0, st, (const int64_t*)lens, B, L, mask, lens32);
  else if (lens_dtype == 3)
    hipLaunchKernelGGL(mask_kernel<int32_t>, grid, dim3(256), 0, st, (const int32_t*)lens, B, L, mask, lens32);
  else {
    vo_set_error("mask_from_lengths: lens dtype must be 0 (f32), 2 (int64) or 3 (int32)");
    return VO_ERR_INVALID;
  }
  VO_RETURN_LAUNCH();
}

extern "C" int vo_vfe_stencil(const float* images, int B, int H, int W, int slice_w, int n_slices, const float* conv,
                              const float* bn, int n_layers, void* out, int out_dtype, void* stream) {
  VO_CHECK_ARG(images && conv && bn && out, "vfe_stencil: null pointer");
  VO_CHECK_ARG(H <= VFE_MAXH && slice_w <= VFE_MAXW && H > 0 && slice_w > 0,
               "vfe_stencil: slice %dx%d exceeds %dx%d", H, slice_w, VFE_MAXH, VFE_MAXW);
  VO_CHECK_ARG(n_slices >= 0 && (int64_t)n_slices * slice_w <= W, "vfe_stencil: %d slices of %d px > width %d",
               n_slices, slice_w, W);
  if (B == 0 || n_slices == 0) return VO_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((unsigned)(B * n_slices));
  if (out_dtype == VO_BF16)
    hipLaunchKernelGGL(vfe_kernel<bf16_t>, grid, dim3(256), 0, st, images, H, W, slice_w, n_slices, conv, bn,
                       n_layers, (bf16_t*)out);
  else
    hipLaunchKernelGGL(vfe_kernel<float>, grid, dim3(256), 0, st, images, H, W, slice_w, n_slices, conv, bn,
                       n_layers, (float*)out);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_add_pos_class(void* x, int x_dtype, const float* pe, const float* cls, const int64_t* cls_idx,
                                int idx_per_token, int B, int T, int D, void* stream) {
  VO_CHECK_ARG(x && (!cls || cls_idx), "add_pos_class: null pointer");
  VO_CHECK_ARG(D % 4 == 0, "add_pos_class: D=%d must be a multiple of 4", D);
  if (B == 0 || T == 0) return VO_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n4 = (int64_t)B * T * D / 4;
  dim3 grid((unsigned)std::min<int64_t>((n4 + 255) / 256, 2048));
  if (x_dtype == VO_BF16)
    hipLaunchKernelGGL(add_pos_class_kernel<bf16_t>, grid, dim3(256), 0, st, (bf16_t*)x, pe, cls, cls_idx, idx_per_token, B, T, D);
  else
    hipLaunchKernelGGL(add_pos_class_kernel<float>, grid, dim3(256), 0, st, (float*)x, pe, cls, cls_idx, idx_per_token, B, T, D);
  VO_RETURN_LAUNCH();
}
