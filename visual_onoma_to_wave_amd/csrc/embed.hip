// Energy bucketize + embedding for the teacher-forced training forward, and its backward
// (config C4; reference: VarianceAdaptor.get_energy_embedding with a target,
// scripts/model/modules.py:53-64, and x + energy_embedding, modules.py:101-104).
//   forward:  idx = bucketize(target, bins) (right=False), out = x + table[idx]   (out of place:
//             the autograd graph keeps x for the energy predictor's backward)
//   backward: dx = dy (the caller's); dtable[e] = sum over the rows r with idx[r] == e of dy[r],
//             rows added in increasing r (deterministic: no atomics), one workgroup per table row.

#include "vo_common.h"

namespace vo {

template <typename TX>
__global__ void __launch_bounds__(256) bucket_embed_kernel(const TX* __restrict__ x, const float* __restrict__ target,
                                                           const float* __restrict__ bins, int n_bins,
                                                           const float* __restrict__ table, int64_t rows, int D,
                                                           TX* __restrict__ out, int32_t* __restrict__ idx_out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;  // uniform per wave
  const float v = target[row];
  int lo = 0, hi = n_bins;   // number of bins strictly below v (torch.bucketize, right=False)
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (bins[mid] < v) lo = mid + 1; else hi = mid;
  }
  if (v != v) lo = n_bins;   // NaN -> n_bins, as torch.bucketize
  if (lane == 0 && idx_out) idx_out[row] = lo;
  const float* e = table + (int64_t)lo * D;
  const TX* xr = x + row * D;
  TX* o = out + row * D;
  for (int c = lane * 4; c < D; c += 256) {
    float q[4], w[4];
    load4(xr + c, q);
    load4(e + c, w);
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] += w[k];
    store4(o + c, q);
  }
}

template <typename TG>
__global__ void __launch_bounds__(256) embed_bwd_kernel(const TG* __restrict__ dy, const int32_t* __restrict__ idx,
                                                        int64_t rows, int D, float* __restrict__ dtable) {
  const int e = blockIdx.x;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float acc = 0.f;
    for (int64_t r = 0; r < rows; ++r)  // idx[r] is uniform across the workgroup: no divergence
      if (idx[r] == e) acc += to_f32(dy[r * D + c]);
    dtable[(int64_t)e * D + c] = acc;
  }
}

}  // namespace vo

using namespace vo;

extern "C" int vo_bucket_embed(const void* x, int x_dtype, const float* target, const float* bins, int n_bins,
                               const float* table, int n_table, int64_t rows, int D, void* out, int32_t* idx_out,
                               void* stream) {
  VO_CHECK_ARG(x && target && bins && table && out, "bucket_embed: null pointer");
  VO_CHECK_ARG(rows >= 0 && D > 0 && D % 4 == 0 && n_bins > 0, "bucket_embed: bad sizes");
  VO_CHECK_ARG(n_table >= n_bins + 1, "bucket_embed: table has %d rows, bucketize over %d bins needs %d", n_table,
               n_bins, n_bins + 1);
  VO_CHECK_ARG(x_dtype == VO_F32 || x_dtype == VO_BF16, "bucket_embed: x must be fp32 or bf16");
  if (rows == 0) return VO_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((unsigned)((rows + 3) / 4));
  if (x_dtype == VO_F32)
    hipLaunchKernelGGL(bucket_embed_kernel<float>, grid, dim3(256), 0, st, (const float*)x, target, bins, n_bins,
                       table, rows, D, (float*)out, idx_out);
  else
    hipLaunchKernelGGL(bucket_embed_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)x, target, bins, n_bins,
                       table, rows, D, (bf16_t*)out, idx_out);
  VO_RETURN_LAUNCH();
}

extern "C" int vo_embed_bwd(const void* dy, int dy_dtype, const int32_t* idx, int64_t rows, int D, int n_table,
                            float* dtable, void* stream) {
  VO_CHECK_ARG(dy && idx && dtable, "embed_bwd: null pointer");
  VO_CHECK_ARG(rows >= 0 && D > 0 && n_table > 0, "embed_bwd: bad sizes");
  VO_CHECK_ARG(dy_dtype == VO_F32 || dy_dtype == VO_BF16, "embed_bwd: dy must be fp32 or bf16");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dy_dtype == VO_F32)
    hipLaunchKernelGGL(embed_bwd_kernel<float>, dim3((unsigned)n_table), dim3(256), 0, st, (const float*)dy, idx,
                       rows, D, dtable);
  else
    hipLaunchKernelGGL(embed_bwd_kernel<bf16_t>, dim3((unsigned)n_table), dim3(256), 0, st, (const bf16_t*)dy, idx,
                       rows, D, dtable);
  VO_RETURN_LAUNCH();
}
