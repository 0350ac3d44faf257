// Variance-adaptor heads: Linear(D -> 1) + pad mask, then duration rounding or energy
// bucketize + embedding add, one wave per token.  The discontinuous steps (round,
// bucketize) are evaluated in fp32 with the reference's exact operation order (no FMA
// contraction) so that they flip only where the reference's own inputs flip.
// Reference: VariancePredictor.linear_layer + masked_fill (scripts/model/modules.py:
// 207-213), VarianceAdaptor.get_energy_embedding (modules.py:53-64), duration rounding
// (modules.py:110-113), x + energy_embedding (modules.py:101-104).

#include "vo_common.h"

namespace vo {

template <typename TH, typename TX>
__global__ void __launch_bounds__(256) head_kernel(vo_head_desc d) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)d.B * d.T) return;
  const int b = (int)(row / d.T), t = (int)(row - (int64_t)b * d.T);
  const TH* h = reinterpret_cast<const TH*>(d.h) + row * d.D;
  float acc = 0.f;
  for (int c = lane * 4; c < d.D; c += 256) {
    float q[4];
    load4(h + c, q);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc += q[e] * d.w[c + e];
  }
  acc = wave_sum(acc) + d.b;
  const bool pad = d.lens && t >= d.lens[b];
  float pred = pad ? 0.f : acc;

  if (d.kind == VO_HEAD_DURATION) {
    if (lane == 0) {
      d.pred[row] = pred;
      if (d.d_round) {
        // clamp(round(exp(log_d) - 1) * d_control, min=0); round = half to even
        const float r = rintf(__fsub_rn(expf(pred), 1.0f));
        d.d_round[row] = fmaxf(__fmul_rn(r, d.d_control), 0.0f);
      }
    }
    return;
  }
  // energy
  float v;
  if (d.target) {
    v = d.target[row];
  } else {
    v = __fadd_rn(__fmul_rn(pred, d.e_std), d.e_mean);
    v = __fmul_rn(v, d.e_control);
    v = __fdiv_rn(__fsub_rn(v, d.e_mean), d.e_std);
    pred = v;
  }
  // bucketize(right=False): number of bins strictly below v; a NaN goes to bucket n_bins, as in
  // torch.bucketize (every comparison with NaN is false there)
  int lo = 0, hi = d.n_bins;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (d.bins[mid] < v) lo = mid + 1; else hi = mid;
  }
  if (v != v) lo = d.n_bins;
  const int idx = lo;
  if (lane == 0) {
    d.pred[row] = pred;
    if (d.idx_out) d.idx_out[row] = idx;
  }
  TX* x = reinterpret_cast<TX*>(d.x) + row * d.D;
  const float* e = d.table + (int64_t)idx * d.D;
  for (int c = lane * 4; c < d.D; c += 256) {
    float q[4], w[4];
    load4(x + c, q);
    load4(e + c, w);
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] += w[k];
    store4(x + c, q);
  }
}

}  // namespace vo

using namespace vo;

extern "C" int vo_variance_head(const vo_head_desc* d, void* stream) {
  VO_CHECK_ARG(d && d->h && d->w && d->pred, "variance_head: null pointer");
  VO_CHECK_ARG(d->D % 4 == 0 && d->B > 0 && d->T > 0, "variance_head: bad sizes");
  if (d->kind == VO_HEAD_ENERGY)
    VO_CHECK_ARG(d->bins && d->table && d->x && d->n_bins > 0, "variance_head: energy head needs bins/table/x");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((unsigned)(((int64_t)d->B * d->T + 3) / 4));
  const int xd = d->kind == VO_HEAD_ENERGY ? d->x_dtype : d->h_dtype;
#define VO_H(TH, TX) hipLaunchKernelGGL((head_kernel<TH, TX>), grid, dim3(256), 0, st, *d)
  if (d->h_dtype == VO_BF16 && xd == VO_BF16) VO_H(bf16_t, bf16_t);
  else if (d->h_dtype == VO_F32 && xd == VO_F32) VO_H(float, float);
  else if (d->h_dtype == VO_BF16 && xd == VO_F32) VO_H(bf16_t, float);
  else if (d->h_dtype == VO_F32 && xd == VO_BF16) VO_H(float, bf16_t);
  else {
    vo_set_error("variance_head: bad dtypes");
    return VO_ERR_INVALID;
  }
#undef VO_H
  VO_RETURN_LAUNCH();
}
