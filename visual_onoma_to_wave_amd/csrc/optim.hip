// Multi-tensor Adam / AdamW step (training configs C4 and C5): one launch updates up to
// VO_OPT_MAX tensors (the tensor table rides in the kernel arguments), every workgroup one
// 4096-element chunk of one tensor.  The learning rate and the step count are read from device
// memory, so the update is graph-capturable (HIP-graph training steps) and needs no host sync.
// Per element, in the order of torch.optim.Adam / AdamW (single-tensor form):
//   AdamW: p *= 1 - lr * wd            Adam: g += wd * p
//   m = m + (g - m) * (1 - b1)          (lerp)
//   v = v * b2 + (1 - b2) * g * g
//   p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)       with t = step + 1
// The step count itself is advanced by vo_opt_step_increment after every chunk launch of a step.
// Replaces: torch.optim.Adam (scripts/model/optimizer.py:9-15, via ScheduledOptim) and the AdamW
// of the HiFi-GAN V1 recipe (scripts/hifigan/config.json: adam_b1 / adam_b2 / learning_rate).

#include "vo_common.h"

namespace vo {

constexpr int OPT_MAX = 64;
constexpr int OPT_CHUNK = 4096;

struct OptArgs {
  float* p[OPT_MAX];
  const float* g[OPT_MAX];
  float* m[OPT_MAX];
  float* v[OPT_MAX];
  int64_t n[OPT_MAX];
  int chunk0[OPT_MAX + 1];  // first chunk of each tensor; chunk0[nt] = total chunks
  int nt;
  const float* lr;
  const float* step;        // steps taken so far (this update is step + 1)
  float b1, b2, eps, wd;
  int decoupled;
};

__global__ void __launch_bounds__(256) adam_multi_kernel(OptArgs a) {
  const int c = blockIdx.x;
  int t = 0;  // the chunk's tensor (uniform: binary search over the argument table)
  {
    int lo = 0, hi = a.nt - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.chunk0[mid] <= c) lo = mid; else hi = mid - 1;
    }
    t = lo;
  }
  const int64_t base = (int64_t)(c - a.chunk0[t]) * OPT_CHUNK;
  const int64_t end = min<int64_t>(a.n[t], base + OPT_CHUNK);
  float* __restrict__ P = a.p[t];
  const float* __restrict__ G = a.g[t];
  float* __restrict__ M = a.m[t];
  float* __restrict__ V = a.v[t];
  const float lr = *a.lr;
  const float st = *a.step + 1.0f;
  const float bc1 = 1.0f - powf(a.b1, st);
  const float bc2s = sqrtf(1.0f - powf(a.b2, st));
  const float step_size = lr / bc1;
  const float decay = a.decoupled ? 1.0f - lr * a.wd : 1.0f;
  const float l2 = a.decoupled ? 0.0f : a.wd;
  const float omb1 = 1.0f - a.b1, omb2 = 1.0f - a.b2;
  auto upd = [&](float& p, float g, float& m, float& v) {
    p *= decay;
    g = fmaf(l2, p, g);
    m = fmaf(g - m, omb1, m);
    v = fmaf(v, a.b2, omb2 * g * g);
    p -= step_size * m / (sqrtf(v) / bc2s + a.eps);
  };
  const bool vec = ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(G) | reinterpret_cast<uintptr_t>(M) |
                     reinterpret_cast<uintptr_t>(V)) & 15) == 0;
  if (vec) {
    const int64_t vend = base + ((end - base) & ~(int64_t)3);
    for (int64_t i = base + threadIdx.x * 4; i < vend; i += 1024) {
      float4 p = *reinterpret_cast<float4*>(P + i), m = *reinterpret_cast<float4*>(M + i);
      float4 v = *reinterpret_cast<float4*>(V + i);
      const float4 g = *reinterpret_cast<const float4*>(G + i);
      upd(p.x, g.x, m.x, v.x); upd(p.y, g.y, m.y, v.y); upd(p.z, g.z, m.z, v.z); upd(p.w, g.w, m.w, v.w);
      *reinterpret_cast<float4*>(P + i) = p;
      *reinterpret_cast<float4*>(M + i) = m;
      *reinterpret_cast<float4*>(V + i) = v;
    }
    for (int64_t i = vend + threadIdx.x; i < end; i += 256) upd(P[i], G[i], M[i], V[i]);
  } else {
    for (int64_t i = base + threadIdx.x; i < end; i += 256) upd(P[i], G[i], M[i], V[i]);
  }
}

__global__ void opt_step_increment_kernel(float* step) { *step += 1.0f; }

}  // namespace vo

using namespace vo;

extern "C" int vo_adam_multi(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                             const int64_t* numel, const float* lr, const float* step, float beta1, float beta2,
                             float eps, float weight_decay, int decoupled, void* stream) {
  VO_CHECK_ARG(nt >= 0 && p && g && m && v && numel && lr && step, "adam_multi: null pointer");
  VO_CHECK_ARG(beta1 >= 0.f && beta1 < 1.f && beta2 >= 0.f && beta2 < 1.f, "adam_multi: betas outside [0, 1)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int t0 = 0; t0 < nt; t0 += OPT_MAX) {
    OptArgs a;
    a.nt = 0;
    int chunks = 0;
    for (int t = t0; t < nt && t < t0 + OPT_MAX; ++t) {
      VO_CHECK_ARG(p[t] && g[t] && m[t] && v[t] && numel[t] >= 0, "adam_multi: bad tensor %d", t);
      if (numel[t] == 0) continue;
      const int k = a.nt++;
      a.p[k] = p[t]; a.g[k] = g[t]; a.m[k] = m[t]; a.v[k] = v[t]; a.n[k] = numel[t];
      a.chunk0[k] = chunks;
      const int64_t c = (numel[t] + OPT_CHUNK - 1) / OPT_CHUNK;
      VO_CHECK_ARG(chunks + c < (int64_t)1 << 30, "adam_multi: too many chunks");
      chunks += (int)c;
    }
    if (a.nt == 0) continue;
    a.chunk0[a.nt] = chunks;
    a.lr = lr; a.step = step;
    a.b1 = beta1; a.b2 = beta2; a.eps = eps; a.wd = weight_decay; a.decoupled = decoupled;
    hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)chunks), dim3(256), 0, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      vo_set_error("adam_multi: launch failed: %s", hipGetErrorString(e));
      return (int)e;
    }
  }
  return VO_OK;
}

extern "C" int vo_opt_step_increment(float* step, void* stream) {
  VO_CHECK_ARG(step, "opt_step_increment: null pointer");
  hipLaunchKernelGGL(opt_step_increment_kernel, dim3(1), dim3(1), 0, reinterpret_cast<hipStream_t>(stream), step);
  VO_RETURN_LAUNCH();
}
