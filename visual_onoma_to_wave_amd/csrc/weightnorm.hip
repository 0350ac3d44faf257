// Weight normalisation w = g * v / ||v|| (norm over every dim but 0, torch.nn.utils.weight_norm's
// dim = 0) and its backward, for MANY layers per launch: the HiFi-GAN generator and discriminators
// (C5) re-derive every conv weight from (weight_v, weight_g) in each training forward, ~80
// generator + 46 discriminator layers per step, which PyTorch ran as one forward and one backward
// kernel per layer (124 + 144 launches of ~7 us, 1.8 ms of a 39 ms step).
//
// One wave per output row (layer l, row r): the row's squared norm (and, backward, its dot product
// with dL/dw) is reduced in a fixed order -- lane-strided partial sums, then a butterfly over the
// wave -- so the result is deterministic.  The layer table rides in the kernel arguments (24
// layers per launch), so the launch is graph-capturable with no device-side table.
//   forward:  w = v * (g / n),                          n = ||v||
//   backward: dg = (dw . v) / n,   dv = (g / n) * (dw - v * (dw . v) / n^2)

#include <algorithm>

#include "vo_common.h"

namespace vo {

constexpr int WN_MAX = 24;

struct WnLayer {
  const float* v; const float* g; float* w;  // forward
  const float* dw; float* dv; float* dg;      // backward
  int rows, len;
};
struct WnArgs {
  WnLayer l[WN_MAX];
  int row0[WN_MAX + 1];  // first global row of each layer; row0[n] = total rows
  int n;
};

template <bool BWD>
__global__ void __launch_bounds__(256) weight_norm_kernel(WnArgs a) {
  const int lane = threadIdx.x & 63;
  // this wave's global row (wave-uniform: the layer lookup below stays scalar)
  const int gr = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (gr >= a.row0[a.n]) return;                       // uniform per wave
  const int li = table_find(a.row0, a.n, gr);
  const WnLayer& L = a.l[li];
  const int r = gr - a.row0[li], len = L.len;
  const int64_t base = (int64_t)r * len;
  const float* v = L.v + base;
  // 16-byte vectors when the row allows it (row starts stay 16-byte aligned iff len % 4 == 0)
  // (every pointer the vector path reads or writes: v and w forward; v, dw and dv backward)
  const bool vec = (len & 3) == 0 && (reinterpret_cast<uintptr_t>(L.v) & 15) == 0 &&
                   (BWD ? ((reinterpret_cast<uintptr_t>(L.dw) | reinterpret_cast<uintptr_t>(L.dv)) & 15) == 0
                        : (reinterpret_cast<uintptr_t>(L.w) & 15) == 0);
  float ss = 0.f, dot = 0.f;
  const float* dw = BWD ? L.dw + base : nullptr;
  if (vec) {
#pragma unroll 4  // several row loads in flight per wave (the loop was latency-bound)
    for (int i = lane * 4; i < len; i += 256) {
      const float4 x = *reinterpret_cast<const float4*>(v + i);
      ss += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
      if constexpr (BWD) {
        const float4 d = *reinterpret_cast<const float4*>(dw + i);
        dot += d.x * x.x + d.y * x.y + d.z * x.z + d.w * x.w;
      }
    }
  } else {
    for (int i = lane; i < len; i += 64) {
      const float x = v[i];
      ss += x * x;
      if constexpr (BWD) dot += dw[i] * x;
    }
  }
  ss = wave_sum(ss);
  const float nrm = sqrtf(ss);
  const float g = L.g[r];
  const float s = g / nrm;
  if constexpr (!BWD) {
    float* w = L.w + base;
    if (vec) {
#pragma unroll 4
      for (int i = lane * 4; i < len; i += 256) {
        const float4 x = *reinterpret_cast<const float4*>(v + i);
        *reinterpret_cast<float4*>(w + i) = make_float4(x.x * s, x.y * s, x.z * s, x.w * s);
      }
    } else {
      for (int i = lane; i < len; i += 64) w[i] = v[i] * s;
    }
  } else {
    dot = wave_sum(dot);
    if (lane == 0) L.dg[r] = dot / nrm;
    const float c = dot / ss;
    float* dv = L.dv + base;
    if (vec) {
#pragma unroll 4
      for (int i = lane * 4; i < len; i += 256) {
        const float4 x = *reinterpret_cast<const float4*>(v + i);
        const float4 d = *reinterpret_cast<const float4*>(dw + i);
        *reinterpret_cast<float4*>(dv + i) =
            make_float4(s * (d.x - x.x * c), s * (d.y - x.y * c), s * (d.z - x.z * c), s * (d.w - x.w * c));
      }
    } else {
      for (int i = lane; i < len; i += 64) dv[i] = s * (dw[i] - v[i] * c);
    }
  }
}

template <bool BWD>
static int wn_launch(int n, const void* const* v, const void* const* g, void* const* w, const void* const* dw,
                     void* const* dv, void* const* dg, const int* rows, const int* len, hipStream_t st) {
  for (int i0 = 0; i0 < n; i0 += WN_MAX) {
    WnArgs a;
    a.n = std::min(WN_MAX, n - i0);
    int total = 0;
    for (int i = 0; i < a.n; ++i) {
      const int k = i0 + i;
      VO_CHECK_ARG(v[k] && g[k] && rows[k] > 0 && len[k] > 0, "weight_norm: layer %d: null pointer or empty", k);
      VO_CHECK_ARG(BWD ? (dw[k] && dv[k] && dg[k]) : (w[k] != nullptr), "weight_norm: layer %d: null output", k);
      VO_CHECK_ARG((int64_t)total + rows[k] < (1 << 30), "weight_norm: too many rows");
      WnLayer& L = a.l[i];
      L.v = (const float*)v[k]; L.g = (const float*)g[k];
      L.w = BWD ? nullptr : (float*)w[k];
      L.dw = BWD ? (const float*)dw[k] : nullptr;
      L.dv = BWD ? (float*)dv[k] : nullptr;
      L.dg = BWD ? (float*)dg[k] : nullptr;
      L.rows = rows[k]; L.len = len[k];
      a.row0[i] = total;
      total += rows[k];
    }
    a.row0[a.n] = total;
    hipLaunchKernelGGL(weight_norm_kernel<BWD>, dim3((unsigned)((total + 3) / 4)), dim3(256), 0, st, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      vo_set_error("weight_norm: launch failed: %s", hipGetErrorString(e));
      return (int)e;
    }
  }
  return VO_OK;
}

}  // namespace vo

using namespace vo;

extern "C" int vo_weight_norm(int n, const void* const* v, const void* const* g, void* const* w, const int* rows,
                              const int* len, void* stream) {
  VO_CHECK_ARG(n >= 0 && (n == 0 || (v && g && w && rows && len)), "weight_norm: null table");
  return wn_launch<false>(n, v, g, w, nullptr, nullptr, nullptr, rows, len, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int vo_weight_norm_bwd(int n, const void* const* v, const void* const* g, const void* const* dw,
                                  void* const* dv, void* const* dg, const int* rows, const int* len, void* stream) {
  VO_CHECK_ARG(n >= 0 && (n == 0 || (v && g && dw && dv && dg && rows && len)), "weight_norm_bwd: null table");
  return wn_launch<true>(n, v, g, nullptr, dw, dv, dg, rows, len, reinterpret_cast<hipStream_t>(stream));
}
