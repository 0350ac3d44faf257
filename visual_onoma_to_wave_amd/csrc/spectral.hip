// Spectral normalisation w = W / sigma(W) with one power iteration per training forward
// (torch.nn.utils.spectral_norm, dim 0, n_power_iterations 1, eps 1e-12 -- the first scale of the
// HiFi-GAN V1 MSD, config C5) for MANY layers per launch.  PyTorch's hook ran ~13 kernels per layer
// and forward (two rocBLAS gemv, norms, clamps, divides, clones, a dot): 8 layers x 3 discriminator
// passes per C5 step.  Here five launches cover every layer of a pass:
//   1. vraw = W^T u           one thread per column over a 64-row slab per workgroup (the partial
//                             sums of the slabs in w, the output's own storage), then the slabs
//                             added in order per column
//   2. s = W vraw / max(|vraw|, eps)   one wave per row (|vraw| summed in a fixed order per block)
//   3. per layer: u = s / max(|s|, eps), sigma = u . s, v = vraw / max(|vraw|, eps)  (buffers + copies)
//   4. w = W / sigma
// (eval mode, no power iteration: vraw = v, the norm taken as 1, u kept: sigma = u . W v).
// Fixed summation orders: deterministic.  Layer tables ride in the kernel arguments.

#include <algorithm>

#include "vo_common.h"

namespace vo {

constexpr int SN_MAX = 16;

struct SnLayer {
  const float* W;  // (rows, L) = weight_orig flattened
  float* u;        // (rows) buffer, updated in place (power iteration)
  float* v;        // (L) buffer, updated in place
  float* u_out;    // copies of the u / v sigma was computed with (saved for the backward)
  float* v_out;
  float* vraw;     // (L) scratch
  float* s;        // (rows) scratch
  float* sigma;    // (1)
  float* w;        // (rows, L) output
  int rows, L;
};
struct SnArgs {
  SnLayer l[SN_MAX];
  int blk0[SN_MAX + 1];  // first workgroup of each layer in the launch
  int n;
  int power;
  float eps;
};

__device__ __forceinline__ int sn_layer(const SnArgs& a, int b) {
  return table_find(a.blk0, a.n, b);
}

// 1a. slab sums: workgroup (column block cb, slab sp) sums rows [64 sp, 64 sp + 64) of 64 columns,
// wave w rows 64 sp + w, + 4, ... -> w[sp][c] (scratch: the slabs of a layer, rows / 64 x L floats,
// fit in its rows x L output, written only by step 4).  The first version ran one workgroup per 64
// columns over every row: 80 workgroups for the MSD's 1024 x 5120 layer, 111 us per pass.
constexpr int SN_SLAB = 64;
__global__ void __launch_bounds__(256) sn_wtu_kernel(SnArgs a) {
  __shared__ float part[4][64];
  const int li = sn_layer(a, blockIdx.x);
  const SnLayer L = a.l[li];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ncb = (L.L + 63) / 64, b = blockIdx.x - a.blk0[li];
  const int sp = b / ncb, c = (b - sp * ncb) * 64 + lane;
  const int r1 = min(L.rows, (sp + 1) * SN_SLAB);
  float acc = 0.f;
  if (c < L.L)
#pragma unroll 4
    for (int r = sp * SN_SLAB + wv; r < r1; r += 4) acc += L.W[(int64_t)r * L.L + c] * L.u[r];
  part[wv][lane] = acc;
  __syncthreads();
  if (wv == 0 && c < L.L) L.w[(int64_t)sp * L.L + c] = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
}

// 1b. vraw[c] = the slab sums of column c added in slab order
__global__ void __launch_bounds__(256) sn_vsum_kernel(SnArgs a) {
  const int li = sn_layer(a, blockIdx.x);
  const SnLayer L = a.l[li];
  const int c = (blockIdx.x - a.blk0[li]) * 256 + threadIdx.x;
  if (c >= L.L) return;
  const int ns = (L.rows + SN_SLAB - 1) / SN_SLAB;
  float v = 0.f;
  for (int sp = 0; sp < ns; ++sp) v += L.w[(int64_t)sp * L.L + c];
  L.vraw[c] = v;
}

__device__ __forceinline__ float sn_block_sumsq(const float* x, int n, float* red) {
  float ss = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) ss += x[i] * x[i];
  ss = wave_sum(ss);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  return ((red[0] + red[1]) + red[2]) + red[3];
}

// 2. s[r] = W[r] . vraw (divided by nv = max(|vraw|, eps) in step 3, which computes nv anyway: the
// first version had every workgroup of this kernel re-reduce |vraw|), one wave per row, 4 rows per
// workgroup
__global__ void __launch_bounds__(256) sn_wv_kernel(SnArgs a) {
  const int li = sn_layer(a, blockIdx.x);
  const SnLayer L = a.l[li];
  const float* vr = a.power ? L.vraw : L.v;
  const int lane = threadIdx.x & 63;
  const int r = (blockIdx.x - a.blk0[li]) * 4 + (threadIdx.x >> 6);
  if (r >= L.rows) return;
  const float* row = L.W + (int64_t)r * L.L;
  float acc = 0.f;
  for (int c = lane; c < L.L; c += 64) acc += row[c] * vr[c];
  acc = wave_sum(acc);
  if (lane == 0) L.s[r] = acc;
}

// 3. one workgroup per layer: u, sigma, v
__global__ void __launch_bounds__(256) sn_finish_kernel(SnArgs a) {
  __shared__ float red[4];
  const SnLayer L = a.l[blockIdx.x];
  float dot;
  if (a.power) {
    const float nv = fmaxf(sqrtf(sn_block_sumsq(L.vraw, L.L, red)), a.eps);
    for (int i = threadIdx.x; i < L.rows; i += 256) L.s[i] = L.s[i] / nv;  // s = W v, v = vraw / nv
    __syncthreads();
    const float nu = fmaxf(sqrtf(sn_block_sumsq(L.s, L.rows, red)), a.eps);
    float d = 0.f;
    for (int i = threadIdx.x; i < L.rows; i += 256) {
      const float u = L.s[i] / nu;
      L.u[i] = u;
      L.u_out[i] = u;
      d += u * L.s[i];
    }
    for (int i = threadIdx.x; i < L.L; i += 256) {
      const float v = L.vraw[i] / nv;
      L.v[i] = v;
      L.v_out[i] = v;
    }
    d = wave_sum(d);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = d;
    __syncthreads();
    dot = ((red[0] + red[1]) + red[2]) + red[3];
  } else {
    float d = 0.f;
    for (int i = threadIdx.x; i < L.rows; i += 256) {
      d += L.u[i] * L.s[i];
      L.u_out[i] = L.u[i];
    }
    for (int i = threadIdx.x; i < L.L; i += 256) L.v_out[i] = L.v[i];
    d = wave_sum(d);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = d;
    __syncthreads();
    dot = ((red[0] + red[1]) + red[2]) + red[3];
  }
  if (threadIdx.x == 0) L.sigma[0] = dot;
}

// 4. w = W / sigma
__global__ void __launch_bounds__(256) sn_scale_kernel(SnArgs a) {
  const int li = sn_layer(a, blockIdx.x);
  const SnLayer L = a.l[li];
  const float sg = L.sigma[0];
  const int64_t n = (int64_t)L.rows * L.L;
  const int64_t i0 = (int64_t)(blockIdx.x - a.blk0[li]) * 1024 + threadIdx.x;
  for (int k = 0; k < 4; ++k) {
    const int64_t i = i0 + k * 256;
    if (i < n) L.w[i] = L.W[i] / sg;
  }
}

// ---- backward (torch.nn.utils.spectral_norm's autograd with u, v held constant):
//   gW = g / sigma - (d / sigma^2) u v^T,  d = sum(g * W)
// for every layer of a pass in three launches (the per-layer PyTorch chain was a multiply, a sum, a
// divide, an outer product, a multiply and a subtract per layer): block partials of d (4096 elements
// per workgroup), their sum per layer in block order, then the elementwise update.
constexpr int SNB_ELEMS = 4096;
struct SnBwdArgs {
  VoSnBwdLayer l[SN_MAX];
  int blk0[SN_MAX + 1];
  int n;
  float* part;  // [blocks] partials, then [n] d values
};

__device__ __forceinline__ float snb_block_sum(float x, float* red) {
  x = wave_sum(x);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  return ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ void __launch_bounds__(256) sn_bwd_dot_kernel(SnBwdArgs a) {
  __shared__ float red[4];
  const int li = table_find(a.blk0, a.n, blockIdx.x);
  const VoSnBwdLayer& L = a.l[li];
  const int64_t n = (int64_t)L.rows * L.L;
  const int64_t i0 = (int64_t)(blockIdx.x - a.blk0[li]) * SNB_ELEMS + threadIdx.x;
  float acc = 0.f;
#pragma unroll 4
  for (int k = 0; k < SNB_ELEMS / 256; ++k) {
    const int64_t i = i0 + k * 256;
    if (i < n) acc += L.g[i] * L.W[i];
  }
  const float s = snb_block_sum(acc, red);
  if (threadIdx.x == 0) a.part[blockIdx.x] = s;
}

__global__ void __launch_bounds__(256) sn_bwd_sum_kernel(SnBwdArgs a) {
  __shared__ float red[4];
  const int li = blockIdx.x;
  float acc = 0.f;
  for (int b = a.blk0[li] + threadIdx.x; b < a.blk0[li + 1]; b += 256) acc += a.part[b];
  const float s = snb_block_sum(acc, red);
  if (threadIdx.x == 0) a.part[a.blk0[a.n] + li] = s;
}

__global__ void __launch_bounds__(256) sn_bwd_apply_kernel(SnBwdArgs a) {
  const int li = table_find(a.blk0, a.n, blockIdx.x);
  const VoSnBwdLayer& L = a.l[li];
  const int64_t n = (int64_t)L.rows * L.L;
  const int64_t i0 = (int64_t)(blockIdx.x - a.blk0[li]) * SNB_ELEMS + threadIdx.x;
  const float sg = L.sigma[0];
  const float c = a.part[a.blk0[a.n] + li] / (sg * sg);
  for (int k = 0; k < SNB_ELEMS / 256; ++k) {
    const int64_t i = i0 + k * 256;
    if (i < n) {
      const int64_t r = i / L.L;
      L.gW[i] = L.g[i] / sg - c * (L.u[r] * L.v[i - r * L.L]);
    }
  }
}

}  // namespace vo

using namespace vo;

extern "C" int64_t vo_spectral_norm_bwd_workspace_size(int n, const VoSnBwdLayer* layers) {
  if (n <= 0 || !layers) return 0;
  int64_t f = 0;
  for (int i0 = 0; i0 < n; i0 += SN_MAX) {
    int64_t blocks = 0;
    const int m = std::min(SN_MAX, n - i0);
    for (int i = 0; i < m; ++i) blocks += ((int64_t)layers[i0 + i].rows * layers[i0 + i].L + SNB_ELEMS - 1) / SNB_ELEMS;
    f = std::max(f, blocks + m);
  }
  return f * (int64_t)sizeof(float);
}

extern "C" int vo_spectral_norm_bwd(int n, const VoSnBwdLayer* layers, float* workspace, void* stream) {
  VO_CHECK_ARG(n >= 0 && (n == 0 || (layers && workspace)), "spectral_norm_bwd: null table / workspace");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int i0 = 0; i0 < n; i0 += SN_MAX) {
    SnBwdArgs a;
    a.n = std::min(SN_MAX, n - i0);
    a.part = workspace;
    int total = 0;
    for (int i = 0; i < a.n; ++i) {
      const VoSnBwdLayer& s = layers[i0 + i];
      VO_CHECK_ARG(s.g && s.W && s.u && s.v && s.sigma && s.gW, "spectral_norm_bwd: layer %d: null pointer", i0 + i);
      VO_CHECK_ARG(s.rows > 0 && s.L > 0 && (int64_t)s.rows * s.L < (1LL << 31), "spectral_norm_bwd: layer %d: bad size",
                   i0 + i);
      a.l[i] = s;
      a.blk0[i] = total;
      total += (int)(((int64_t)s.rows * s.L + SNB_ELEMS - 1) / SNB_ELEMS);
    }
    a.blk0[a.n] = total;
    hipLaunchKernelGGL(sn_bwd_dot_kernel, dim3((unsigned)total), dim3(256), 0, st, a);
    hipLaunchKernelGGL(sn_bwd_sum_kernel, dim3((unsigned)a.n), dim3(256), 0, st, a);
    hipLaunchKernelGGL(sn_bwd_apply_kernel, dim3((unsigned)total), dim3(256), 0, st, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      vo_set_error("spectral_norm_bwd: launch failed: %s", hipGetErrorString(e));
      return (int)e;
    }
  }
  return VO_OK;
}

extern "C" int vo_spectral_norm(int n, const VoSnLayer* layers, int power, float eps, void* stream) {
  VO_CHECK_ARG(n >= 0 && (n == 0 || layers), "spectral_norm: null table");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int i0 = 0; i0 < n; i0 += SN_MAX) {
    SnArgs a;
    a.n = std::min(SN_MAX, n - i0);
    a.power = power ? 1 : 0;
    a.eps = eps;
    for (int i = 0; i < a.n; ++i) {
      const VoSnLayer& s = layers[i0 + i];
      VO_CHECK_ARG(s.W && s.u && s.v && s.u_out && s.v_out && s.vraw && s.s && s.sigma && s.w,
                   "spectral_norm: layer %d: null pointer", i0 + i);
      VO_CHECK_ARG(s.rows > 0 && s.L > 0 && (int64_t)s.rows * s.L < (1LL << 31),
                   "spectral_norm: layer %d: bad size", i0 + i);
      VO_CHECK_ARG(s.w != s.W, "spectral_norm: layer %d: w must not alias W (it holds the W^T u slab sums)", i0 + i);
      a.l[i] = SnLayer{s.W, s.u, s.v, s.u_out, s.v_out, s.vraw, s.s, s.sigma, s.w, s.rows, s.L};
    }
    auto launch = [&](void (*k)(SnArgs), int (*blocks)(const SnLayer&)) -> int {
      int total = 0;
      for (int i = 0; i < a.n; ++i) {
        a.blk0[i] = total;
        total += blocks(a.l[i]);
      }
      a.blk0[a.n] = total;
      hipLaunchKernelGGL(k, dim3((unsigned)total), dim3(256), 0, st, a);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) {
        vo_set_error("spectral_norm: launch failed: %s", hipGetErrorString(e));
        return (int)e;
      }
      return VO_OK;
    };
    int rc;
    if (a.power) {
      if ((rc = launch(sn_wtu_kernel, [](const SnLayer& l) {
             return (l.L + 63) / 64 * ((l.rows + SN_SLAB - 1) / SN_SLAB);
           })) != VO_OK)
        return rc;
      if ((rc = launch(sn_vsum_kernel, [](const SnLayer& l) { return (l.L + 255) / 256; })) != VO_OK) return rc;
    }
    if ((rc = launch(sn_wv_kernel, [](const SnLayer& l) { return (l.rows + 3) / 4; })) != VO_OK) return rc;
    hipLaunchKernelGGL(sn_finish_kernel, dim3((unsigned)a.n), dim3(256), 0, st, a);
    if ((rc = launch(sn_scale_kernel, [](const SnLayer& l) {
           return (int)(((int64_t)l.rows * l.L + 1023) / 1024);
         })) != VO_OK)
      return rc;
  }
  return VO_OK;
}
