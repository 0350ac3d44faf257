// Probe of ds_read_b64_tr_b16 lane semantics: LDS holds v = row * 100 + col (16-bit) for a
// [8][72] tile; lane 4q+p of each 16-lane group points at row q (+ 4 * group), col 4p.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short v4s __attribute__((ext_vector_type(4)));
__global__ void k(short* out) {
  __shared__ __attribute__((aligned(16))) short lds[16 * 72];
  for (int i = threadIdx.x; i < 16 * 72; i += 64) lds[i] = (short)((i / 72) * 100 + (i % 72));
  __syncthreads();
  const int lane = threadIdx.x, g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const short* base = lds + (4 * g + q) * 72 + 4 * p;
  typedef __attribute__((address_space(3))) v4s lv;
  v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lv*)base);
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = v[e];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  short h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) printf("lane %2d: %4d %4d %4d %4d\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
  return 0;
}
