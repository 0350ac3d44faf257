// Training input pipeline on device: the per-character centring of the
// rendered onomatopoeia strip into fixed-width cells, the batch's white right-padding and
// margins, and torchvision ToTensor (uint8 -> float / 255), in one gather launch.
//
// Reference (host, per sample with cv2 + numpy, then per batch):
//   Dataset.character_padding_forinput (scripts/dataset.py:71-92): character j of width len_j
//     (columns [start_j, start_j + len_j) of the strip) is padded with white to `cell` columns,
//     pleft = (cell - len_j) / 2 + (cell - len_j) % 2, pright = (cell - len_j) / 2;
//   pad_2D_gray_image (scripts/utils/tools.py:616-635): right-pad with 255 to the batch's widest
//     strip, then (stride // 2) * cell white columns on both sides;
//   to_device's transforms.ToTensor (tools.py:18-20,50-51): (B, 1, H, W) float = uint8 / 255.
// Here: out[b, 0, y, x] = v / 255 with v the source pixel or 255 (white), one thread per pixel.
// chars == NULL: the strips are already centred (B strips of img_w[b] columns): copy + pad.

#include "vo_common.h"

namespace vo {

__global__ void __launch_bounds__(256) glyph_batch_kernel(const uint8_t* __restrict__ px, const int64_t* __restrict__ img_off,
                                                          const int32_t* __restrict__ img_w,
                                                          const int32_t* __restrict__ char_off,
                                                          const int32_t* __restrict__ char_start,
                                                          const int32_t* __restrict__ char_len, int H, int cell,
                                                          int margin, int W_out, float* __restrict__ out) {
  const int b = blockIdx.z, y = blockIdx.y;
  const int x = blockIdx.x * 256 + threadIdx.x;
  if (x >= W_out) return;
  const uint8_t* row = px + img_off[b] + (int64_t)y * img_w[b];
  int v = 255;
  const int xm = x - margin;
  if (xm >= 0) {
    if (char_off) {
      const int j = xm / cell, c = xm - j * cell;
      if (j < char_off[b + 1] - char_off[b]) {
        const int len = char_len[char_off[b] + j];
        const int pleft = (cell - len) / 2 + (cell - len) % 2;
        const int sc = c - pleft;
        if (sc >= 0 && sc < len) v = row[char_start[char_off[b] + j] + sc];
      }
    } else if (xm < img_w[b]) {
      v = row[xm];
    }
  }
  out[(((int64_t)b * H) + y) * W_out + x] = __fdiv_rn((float)v, 255.f);
}

}  // namespace vo

using namespace vo;

extern "C" int vo_glyph_batch(const uint8_t* px, const int64_t* img_off, const int32_t* img_w, const int32_t* char_off,
                              const int32_t* char_start, const int32_t* char_len, int B, int H, int cell, int margin,
                              int W_out, float* out, void* stream) {
  VO_CHECK_ARG(px && img_off && img_w && out, "glyph_batch: null pointer");
  VO_CHECK_ARG(!char_off || (char_start && char_len && cell > 0), "glyph_batch: incomplete character table");
  VO_CHECK_ARG(B > 0 && H > 0 && W_out > 0 && margin >= 0 && H <= 65535 && B <= 65535, "glyph_batch: bad sizes");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((unsigned)((W_out + 255) / 256), (unsigned)H, (unsigned)B);
  hipLaunchKernelGGL(glyph_batch_kernel, grid, dim3(256), 0, st, px, img_off, img_w, char_off, char_start, char_len, H,
                     cell, margin, W_out, out);
  VO_RETURN_LAUNCH();
}
