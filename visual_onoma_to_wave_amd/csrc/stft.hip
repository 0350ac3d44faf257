// placeholder: replaced by the LDS radix FFT mel front-end (row a21)
#include "vo_common.h"
extern "C" int vo_stft_mel(const float*, int, int, const float*, const float*, int, int, int, float, float*, float*,
                           void*) {
  vo_set_error("stft_mel: not built yet");
  return VO_ERR_INVALID;
}
