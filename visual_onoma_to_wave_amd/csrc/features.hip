// Character-level acoustic features of the offline feature extraction:
// frame energies / power-spectrum statistics (from vo_stft_mel_ex) -> per-character mean energy
// and spectral kurtosis over each character's duration span.
// Reference: Preprocessor._process (scripts/preprocessor/preprocessor.py:395-403, energy
// frame -> character) and Preprocessor._get_kurtosis (:339-357).  One thread per character
// (spans are a few frames to a few hundred; the frame statistics are already reduced over
// frequency by the STFT kernel).

#include "vo_common.h"

namespace vo {

__global__ void __launch_bounds__(256) char_features_kernel(const float* __restrict__ energy,
                                                            const float* __restrict__ fstats, int F,
                                                            const int32_t* __restrict__ dur,
                                                            const int32_t* __restrict__ char_off, int B, int n_bins,
                                                            float* __restrict__ e_char, float* __restrict__ k_char) {
  const int b = blockIdx.y;
  const int j0 = char_off[b], n = char_off[b + 1] - j0;
  for (int j = blockIdx.x * 256 + threadIdx.x; j < n; j += gridDim.x * 256) {
    int pos = 0;
    for (int i = 0; i < j; ++i) pos += dur[j0 + i];
    const int d = dur[j0 + j];
    float se = 0.f, sp = 0.f, sl = 0.f;
    for (int t = pos; t < pos + d && t < F; ++t) {
      se += energy[(int64_t)b * F + t];
      if (fstats) {
        sp += fstats[((int64_t)b * F + t) * 2];
        sl += fstats[((int64_t)b * F + t) * 2 + 1];
      }
    }
    if (e_char) e_char[j0 + j] = d > 0 ? se / (float)d : 0.f;
    if (k_char && fstats) {
      const float cnt = (float)n_bins * (float)d;
      const float g = logf(sp / cnt + 1e-8f) - sl / cnt;
      const float eta = (3.f - g + sqrtf((g - 3.f) * (g - 3.f) + 24.f * g)) / (12.f * g);
      k_char[j0 + j] = (eta + 2.f) * (eta + 3.f) / (eta * (eta + 1.f) + 1e-8f);
    }
  }
}

}  // namespace vo

using namespace vo;

extern "C" int vo_char_features(const float* energy, const float* fstats, int F, const int32_t* dur,
                                const int32_t* char_off, int B, int n_bins, float* e_char, float* k_char,
                                void* stream) {
  VO_CHECK_ARG(energy && dur && char_off && B > 0 && F > 0, "char_features: bad arguments");
  VO_CHECK_ARG(!k_char || (fstats && n_bins > 0), "char_features: kurtosis needs the frame statistics");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(char_features_kernel, dim3(1, (unsigned)B), dim3(256), 0, st, energy, fstats, F, dur, char_off, B,
                     n_bins, e_char, k_char);
  VO_RETURN_LAUNCH();
}
