// Mel / STFT front-end: framing + Hann window + 1024-point real FFT in LDS + |X| + mel
// projection + log, and the frame energy, one workgroup per frame.
//
// Semantics (scripts/preprocessor/preprocessor.py:22-36,323-337 -- torchaudio
// Spectrogram(n_fft, win=n_fft, hop, power=1, center=True) -> MelScale(slaney norm) ->
// log(clamp_min(., 1e-5)); energy = L2 norm of |X| over frequency), and with a slaney-scale
// filterbank the TacotronSTFT.mel_spectrogram variant (scripts/audio/stft.py:159-178):
//   * input clipped to [-1, 1], reflect-padded by n_fft/2 at both ends (center=True);
//   * frame f covers padded samples [f*hop, f*hop + n_fft), F = 1 + N / hop frames;
//   * the real FFT of n points runs as an n/2-point complex radix-2 Stockham FFT of the
//     even/odd-packed frame (z[m] = x[2m] + i x[2m+1]) plus the split step
//     X[k] = (Z[k] + Z*[n/2-k])/2 - i e^{-2 pi i k / n} (Z[k] - Z*[n/2-k])/2;
//   * twiddles from sincospif (accurate fp32), accumulation in fp32.

#include "vo_common.h"

namespace vo {

constexpr int STFT_MAX_N = 2048;

__device__ __forceinline__ int reflect(int i, int n) {
  // torch reflect padding (edge sample not repeated); |i| < n guaranteed by n_fft/2 < N
  if (i < 0) i = -i;
  if (i >= n) i = 2 * (n - 1) - i;
  return i;
}

__global__ void __launch_bounds__(256) stft_mel_kernel(const float* __restrict__ wav, int N, int F,
                                                       const float* __restrict__ window,
                                                       const float* __restrict__ fb, int n_fft, int hop,
                                                       int n_mels, float log_floor, float* __restrict__ mel,
                                                       float* __restrict__ energy, int pad, float mag_eps,
                                                       int clip, float* __restrict__ fstats) {
  __shared__ float2 buf[2][STFT_MAX_N / 2];
  __shared__ float mag[STFT_MAX_N / 2 + 1];
  __shared__ float red[4], red_p[4], red_l[4];
  const int f = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x;
  const int half = n_fft / 2;
  const float* x = wav + (int64_t)b * N;
  const int start = f * hop - pad;  // unpadded index of frame sample 0

  // load + clip + window, packed even/odd into complex
  for (int m = tid; m < half; m += 256) {
    const int i0 = reflect(start + 2 * m, N), i1 = reflect(start + 2 * m + 1, N);
    const float x0 = clip ? fminf(fmaxf(x[i0], -1.f), 1.f) : x[i0];
    const float x1 = clip ? fminf(fmaxf(x[i1], -1.f), 1.f) : x[i1];
    const float a = x0 * window[2 * m];
    const float c = x1 * window[2 * m + 1];
    buf[0][m] = make_float2(a, c);
  }
  __syncthreads();

  // radix-2 Stockham autosort FFT of length L = half (power of two)
  int src = 0;
  const int L = half;
  for (int ns = 1; ns < L; ns <<= 1) {
    for (int j = tid; j < L / 2; j += 256) {
      const int k = j & (ns - 1);                  // position within the current sub-transform
      const float2 u = buf[src][j];
      const float2 v = buf[src][j + L / 2];
      float s, c;
      sincospif(-(float)k / (float)ns, &s, &c);   // e^{-i pi k / ns}
      const float2 tv = make_float2(v.x * c - v.y * s, v.x * s + v.y * c);
      const int out = (j - k) * 2 + k;            // (j / ns) * 2 * ns + k
      buf[src ^ 1][out] = make_float2(u.x + tv.x, u.y + tv.y);
      buf[src ^ 1][out + ns] = make_float2(u.x - tv.x, u.y - tv.y);
    }
    __syncthreads();
    src ^= 1;
  }

  // split into the n_fft-point real spectrum, magnitudes
  float e2 = 0.f, sp = 0.f, sl = 0.f;
  for (int k = tid; k <= half; k += 256) {
    const float2 zk = buf[src][k & (L - 1)];
    const float2 zn = buf[src][(L - k) & (L - 1)];
    // E = (Z[k] + conj Z[L-k]) / 2 ; O = (Z[k] - conj Z[L-k]) / (2i)
    const float er = 0.5f * (zk.x + zn.x), ei = 0.5f * (zk.y - zn.y);
    const float orr = 0.5f * (zk.y + zn.y), oi = -0.5f * (zk.x - zn.x);
    float s, c;
    sincospif(-2.f * (float)k / (float)n_fft, &s, &c);
    const float xr = er + (orr * c - oi * s);
    const float xi = ei + (orr * s + oi * c);
    const float mg = sqrtf(xr * xr + xi * xi + mag_eps);
    mag[k] = mg;
    e2 += mg * mg;
    if (fstats) {  // power-spectrum statistics of the frame (kurtosis feature)
      const float p = mg * mg;
      sp += p;
      sl += logf(p + 1e-8f);
    }
  }
  e2 = wave_sum(e2);
  if ((tid & 63) == 0) red[tid >> 6] = e2;
  if (fstats) {
    sp = wave_sum(sp);
    sl = wave_sum(sl);
    if ((tid & 63) == 0) {
      red_p[tid >> 6] = sp;
      red_l[tid >> 6] = sl;
    }
  }
  __syncthreads();
  if (tid == 0 && energy) energy[(int64_t)b * F + f] = sqrtf(red[0] + red[1] + red[2] + red[3]);
  if (tid == 0 && fstats) {
    fstats[((int64_t)b * F + f) * 2] = red_p[0] + red_p[1] + red_p[2] + red_p[3];
    fstats[((int64_t)b * F + f) * 2 + 1] = red_l[0] + red_l[1] + red_l[2] + red_l[3];
  }

  // mel projection: wave w handles bins w, w+4, ...; lanes stride over frequency
  const int lane = tid & 63, wave = tid >> 6;
  const int nf = half + 1;
  for (int m = wave; m < n_mels; m += 4) {
    float acc = 0.f;
    for (int k = lane; k < nf; k += 64) acc += fb[(int64_t)k * n_mels + m] * mag[k];
    acc = wave_sum(acc);
    if (lane == 0) mel[((int64_t)b * n_mels + m) * F + f] = logf(fmaxf(acc, log_floor));
  }
}

}  // namespace vo

using namespace vo;

extern "C" int vo_stft_mel_ex(const float* wav, int B, int N, const float* window, const float* fb, int n_fft,
                              int hop, int n_mels, int pad, float mag_eps, int clip, float log_floor, float* mel,
                              float* energy, float* fstats, void* stream) {
  VO_CHECK_ARG(wav && window && fb && mel, "stft_mel: null pointer");
  VO_CHECK_ARG(n_fft >= 8 && n_fft <= STFT_MAX_N && (n_fft & (n_fft - 1)) == 0, "stft_mel: n_fft=%d must be a power of "
               "two in [8, %d]", n_fft, STFT_MAX_N);
  VO_CHECK_ARG(hop > 0 && n_mels > 0 && B > 0 && pad >= 0, "stft_mel: bad sizes");
  VO_CHECK_ARG(N > pad, "stft_mel: reflect padding needs N (%d) > pad (%d)", N, pad);
  VO_CHECK_ARG(N + 2 * pad >= n_fft, "stft_mel: signal shorter than one frame");
  const int F = 1 + (N + 2 * pad - n_fft) / hop;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(stft_mel_kernel, dim3((unsigned)F, (unsigned)B), dim3(256), 0, st, wav, N, F, window, fb, n_fft,
                     hop, n_mels, log_floor, mel, energy, pad, mag_eps, clip, fstats);
  VO_RETURN_LAUNCH();
}

// torchaudio center=True framing (pad n_fft / 2, F = 1 + N / hop), clipped input, |X|
extern "C" int vo_stft_mel(const float* wav, int B, int N, const float* window, const float* fb, int n_fft, int hop,
                           int n_mels, float log_floor, float* mel, float* energy, void* stream) {
  return vo_stft_mel_ex(wav, B, N, window, fb, n_fft, hop, n_mels, n_fft / 2, 0.f, 1, log_floor, mel, energy, nullptr,
                        stream);
}
