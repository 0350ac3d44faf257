"""Offline acoustic feature extraction on the GPU: the producer of the
``mel/*.npy`` (T, 80), ``energy/*.npy`` and ``kurtosis/*.npy`` character-level features and
their corpus z-normalisation that the training Dataset reads.

Reference: scripts/preprocessor/preprocessor.py -- ``Preprocessor._get_spec`` (:323-337,
torchaudio Spectrogram(power=1, center=True) + MelScale(slaney) + log clamp 1e-5, energy = L2
norm of |X| over frequency), the frame -> character energy averaging of ``_process``
(:395-403), ``_get_kurtosis`` (:339-357) and the StandardScaler + ``_normalize`` pass of
``build_from_path`` (:113-129, :624-645).  Corpus walking, TextGrid alignment, resampling
(librosa.load) and glyph rendering stay host-side and are out of scope.

GPU work per batch of utterances: one ``vo_stft_mel_ex`` launch (framing, FFT, |X|, mel, log,
frame energy and the power statistics the kurtosis needs) and one ``vo_char_features``
launch (per-character reductions over the duration spans).
"""

import numpy as np
import torch

from .. import ops
from ..audio import melscale_fbanks


class FeatureExtractor:
    def __init__(self, config, device="cuda"):
        a = config["audio"]
        st, mel = a["stft"], a["mel"]
        self.n_fft, self.hop, self.win = st["filter_length"], st["hop_length"], st["win_length"]
        if self.win != self.n_fft:
            raise NotImplementedError("win_length != filter_length")
        self.n_mels = mel["n_mel_channels"]
        self.device = torch.device(device)
        self.fb = melscale_fbanks(self.n_fft // 2 + 1, mel["mel_fmin"], mel["mel_fmax"], self.n_mels,
                                  a["sampling_rate"]).float().contiguous().to(self.device)
        self.window = torch.hann_window(self.n_fft, periodic=True).to(self.device)

    def get_spec(self, audio):
        """Preprocessor._get_spec: 1-D waveform -> (log-mel (80, F), energy (F,)) numpy."""
        w = torch.as_tensor(np.asarray(audio, np.float32), device=self.device)[None].contiguous()
        mel, energy, _ = ops.spec_features(w, self.window, self.fb, self.n_fft, self.hop)
        return mel[0].cpu().numpy(), energy[0].cpu().numpy()

    def process(self, wavs, durations):
        """Batch of utterances (1-D float arrays, trimmed as in _process) and their per-character
        durations (frames) -> list of dicts {mel (sum(d), 80), energy (n_chars,), kurtosis (n_chars,)}
        exactly as _process saves them (mel transposed, truncated to sum(duration))."""
        B = len(wavs)
        # utterances of different lengths are framed separately (reflect padding is per signal);
        # equal-length groups share one launch
        by_len = {}
        for i, w in enumerate(wavs):
            by_len.setdefault(len(w), []).append(i)
        res = [None] * B
        for n, idx in by_len.items():
            w = torch.as_tensor(np.stack([np.asarray(wavs[i], np.float32) for i in idx]), device=self.device)
            mel, energy, fstats = ops.spec_features(w.contiguous(), self.window, self.fb, self.n_fft, self.hop)
            e_c, k_c = ops.char_features(energy, fstats, [durations[i] for i in idx], self.n_fft // 2 + 1)
            for j, i in enumerate(idx):
                T = int(np.sum(durations[i]))
                res[i] = dict(mel=mel[j, :, :T].t().contiguous().cpu().numpy(), energy=e_c[j].cpu().numpy(),
                              kurtosis=k_c[j].cpu().numpy().astype(np.float64))
        return res


def normalize_features(arrays):
    """StandardScaler.partial_fit over every value + _normalize: returns (normalised arrays,
    mean, std, min, max) with the population std (ddof 0) StandardScaler uses."""
    flat = np.concatenate([np.asarray(a, np.float64).reshape(-1) for a in arrays])
    mean = float(flat.mean())
    std = float(np.sqrt(np.mean((flat - mean) ** 2)))
    if std == 0.0:
        std = 1.0  # StandardScaler's handling of a zero variance
    normed = [(np.asarray(a) - mean) / std for a in arrays]
    mn = min(float(np.min(v)) for v in normed)
    mx = max(float(np.max(v)) for v in normed)
    return normed, mean, std, mn, mx
