"""Mel / STFT front-end on the HIP ``vo_stft_mel`` kernel.

get_spec / MelSpectrogram  <- scripts/preprocessor/preprocessor.py:22-36,323-337 (torchaudio
                              Spectrogram(power=1, center=True) + MelScale(norm="slaney",
                              mel_scale="htk") + log(clamp_min(., 1e-5)); energy = ||X||_2)
TacotronSTFT               <- scripts/audio/stft.py:130-178 (librosa slaney-scale mel basis,
                              dynamic_range_compression = log(clamp(x, 1e-5)))
The filterbanks are built once on the host (float64 -> float32, the published torchaudio /
librosa formulas); the per-frame work -- framing, window, FFT, |X|, mel projection, log,
energy -- is one kernel launch.
"""

import numpy as np
import torch

from .. import ops


def _hz_to_mel_htk(f):
    return 2595.0 * np.log10(1.0 + np.asarray(f, np.float64) / 700.0)


def melscale_fbanks(n_freqs, f_min, f_max, n_mels, sample_rate):
    """torchaudio.functional.melscale_fbanks(norm="slaney", mel_scale="htk") -> (n_freqs, n_mels)."""
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_pts = torch.linspace(float(_hz_to_mel_htk(f_min)), float(_hz_to_mel_htk(f_max)), n_mels + 2)
    f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_freqs[:, None]
    fb = torch.clamp(torch.minimum((-slopes[:, :-2]) / f_diff[:-1], slopes[:, 2:] / f_diff[1:]), min=0.0)
    return fb * (2.0 / (f_pts[2:n_mels + 2] - f_pts[:n_mels]))[None, :]


def _hz_to_mel_slaney(f):
    f = np.asarray(f, np.float64)
    f_sp, min_log_hz, logstep = 200.0 / 3, 1000.0, np.log(6.4) / 27.0
    mel = f / f_sp
    return np.where(f >= min_log_hz, min_log_hz / f_sp + np.log(np.maximum(f, 1e-30) / min_log_hz) / logstep, mel)


def _mel_to_hz_slaney(m):
    m = np.asarray(m, np.float64)
    f_sp, min_log_hz, logstep = 200.0 / 3, 1000.0, np.log(6.4) / 27.0
    min_log_mel = min_log_hz / f_sp
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def librosa_mel(sr, n_fft, n_mels=128, fmin=0.0, fmax=None):
    """librosa.filters.mel(htk=False, norm="slaney") -> (n_mels, 1 + n_fft // 2) float32."""
    fmax = sr / 2.0 if fmax is None else fmax
    fftfreqs = np.linspace(0, sr / 2.0, 1 + n_fft // 2)
    mel_f = _mel_to_hz_slaney(np.linspace(_hz_to_mel_slaney(fmin), _hz_to_mel_slaney(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    w = np.zeros((n_mels, 1 + n_fft // 2), np.float64)
    for i in range(n_mels):
        w[i] = np.maximum(0, np.minimum(-ramps[i] / fdiff[i], ramps[i + 2] / fdiff[i + 1]))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w.astype(np.float32)


class MelSpectrogram:
    """Spectrogram(n_fft, win=n_fft, hop, power=1, center=True) -> MelScale -> log, on HIP."""

    def __init__(self, n_fft=1024, hop_length=256, n_mels=80, sample_rate=22050, f_min=0.0, f_max=8000.0,
                 fb=None, log_floor=1e-5):
        self.n_fft, self.hop, self.n_mels, self.log_floor = n_fft, hop_length, n_mels, log_floor
        self.fb = (melscale_fbanks(n_fft // 2 + 1, f_min, f_max, n_mels, sample_rate) if fb is None
                   else torch.as_tensor(fb)).float().contiguous()
        self.window = torch.hann_window(n_fft, periodic=True)
        self._dev = {}

    def _on(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = (self.window.to(device), self.fb.to(device).contiguous())
        return self._dev[key]

    def __call__(self, wav):
        """wav (N,) or (B, N) fp32 on the GPU -> (log-mel (B, n_mels, F), energy (B, F))."""
        squeeze = wav.dim() == 1
        w = wav.reshape(1, -1) if squeeze else wav
        window, fb = self._on(w.device)
        logmel, energy = ops.stft_mel(w.float().contiguous(), window, fb, self.n_fft, self.hop, self.n_mels,
                                      self.log_floor)
        return (logmel[0], energy[0]) if squeeze else (logmel, energy)


def get_spec(wav, preprocess_config=None):
    """Preprocessor._get_spec: (log-mel (80, F), energy (F,)) of a 1-D waveform."""
    a = (preprocess_config or {}).get("audio", {})
    st, mel = a.get("stft", {}), a.get("mel", {})
    m = MelSpectrogram(st.get("filter_length", 1024), st.get("hop_length", 256), mel.get("n_mel_channels", 80),
                       a.get("sampling_rate", 22050), mel.get("mel_fmin", 0), mel.get("mel_fmax", 8000))
    return m(wav)


class TacotronSTFT(torch.nn.Module):
    """TacotronSTFT with the librosa slaney mel basis; mel_spectrogram(y) -> (mel, energy)."""

    def __init__(self, filter_length, hop_length, win_length, n_mel_channels, sampling_rate, mel_fmin,
                 mel_fmax):
        super().__init__()
        if win_length != filter_length:
            raise NotImplementedError("the HIP front-end uses win_length == filter_length (the ICASSP config)")
        self.n_mel_channels, self.sampling_rate = n_mel_channels, sampling_rate
        basis = torch.from_numpy(librosa_mel(sampling_rate, filter_length, n_mel_channels, mel_fmin, mel_fmax))
        self.register_buffer("mel_basis", basis)
        self._mel = MelSpectrogram(filter_length, hop_length, n_mel_channels, fb=basis.t().contiguous())

    def mel_spectrogram(self, y):
        if float(y.min()) < -1 or float(y.max()) > 1:
            raise AssertionError("waveform must lie in [-1, 1]")
        return self._mel(y)
