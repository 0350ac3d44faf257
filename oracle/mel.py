"""ORACLE (test infrastructure only) -- mel/STFT front-end restated on the CPU.

PARITY-UNPINNED: the reference computes these features with torchaudio
(``scripts/preprocessor/preprocessor.py:22-36,323-337``) and librosa
(``scripts/audio/stft.py:145-178``); neither is installed here and no file in the
reference holds their outputs.  This module restates the *published* algorithms
of those libraries (versions are unpinned in ``requirements.txt``):

* torchaudio ``Spectrogram(n_fft, win_length, hop_length, power=1, center=True)``
  = ``|torch.stft(x, n_fft, hop, win, hann_window(win, periodic=True),
  center=True, pad_mode="reflect", onesided=True)|``;
* torchaudio ``melscale_fbanks(n_freqs, f_min, f_max, n_mels, sr, norm="slaney",
  mel_scale="htk")``: HTK mel points, triangular filters on
  ``linspace(0, sr // 2, n_freqs)``, slaney area normalisation 2 / (f[i+2] - f[i]);
* ``_get_spec``: log(clamp_min(fb^T |X|, 1e-5)); energy = L2 norm of |X| over
  frequency.
"""

import numpy as np
import torch


def hz_to_mel_htk(f):
    return 2595.0 * np.log10(1.0 + np.asarray(f, dtype=np.float64) / 700.0)


def mel_to_hz_htk(m):
    return 700.0 * (10.0 ** (np.asarray(m, dtype=np.float64) / 2595.0) - 1.0)


def melscale_fbanks(n_freqs=513, f_min=0.0, f_max=8000.0, n_mels=80, sample_rate=22050):
    """(n_freqs, n_mels) float32 HTK-scale, slaney-normalised triangular filterbank."""
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_pts = torch.linspace(float(hz_to_mel_htk(f_min)), float(hz_to_mel_htk(f_max)), n_mels + 2)
    f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_freqs[:, None]
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    fb = torch.clamp(torch.minimum(down, up), min=0.0)
    enorm = 2.0 / (f_pts[2: n_mels + 2] - f_pts[:n_mels])
    return fb * enorm[None, :]


def magnitude(wav, n_fft=1024, hop=256, win=1024):
    """|STFT| (..., n_fft//2+1, frames) as torchaudio Spectrogram(power=1, center=True)."""
    wav = torch.as_tensor(wav, dtype=torch.float32)
    window = torch.hann_window(win, periodic=True)
    X = torch.stft(wav, n_fft, hop_length=hop, win_length=win, window=window, center=True,
                   pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    return X.abs()


def get_spec(wav, n_fft=1024, hop=256, win=1024, n_mels=80, sr=22050, fmin=0.0, fmax=8000.0):
    """Preprocessor._get_spec, preprocessor.py:323-337 -> (log-mel (..., 80, F), energy (..., F))."""
    wav = torch.clamp(torch.as_tensor(wav, dtype=torch.float32), -1, 1)
    mag = magnitude(wav, n_fft, hop, win)
    fb = melscale_fbanks(n_fft // 2 + 1, fmin, fmax, n_mels, sr)
    mel = torch.matmul(mag.transpose(-1, -2), fb).transpose(-1, -2)
    logmel = torch.log(torch.clamp_min(mel, 1.0e-5) * 1.0)
    energy = torch.linalg.vector_norm(mag, dim=-2)
    return logmel, energy


def _hz_to_mel_slaney(f):
    f = np.asarray(f, np.float64)
    f_sp, min_log_hz, logstep = 200.0 / 3, 1000.0, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_hz / f_sp + np.log(np.maximum(f, 1e-30) / min_log_hz) / logstep,
                    f / f_sp)


def _mel_to_hz_slaney(m):
    m = np.asarray(m, np.float64)
    f_sp, min_log_hz, logstep = 200.0 / 3, 1000.0, np.log(6.4) / 27.0
    mm = min_log_hz / f_sp
    return np.where(m >= mm, min_log_hz * np.exp(logstep * (m - mm)), f_sp * m)


def librosa_mel(sr, n_fft, n_mels, fmin, fmax):
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax) (htk=False, norm="slaney"), the basis
    of TacotronSTFT (scripts/audio/stft.py:145-149) -> (n_mels, 1 + n_fft // 2)."""
    fft = np.linspace(0, sr / 2.0, 1 + n_fft // 2)
    mel_f = _mel_to_hz_slaney(np.linspace(_hz_to_mel_slaney(fmin), _hz_to_mel_slaney(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fft)
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    w = np.maximum(0, np.minimum(lower, upper)) * (2.0 / (mel_f[2:] - mel_f[:-2]))[:, None]
    return w.astype(np.float32)


def tacotron_mel(wav, n_fft=1024, hop=256, n_mels=80, sr=22050, fmin=0.0, fmax=8000.0):
    """TacotronSTFT.mel_spectrogram (scripts/audio/stft.py:159-178): |STFT| (reflect pad n_fft/2,
    hann) -> librosa mel basis -> log(clamp(., 1e-5)); energy = ||X||_2 over frequency."""
    mag = magnitude(torch.as_tensor(wav, dtype=torch.float32), n_fft, hop, n_fft)
    basis = torch.from_numpy(librosa_mel(sr, n_fft, n_mels, fmin, fmax))
    mel = torch.matmul(basis, mag)
    return torch.log(torch.clamp(mel, min=1e-5)), torch.linalg.vector_norm(mag, dim=-2)


def char_features(wav, duration, n_fft=1024, hop=256, n_mels=80, sr=22050, fmin=0.0, fmax=8000.0):
    """Preprocessor._process feature steps (scripts/preprocessor/preprocessor.py:386-403) and
    _get_kurtosis (:339-357): (mel (sum d, 80), char energy, char kurtosis)."""
    wav = torch.clip(torch.as_tensor(np.asarray(wav, np.float32)), -1, 1)
    logmel, energy = get_spec(wav, n_fft, hop, n_fft, n_mels, sr, fmin, fmax)
    d = [int(x) for x in duration]
    T = sum(d)
    mel = logmel[:, :T].numpy().T
    e = energy[:T].numpy().copy()
    pos = 0
    for i, di in enumerate(d):
        e[i] = np.mean(e[pos:pos + di]) if di > 0 else 0
        pos += di
    e = e[:len(d)]
    eps = 1e-8
    power = magnitude(wav, n_fft, hop, n_fft) ** 2
    dd = [0] + d
    kurt = np.zeros(len(d))
    for i in range(len(d)):
        spec = power[:, sum(dd[:i + 1]): sum(dd[:i + 2])]
        gamma = torch.log(torch.mean(spec) + eps) - torch.mean(torch.log(spec + eps))
        eta = (3 - gamma + torch.sqrt((gamma - 3) ** 2 + 24 * gamma)) / (12 * gamma)
        kurt[i] = (eta + 2) * (eta + 3) / (eta * (eta + 1) + eps)
    return mel, e, kurt
