"""Mel / STFT front-end (row a21).

Pinned (round 3): the STFT magnitude, its log compression and the Tacotron mel composition
(basis product, ``dynamic_range_compression``, energy) against the reference's OWN code --
``scripts/audio/stft.py:52-81`` ``STFT.transform`` and ``:159-178`` ``TacotronSTFT.mel_spectrogram``,
``audio_processing.py:85-91`` -- run on CPU by ``tests/golden/make_goldens.py stft``
(goldens ``stft_ref_22050`` / ``stft_ref_9001``): the oracle (CPU) and the HIP kernels (GPU)
are both checked against them, magnitude rel-L2 <= 1e-5 (fp32).
PARITY-UNPINNED: the mel filterbanks themselves (torchaudio ``MelScale`` and
``librosa.filters.mel`` are not installed and no reference file holds their outputs): the
oracle restates their published algorithms and is cross-checked here against an independent
float64 DFT; the HIP kernel is checked against the oracle.

Tolerances: log-mel abs error <= 2e-3 where mel >= 1e-3 (fp32 FFT vs fp32 FFT; log amplifies
relative error near the 1e-5 floor), energy rel error <= 1e-4."""

import numpy as np
import pytest
import torch

from oracle import mel as M


def _wav(B, N, seed=0):
    rng = np.random.default_rng(seed)
    t = np.arange(N) / 22050.0
    w = np.zeros((B, N), np.float64)
    for b in range(B):
        for f in rng.uniform(80, 7000, size=5):
            w[b] += rng.uniform(0.05, 0.3) * np.sin(2 * np.pi * f * t + rng.uniform(0, 6.28))
        w[b] += 0.01 * rng.normal(size=N)
    w[:, : N // 10] *= 1.3  # a little clipping at +-1
    return np.clip(w, -1.2, 1.2).astype(np.float32)


def test_oracle_stft_matches_float64_dft():
    wav = _wav(1, 3000)[0]
    n_fft, hop = 1024, 256
    x = np.clip(wav.astype(np.float64), -1, 1)
    xp = np.pad(x, (n_fft // 2, n_fft // 2), mode="reflect")
    win = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n_fft) / n_fft)
    F = 1 + len(x) // hop
    frames = np.stack([xp[f * hop: f * hop + n_fft] * win for f in range(F)])
    mag = np.abs(np.fft.rfft(frames, axis=1)).T  # (513, F)
    fb = M.melscale_fbanks().double().numpy()
    ref = np.log(np.maximum(fb.T @ mag, 1e-5))
    logmel, energy = M.get_spec(torch.from_numpy(wav))
    assert logmel.shape == (80, F)
    np.testing.assert_allclose(logmel.numpy(), ref, atol=2e-3)
    np.testing.assert_allclose(energy.numpy(), np.linalg.norm(mag, axis=0), rtol=1e-4)


def test_librosa_basis_properties():
    w = M.librosa_mel(22050, 1024, 80, 0.0, 8000.0)
    assert w.shape == (80, 513) and (w >= 0).all()
    # slaney normalisation: each filter's area (in Hz) is ~1 (2 / bandwidth * bandwidth / 2)
    freqs = np.linspace(0, 11025, 513)
    area = (w * np.gradient(freqs)[None]).sum(1)
    assert np.allclose(area, 1.0, rtol=0.1)


def _check(mel, energy, ref_mel, ref_e):
    mel, ref_mel = mel.cpu().numpy(), ref_mel.numpy()
    m = ref_mel > np.log(1e-3)
    assert np.abs(mel - ref_mel)[m].max() < 2e-3
    assert np.abs(mel - ref_mel).max() < 5e-2
    np.testing.assert_allclose(energy.cpu().numpy(), ref_e.numpy(), rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("B,N", [(2, 22050), (3, 600), (1, 5 * 22050 + 77)])
def test_get_spec_vs_oracle(B, N):
    from visual_onoma_to_wave_amd.audio import MelSpectrogram
    wav = _wav(B, N, seed=N)
    logmel, energy = MelSpectrogram()(torch.from_numpy(wav).cuda())
    ref = [M.get_spec(torch.from_numpy(w)) for w in wav]
    _check(logmel, energy, torch.stack([r[0] for r in ref]), torch.stack([r[1] for r in ref]))


@pytest.mark.gpu
def test_tacotron_stft_vs_oracle():
    from visual_onoma_to_wave_amd.audio import TacotronSTFT
    wav = np.clip(_wav(2, 12800, seed=3), -1, 1)
    stft = TacotronSTFT(1024, 256, 1024, 80, 22050, 0.0, 8000.0).cuda()
    mel, energy = stft.mel_spectrogram(torch.from_numpy(wav).cuda())
    ref = [M.tacotron_mel(torch.from_numpy(w)) for w in wav]
    _check(mel, energy, torch.stack([r[0] for r in ref]), torch.stack([r[1] for r in ref]))
    assert mel.shape == (2, 80, 51)


# ------------------------------------------------------------- pinned to the reference's STFT code

REF_STFT = ["stft_ref_22050", "stft_ref_9001"]


def _ref(name):
    from helpers import golden
    return golden(name)


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


@pytest.mark.parametrize("name", REF_STFT)
def test_oracle_pinned_to_reference_stft(name):
    """Oracle |STFT| (torch.stft, periodic Hann) == the reference's DFT-basis conv magnitude."""
    g = _ref(name)
    np.testing.assert_allclose(g["window"], torch.hann_window(1024, periodic=True).numpy(), atol=5e-7)
    mag = M.magnitude(torch.from_numpy(g["wav"])).numpy()
    assert mag.shape == g["magnitude"].shape
    assert _rel(mag, g["magnitude"]) < 1e-5
    mel = np.log(np.maximum(np.einsum("mk,bkf->bmf", g["mel_basis"].astype(np.float64), mag), 1e-5))
    ok = g["mel"] > np.log(1e-3)
    assert np.abs(mel - g["mel"])[ok].max() < 2e-3
    np.testing.assert_allclose(np.linalg.norm(mag, axis=1), g["energy"], rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("name", REF_STFT)
def test_stft_magnitude_vs_reference(name):
    """vo_stft_mag (LDS FFT) against STFT.transform's magnitude, and its log compression against
    dynamic_range_compression's."""
    from visual_onoma_to_wave_amd import ops
    g = _ref(name)
    wav = torch.from_numpy(g["wav"]).cuda()
    mag = ops.stft_mag(wav, torch.from_numpy(g["window"]).cuda(), 1024, 256, eps=0.0)
    mag = mag.transpose(1, 2).cpu().numpy()                      # (B, bins, frames) as the reference
    assert mag.shape == g["magnitude"].shape
    assert _rel(mag, g["magnitude"]) < 1e-5
    drc = np.log(np.maximum(mag, 1e-5))
    ok = g["magnitude"] > 1e-3
    assert np.abs(drc - g["log_magnitude"])[ok].max() < 2e-3
    assert np.abs(drc - g["log_magnitude"]).max() < 5e-2


@pytest.mark.gpu
@pytest.mark.parametrize("name", REF_STFT)
def test_tacotron_mel_vs_reference(name):
    """The HIP mel front end with the reference's composition: TacotronSTFT.mel_spectrogram on the
    same mel basis (the basis itself is the oracle's librosa restatement, unpinned)."""
    from visual_onoma_to_wave_amd.audio import MelSpectrogram
    g = _ref(name)
    m = MelSpectrogram(1024, 256, 80, fb=torch.from_numpy(g["mel_basis"]).t().contiguous())
    mel, energy = m(torch.from_numpy(g["wav"]).cuda())
    _check(mel, energy, torch.from_numpy(g["mel"]), torch.from_numpy(g["energy"]))
