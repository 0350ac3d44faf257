"""Offline feature extraction on the GPU vs the CPU oracle restatement of
Preprocessor._get_spec / _process / _get_kurtosis (parity unpinned: torchaudio is absent, see
oracle/mel.py), and the StandardScaler normalisation."""

import numpy as np
import pytest

from helpers import configs, rel_l2


def test_normalize_matches_standard_scaler():
    from sklearn.preprocessing import StandardScaler
    from visual_onoma_to_wave_amd.preprocessor import normalize_features
    rng = np.random.default_rng(0)
    arrays = [rng.standard_normal(int(rng.integers(1, 9))) * 3 + 1 for _ in range(20)]
    sc = StandardScaler()
    for a in arrays:
        sc.partial_fit(a.reshape(-1, 1))
    normed, mean, std, mn, mx = normalize_features(arrays)
    assert abs(mean - sc.mean_[0]) < 1e-12 and abs(std - sc.scale_[0]) < 1e-12
    ref = [(a - sc.mean_[0]) / sc.scale_[0] for a in arrays]
    assert all(np.allclose(x, y) for x, y in zip(normed, ref))
    assert abs(mn - min(r.min() for r in ref)) < 1e-12 and abs(mx - max(r.max() for r in ref)) < 1e-12


@pytest.mark.gpu
def test_char_features_vs_oracle():
    from oracle import mel as O
    from visual_onoma_to_wave_amd.preprocessor import FeatureExtractor
    rng = np.random.default_rng(3)
    fx = FeatureExtractor(configs()[0])
    wavs, durs = [], []
    for n in (12800, 12800, 20000, 7000):
        t = np.arange(n) / 22050.0
        wavs.append((0.4 * np.sin(2 * np.pi * rng.uniform(100, 900) * t) * np.exp(-t) +
                     0.02 * rng.standard_normal(n)).astype(np.float32))
        F = 1 + n // 256
        d = rng.integers(0, 12, 6)
        d = (d * min(1.0, (F - 1) / max(d.sum(), 1))).astype(int)
        durs.append(d)
    out = fx.process(wavs, durs)
    for w, d, o in zip(wavs, durs, out):
        mel, e, k = O.char_features(w, d)
        assert o["mel"].shape == mel.shape
        assert rel_l2(o["mel"], mel) < 1e-5
        assert rel_l2(o["energy"], e) < 1e-5
        fin = np.isfinite(k)
        assert np.array_equal(fin, np.isfinite(o["kurtosis"]))  # zero-length spans: nan both sides
        assert rel_l2(o["kurtosis"][fin], k[fin]) < 1e-4
