#!/usr/bin/env python3
"""Measurement of the SURVEY.md 8(f) rows 2-3 on one MI355X (one JSON line each):

* glyph batch (vo_glyph_batch): a C4 training batch of 48 utterances (12 x group 4) of up to 21
  characters, 24 x 102 px cells -> (B, 1, 24, W) fp32; HBM roofline on the algorithmic bytes
  (uint8 strips in + fp32 out); CPU baseline = the reference's numpy layout (oracle/data.py).
* feature extraction (vo_stft_mel_ex + vo_char_features): 64 utterances of 2 s at 22.05 kHz
  -> mel + character energy + kurtosis; CPU baseline = oracle/mel.char_features (torch-CPU).

    python tools/bench_aux.py
"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0


def timed(fn, n):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n / 1e3


def glyph():
    from oracle import data as O
    from visual_onoma_to_wave_amd import ops
    rng = np.random.default_rng(0)
    B, H, cell = 48, 24, 102
    widths = [rng.integers(30, cell + 1, int(rng.integers(4, 22))) for _ in range(B)]
    strips = [rng.integers(0, 256, (H, int(w.sum()))).astype(np.uint8) for w in widths]
    dev = torch.device("cuda")
    # device-resident strips: time the layout kernel itself (the host packs / uploads once per batch)
    out = ops.glyph_batch(strips, widths, cell, 0, dev)
    n_in = sum(s.size for s in strips)
    t_e2e = timed(lambda: ops.glyph_batch(strips, widths, cell, 0, dev), 20)  # incl. pack + H2D
    # kernel only: replay with pre-uploaded buffers through the C ABI
    import ctypes
    from visual_onoma_to_wave_amd import _lib
    offs = np.zeros(B, np.int64)
    offs[1:] = np.cumsum([s.size for s in strips])[:-1]
    cw = np.concatenate(widths).astype(np.int32)
    co = np.zeros(B + 1, np.int32)
    co[1:] = np.cumsum([len(w) for w in widths])
    cs = np.concatenate([np.concatenate([[0], np.cumsum(w)[:-1]]) for w in widths]).astype(np.int32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    px, of, iw, cod, csd, cwd = (t(np.concatenate([s.reshape(-1) for s in strips])), t(offs),
                                 t(np.array([s.shape[1] for s in strips], np.int32)), t(co), t(cs), t(cw))
    W = out.shape[-1]
    P = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def k():
        _lib.lib().vo_glyph_batch(P(px), P(of), P(iw), P(cod), P(csd), P(cwd), B, H, cell, 0, W, P(out), st)
    t_k = timed(k, 200)
    nbytes = n_in + out.numel() * 4
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 2.0:
        O.glyph_batch(strips, widths, cell, 1)
        n += 1
    t_cpu = (time.perf_counter() - t0) / n
    return {"metric": "glyph batch layout (training input pipeline, SURVEY 8(f) row 2)", "unit": "batches/s",
            "value": round(1 / t_k, 1), "e2e_batches_per_s_incl_host_pack_h2d": round(1 / t_e2e, 1),
            "config": {"batch": B, "cell": cell, "height": H, "out_width": W},
            "roofline": {"bound": "hbm", "achieved": round(nbytes / t_k / 1e9, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(nbytes / t_k / 1e9 / HBM_PEAK_GBS, 4),
                         "bytes_per_launch": nbytes, "avg_launch_us": round(t_k * 1e6, 2)},
            "cpu_baseline": {"value": round(1 / t_cpu, 1), "unit": "batches/s", "cores": 1, "kind": "port",
                             "sample": f"{n} batches, oracle/data.py numpy layout"}}


def features():
    from helpers import configs
    from oracle import mel as O
    from visual_onoma_to_wave_amd.preprocessor import FeatureExtractor
    rng = np.random.default_rng(1)
    n_utt, N = 64, 44100
    wavs = [(0.3 * rng.standard_normal(N)).astype(np.float32) for _ in range(n_utt)]
    F = 1 + N // 256
    durs = [np.full(8, (F - 1) // 8) for _ in range(n_utt)]
    fx = FeatureExtractor(configs()[0])
    fx.process(wavs, durs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        fx.process(wavs, durs)
    torch.cuda.synchronize()
    t_gpu = (time.perf_counter() - t0) / reps
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 5.0 and n < n_utt:
        O.char_features(wavs[n], durs[n])
        n += 1
    t_cpu = (time.perf_counter() - t0) / n
    return {"metric": "offline feature extraction (mel + char energy + kurtosis, SURVEY 8(f) row 3)",
            "unit": "utterances/s (2 s @ 22.05 kHz)", "value": round(n_utt / t_gpu, 1),
            "config": {"utterances": n_utt, "samples": N, "frames": F},
            "note": "host-inclusive (numpy in, numpy out per utterance)",
            "cpu_baseline": {"value": round(1 / t_cpu, 1), "unit": "utterances/s", "cores": torch.get_num_threads(),
                             "kind": "port", "sample": f"{n} utterances, oracle/mel.char_features torch-CPU"}}


if __name__ == "__main__":
    print(json.dumps(glyph()))
    print(json.dumps(features()))
