#!/usr/bin/env python3
"""A/B of vo_conv1d_wgrad settings (wgrad_cfg) on the HiFi-GAN V1 training shapes (B = 16,
8192-sample segments): generator MRF stages, upsampler (transposed form), MPD / MSD layers.

    python tools/ab_wgrad.py [cfg ...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402

# (name, rows B*T_A, M, N, K, S, dil, pad, T_A, T_B, groups)
SHAPES = [
    ("s0 C256 k11 d5", 16, 256, 256, 11, 1, 5, 25, 256, 256, 1),
    ("s1 C128 k7 d3", 16, 128, 128, 7, 1, 3, 9, 2048, 2048, 1),
    ("s2 C64 k11 d5", 16, 64, 64, 11, 1, 5, 25, 4096, 4096, 1),
    ("s3 C32 k3 d1", 16, 32, 32, 3, 1, 1, 1, 8192, 8192, 1),
    ("mpd 512->1024 k5 s3", 32, 1024, 512, 5, 3, 1, 2, 365, 1093, 1),
    ("msd 1024 g16 k41 s4", 32, 64, 64, 41, 4, 1, 20, 128, 512, 16),
    ("msd 256->512 g16 k41 s4", 32, 32, 16, 41, 4, 1, 20, 2048, 8192, 16),
]


def t_ms(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    cfgs = [int(c) for c in sys.argv[1:]] or [0]
    for name, B, M, N, K, S, dil, pad, T_A, T_B, g in SHAPES:
        torch.manual_seed(0)
        a = torch.randn(B, T_A, M * g, device="cuda").to(torch.bfloat16)
        b = torch.randn(B, T_B, N * g, device="cuda").to(torch.bfloat16)
        f = lambda: ops.conv1d_wgrad(a, b, K, S=S, dil=dil, pad=pad, pre_b=0.1, groups=g)  # noqa: E731
        fl = 2.0 * B * T_A * M * N * g * K
        ref, best, errs = None, {}, {}
        for c in cfgs:
            _lib.lib().vo_tune(b"wgrad_cfg", c)
            out = f()
            torch.cuda.synchronize()
            ref = out if ref is None else ref
            errs[c] = float((out - ref).abs().max() / ref.abs().max())
        for _ in range(3):
            for c in cfgs:
                _lib.lib().vo_tune(b"wgrad_cfg", c)
                best[c] = min(best.get(c, 1e9), t_ms(f))
        _lib.lib().vo_tune(b"wgrad_cfg", 0)
        print(f"{name}:" + "".join(f"  [{c}] {best[c]:.4f} ms {fl / best[c] / 1e9:.0f} TF/s d={errs[c]:.1e}"
                                    for c in cfgs), flush=True)


if __name__ == "__main__":
    main()
