#!/usr/bin/env python3
"""Fused ResBlock pair vs two conv launches on the MRF stage-2/3 shapes (B=32), one process."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402


def t_ms(fn, n=10):
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
    B = 32
    for C, T in ((128, 32768), (64, 65536), (32, 131072)):
        for k, d in ((3, 1), (7, 3), (11, 5)):
            x = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
            w1 = ops.pack_conv_weight(torch.randn(C, C, k, device="cuda") / (C * k) ** 0.5, torch.bfloat16)
            w2 = ops.pack_conv_weight(torch.randn(C, C, k, device="cuda") / (C * k) ** 0.5, torch.bfloat16)
            b = torch.zeros(C, device="cuda")
            y = torch.empty_like(x)
            t = torch.empty_like(x)
            var = {128: 2, 64: 3, 32: 4}[C]

            def unfused():
                ops.conv1d(x, w1, b, Co=C, K=k, dil=d, pad=d * (k - 1) // 2, pre_act=ops.ACT_LRELU, pre_slope=0.1,
                           post_act=ops.ACT_LRELU, post_slope=0.1, out=t, variant=var)
                ops.conv1d(t, w2, b, Co=C, K=k, pad=(k - 1) // 2, res1=x, out=y, variant=var)

            fused = lambda: ops.resblock_pair(x, w1, b, w2, b, k, d, 0.1, out=y)  # noqa: E731
            fl = 2 * 2.0 * B * T * C * C * k
            a = t_ms(unfused)
            line = f"C={C} k={k} d={d}: unfused {a:.4f} ms ({fl / a / 1e9:.0f} TF/s)"
            for cfg in {128: (0, 6), 64: (0,), 32: (0,)}[C]:
                _lib.lib().vo_tune(b"pair_cfg", cfg)
                f = t_ms(fused)
                line += f"  fused[{cfg}] {f:.4f} ms ({fl / f / 1e9:.0f} TF/s)"
            _lib.lib().vo_tune(b"pair_cfg", 0)
            print(line, flush=True)


if __name__ == "__main__":
    main()
