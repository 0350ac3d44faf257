#!/usr/bin/env python3
"""vo_resblock3 (one launch per k = 3 ResBlock) against three vo_resblock_pair launches on the
MRF stage shapes (B = 32), with the MRF accumulator, plus HBM bytes / TF/s of each.

    python tools/ab_rb3.py [rb3_cfg ...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402


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
    B, dils = 32, (1, 3, 5)
    for C, T in ((128, 32768), (64, 65536), (32, 131072)):
        torch.manual_seed(C)
        x = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
        acc = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
        p1 = [ops.pack_conv_weight(torch.randn(C, C, 3, device="cuda") / (3 * C) ** 0.5, torch.bfloat16) for _ in dils]
        p2 = [ops.pack_conv_weight(torch.randn(C, C, 3, device="cuda") / (3 * C) ** 0.5, torch.bfloat16) for _ in dils]
        b1 = [torch.randn(C, device="cuda") * 0.1 for _ in dils]
        b2 = [torch.randn(C, device="cuda") * 0.1 for _ in dils]
        y = torch.empty_like(x)

        def pairs():
            cur = x
            for s, d in enumerate(dils):
                cur = ops.resblock_pair(cur, p1[s], b1[s], p2[s], b2[s], 3, d, 0.1, out=y if s == 2 else None,
                                        out_scale=1.0 / 3 if s == 2 else 1.0, acc=acc if s == 2 else None)
        fl = 3 * 2 * 2.0 * B * T * C * C * 3
        line = f"C={C} T={T}: 3 pairs {t_ms(pairs):.4f} ms"
        ref = None
        for c in cfgs:
            _lib.lib().vo_tune(b"rb3_cfg", c)
            ops.resblock3(x, p1, b1, p2, b2, dils, 0.1, out=y, out_scale=1.0 / 3, acc=acc)
            if ref is None:
                ref = y.clone()
            same = "==" if torch.equal(y, ref) else "DIFF"
            ms = t_ms(lambda: ops.resblock3(x, p1, b1, p2, b2, dils, 0.1, out=y, out_scale=1.0 / 3, acc=acc))
            line += f" | rb3[{c}]{same} {ms:.4f} ms {fl / ms / 1e9:.0f} TF/s {4 * x.numel() * 2 / ms / 1e6:.0f} GB/s(4 passes)"
        _lib.lib().vo_tune(b"rb3_cfg", 0)
        print(line, flush=True)


if __name__ == "__main__":
    main()
