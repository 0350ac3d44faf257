#!/usr/bin/env python3
"""MRF stage-0 conv (C = 256, T = 4096, vo_conv1d variant 1) time against the batch size: separates
the per-launch / per-tile fixed cost from the per-tap cost.  Prints ms and TF/s per (k, B)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
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
    C, T = 256, 4096
    cfgs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "0").split(",")]
    res = os.environ.get("S0_RES", "1") == "1"  # S0_RES=0: no residual operand (the ResBlock's c1)
    Bs = [int(b) for b in os.environ.get("S0_B", "8,16,32,64").split(",")]
    for k, d in ((3, 1), (7, 3), (11, 5)):
        w = ops.pack_conv_weight(torch.randn(C, C, k, device="cuda") / (C * k) ** 0.5, torch.bfloat16)
        b = torch.zeros(C, device="cuda")
        for B in Bs:
            x = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
            y = torch.empty_like(x)
            fl = 2.0 * B * T * C * C * k
            line = f"k={k} d={d} B={B}:"
            ref = None
            for cfg in cfgs:
                _lib.lib().vo_tune(b"conv_cfg", cfg)
                f = lambda: ops.conv1d(x, w, b, Co=C, K=k, dil=d, pad=d * (k - 1) // 2,  # noqa: E731
                                       pre_act=ops.ACT_LRELU, pre_slope=0.1, out=y, res1=x if res else None, variant=1)
                ms = t_ms(f)
                f()
                torch.cuda.synchronize()
                err = 0.0 if ref is None else float((y.float() - ref).abs().max())
                ref = y.float().clone() if ref is None else ref
                line += f"  [{cfg}] {ms:.4f} ms {fl / ms / 1e9:.0f} TF/s (diff {err:.1e})"
            _lib.lib().vo_tune(b"conv_cfg", 0)
            print(line, flush=True)


if __name__ == "__main__":
    main()
