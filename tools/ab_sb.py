#!/usr/bin/env python3
"""A/B of kernel variants on the MRF shapes (B=32): each variant's output is compared with
config 0's (same MFMA accumulation order -> bit-identical unless the tiling changes).

    python tools/ab_sb.py [pair|conv] [cfg ...]
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


def run(kind, C, T, cfgs, key):
    B = 32
    for k, d in ((3, 1), (7, 3), (11, 5)):
        torch.manual_seed(k)
        x = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
        w1 = ops.pack_conv_weight(torch.randn(C, C, k, device="cuda") / (C * k) ** 0.5, torch.bfloat16)
        w2 = ops.pack_conv_weight(torch.randn(C, C, k, device="cuda") / (C * k) ** 0.5, torch.bfloat16)
        b = torch.randn(C, device="cuda") * 0.1
        y = torch.empty_like(x)
        if kind == "pair":
            f = lambda: ops.resblock_pair(x, w1, b, w2, b, k, d, 0.1, out=y)  # noqa: E731
            fl = 2 * 2.0 * B * T * C * C * k
        else:
            f = lambda: ops.conv1d(x, w1, b, Co=C, K=k, dil=d, pad=d * (k - 1) // 2,  # noqa: E731
                                   pre_act=ops.ACT_LRELU, pre_slope=0.1, out=y, variant=1)
            fl = 2.0 * B * T * C * C * k
        line = f"{kind} C={C} k={k} d={d}:"
        ref = None
        errs, best = {}, {}
        for cfg in cfgs:
            _lib.lib().vo_tune(key, cfg)
            y.zero_()
            f()
            torch.cuda.synchronize()
            out = y.float().clone()
            if ref is None:
                ref = out
            errs[cfg] = float((out - ref).abs().max())
        for _ in range(3):  # round-robin, best of 3: the clock drifts between configs
            for cfg in cfgs:
                _lib.lib().vo_tune(key, cfg)
                best[cfg] = min(best.get(cfg, 1e9), t_ms(f))
        for cfg in cfgs:
            ms = best[cfg]
            line += f"  [{cfg}] {ms:.4f} ms {fl / ms / 1e9:.0f} TF/s d={errs[cfg]:.1e}"
        _lib.lib().vo_tune(key, 0)
        print(line, flush=True)


def run_gen(cfgs, dt=torch.bfloat16, T=512):
    """decoder / PostNet / upsampler shapes through the generic bf16 path (gen_cfg); with
    dt=float32, T=12: the glyph encoder / variance predictor shapes"""
    B = 32
    shapes = [(256, 1024, 9, 1), (1024, 256, 1, 1), (256, 768, 1, 1), (256, 256, 1, 1), (512, 512, 5, 1),
              (80, 512, 5, 1)] if T > 16 else [(256, 1024, 9, 1), (1024, 256, 1, 1), (256, 768, 1, 1),
                                                 (256, 256, 1, 1), (256, 256, 3, 1)]
    for Ci, Co, k, d in shapes:
        torch.manual_seed(k)
        x = torch.randn(B, T, Ci, device="cuda").to(dt)
        w = ops.pack_conv_weight(torch.randn(Co, Ci, k, device="cuda") / (Ci * k) ** 0.5, dt)
        b = torch.randn(Co, device="cuda") * 0.1
        y = torch.empty(B, T, Co, device="cuda", dtype=dt)
        f = lambda: ops.conv1d(x, w, b, Co=Co, K=k, dil=d, pad=d * (k - 1) // 2, out=y,  # noqa: E731
                               compute_dtype=dt)
        fl = 2.0 * B * T * Ci * Co * k
        errs, best, ref = {}, {}, None
        for cfg in cfgs:
            _lib.lib().vo_tune(b"gen_cfg", cfg)
            f()
            torch.cuda.synchronize()
            out = y.float().clone()
            ref = out if ref is None else ref
            errs[cfg] = float((out - ref).abs().max())
        for _ in range(3):
            for cfg in cfgs:
                _lib.lib().vo_tune(b"gen_cfg", cfg)
                best[cfg] = min(best.get(cfg, 1e9), t_ms(f))
        line = f"gen Ci={Ci} Co={Co} k={k}:"
        for cfg in cfgs:
            line += f"  [{cfg}] {best[cfg]:.4f} ms {fl / best[cfg] / 1e9:.0f} TF/s d={errs[cfg]:.1e}"
        _lib.lib().vo_tune(b"gen_cfg", 0)
        print(line, flush=True)


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "pair"
    cfgs = [int(c) for c in sys.argv[2:]] or [0]
    if kind == "pair":
        run("pair", 128, 32768, cfgs, b"pair_cfg")
    elif kind == "pair64":
        run("pair", 64, 65536, cfgs, b"pair_cfg")
    elif kind == "pair32":
        run("pair", 32, 131072, cfgs, b"pair_cfg")
    elif kind == "gen":
        run_gen(cfgs)
    elif kind == "genf32":
        run_gen(cfgs, torch.float32, 12)
    else:
        run("conv", 256, 4096, cfgs, b"conv_cfg")


if __name__ == "__main__":
    main()
