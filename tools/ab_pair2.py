#!/usr/bin/env python3
"""A/B of vo_resblock_pair kernel configurations (pair_cfg) on the bench's MRF shapes (B=32, MRF
accumulate on), interleaved rounds in one process; prints ms per launch, TF/s and the max |diff|
against pair_cfg 0.

    python tools/ab_pair2.py "128:0,20,21" "64:0,20,21"
    python tools/ab_pair2.py "rb3:128,64,32"          # the fused k = 3 ResBlock (vo_resblock3)
    AB_RB3_CFG=0,4 python tools/ab_pair2.py "rb3:128"  # rb3_cfg values (interleaved)

Set VO_LIB_PATH to time another build of the library (tools/ab_libs.sh runs two builds).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402

T_OF = {128: 32768, 64: 65536, 32: 131072}


def timed(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    B = int(os.environ.get("AB_B", "32"))
    for spec in sys.argv[1:]:
        if spec.startswith("rb3:"):
            for C in [int(c) for c in spec[4:].split(",")]:
                rb3(B, C)
            continue
        C, cfgs = spec.split(":")
        C, cfgs = int(C), [int(c) for c in cfgs.split(",")]
        T = T_OF[C]
        for k, d in ((7, 3), (7, 5), (11, 1), (11, 5)):
            g = torch.Generator(device="cuda").manual_seed(k * 10 + d)
            x = torch.randn(B, T, C, device="cuda", generator=g).to(torch.bfloat16)
            acc0 = torch.randn(B, T, C, device="cuda", generator=g).to(torch.bfloat16)
            w1 = ops.pack_conv_weight(torch.randn(C, C, k, device="cuda", generator=g) / (C * k) ** 0.5, torch.bfloat16)
            w2 = ops.pack_conv_weight(torch.randn(C, C, k, device="cuda", generator=g) / (C * k) ** 0.5, torch.bfloat16)
            b = torch.randn(C, device="cuda", generator=g) * 0.1
            y = acc0.clone()
            fl = 2 * 2.0 * B * T * C * C * k
            outs, times = {}, {c: [] for c in cfgs}
            for c in cfgs:  # correctness (one launch from the same accumulator)
                _lib.lib().vo_tune(b"pair_cfg", c)
                o = acc0.clone()
                ops.resblock_pair(x, w1, b, w2, b, k, d, 0.1, out=o, out_scale=1.0 / 3, acc=o)
                outs[c] = o.float()
            for _ in range(3):  # interleaved timing rounds (y accumulates: values irrelevant)
                for c in cfgs:
                    _lib.lib().vo_tune(b"pair_cfg", c)
                    fn = lambda: ops.resblock_pair(x, w1, b, w2, b, k, d, 0.1, out=y, out_scale=1.0 / 3,  # noqa: E731
                                                   acc=y)
                    fn()
                    times[c].append(timed(fn, 10))
            _lib.lib().vo_tune(b"pair_cfg", 0)
            line = f"C={C} k={k} d={d}:"
            for c in cfgs:
                t = min(times[c])
                diff = float((outs[c] - outs[cfgs[0]]).abs().max())
                line += f"  [{c}] {t:.4f} ms {fl / t / 1e9:.0f} TF/s diff {diff:.1e}"
            print(line, flush=True)


def rb3(B, C):
    T = T_OF[C]
    g = torch.Generator(device="cuda").manual_seed(C)
    x = torch.randn(B, T, C, device="cuda", generator=g).to(torch.bfloat16)
    acc0 = torch.randn(B, T, C, device="cuda", generator=g).to(torch.bfloat16)
    w1 = [ops.pack_conv_weight(torch.randn(C, C, 3, device="cuda", generator=g) / (C * 3) ** 0.5, torch.bfloat16)
          for _ in range(3)]
    w2 = [ops.pack_conv_weight(torch.randn(C, C, 3, device="cuda", generator=g) / (C * 3) ** 0.5, torch.bfloat16)
          for _ in range(3)]
    b = [torch.randn(C, device="cuda", generator=g) * 0.1 for _ in range(3)]
    fl = 3 * 2 * 2.0 * B * T * C * C * 3
    for cfg in [int(c) for c in os.environ.get("AB_RB3_CFG", "0").split(",")]:
        _lib.lib().vo_tune(b"rb3_cfg", cfg)
        o = acc0.clone()
        ops.resblock3(x, w1, b, w2, b, (1, 3, 5), 0.1, out=o, out_scale=1.0 / 3, acc=o)
        chk = float(o.float().abs().sum())
        y = acc0.clone()
        fn = lambda: ops.resblock3(x, w1, b, w2, b, (1, 3, 5), 0.1, out=y, out_scale=1.0 / 3, acc=y)  # noqa: E731
        fn()
        t = min(timed(fn, 10) for _ in range(3))
        print(f"rb3 C={C} [{cfg}]: {t:.4f} ms {fl / t / 1e9:.0f} TF/s checksum {chk:.6e}", flush=True)
    _lib.lib().vo_tune(b"rb3_cfg", 0)


if __name__ == "__main__":
    main()
