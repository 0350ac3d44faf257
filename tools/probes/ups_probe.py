"""Per-launch time of the bf16 polyphase upsamplers ups2 (128 -> 64) and ups3 (64 -> 32), k4 s2,
at C3-like B = 32 x 512 frames: streaming kernel (ups_cfg 0, upsample.hip) vs the generic tiled
conv (ups_cfg 1).  Usage: python tools/probes/ups_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402


def t_us(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    for Ci, Cout, T, u, k in ((256, 128, 4096, 8, 16), (128, 64, 32768, 2, 4), (64, 32, 65536, 2, 4)):
        xb = torch.randn(32, T, Ci, device="cuda").to(torch.bfloat16)
        wb = ops.pack_conv_weight(torch.randn(Ci, Cout, k, device="cuda") * 0.05, torch.bfloat16, transposed_stride=u)
        bb = torch.randn(Cout, device="cuda")
        out = torch.empty(32, u * T, Cout, device="cuda", dtype=torch.bfloat16)
        line = f"ConvT Ci={Ci} Cout={Cout} T={T}:"
        ref = None
        for c in ((0, 5, 1) if Ci == 256 else (0, 2, 3, 1)):
            _lib.lib().vo_tune(b"ups_cfg", c)
            f = lambda: ops.conv1d(xb, wb, bb, Co=u * Cout, K=2, pad=1, pre_act=ops.ACT_LRELU, pre_slope=0.1,  # noqa: E731
                                   transposed=dict(stride=u, pad=(k - u) // 2, cout=Cout), out=out)
            y = f().clone()
            ref = y if ref is None else ref
            same = bool(torch.equal(y, ref))
            us = t_us(f)
            gbs = (xb.numel() + y.numel()) * 2 / us / 1e3
            line += f" [ups_cfg {c}] {us:.1f} us {gbs:.0f} GB/s ({gbs / 8000:.2f} of 8 TB/s){'' if same else ' MISMATCH'}"
        _lib.lib().vo_tune(b"ups_cfg", 0)
        print(line, flush=True)


if __name__ == "__main__":
    main()
