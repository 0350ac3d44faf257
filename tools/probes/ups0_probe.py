"""ups0 (ConvTranspose1d 512 -> 256, k 16, s 8) at B = 32 x 512 frames on the tiled polyphase conv:
role-split staging (conv_cfg 0, default) vs the plain 256 x 256 tile (conv_cfg 6); bit-identity and
time.  Usage: python tools/probes/ups0_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402
from ups_probe import t_us  # noqa: E402


def main():
    Ci, Cout, T, u, k = 512, 256, 512, 8, 16
    for B in (32, 64):
        xb = torch.randn(B, T, Ci, device="cuda").to(torch.bfloat16)
        wb = ops.pack_conv_weight(torch.randn(Ci, Cout, k, device="cuda") * 0.05, torch.bfloat16, transposed_stride=u)
        bb = torch.randn(Cout, device="cuda")
        out = torch.empty(B, u * T, Cout, device="cuda", dtype=torch.bfloat16)
        line, ref = f"ups0 B={B}:", None
        for c in (6, 0, 6, 0):
            _lib.lib().vo_tune(b"conv_cfg", c)
            f = lambda: ops.conv1d(xb, wb, bb, Co=u * Cout, K=2, pad=1, pre_act=ops.ACT_LRELU, pre_slope=0.1,  # noqa: E731
                                   transposed=dict(stride=u, pad=(k - u) // 2, cout=Cout), out=out)
            y = f().clone()
            ref = y if ref is None else ref
            us = t_us(f)
            fl = 2.0 * B * (T + 1) * Ci * 2 * u * Cout
            line += f" [conv_cfg {c}] {us:.1f} us {fl / us / 1e6:.0f} TF/s{'' if torch.equal(y, ref) else ' MISMATCH'}"
        _lib.lib().vo_tune(b"conv_cfg", 0)
        print(line, flush=True)


if __name__ == "__main__":
    main()
