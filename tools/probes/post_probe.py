"""Per-launch time of the HiFi-GAN conv_post (lrelu 0.01 -> 32 -> 1 k7 -> tanh) at C3 B = 32 x 131072
samples: row-partials kernel (post_cfg 0) vs the LDS-stencil kernel (post_cfg 1).
Usage: python tools/probes/post_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402
from ups_probe import t_us  # noqa: E402

x = torch.randn(32, 131072, 32, device="cuda").to(torch.bfloat16)
w = torch.randn(7, 32, device="cuda") * 0.1
line = "conv_post B=32 T=131072:"
for c in (0, 1):
    _lib.lib().vo_tune(b"post_cfg", c)
    us = t_us(lambda: ops.conv_post(x, w, 0.05, slope=0.01))
    gbs = (x.numel() * 2 + x.shape[0] * x.shape[1] * 4) / us / 1e3
    line += f" [post_cfg {c}] {us:.1f} us {gbs:.0f} GB/s"
_lib.lib().vo_tune(b"post_cfg", 0)
print(line, flush=True)
