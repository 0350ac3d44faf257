"""Per-launch time of the C4 decoder's widest bf16 input-gradient conv (FFN w_1's dgrad: 1024 -> 256
channels, K = 9, B*T = 16384 rows) and the forward 1x1 / k9 convs at that size, by gen_cfg tile:
0 = default, 9 = 128 x 256, 10 = 256 x 128, 11 = 64 x 128, 12 = 256 x 256 (co x rows).
Usage: python tools/probes/dgrad_tiles.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402


def t_us(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for Ci, Co, K in ((1024, 256, 9), (256, 1024, 9), (1024, 256, 1), (256, 256, 1), (512, 512, 5)):
    xb = torch.randn(32, 512, Ci, device="cuda").to(torch.bfloat16)
    wb = ops.pack_conv_weight(torch.randn(Co, Ci, K, device="cuda") * 0.02, torch.bfloat16)
    line = f"Ci={Ci} Co={Co} K={K}:"
    ref = None
    for c in (0, 9, 10, 11, 12):
        _lib.lib().vo_tune(b"gen_cfg", c)
        y = ops.conv1d(xb, wb, None, Co=Co, K=K, pad=(K - 1) // 2)
        ref = y if ref is None else ref
        same = bool(torch.equal(y, ref))
        us = t_us(lambda: ops.conv1d(xb, wb, None, Co=Co, K=K, pad=(K - 1) // 2))
        tf = 2 * 32 * 512 * Co * Ci * K / us / 1e6
        line += f" [{c}] {us:.1f} us {tf:.0f} TF/s{'' if same else ' MISMATCH'}"
    _lib.lib().vo_tune(b"gen_cfg", 0)
    print(line, flush=True)
