"""Per-launch time of the mid-width bf16 convs of the inference step (PostNet 512 -> 512 k5,
conv_pre-like 80 -> 512 k7, PostNet 80 -> 512 k5 at B*T = 16384 rows) by gen_cfg tile:
0 = default (128 x 128), 9 = 128 x 256, 10 = 256 x 128.  Usage: python tools/probes/mid_convs.py"""
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


for Ci, Co, K in ((512, 512, 5), (80, 512, 5), (80, 512, 7), (256, 512, 3)):
    xb = torch.randn(32, 512, Ci, device="cuda").to(torch.bfloat16)
    wb = ops.pack_conv_weight(torch.randn(Co, Ci, K, device="cuda") * 0.02, torch.bfloat16)
    bb = torch.randn(Co, device="cuda")
    line = f"Ci={Ci} Co={Co} K={K}:"
    ref = None
    for c in (0, 9, 10):
        _lib.lib().vo_tune(b"gen_cfg", c)
        y = ops.conv1d(xb, wb, bb, Co=Co, K=K, pad=(K - 1) // 2, post_act=ops.ACT_TANH)
        ref = y if ref is None else ref
        same = bool(torch.equal(y, ref))
        us = t_us(lambda: ops.conv1d(xb, wb, bb, Co=Co, K=K, pad=(K - 1) // 2, post_act=ops.ACT_TANH))
        tf = 2 * 32 * 512 * Co * Ci * K / us / 1e6
        line += f" [{c}] {us:.1f} us {tf:.0f} TF/s{'' if same else ' MISMATCH'}"
    _lib.lib().vo_tune(b"gen_cfg", 0)
    print(line, flush=True)

# HiFi-GAN upsamplers ups2 (128 -> 64, k4 s2) and ups3 (64 -> 32, k4 s2) at C3-like B = 32 x 512
# frames (polyphase ConvTranspose1d: Co = s * C_out, K = 2), pre-lrelu 0.1 as in the generator
for Ci, Cout, T in ((128, 64, 32768), (64, 32, 65536)):
    u, k = 2, 4
    xb = torch.randn(32, T, Ci, device="cuda").to(torch.bfloat16)
    wt = torch.randn(Ci, Cout, k, device="cuda") * 0.05
    wb = ops.pack_conv_weight(wt, torch.bfloat16, transposed_stride=u)
    bb = torch.randn(Cout, device="cuda")
    line = f"ConvT Ci={Ci} Cout={Cout} T={T}:"
    ref = None
    for c in (0, 6, 7, 9, 10):
        _lib.lib().vo_tune(b"gen_cfg", c)
        f = lambda: ops.conv1d(xb, wb, bb, Co=u * Cout, K=2, pad=1, pre_act=ops.ACT_LRELU, pre_slope=0.1,  # noqa: E731
                               transposed=dict(stride=u, pad=(k - u) // 2, cout=Cout))
        y = f()
        ref = y if ref is None else ref
        same = bool(torch.equal(y, ref))
        us = t_us(f)
        gbs = (xb.numel() + y.numel()) * 2 / us / 1e3
        line += f" [{c}] {us:.1f} us {gbs:.0f} GB/s{'' if same else ' MISMATCH'}"
    _lib.lib().vo_tune(b"gen_cfg", 0)
    print(line, flush=True)
