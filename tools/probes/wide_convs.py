"""Per-launch time of the wide bf16 convs of the inference step that share the 256 x 256 tile:
decoder FFN w_1 (256 -> 1024, k9) and fused q/k/v (256 -> 768, k1) at B*T = 16384 rows, and the
polyphase upsamplers ups0 (512 -> 256, k16 s8; 16384 input steps) and ups1 (256 -> 128, k16 s8;
131072 input steps), by gen_cfg tile (0 = shipped, 1 = 128 x 128, 9 = 128 x 256, 10 = 256 x 128).
Usage: python tools/probes/wide_convs.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402
from ups_probe import t_us  # noqa: E402

CFGS = (0, 1, 9, 10)
for Ci, Co, K in ((256, 1024, 9), (256, 768, 1)):
    xb = torch.randn(32, 512, Ci, device="cuda").to(torch.bfloat16)
    wb = ops.pack_conv_weight(torch.randn(Co, Ci, K, device="cuda") * 0.02, torch.bfloat16)
    bb = torch.randn(Co, device="cuda")
    line = f"Ci={Ci} Co={Co} K={K}:"
    for c in CFGS:
        _lib.lib().vo_tune(b"gen_cfg", c)
        us = t_us(lambda: ops.conv1d(xb, wb, bb, Co=Co, K=K, pad=(K - 1) // 2, post_act=ops.ACT_RELU))
        line += f" [{c}] {us:.1f} us {2 * 32 * 512 * Co * Ci * K / us / 1e6:.0f} TF/s"
    _lib.lib().vo_tune(b"gen_cfg", 0)
    print(line, flush=True)

for Ci, Cout, T in ((512, 256, 512), (256, 128, 4096)):
    u, k = 8, 16
    xb = torch.randn(32, T, Ci, device="cuda").to(torch.bfloat16)
    wb = ops.pack_conv_weight(torch.randn(Ci, Cout, k, device="cuda") * 0.02, torch.bfloat16, transposed_stride=u)
    bb = torch.randn(Cout, device="cuda")
    line = f"ConvT Ci={Ci} Cout={Cout} T={T}:"
    ref = None
    for c in CFGS:
        _lib.lib().vo_tune(b"gen_cfg", c)
        f = lambda: ops.conv1d(xb, wb, bb, Co=u * Cout, K=2, pad=1, pre_act=ops.ACT_LRELU, pre_slope=0.1,  # noqa: E731
                               transposed=dict(stride=u, pad=(k - u) // 2, cout=Cout))
        y = f()
        ref = y if ref is None else ref
        us = t_us(f)
        tf = 2 * 32 * (T + 1) * u * Cout * Ci * 2 / us / 1e6
        gbs = (xb.numel() + y.numel()) * 2 / us / 1e3
        line += f" [{c}] {us:.1f} us {tf:.0f} TF/s {gbs:.0f} GB/s{'' if torch.equal(y, ref) else ' MISMATCH'}"
    _lib.lib().vo_tune(b"gen_cfg", 0)
    print(line, flush=True)
