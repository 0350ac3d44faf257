"""Latency of the small convs of the inference step: VFE bridge (fp32 2448 -> 256 on 384 rows)
through vo_conv1d vs torch (hipBLASLt) addmm; the Co = 80 convs (PostNet last, mel_linear) by
gen_cfg tile."""
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


x = torch.randn(1, 384, 2448, device="cuda")
w = torch.randn(256, 2448, device="cuda") * 0.02
b = torch.randn(256, device="cuda")
wp = ops.pack_conv_weight(w[:, :, None], torch.float32)
print("vfe bridge vo_conv1d fp32: %.1f us" % t_us(lambda: ops.conv1d(x, wp, b, Co=256, K=1, post_act=ops.ACT_RELU,
                                                                   compute_dtype=torch.float32)))
print("vfe bridge torch addmm fp32: %.1f us" % t_us(lambda: torch.relu(torch.addmm(b, x[0], w.t()))))
for Ci, Co, K in ((512, 80, 5), (256, 80, 1), (80, 512, 5), (80, 512, 7)):
    xb = torch.randn(32, 512, Ci, device="cuda").to(torch.bfloat16)
    wb = ops.pack_conv_weight(torch.randn(Co, Ci, K, device="cuda") * 0.02, torch.bfloat16)
    bb = torch.randn(Co, device="cuda")
    line = f"Ci={Ci} Co={Co} K={K}:"
    for c in (0, 1, 6, 7):
        _lib.lib().vo_tune(b"gen_cfg", c)
        line += f" [{c}] {t_us(lambda: ops.conv1d(xb, wb, bb, Co=Co, K=K, pad=(K - 1) // 2)):.1f} us"
    _lib.lib().vo_tune(b"gen_cfg", 0)
    print(line, flush=True)
