"""Per-call time of the fp32 convs over short utterances (glyph encoder FFT blocks and variance
predictors: B = 32, T_src = 12), as shipped (per-utterance time tiles, split reduction) and with the
batch run as ONE zero-gapped sequence (utterances separated by pad = (K - 1) / 2 zero rows, so a plain
conv over it never mixes utterances).  Round 5: the gapped sequence 78 vs 52 us (w_1 k9) and 24 vs 16 us
(predictor k3); pointwise convs flattened over the batch 33 vs ~10 us (w_2): both dropped.
Usage: python tools/probes/short_convs.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from visual_onoma_to_wave_amd import ops  # noqa: E402


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


B, T = 32, 12
for Ci, Co, K in ((256, 1024, 9), (1024, 256, 1), (256, 768, 1), (256, 256, 1), (256, 256, 3)):
    g = torch.Generator(device="cuda").manual_seed(Ci + Co + K)
    x = torch.randn(B, T, Ci, device="cuda", generator=g)
    w = ops.pack_conv_weight(torch.randn(Co, Ci, K, device="cuda", generator=g) * 0.02, torch.float32)
    b = torch.randn(Co, device="cuda", generator=g)
    pad = (K - 1) // 2
    f0 = lambda: ops.conv1d(x, w, b, Co=Co, K=K, pad=pad, compute_dtype=torch.float32)  # noqa: E731
    y0 = f0()
    line = f"Ci={Ci} Co={Co} K={K}: shipped {t_us(f0):.1f} us"
    if K > 1:
        L = pad + B * (T + pad)
        xp = torch.zeros(1, L, Ci, device="cuda")
        xp[0, pad:].view(B, T + pad, Ci)[:, :T] = x
        f1 = lambda: ops.conv1d(xp, w, b, Co=Co, K=K, pad=pad, compute_dtype=torch.float32)  # noqa: E731
        yp = f1()
        y1 = yp[0, pad:].view(B, T + pad, Co)[:, :T]
        err = float((y1 - y0).abs().max())
        line += f" | gapped sequence {t_us(f1):.1f} us (max diff {err:.1e})"
    print(line, flush=True)
